// bindings.cpp — pybind11 module `quorum_amd._qmx` (CPU engine, HIP engine, text ops).
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "qmx_env.h"
#include "qmx_engine.h"
#include "qmx_hip.h"
#include "qmx_json.h"
#include <chrono>
#include <condition_variable>
#include <map>
#include <set>
#include <mutex>
#include <thread>

#include "qmx_exchange.h"
#include "qmx_server.h"

namespace py = pybind11;
using namespace qmx;

namespace {

struct PyStreamFilter {
  TagSet ts;
  FilterState fs;
  explicit PyStreamFilter(const std::vector<std::string>& tags) : ts(make_tagset(tags)) {}
  py::bytes feed(const std::string& s) {
    std::string out;
    filter_feed(ts, fs, (const uint8_t*)s.data(), s.size(), out);
    return py::bytes(out);
  }
  py::bytes flush() {
    fs = FilterState();
    return py::bytes("");
  }
};

struct PyStripper {
  TagSet ts;
  explicit PyStripper(const std::vector<std::string>& tags) : ts(make_tagset(tags)) {}
  py::bytes strip(const std::string& s) { return py::bytes(strip_final(ts, (const uint8_t*)s.data(), s.size())); }
};

py::tuple tick_to_py(HostEngine& e, int64_t created, int lane = 0, std::vector<int>* taken = nullptr,
                     bool with_gen = false) {
  std::vector<SlotResult> results;
  std::vector<FinalizeRes> fres;
  {
    py::gil_scoped_release nogil;
    e.tick(created, results, fres, lane, taken);
  }
  py::list r;
  for (auto& x : results) {
    if (with_gen) r.append(py::make_tuple(x.slot, py::bytes(x.data(), x.size()), x.flags, x.gen));
    else r.append(py::make_tuple(x.slot, py::bytes(x.data(), x.size()), x.flags));
  }
  py::list f;
  for (auto& x : fres) {
    if (x.kind == 0) {
      f.append(py::make_tuple(x.id, 0, py::none()));
    } else if (x.kind == 1) {
      f.append(py::make_tuple(x.id, 1, py::bytes(x.event)));
    } else {
      py::list t;
      for (auto& s : x.texts) t.append(py::bytes(s));
      f.append(py::make_tuple(x.id, 2, t));
    }
  }
  return py::make_tuple(r, f);
}

template <class E>
void bind_engine(py::class_<E>& c) {
  c.def("open", [](E& e, int index, bool filter, bool emit) { return e.open(index, filter, emit); },
        py::arg("index"), py::arg("filter"), py::arg("emit"))
      // (slot, generation): a slot's results carry the generation of the open() they belong to
      .def("open_gen", [](E& e, int index, bool filter, bool emit) {
        uint32_t g = 0;
        int slot = e.open(index, filter, emit, &g);
        return py::make_tuple(slot, g);
      })
      .def("feed", [](E& e, int slot, const py::bytes& b) { e.feed(slot, std::string(b)); })
      .def("finish", &E::finish)
      .def("release", &E::release)
      .def("submit_finalize", &E::submit_finalize)
      .def("has_work", &E::has_work)
      .def("tick", [](E& e, int64_t created, int lane) { return tick_to_py(e, created, lane); }, py::arg("created"),
           py::arg("lane") = 0)
      // multi-lane protocol: the slots of an unsettled tick stay busy (skipped by other lanes)
      // until settle(taken) — callers deliver the results first, keeping per-stream order
      .def("tick_unsettled", [](E& e, int64_t created, int lane) {
        std::vector<int> taken;
        py::tuple t = tick_to_py(e, created, lane, &taken);
        return py::make_tuple(t[0], t[1], taken);
      })
      // same, results as (slot, sse, flags, generation)
      .def("tick_unsettled_gen", [](E& e, int64_t created, int lane) {
        std::vector<int> taken;
        py::tuple t = tick_to_py(e, created, lane, &taken, true);
        return py::make_tuple(t[0], t[1], taken);
      })
      .def("settle", [](E& e, const std::vector<int>& taken) {
        py::gil_scoped_release nogil;
        e.settle(taken);
      })
      .def("text", [](E& e, int slot) { return py::bytes(e.text(slot)); })
      // spread owner's shadow slot: its HBM content area (0: none) and a remote final text —
      // `data` None: already written into that area (an RCCL round), bytes: over the mesh
      .def("content_device_ptr", [](E& e, int slot) {
        size_t cap = 0;
        void* p = e.content_device_ptr(slot, &cap);
        return py::make_tuple((uintptr_t)p, cap);
      })
      .def("set_remote_content", [](E& e, int slot, const py::object& data, size_t len) {
        if (data.is_none()) return e.set_remote_content(slot, nullptr, len);
        std::string b = py::cast<std::string>(py::bytes(data));
        e.set_remote_content(slot, &b, b.size());
      })
      .def("stats", &E::stats);
}

}  // namespace

ServerCfg server_cfg_from(const py::dict& d) {
  ServerCfg c;
  auto gs = [&](const char* k, std::string& v) { if (d.contains(k)) v = py::cast<std::string>(d[k]); };
  auto gi = [&](const char* k, int& v) { if (d.contains(k)) v = py::cast<int>(d[k]); };
  auto gd = [&](const char* k, double& v) { if (d.contains(k)) v = py::cast<double>(d[k]); };
  auto gb = [&](const char* k, bool& v) { if (d.contains(k)) v = py::cast<bool>(d[k]); };
  gs("host", c.host); gi("port", c.port); gi("threads", c.threads);
  gs("engine", c.engine); gi("device", c.device); gi("tile", c.tile); gi("max_slots", c.max_slots);
  gi("content_cap", c.content_cap);
  gb("has_iterations_and_strategy", c.has_iterations_and_strategy);
  gd("timeout", c.timeout); gd("total_timeout", c.total_timeout);
  gs("separator", c.separator); gb("hide_intermediate", c.hide_intermediate); gb("hide_final", c.hide_final);
  gb("skip_final", c.skip_final); gb("suppress", c.suppress);
  if (d.contains("tags")) c.tags = py::cast<std::vector<std::string>>(d["tags"]);
  gs("aggregator_name", c.aggregator_name); gs("prompt_template", c.prompt_template);
  gs("intermediate_separator", c.intermediate_separator); gs("query_format", c.query_format);
  gs("source_label_format", c.source_label_format); gb("include_original_query", c.include_original_query);
  gb("include_source_names", c.include_source_names); gs("env_api_key", c.env_api_key);
  gb("documented", c.documented); gb("strip_intermediate", c.strip_intermediate);
  gb("hide_aggregator_think", c.hide_aggregator_think); gb("sources_all", c.sources_all);
  if (d.contains("sources")) c.sources = py::cast<std::vector<std::string>>(d["sources"]);
  gb("api_key_from_env", c.api_key_from_env); gs("openapi_json", c.openapi_json); gs("docs_html", c.docs_html);
  gs("redoc_html", c.redoc_html); gs("oauth2_redirect_html", c.oauth2_redirect_html);
  gb("install_signals", c.install_signals);
  gi("rank", c.rank); gi("world", c.world); gs("placement", c.placement); gs("xchg", c.xchg);
  gs("xchg_addr", c.xchg_addr); gi("xchg_port", c.xchg_port); gi("xchg_bulk_port", c.xchg_bulk_port); gs("xchg_id_file", c.xchg_id_file);
  gi("xchg_round_us", c.xchg_round_us); gi("xchg_eager_bytes", c.xchg_eager_bytes);
  gi("xchg_links", c.xchg_links); gd("xchg_timeout", c.xchg_timeout);
  gd("drain_s", c.drain_s); gs("ready_file", c.ready_file); gb("verify", c.verify); gi("admin_port", c.admin_port);
  gi("shared_engine", c.shared_engine); gi("tick_lanes", c.tick_lanes); gs("tick_mode", c.tick_mode);
  gi("read_pace_us", c.read_pace_us); gi("light_host", c.light_host);
  gs("ca_file", c.ca_file); gb("tls_verify", c.tls_verify);
  if (d.contains("backends")) {
    for (auto item : py::cast<py::list>(d["backends"])) {
      py::dict b = py::cast<py::dict>(item);
      BackendCfg bc;
      bc.name = py::cast<std::string>(b["name"]);
      bc.url = py::cast<std::string>(b["url"]);
      bc.model = py::cast<std::string>(b["model"]);
      bc.has_model_key = py::cast<bool>(b["has_model_key"]);
      bc.valid = py::cast<bool>(b["valid"]);
      bc.host = py::cast<std::string>(b["host"]);
      bc.port = py::cast<int>(b["port"]);
      bc.path = py::cast<std::string>(b["path"]);
      bc.https = py::cast<bool>(b["https"]);
      c.backends.push_back(bc);
    }
  }
  return c;
}

PYBIND11_MODULE(_qmx, m) {
  m.doc() = "qmx native core: CPU stream engine, CDNA4 HIP stream engine, text ops";
  m.def("device_count", []() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
  });
  m.def("classify", [](const py::bytes& b) -> py::tuple {
    std::string s(b);
    EvResult r = classify_event((const uint8_t*)s.data(), (int)s.size());
    if (r.kind != EV_CONTENT) return py::make_tuple(r.kind, py::none());
    int n = json_unescape((const uint8_t*)s.data(), r.str_a, r.str_b, nullptr);
    std::string out(n, '\0');
    json_unescape((const uint8_t*)s.data(), r.str_a, r.str_b, (uint8_t*)&out[0]);
    return py::make_tuple(r.kind, py::bytes(out));
  });
  // the native side never calls getenv on its threads (qmx_env.h): it reads a snapshot
  // taken here, on the calling thread, before any server thread starts
  m.def("env_refresh", &env_refresh,
        "re-snapshot the process environment for the native side (e.g. a rotated OPENAI_API_KEY)");
  m.def("run_server", [](const py::dict& d) {
    ServerCfg c = server_cfg_from(d);
    env_refresh();
    py::gil_scoped_release nogil;
    return run_server(c);
  });
  m.def("server_counters", &server_counters);
  m.def("rccl_unique_id", &rccl_unique_id_hex);
  // Exchange self-test: every rank sends every other rank `rounds` delta messages over the
  // mesh and `rounds` final texts through the bulk plane (RCCL p2p rounds from HBM into HBM
  // sinks with transport=rccl, the mesh with tcp); receivers verify every byte and that each
  // text arrives exactly once.  Options: pace_ms spaces the sends so they form many rounds;
  // min_epochs waits for re-formed communicators; wave2 then sends that many more rounds
  // and reports how many bulk rounds / mesh finals carried them (the re-formed epoch's work).
  m.def("exchange_selftest", [](const py::dict& d, int rounds) {
    env_refresh();  // fault-injection knobs set by the caller
    XOptions o;
    auto gs = [&](const char* k, std::string& v) { if (d.contains(k)) v = py::cast<std::string>(d[k]); };
    auto gi = [&](const char* k, int& v) { if (d.contains(k)) v = py::cast<int>(d[k]); };
    gi("rank", o.rank); gi("world", o.world); gs("transport", o.transport); gs("addr", o.addr);
    gi("port", o.port); gi("device", o.device); gi("bulk_port", o.bulk_port);
    if (d.contains("timeout")) o.timeout_s = py::cast<double>(d["timeout"]);
    const double wait_s = o.timeout_s;  // the whole test; round_timeout: the exchange's own round limit
    if (d.contains("round_timeout")) o.timeout_s = py::cast<double>(d["round_timeout"]);
    const uint64_t min_epochs = d.contains("min_epochs") ? py::cast<uint64_t>(d["min_epochs"]) : 0;
    const double pace_ms = d.contains("pace_ms") ? py::cast<double>(d["pace_ms"]) : 0.0;
    int wave2 = 0;
    gi("wave2", wave2);
    const bool dev = o.transport == "rccl";
    auto payload = [](int r, int src, int dst, int kind) {
      uint64_t x = 1234567 ^ ((uint64_t)r * 1000003ull) ^ ((uint64_t)src * 7919ull) ^ ((uint64_t)dst * 104729ull) ^
                   ((uint64_t)kind << 40);
      size_t n = kind ? 1 + (x % 20000) : 1 + (x % 3000);
      std::string s(n, '\0');
      for (size_t i = 0; i < n; ++i) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        s[i] = (char)(x >> 56);
      }
      return s;
    };
    std::mutex mu;
    std::condition_variable cv;
    std::vector<XMsg> got;
    bool ok = true;
    int bad = 0, dups = 0, n_data = 0, n_bulk = 0, n_sent = 0;
    double data_us = 0, wall = 0;
    uint64_t rounds_done = 0, mesh_finals = 0, epochs = 0, w2_rounds = 0, w2_mesh = 0, rescued = 0, sweeps = 0, early_reports = 0;
    std::string why;
    {
      py::gil_scoped_release nogil;
      std::vector<void*> bufs;
      auto dalloc = [&](size_t n) -> void* {
        void* p = nullptr;
        if (hipSetDevice(o.device) != hipSuccess || hipMalloc(&p, std::max<size_t>(n, 16)) != hipSuccess) return nullptr;
        bufs.push_back(p);
        return p;
      };
      Exchange x(o, 1, [&](int, std::vector<XMsg>&& v) {
        std::lock_guard<std::mutex> g(mu);
        for (auto& m : v) got.push_back(std::move(m));
        cv.notify_all();
      });
      const bool loop1 = o.world == 1;  // one rank: everything goes to itself (RCCL send/recv to self)
      const int total = rounds + wave2;  // message round r: skey r + 1 (wave 2: r >= rounds)
      // sinks first: a bulk that finds no sink is dropped
      std::map<std::pair<int, int>, void*> sinks;
      for (int r = 0; r < total; ++r)
        for (int src = 0; src < o.world; ++src) {
          if (src == o.rank && !loop1) continue;
          const size_t n = payload(r, src, o.rank, 1).size();
          void* p = dev ? dalloc(n) : nullptr;
          // (skey, bi) names ONE stream: bi = src x world + dst, as a session key names one owner
          sinks[{r, src}] = p;
          x.expect_bulk((uint64_t)(r + 1), src * o.world + o.rank, p, n);
        }
      const auto t0 = std::chrono::steady_clock::now();
      auto secs = [&] { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); };
      auto wait_bulk_ready = [&] {
        while (!x.healthy() || (x.bulk_transport() && !x.rccl_active())) {
          if (secs() > wait_s) {
            why = "bulk plane not ready";
            return false;
          }
          std::this_thread::sleep_for(std::chrono::milliseconds(5));
        }
        return true;
      };
      ok = wait_bulk_ready();
      const auto t1 = std::chrono::steady_clock::now();
      std::set<std::pair<uint64_t, int>> seen_bulk, seen_sent;
      auto send_rounds = [&](int r0, int r1) {
        for (int r = r0; r < r1 && ok; ++r) {
          for (int p = 0; p < o.world; ++p) {
            if (p == o.rank && !loop1) continue;
            XMsg m;
            m.type = X_DATA;
            m.dst_rank = p;
            m.src_rank = o.rank;
            m.skey = (uint64_t)(r + 1);
            m.bi = o.rank;
            m.payload = payload(r, o.rank, p, 0);
            x.post(std::move(m));
            std::string b = payload(r, o.rank, p, 1);
            void* src = nullptr;
            if (dev) {
              src = dalloc(b.size());
              if (!src || hipMemcpy(src, b.data(), b.size(), hipMemcpyHostToDevice) != hipSuccess) ok = false;
            }
            XMsg h;
            h.dst_rank = p;
            h.src_rank = o.rank;
            h.skey = (uint64_t)(r + 1);
            h.bi = o.rank * o.world + p;
            h.flags = XF_TEXT;
            x.send_bulk(std::move(h), src, b.size(), [b] { return b; });
          }
          if (pace_ms > 0) std::this_thread::sleep_for(std::chrono::microseconds((int64_t)(pace_ms * 1000)));
        }
      };
      // drain deliveries until `want` of each kind (and the epochs) are in
      auto collect = [&](int want, uint64_t epochs_needed) {
        std::unique_lock<std::mutex> lk(mu);
        while (ok) {
          for (auto& m : got) {
            if (m.type == X_DATA) {
              ++n_data;
              if (m.payload != payload((int)m.skey - 1, m.bi, o.rank, 0)) ++bad;
              if (n_data == want) data_us = 1e6 * std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
            } else if (m.type == X_BULK) {
              ++n_bulk;
              const int src = m.bi / o.world;
              if (!seen_bulk.insert({m.skey, m.bi}).second) ++dups;
              const std::string exp = payload((int)m.skey - 1, src, o.rank, 1);
              std::string have = m.payload;
              if (have.empty() && m.a > 0) {  // RCCL: in the HBM sink
                have.assign((size_t)m.a, '\0');
                void* sp = sinks[{(int)m.skey - 1, src}];
                if (!sp || hipMemcpy(&have[0], sp, have.size(), hipMemcpyDeviceToHost) != hipSuccess) have.clear();
              }
              if (have != exp) ++bad;
            } else if (m.type == X_SENT) {
              ++n_sent;
              if (!seen_sent.insert({m.skey, m.bi}).second) ++dups;
            }
          }
          got.clear();
          if (n_data >= want && n_bulk >= want && n_sent >= want && x.epochs() >= epochs_needed) break;
          if (secs() > wait_s) {
            ok = false;
            why = "deadline: data " + std::to_string(n_data) + " bulk " + std::to_string(n_bulk) + " sent " +
                  std::to_string(n_sent) + " of " + std::to_string(want) + ", epochs " + std::to_string(x.epochs());
            break;
          }
          cv.wait_for(lk, std::chrono::milliseconds(20));
        }
      };
      const int per = loop1 ? 1 : o.world - 1;
      send_rounds(0, rounds);
      collect(rounds * per, min_epochs);
      if (ok && wave2 > 0) {
        // the communicator re-formed: the next texts must travel in its rounds again
        ok = wait_bulk_ready();
        const uint64_t r0 = x.rounds(), m0 = x.mesh_bulk();
        send_rounds(rounds, total);
        collect(total * per, min_epochs);
        // let the peers finish the rounds that carry our receives' counterparts
        w2_rounds = x.rounds() - r0;
        w2_mesh = x.mesh_bulk() - m0;
      }
      wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
      rounds_done = x.rounds();
      mesh_finals = x.mesh_bulk();
      epochs = x.epochs();
      rescued = x.rescued();
      sweeps = x.sweeps();
      early_reports = x.early_reports();
      // linger so peers still waiting for our bytes (or reports) get them, then stop
      std::this_thread::sleep_for(std::chrono::milliseconds(300));
      {  // nothing may arrive twice, not even late
        std::lock_guard<std::mutex> lk(mu);
        for (auto& m : got) {
          if (m.type == X_BULK && !seen_bulk.insert({m.skey, m.bi}).second) ++dups;
          if (m.type == X_SENT && !seen_sent.insert({m.skey, m.bi}).second) ++dups;
        }
        got.clear();
      }
      x.request_stop();
      x.join();
      for (void* p : bufs) hipFree(p);
    }
    return py::dict(py::arg("ok") = ok && bad == 0 && dups == 0, py::arg("bad") = bad, py::arg("dups") = dups,
                    py::arg("rounds") = rounds, py::arg("data") = n_data, py::arg("bulk") = n_bulk,
                    py::arg("sent") = n_sent, py::arg("data_wall_us") = data_us, py::arg("wall_s") = wall,
                    py::arg("rccl_rounds") = rounds_done, py::arg("mesh_finals") = mesh_finals,
                    py::arg("epochs") = epochs, py::arg("wave2_rounds") = w2_rounds,
                    py::arg("wave2_mesh_finals") = w2_mesh, py::arg("rescued") = rescued, py::arg("sweeps") = sweeps, py::arg("early_reports") = early_reports,
                    py::arg("why") = why);
  });
  // One-rank RCCL rounds into given HBM sinks (GPU tests of the owner's remote-final path):
  // each payload is copied to a fresh device buffer and sent with send_bulk into its sink
  // through the exchange's own manifests / epoch / ncclSend+ncclRecv rounds.
  m.def("rccl_deliver", [](const py::dict& d, const py::list& items) {
    XOptions o;
    o.transport = "rccl";
    if (d.contains("port")) o.port = py::cast<int>(d["port"]);
    if (d.contains("device")) o.device = py::cast<int>(d["device"]);
    const double wait_s = d.contains("timeout") ? py::cast<double>(d["timeout"]) : 60.0;
    std::vector<std::pair<uintptr_t, std::string>> v;
    for (auto it : items) {
      py::tuple t = py::cast<py::tuple>(it);
      v.emplace_back(py::cast<uintptr_t>(t[0]), py::cast<std::string>(t[1]));
    }
    int got = 0, sent = 0;
    uint64_t rounds = 0, mesh = 0;
    bool ok = true;
    {
      py::gil_scoped_release nogil;
      std::mutex mu;
      std::condition_variable cv;
      Exchange x(o, 1, [&](int, std::vector<XMsg>&& ms) {
        std::lock_guard<std::mutex> g(mu);
        for (auto& m : ms) {
          if (m.type == X_BULK) ++got;
          if (m.type == X_SENT) ++sent;
        }
        cv.notify_all();
      });
      const auto t0 = std::chrono::steady_clock::now();
      auto secs = [&] { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); };
      while (ok && (!x.healthy() || !x.rccl_active())) {
        if (secs() > wait_s) ok = false;
        std::this_thread::sleep_for(std::chrono::milliseconds(5));
      }
      std::vector<void*> bufs;
      for (size_t i = 0; i < v.size() && ok; ++i) {
        x.expect_bulk(1000 + i, 0, (void*)v[i].first, v[i].second.size());
        void* src = nullptr;
        if (hipSetDevice(o.device) != hipSuccess || hipMalloc(&src, std::max<size_t>(v[i].second.size(), 16)) != hipSuccess ||
            hipMemcpy(src, v[i].second.data(), v[i].second.size(), hipMemcpyHostToDevice) != hipSuccess) {
          ok = false;
          break;
        }
        bufs.push_back(src);
        XMsg h;
        h.skey = 1000 + i;
        h.bi = 0;
        h.flags = XF_TEXT;
        std::string b = v[i].second;
        x.send_bulk(std::move(h), src, b.size(), [b] { return b; });
      }
      {
        std::unique_lock<std::mutex> lk(mu);
        while (ok && (got < (int)v.size() || sent < (int)v.size())) {
          if (secs() > wait_s) ok = false;
          cv.wait_for(lk, std::chrono::milliseconds(20));
        }
      }
      rounds = x.rounds();
      mesh = x.mesh_bulk();
      x.request_stop();
      x.join();
      for (void* p : bufs) hipFree(p);
    }
    return py::dict(py::arg("ok") = ok, py::arg("bulk") = got, py::arg("sent") = sent, py::arg("rounds") = rounds,
                    py::arg("mesh_finals") = mesh);
  });
  m.def("stop_server", &stop_server);
  m.def("json_roundtrip", [](const py::bytes& b) -> py::object {
    std::string s(b), err;
    JVal v;
    if (!json_parse(s.data(), s.size(), v, &err)) return py::make_tuple(false, err);
    return py::make_tuple(true, py::bytes(json_dumps(v)));
  });
  m.def("py_float_repr", &py_float_repr);
  m.def("escape", [](const py::bytes& b) {
    std::string s(b), out;
    escape_append((const uint8_t*)s.data(), s.size(), out);
    return py::bytes(out);
  });
  py::class_<PyStreamFilter>(m, "StreamFilter")
      .def(py::init<const std::vector<std::string>&>())
      .def("feed", &PyStreamFilter::feed)
      .def("flush", &PyStreamFilter::flush);
  py::class_<PyStripper>(m, "Stripper")
      .def(py::init<const std::vector<std::string>&>())
      .def("strip", &PyStripper::strip);
  env_refresh();
  py::class_<CpuEngine> ce(m, "CpuEngine");
  ce.def(py::init([](const std::vector<std::string>& tags) {
    env_refresh();
    return new CpuEngine(tags);
  }));
  bind_engine(ce);
  // the multi-door grid of loop ticks (tests drive several door engines from Python threads)
  py::class_<HipGrid>(m, "HipGrid")
      .def(py::init([](int device, int doors, int wg_per_door, int idle_ms) {
             env_refresh();
             return new HipGrid(device, doors, wg_per_door, idle_ms);
           }),
           py::arg("device"), py::arg("doors"), py::arg("wg_per_door") = 8, py::arg("idle_ms") = 50)
      .def("housekeep", &HipGrid::housekeep)
      .def("stop", &HipGrid::stop, py::call_guard<py::gil_scoped_release>())
      .def("stats", &HipGrid::stats);
  m.def("_free_doors", [](HipEngine& e) { return e.free_doors(); });
  m.def("stream_stats", &stream_stats);
  m.def("stream_probe", &stream_probe, py::arg("n"), py::arg("wait_ms") = 200.0,
        py::call_guard<py::gil_scoped_release>());
  py::class_<HipEngine> he(m, "HipEngine");
  he.def(py::init([](const std::vector<std::string>& tags, int device, int tile, int max_slots, int content_cap,
                      int lanes, HipGrid* grid, int door, int ndoors) {
           env_refresh();
           return new HipEngine(tags, device, tile, max_slots, content_cap, lanes, grid, door, ndoors);
         }),
         py::arg("tags"), py::arg("device"), py::arg("tile_bytes") = 16384, py::arg("max_slots") = 8192,
         py::arg("content_cap") = 1 << 20, py::arg("lanes") = 1, py::arg("grid") = nullptr, py::arg("door") = -1,
         py::arg("ndoors") = 1, py::keep_alive<1, 8>());
  bind_engine(he);
  he.def("kernel_stats", &HipEngine::kernel_stats);
  he.def("debug_poison_results", &HipEngine::debug_poison_results, py::arg("ahead") = 1);
  he.def("set_remote_hbm_direct", &HipEngine::set_remote_hbm_direct, py::arg("on"));
}
