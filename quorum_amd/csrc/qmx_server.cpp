// qmx_server.cpp — native epoll data plane (see qmx_server.h).
#include "qmx_env.h"
#include "qmx_server.h"

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <sys/epoll.h>
#include <sys/syscall.h>
#include <dirent.h>
#include <sys/resource.h>
#include <sys/ioctl.h>
#include <sys/eventfd.h>
#include <sys/prctl.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>

#include <functional>
#include <map>

#include <openssl/err.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>

#include "qmx_engine.h"
#include "qmx_exchange.h"
#include "qmx_hip.h"
#include "qmx_json.h"
#include "qmx_prof.h"

namespace qmx {
namespace {

std::atomic<bool> g_stop{false};
std::atomic<bool> g_drain{false};  // SIGTERM: stop accepting, finish in-flight sessions, then exit
std::atomic<int> g_ready{0};       // io loops with a bound listener
std::atomic<uint64_t> c_requests{0}, c_stream{0}, c_nonstream{0}, c_errors{0}, c_up_fail{0}, c_ticks{0},
    c_tick_slots{0}, c_up_conns{0}, c_clients{0}, c_remote_streams{0},
    c_route_ns{0},  // tick lanes: tick returned -> results handed to the io loops + streams settled
    c_flush_ns{0}, c_flushes{0},  // io loop: oldest upstream bytes of a batch -> handed to the engine
    c_apply_ns{0}, c_applies{0},  // io loop: a tick's results routed -> applied (sent to clients)
    c_link_msgs{0},  // spread: exchange messages sent over the io loops' own links (no mesh thread)
    c_coalesced{0},  // deltas held for their stream's next output instead of a send of their own
    c_hold_ns{0}, c_holds{0},  // a client's held (corked) output: hold start -> released (its added latency)
    c_hold_deadline{0};        // ... released by the coalescing deadline, not by its stream
// failures by class
std::atomic<uint64_t> c_fail_connect{0}, c_fail_timeout{0}, c_fail_status{0}, c_fail_disconnect{0},
    c_fail_protocol{0}, c_stream_aborts{0},
    c_host_path_opens{0};  // HIP engine: streams opened past max_slots (host path)
// spread placement accounting (owner side unless noted): how every remote stream ended, and
// the delta invariant — the owner must have received exactly the deltas the worker sent
// before it applies the stream's final (X_BULK / X_FINAL carry the worker's count in b)
std::atomic<uint64_t> c_sp_failed{0}, c_sp_aborted{0}, c_sp_empty{0}, c_sp_text{0}, c_sp_down{0},
    c_sp_delta_mismatch{0}, c_sp_nodata{0} /* worker: content but no delta sent */,
    c_sp_eager{0} /* worker: final texts sent eagerly over the mesh (no round) */,
    c_sp_release_deferred{0} /* owner: shadow slots released after the round writing them (X_RELEASE) */,
    c_sp_fetched{0} /* worker: final texts copied out of HBM by a tick's finalize item */;
// io loop passes (epoll return -> next wait) longer than 1 ms / 5 ms: anything that blocks a
// loop (a synchronous device copy, a lock held by another thread) shows here
std::atomic<uint64_t> c_loop_pass_1ms{0}, c_loop_pass_5ms{0};
std::atomic<uint64_t> c_paced{0};  // loop passes stretched by read pacing (QMX_READ_PACE_US)
std::atomic<int> g_sp_logs{0};  // rate limit: the first 20 anomalies are logged with their state

// Prometheus histogram with lock-free buckets (seconds)
struct Hist {
  static constexpr int N = 17;
  static constexpr double le[N] = {1e-4, 2.5e-4, 5e-4, 1e-3, 2.5e-3, 5e-3, 1e-2, 2.5e-2, 5e-2,
                                   0.1,  0.25,   0.5,  1.0,  2.5,    5.0,  10.0, 30.0};
  std::atomic<uint64_t> b[N + 1];
  std::atomic<uint64_t> count{0}, sum_ns{0};
  Hist() {
    for (auto& x : b) x.store(0);
  }
  void observe(double sec) {
    int i = 0;
    while (i < N && sec > le[i]) ++i;
    b[i]++;
    count++;
    sum_ns += (uint64_t)(sec * 1e9);
  }
  void render(std::string& m, const std::string& name, const std::string& labels = std::string()) const {
    uint64_t acc = 0;
    const std::string sep = labels.empty() ? "" : ",";
    for (int i = 0; i <= N; ++i) {
      acc += b[i].load();
      char le_s[32];
      if (i < N) snprintf(le_s, sizeof(le_s), "%g", le[i]);
      else snprintf(le_s, sizeof(le_s), "+Inf");
      m += name + "_bucket{" + labels + sep + "le=\"" + le_s + "\"} " + std::to_string(acc) + "\n";
    }
    m += name + "_sum" + (labels.empty() ? "" : "{" + labels + "}") + " " + std::to_string(sum_ns.load() / 1e9) + "\n";
    m += name + "_count" + (labels.empty() ? "" : "{" + labels + "}") + " " + std::to_string(acc) + "\n";
  }
};
constexpr double Hist::le[Hist::N];
// h_engine: a stream's first upstream body bytes handed to the engine -> its final result
// applied in the io loop (queueing for a tick lane + tick(s) + routing back)
Hist h_ttft, h_latency, h_tick, h_upstream_ttfb, h_engine;
// spread placement, owner side: a remote stream's X_OPEN queued -> its first delta applied
// (the mesh hop both ways + the worker's upstream and engine), and its last delta (or open)
// -> its final text applied (the bulk round or mesh transfer of the final)
Hist h_sp_first, h_sp_final;

using Clock = std::chrono::steady_clock;
inline double now_s() { return std::chrono::duration<double>(Clock::now().time_since_epoch()).count(); }
// QMX_* on/off knobs, read once where a loop or engine is built ("0" / "false": off)
inline bool env_flag(const char* name, bool dflt) {
  const char* v = env_get(name);
  if (!v || !*v) return dflt;
  return !(std::strcmp(v, "0") == 0 || std::strcmp(v, "false") == 0);
}

// Header block [p, p+n) ("k: v\r\n" lines, no start line): calls f(lower(trim(k)), trim(v)) per line that
// has a colon, building each key and value string once (no per-line/per-field temporaries).
// ASCII lower case (what tolower does in the C locale, inline: no locale lookup per byte)
inline char alow(unsigned char c) { return (char)(c - 'A' < 26u ? c | 0x20 : c); }
// "\r\n" / "\r\n\r\n" in [p, p+n): memchr for the '\r' (vectorised) and a look at the next
// bytes — glibc's memmem sets up a two-way search per call, which for these 2- and 4-byte
// needles over short HTTP heads and chunk-size lines cost more than the search itself
inline const char* find_crlf(const char* p, size_t n) {
  const char* e = p + n;
  while (p < e) {
    const char* r = (const char*)memchr(p, '\r', (size_t)(e - p));
    if (!r || r + 1 >= e) return nullptr;
    if (r[1] == '\n') return r;
    p = r + 1;
  }
  return nullptr;
}
inline const char* find_crlfcrlf(const char* p, size_t n) {
  const char* e = p + n;
  while (p < e) {
    const char* r = find_crlf(p, (size_t)(e - p));
    if (!r || r + 3 >= e) return nullptr;
    if (r[2] == '\r' && r[3] == '\n') return r;
    p = r + 2;
  }
  return nullptr;
}
template <class F>
void for_each_header(const char* p, size_t n, F&& f) {
  auto ws = [](char ch) { return ch == ' ' || ch == '\t'; };
  size_t pos = 0;
  while (pos < n) {
    const char* e0 = find_crlf(p + pos, n - pos);
    size_t e = e0 ? (size_t)(e0 - p) : n;
    const char* colon = (const char*)memchr(p + pos, ':', e - pos);
    if (colon) {
      size_t ka = pos, kb = (size_t)(colon - p);
      while (ka < kb && ws(p[ka])) ++ka;
      while (kb > ka && (ws(p[kb - 1]) || p[kb - 1] == '\r')) --kb;
      size_t va = (size_t)(colon - p) + 1, vb = e;
      while (va < vb && ws(p[va])) ++va;
      while (vb > va && (ws(p[vb - 1]) || p[vb - 1] == '\r')) --vb;
      std::string k(p + ka, kb - ka);
      for (auto& ch : k) ch = alow((unsigned char)ch);
      f(std::move(k), std::string(p + va, vb - va));
    }
    pos = e + 2;
  }
}
// ASCII case-insensitive equality / substring search of a lower-case needle
bool ieq(const std::string& s, const char* lw) {
  size_t n = strlen(lw);
  if (s.size() != n) return false;
  for (size_t i = 0; i < n; ++i)
    if (alow((unsigned char)s[i]) != lw[i]) return false;
  return true;
}
bool icontains(const std::string& s, const char* lw) {
  size_t n = strlen(lw);
  for (size_t i = 0; i + n <= s.size(); ++i) {
    size_t j = 0;
    while (j < n && alow((unsigned char)s[i + j]) == lw[j]) ++j;
    if (j == n) return true;
  }
  return false;
}
const char* reason(int st) {
  switch (st) {
    case 200: return "OK";
    case 400: return "Bad Request";
    case 401: return "Unauthorized";
    case 404: return "Not Found";
    case 500: return "Internal Server Error";
    case 502: return "Bad Gateway";
    case 503: return "Service Unavailable";
    default: return "Status";
  }
}
// "<hex len>\r\n" into h (>= 20 bytes), its length returned: the chunk header of every
// client write (snprintf's format machinery showed in the proxy's CPU profile)
inline int chunk_head(char* h, size_t len) {
  static const char* d = "0123456789abcdef";
  char t[16];
  int k = 0;
  do {
    t[k++] = d[len & 15];
    len >>= 4;
  } while (len);
  for (int i = 0; i < k; ++i) h[i] = t[k - 1 - i];
  h[k] = '\r';
  h[k + 1] = '\n';
  return k + 2;
}
inline int dec_str(char* o, size_t v) {
  char t[24];
  int k = 0;
  do {
    t[k++] = (char)('0' + v % 10);
    v /= 10;
  } while (v);
  for (int i = 0; i < k; ++i) o[i] = t[k - 1 - i];
  return k;
}
std::string chunk(const std::string& s) {
  char h[24];
  const int n = chunk_head(h, s.size());
  std::string r;
  r.reserve(n + s.size() + 2);
  r.append(h, n).append(s).append("\r\n");
  return r;
}
std::string err_json(const std::string& msg, const char* type) {
  JVal e;
  e.t = JVal::OBJ;
  e.set("message", JVal::str(msg));
  e.set("type", JVal::str(type));
  JVal o;
  o.t = JVal::OBJ;
  o.set("error", e);
  return json_dumps(o);
}
std::string http_response(int status, const std::string& ctype, const std::string& body,
                          const std::vector<std::pair<std::string, std::string>>* extra = nullptr) {
  std::string r = "HTTP/1.1 " + std::to_string(status) + " " + reason(status) + "\r\n";
  r += "content-length: " + std::to_string(body.size()) + "\r\ncontent-type: " + ctype + "\r\n";
  if (extra)
    for (auto& h : *extra) r += h.first + ": " + h.second + "\r\n";
  r += "\r\n";
  r += body;
  return r;
}
const char* kSseHdr =
    "HTTP/1.1 200 OK\r\ncontent-type: text/event-stream; charset=utf-8\r\ntransfer-encoding: chunked\r\n\r\n";
const char* kDone = "data: [DONE]\n\n";

std::string chunk_event_json(const char* id, int64_t created, const std::string& model_json,
                             const std::string& delta_json, const char* finish) {
  return std::string("data: {\"id\": \"") + id + "\", \"object\": \"chat.completion.chunk\", \"created\": " +
         std::to_string(created) + ", \"model\": " + model_json + ", \"choices\": [{\"index\": 0, \"delta\": " +
         delta_json + ", \"finish_reason\": " + finish + "}]}\n\n";
}

// --------------------------------------------------------------------------------------
// incremental HTTP/1.1 response parser (upstream side)
// --------------------------------------------------------------------------------------
struct RespParser {
  int phase = 0;  // 0 headers, 1 length body, 2 chunk size, 3 chunk data, 4 chunk crlf, 5 trailers, 6 until close, 7 done
  int status = 0;
  bool keep_headers = true;  // engine-fed streams need only status + framing (no per-header strings)
  std::vector<std::pair<std::string, std::string>> headers;
  long remaining = 0;
  bool close = false;
  std::string buf;
  // returns -1 on protocol error; appends body bytes to out.  Parses straight from the read
  // buffer when nothing is pending (the common case): only an unconsumed tail is copied.
  int feed(const char* p, size_t n, std::string& out) {
    const char* d = p;
    size_t len = n;
    if (!buf.empty()) {
      buf.append(p, n);
      d = buf.data();
      len = buf.size();
    }
    out.reserve(out.size() + n);  // at most n body bytes arrive with n bytes
    auto find = [&](const char* pat, size_t pl, size_t from) -> size_t {
      if (from > len) return std::string::npos;
      const void* f = pl == 2 && pat[0] == '\r' && pat[1] == '\n' ? find_crlf(d + from, len - from)
                      : pl == 4 && memcmp(pat, "\r\n\r\n", 4) == 0 ? find_crlfcrlf(d + from, len - from)
                                                                  : memmem(d + from, len - from, pat, pl);
      return f ? (size_t)((const char*)f - d) : std::string::npos;
    };
    size_t i = 0;
    while (phase != 7) {
      if (phase == 0) {
        size_t he = find("\r\n\r\n", 4, i);
        if (he == std::string::npos) break;
        const char* hp = d + i;
        size_t hn = he - i;
        i = he + 4;
        const char* le0 = find_crlf(hp, hn);
        size_t le = le0 ? (size_t)(le0 - hp) : hn;
        if (le < 12 || memcmp(hp, "HTTP/", 5) != 0) return -1;
        status = 0;
        for (size_t k = 9; k < le && hp[k] >= '0' && hp[k] <= '9'; ++k) status = status * 10 + (hp[k] - '0');
        bool chunked = false, has_len = false;
        size_t pos = le0 ? le + 2 : hn;
        for_each_header(hp + pos, hn - pos, [&](std::string&& k, std::string&& v) {
          if (k == "transfer-encoding" && icontains(v, "chunked")) chunked = true;
          if (k == "content-length") {
            has_len = true;
            remaining = atol(v.c_str());
          }
          if (k == "connection" && ieq(v, "close")) close = true;
          if (keep_headers) headers.emplace_back(std::move(k), std::move(v));
        });
        if (status == 204 || status == 304) phase = 7;
        else if (chunked) phase = 2;
        else if (has_len) phase = remaining > 0 ? 1 : 7;
        else {
          phase = 6;
          close = true;
        }
        continue;
      }
      if (phase == 1) {
        size_t take = std::min((size_t)remaining, len - i);
        out.append(d + i, take);
        i += take;
        remaining -= take;
        if (remaining == 0) phase = 7;
        break;
      }
      if (phase == 6) {
        out.append(d + i, len - i);
        i = len;
        break;
      }
      if (phase == 2) {
        size_t le = find("\r\n", 2, i);
        if (le == std::string::npos) break;
        remaining = strtol(d + i, nullptr, 16);  // stops at the CR
        i = le + 2;
        phase = remaining == 0 ? 5 : 3;
        continue;
      }
      if (phase == 3) {
        size_t take = std::min((size_t)remaining, len - i);
        out.append(d + i, take);
        i += take;
        remaining -= take;
        if (remaining > 0) break;
        phase = 4;
        continue;
      }
      if (phase == 4) {
        if (len - i < 2) break;
        i += 2;
        phase = 2;
        continue;
      }
      if (phase == 5) {
        size_t le = find("\r\n", 2, i);
        if (le == std::string::npos) break;
        bool empty = le == i;
        i = le + 2;
        if (empty) phase = 7;
        continue;
      }
    }
    if (d == p) buf.assign(p + i, n - i);  // the unconsumed tail only
    else buf.erase(0, i);
    return 0;
  }
  bool done() const { return phase == 7; }
  const std::string* header(const std::string& k) const {
    for (auto& h : headers)
      if (h.first == k) return &h.second;
    return nullptr;
  }
};

// --------------------------------------------------------------------------------------
// connection / session state
// --------------------------------------------------------------------------------------
struct Session;
struct Client {
  int fd = -1;
  std::string in, out;
  size_t out_off = 0;
  Session* sess = nullptr;
  bool keepalive = true;
  bool dead = false;         // error: close now
  bool close_after = false;  // graceful: close once output is flushed
  bool queued = false;       // in the loop's end-of-iteration flush list
  int served = 0;            // requests handled on this connection
  uint64_t serial = 0;       // per-loop connection serial (fd numbers are reused)
  double t_accept = 0;
  bool want_out = false;     // EPOLLOUT armed (socket buffer was full)
  bool held = false;         // corked output held for a stream's next delta (a deferral entry is out)
  double held_t0 = 0;        // when the hold began (qmx_output_hold_seconds)
};

enum UpMode { UP_ENGINE, UP_BUFFER, UP_PASS };
struct Up {
  int fd = -1;
  int backend = -1;  // index into cfg.backends
  Session* sess = nullptr;
  int bi = -1;  // index into sess->bs, -1 = aggregator call
  UpMode mode = UP_BUFFER;
  std::string req;
  size_t req_off = 0;
  bool connecting = false, reused = false, got_bytes = false, headers_seen = false;
  RespParser rp;
  std::string body;  // buffered body (UP_BUFFER / non-200)
  double last_io = 0, deadline = 0, timeout = 60, t_open = 0;
  SSL* ssl = nullptr;     // https backend
  bool tls_hs = false;    // handshake in progress
  bool out_armed = false;  // EPOLLOUT registered (connect / a send that hit EAGAIN)
};

struct BState {
  int backend = -1;
  int slot = -1;          // engine slot (spread: the owner's shadow slot of a remote stream)
  int remote = -1;        // spread placement: rank running this stream (-1 = local)
  int rx_data = 0;        // spread: delta messages received from the worker
  double t_sp_open = 0, t_sp_last = 0;  // spread: X_OPEN queued / last delta applied (h_sp_*)
  bool via_link = false;      // spread: this remote stream's messages use the io loop's link to its rank
  bool bulk_waiting = false;  // spread: the final text arrived before some of its deltas
  XMsg bulk_msg;
  Up* up = nullptr;
  int state = 0;  // 0 running, 1 done, 2 failed
  int status = 0;
  bool aborted = false;
  double t_fed = 0;  // first body bytes handed to the engine (h_engine)
  // buffered (non-stream) result, call_backend contract
  bool is_json = false;
  JVal js;
  std::string text;
  std::vector<std::pair<std::string, std::string>> rheaders;
};

enum SKind { K_PAR, K_SINGLE, K_NONSTREAM, K_REMOTE };  // K_REMOTE: worker side of a spread stream
struct Session {
  Client* cl = nullptr;
  SKind kind = K_PAR;
  JVal body;
  std::string raw;
  std::vector<std::pair<std::string, std::string>> fwd;  // forwarded headers
  std::string auth;                                      // normalized Authorization value
  std::vector<BState> bs;
  int finished = 0;
  bool filter = true, emit = true;
  int stage = 0;  // 0 streaming, 1 finalize pending, 2 aggregator pending, 3 done
  int fin_id = -1;
  bool fin_texts = false;
  std::vector<std::string> texts;
  std::vector<std::string> text_names;  // documented semantics: each text's backend name
  Up* agg = nullptr;
  // single-stream passthrough
  // body with "model" replaced = mpre + dumps(model) + mpost (built once per request,
  // reused for every backend whose config model overrides the request's)
  bool msplit = false;
  std::string mpre, mpost;
  std::string first_buf;
  bool first_decided = false, saw_done = false, pass_started = false;
  std::string done_tail;
  std::string role_model_json;
  double t0 = 0;
  // spread placement
  uint64_t skey = 0;  // owner: key under which workers address this session
  int remote_n = 0;
  int owner_rank = -1, owner_loop = 0, shadow_bi = 0;  // worker (K_REMOTE)
  bool via_link = false;  // worker: the X_OPEN came over this loop's link (replies take it too)
  uint64_t owner_skey = 0;
  int data_sent = 0;          // worker: delta messages posted to the owner
  bool bulk_pending = false;  // worker: the final text is in flight (the slot must stay)
  // worker, HIP engine: the final text is being fetched from HBM by a texts-kind finalize item
  // of the loop's next tick (no synchronous device copy on the io loop); then it is here
  bool fetching = false, fetched = false;
  std::string fetched_text;
  bool first_content = false;  // TTFT recorded
};

struct ResultBatch {
  std::vector<SlotResult> r;
  std::vector<FinalizeRes> f;
  double t_routed = 0;
};

// --------------------------------------------------------------------------------------
// verify mode (QMX_VERIFY / runtime.verify): a shadow C++ CPU engine sees every open / feed /
// finish / finalize of the primary (HIP) engine and is ticked right after it; per-stream
// SSE output, terminal flags and finalize results must be byte-identical (the SURVEY §5.2
// "run the CPU oracle on every tick and compare" debug mode).  Mismatches are counted in
// /metrics and logged.
// --------------------------------------------------------------------------------------
std::atomic<uint64_t> c_verify_checked{0}, c_verify_mismatch{0};

class Verifier {
 public:
  explicit Verifier(const std::vector<std::string>& tags) : cpu_(tags) {}
  void open(int slot, uint32_t gen, int index, bool f, bool e) {
    std::lock_guard<std::mutex> g(mu_);
    Track t;
    t.gen = gen;
    t.shadow = cpu_.open(index, f, e);
    rmap_[t.shadow] = slot;
    map_[slot] = std::move(t);
  }
  void feed(int slot, const std::string& d) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = map_.find(slot);
    if (it != map_.end()) cpu_.feed(it->second.shadow, d);
  }
  void finish(int slot) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = map_.find(slot);
    if (it != map_.end()) cpu_.finish(it->second.shadow);
  }
  void release(int slot) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = map_.find(slot);
    if (it == map_.end()) return;
    if (!it->second.compared && !it->second.acc[0].empty()) {
      // released before both sides terminated (a failed sibling backend's slot, a client that
      // left): what the primary emitted must still be a prefix of the oracle's output for the
      // same feeds — a spurious event on a stream that never terminates is caught here
      drain_locked(last_created_);
      Track& t = map_[slot];
      const std::string a0 = norm(t.acc[0]), a1 = norm(t.acc[1]);
      c_verify_checked++;
      if (a1.compare(0, a0.size(), a0) != 0) report("released stream", slot, t.acc[0], t.acc[1]);
      it = map_.find(slot);
    }
    rmap_.erase(it->second.shadow);
    cpu_.release(it->second.shadow);
    map_.erase(it);
  }
  void apply_ops(const std::vector<EngineOp>& ops) {
    for (auto& op : ops) {
      if (op.kind == EngineOp::FEED) feed(op.slot, op.data);
      else if (op.kind == EngineOp::FINISH) finish(op.slot);
      else release(op.slot);
    }
  }
  void submit(int fid, const std::vector<int>& slots, bool strip, bool texts, const std::string& joiner,
              int64_t created) {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<int> sh;
    for (int s : slots) {
      auto it = map_.find(s);
      if (it == map_.end()) return;  // not tracked (opened before verify): skip
      sh.push_back(it->second.shadow);
    }
    fin_[cpu_.submit_finalize(sh, strip, texts, joiner, created)] = fid;
  }
  // the oracle ticked until it has nothing left: its outputs appended to the tracks
  void drain_locked(int64_t created, std::vector<FinalizeRes>* sf_out = nullptr) {
    std::vector<SlotResult> sr;
    std::vector<FinalizeRes> sf;
    for (int k = 0; k < 64 && cpu_.has_work(); ++k) cpu_.tick(created, sr, sf);
    for (auto& x : sr) {
      auto rit = rmap_.find(x.slot);
      if (rit == rmap_.end()) continue;
      Track& t = map_[rit->second];
      t.acc[1].append(x.data(), x.size());
      t.term[1] |= x.flags & (RF_DONE | RF_ABORTED);
    }
    if (sf_out) {
      for (auto& x : sf) sf_out->push_back(std::move(x));
    } else {
      for (auto& x : sf) pending_sf_.push_back(std::move(x));
    }
  }
  // tick thread, right after the primary engine's tick(created)
  void check(int64_t created, const std::vector<SlotResult>& r, const std::vector<FinalizeRes>& f) {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& x : r) {
      auto it = map_.find(x.slot);
      if (it == map_.end() || it->second.gen != x.gen) continue;  // stale: slot re-opened
      it->second.acc[0].append(x.data(), x.size());
      it->second.term[0] |= x.flags & (RF_DONE | RF_ABORTED);
    }
    for (auto& x : f) pfin_[x.id] = x;
    last_created_ = created;
    std::vector<FinalizeRes> sf;
    drain_locked(created, &sf);
    for (auto& kv : map_) {
      Track& t = kv.second;
      if (t.compared || !t.term[0] || !t.term[1]) continue;
      t.compared = true;
      c_verify_checked++;
      if (t.term[0] != t.term[1] || norm(t.acc[0]) != norm(t.acc[1])) report("stream", kv.first, t.acc[0], t.acc[1]);
    }
    for (auto& x : pending_sf_) sf.push_back(std::move(x));
    pending_sf_.clear();
    for (auto& x : sf) {
      auto it = fin_.find(x.id);
      if (it == fin_.end()) continue;
      sfin_[it->second] = x;
      fin_.erase(it);
    }
    for (auto it = sfin_.begin(); it != sfin_.end();) {
      auto p = pfin_.find(it->first);
      if (p == pfin_.end()) {
        ++it;
        continue;
      }
      c_verify_checked++;
      const FinalizeRes &a = p->second, &b = it->second;
      if (a.kind != b.kind || norm(a.event) != norm(b.event) || a.texts != b.texts)
        report("finalize", a.id, a.event, b.event);
      pfin_.erase(p);
      it = sfin_.erase(it);
    }
  }

 private:
  struct Track {
    int shadow = -1;
    uint32_t gen = 0;
    std::string acc[2];
    int term[2] = {0, 0};
    bool compared = false;
  };
  // a stream's bytes can straddle a one-second boundary differently in the two engines
  static std::string norm(const std::string& x) {
    std::string o;
    o.reserve(x.size());
    static const std::string key = "\"created\": ";
    for (size_t i = 0; i < x.size();) {
      if (x.compare(i, key.size(), key) == 0) {
        o += key;
        i += key.size();
        while (i < x.size() && x[i] >= '0' && x[i] <= '9') ++i;
        continue;
      }
      o.push_back(x[i++]);
    }
    return o;
  }
  void report(const char* what, int id, const std::string& a, const std::string& b) {
    if (c_verify_mismatch++ < 20)
      fprintf(stderr, "qmx verify: %s %d differs (primary %zu B, cpu oracle %zu B)\n  primary: %.300s\n  oracle:  %.300s\n",
              what, id, a.size(), b.size(), a.c_str(), b.c_str());
  }
  std::mutex mu_;
  CpuEngine cpu_;
  int64_t last_created_ = 0;
  std::vector<FinalizeRes> pending_sf_;  // oracle finalize results drained by a release
  std::unordered_map<int, Track> map_;
  std::unordered_map<int, int> rmap_, fin_;
  std::unordered_map<int, FinalizeRes> pfin_, sfin_;
};

// --------------------------------------------------------------------------------------
// GPU hub: ONE HIP engine per process shared by every io loop (the SURVEY's "pack pending
// upstream bytes of ALL active streams on this rank").  `tick_lanes` tick threads each own
// a lane of the engine (HIP stream + host-mapped arenas): a lane takes every dirty stream
// that is not in flight on another lane, launches the fused tick kernel, waits, routes each
// stream's results to the loop that owns it (per-loop queue + eventfd) and only then
// settles its streams — so a stream's outputs stay in order while a second lane already
// has the next kernel in flight for the bytes that arrived meanwhile (the tick kernel is
// latency-bound: two launches in flight cost the GPU nothing and halve the tick period).
// --------------------------------------------------------------------------------------
// Round-delivered remote finals read straight from HBM (HipEngine::set_remote_hbm_direct):
// tcpbulk rounds copy them in from the host (a runtime dispatch on this device: coherent), and
// RCCL at world 1 is its own kernel on this device; RCCL at world > 1 (a peer GPU's writes)
// only with QMX_REMOTE_HBM=1 until a multi-GPU run has pinned it
static bool remote_hbm_direct(const ServerCfg& cfg) {
  if (const char* e = env_get("QMX_REMOTE_HBM")) return atoi(e) != 0;
  const char* x = env_get("QMX_XCHG");
  const std::string t = x && *x ? x : cfg.xchg;
  return cfg.world <= 1 || t != "rccl";
}

class GpuHub {
 public:
  using Sink = std::function<void(ResultBatch&&)>;
  GpuHub(const ServerCfg& cfg, int nloops) : cfg_(cfg), sinks_(nloops), pools_(nloops) {
    lanes_ = std::max(1, std::min(cfg.tick_lanes, 8));
    if (cfg.engine == "hip") {
      HipEngine* he = new HipEngine(cfg.tags, cfg.device, cfg.tile, cfg.max_slots, cfg.content_cap, lanes_);
      he->set_remote_hbm_direct(remote_hbm_direct(cfg));
      // (spread placement: an RCCL round writes a remote final text into the content arena
      // and its stream is synchronised before the text is applied; the finalize that reads it
      // is a later tick, whose items start with a system-scope acquire — one-shot launches and
      // persistent grids alike)
      eng_.reset(he);
    } else
      eng_.reset(new CpuEngine(cfg.tags));  // shared CPU engine: exercises the hub routing on CPU
    if (cfg.verify) ver_.reset(new Verifier(cfg.tags));
  }
  ~GpuHub() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_)
      if (t.joinable()) t.join();
  }
  void start() {
    for (int i = 0; i < lanes_; ++i) th_.emplace_back([this, i] { run(i); });
  }
  void attach(int loop, Sink s) { sinks_[loop] = std::move(s); }
  // called by io loop `loop` only: slots come from that loop's reserve, refilled a chunk at
  // a time under one engine lock + one owner-map lock (not two locks per open).  The chunk is
  // at most max_slots / (4 x loops): reserves parked in idle loops can never push the other
  // loops' opens past max_slots (the device state table) onto the slow host path.
  int open(int loop, int index, bool f, bool e, uint32_t* gen, bool verify = true) {
    std::vector<int>& pool = pools_[loop];
    if (pool.empty()) {
      const int chunk = std::max(1, std::min(32, cfg_.max_slots / (4 * (int)pools_.size())));
      eng_->reserve(chunk, pool);
      std::lock_guard<std::mutex> g(omu_);
      for (int slot : pool) {
        if ((int)owner_.size() <= slot) owner_.resize(slot + 1024, -1);
        owner_[slot] = loop;
      }
    }
    const int slot = pool.back();
    pool.pop_back();
    if (cfg_.engine == "hip" && slot >= cfg_.max_slots) c_host_path_opens++;  // beyond HBM slot state
    eng_->open_reserved(slot, index, f, e, gen);
    if (ver_ && verify) ver_->open(slot, *gen, index, f, e);
    return slot;
  }
  HostEngine& engine() { return *eng_; }
  void feed(int slot, const std::string& d) {
    eng_->feed(slot, d);
    if (ver_) ver_->feed(slot, d);
  }
  void finish(int slot) {
    eng_->finish(slot);
    if (ver_) ver_->finish(slot);
  }
  void release(int slot) {
    eng_->release(slot);
    if (ver_) ver_->release(slot);
  }
  void apply_ops(std::vector<EngineOp>& ops) {
    if (ver_) ver_->apply_ops(ops);
    eng_->apply_ops(ops, true);
  }
  int submit(int loop, const std::vector<int>& slots, bool strip, bool texts, const std::string& joiner,
             int64_t created) {
    std::lock_guard<std::mutex> g(omu_);  // the id must be routable before a tick lane sees it
    int id = eng_->submit_finalize(slots, strip, texts, joiner, created);
    fin_owner_[id] = loop;
    if (ver_) ver_->submit(id, slots, strip, texts, joiner, created);
    return id;
  }
  void kick() {
    {
      std::lock_guard<std::mutex> g(mu_);
      work_ = true;
    }
    cv_.notify_one();  // an idle lane, if any: a busy lane re-checks for work when it settles
  }
  std::unordered_map<std::string, double> snapshot() {
    std::lock_guard<std::mutex> g(smu_);
    return snap_;
  }

 private:
  // A tick lane that throws (a device fault surfaced by a synchronise, output arenas never
  // released, a lost tick) cannot know which of its streams' bytes were consumed: the process
  // exits with a message and a distinct code (the supervisor restarts it; clients see their
  // connections close) instead of dying in std::terminate.
  void run(int lane) {
    try {
      run_lane(lane);
    } catch (const std::exception& e) {
      fprintf(stderr, "qmx: tick lane %d failed: %s — exiting\n", lane, e.what());
      fflush(stderr);
      _exit(70);
    }
  }
  void run_lane(int lane) {
    prof_thread();
    crash_thread();
    if (cfg_.engine == "hip") hipSetDevice(cfg_.device);
    std::vector<ResultBatch> per(sinks_.size());
    if (eng_->pipelined()) return run_pipelined(lane, per);
    std::vector<int> taken;
    while (true) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait_for(lk, std::chrono::milliseconds(2), [this] { return work_ || stop_; });
        if (stop_) break;
        work_ = false;
      }
      while (true) {
        ResultBatch rb;
        taken.clear();
        const double tt = now_s();
        const int64_t created = (int64_t)time(nullptr);
        if (!eng_->tick(created, rb.r, rb.f, lane, &taken)) break;  // nothing this lane may take
        const double t_ticked = now_s();
        h_tick.observe(t_ticked - tt);
        if (ver_) ver_->check(created, rb.r, rb.f);
        deliver(rb, per, taken, t_ticked);
        if (stop_) break;
      }
    }
  }
  // A pipelined lane (HipEngine with polled completion): while its tick runs on the device,
  // the lane takes and prepares the next one, posts it the moment the running one completes,
  // and only then turns the completed tick into results and routes them — the lane's host
  // work (preparation, routing, settling) overlaps its device time instead of adding to it.
  void run_pipelined(int lane, std::vector<ResultBatch>& per) {
    HostEngine::Job jobs[2];
    double t_post[2] = {0.0, 0.0};
    std::vector<int> taken;
    int c = 0;
    while (!stop_) {
      HostEngine::Job& cur = jobs[c];
      if (!cur.live) {
        {
          std::unique_lock<std::mutex> lk(mu_);
          cv_.wait_for(lk, std::chrono::milliseconds(2), [this] { return work_ || stop_; });
          if (stop_) break;
          work_ = false;
        }
        cur.created = (int64_t)time(nullptr);
        cur.lane = lane;
        if (!eng_->job_take(cur, true)) continue;
        t_post[c] = now_s();
        eng_->job_prepare(cur);
        eng_->job_post(cur);
        cur.live = true;
      }
      HostEngine::Job& nxt = jobs[c ^ 1];
      eng_->job_wait_near(cur);
      nxt.created = (int64_t)time(nullptr);
      nxt.lane = lane;
      // finalize requests use the lane's single finalize arenas: one tick in flight with them
      const bool have = !stop_ && eng_->job_take(nxt, cur.fin.empty());
      if (have) eng_->job_prepare(nxt);
      ResultBatch rb;
      taken.clear();
      eng_->job_complete(cur, rb.r, rb.f);
      eng_->job_finish(cur, rb.r, taken);
      cur.live = false;
      if (have) {
        t_post[c ^ 1] = now_s();
        eng_->job_post(nxt);
        nxt.live = true;
      }
      const double t_ticked = now_s();
      h_tick.observe(t_ticked - t_post[c]);
      if (ver_) ver_->check(cur.created, rb.r, rb.f);
      deliver(rb, per, taken, t_ticked);
      c ^= 1;
    }
    for (HostEngine::Job& j : jobs) {  // stopping: a posted tick still completes (its slots are busy)
      if (!j.live) continue;
      ResultBatch rb;
      taken.clear();
      eng_->job_complete(j, rb.r, rb.f);
      eng_->job_finish(j, rb.r, taken);
      j.live = false;
      deliver(rb, per, taken, now_s());
    }
  }
  // a tick's results → the owning io loops, then its streams settle (in that order: a
  // stream's next results cannot overtake these)
  void deliver(ResultBatch& rb, std::vector<ResultBatch>& per, const std::vector<int>& taken, double t_ticked) {
    c_ticks++;
    c_tick_slots += rb.r.size();
    {
      std::lock_guard<std::mutex> g(omu_);
      for (auto& r : rb.r) {
        const int l = r.slot < (int)owner_.size() ? owner_[r.slot] : -1;
        if (l >= 0) per[l].r.push_back(std::move(r));
      }
      for (auto& f : rb.f) {
        auto it = fin_owner_.find(f.id);
        if (it == fin_owner_.end()) continue;
        per[it->second].f.push_back(std::move(f));
        fin_owner_.erase(it);
      }
    }
    for (size_t l = 0; l < per.size(); ++l) {
      if (per[l].r.empty() && per[l].f.empty()) continue;
      per[l].t_routed = now_s();
      if (sinks_[l]) sinks_[l](std::move(per[l]));
      per[l] = ResultBatch();
    }
    eng_->settle(taken);
    c_route_ns += (uint64_t)((now_s() - t_ticked) * 1e9);
    if (t_ticked - last_snap_.load() > 0.05) {
      last_snap_.store(t_ticked);
      std::unordered_map<std::string, double> m;
      for (auto& kv : eng_->stats()) m["qmx_engine_" + kv.first] = kv.second;
      if (auto* h = dynamic_cast<HipEngine*>(eng_.get()))
        for (auto& kv : h->kernel_stats()) m["qmx_kernel_" + kv.first] = kv.second;
      std::lock_guard<std::mutex> g(smu_);
      snap_.swap(m);
    }
  }
  const ServerCfg& cfg_;
  int lanes_ = 1;
  std::unique_ptr<HostEngine> eng_;
  std::unique_ptr<Verifier> ver_;
  std::vector<Sink> sinks_;
  std::vector<std::vector<int>> pools_;  // per io loop: reserved, not yet opened slots
  std::mutex mu_, omu_, smu_;
  std::condition_variable cv_;
  bool work_ = false;
  std::atomic<bool> stop_{false};  // set under mu_ (cv predicate); lanes also poll it between ticks
  std::atomic<double> last_snap_{0.0};
  std::vector<int> owner_;                  // slot → io loop
  std::unordered_map<int, int> fin_owner_;  // finalize id → io loop
  std::unordered_map<std::string, double> snap_;
  std::vector<std::thread> th_;
};

// --------------------------------------------------------------------------------------
// io loop (one per thread)
// --------------------------------------------------------------------------------------
class Loop {
 public:
  Loop(const ServerCfg& cfg, int idx) : cfg_(cfg), idx_(idx) { xfd_ = eventfd(0, EFD_NONBLOCK); }
  void attach_exchange(Exchange* x) { xch_ = x; }
  int index() const { return idx_; }
  void attach_hub(GpuHub* h) {
    hub_ = h;
    if (h)
      h->attach(idx_, [this](ResultBatch&& rb) {
        {
          std::lock_guard<std::mutex> g(rmu_);
          rq_.push_back(std::move(rb));
        }
        rq_pending_.store(true, std::memory_order_seq_cst);
        // QMX_LAZY_WAKE: a loop that is not parked in epoll_wait picks the batch up itself
        // (between events, or before it waits: the Dekker pair in_wait_ / rq_pending_), so
        // only a parked loop costs the lane an eventfd write
        if (lazy_wake_ && !in_wait_.load(std::memory_order_seq_cst)) return;
        uint64_t one = 1;
        ssize_t w = write(evfd_, &one, 8);
        (void)w;
      });
  }
  void attach_tls(SSL_CTX* t) { tls_ = t; }
  // loop ticks: this loop's HIP engine posts into door idx_ of the shared grid
  void attach_grid(HipGrid* g) { grid_ = g; }
  void attach_loops(const std::vector<Loop*>* ls) { loops_ = ls; }
  std::mutex smu_;
  std::unordered_map<std::string, double> snap_;  // engine stats snapshot (read by /metrics on any loop)
  std::atomic<double> pass_max_{0.0};  // this loop's longest pass over 1 ms (/metrics)
  // QMX_LOOP_STALL_LOG watchdog: the running pass's start (0: waiting in epoll) and the thread
  std::atomic<double> pass_t0_{0.0};
  std::atomic<int> tid_{0};
  // syscalls issued by this loop's thread (single writer; /metrics reads them from any loop)
  enum { SC_CLIENT_SEND, SC_UP_SEND, SC_RECV, SC_EPOLL_WAIT, SC_EPOLL_CTL, SC_WAKE_READ, SC_N };
  std::atomic<uint64_t> sc_[SC_N] = {};
  void cnt(int i) { sc_[i].store(sc_[i].load(std::memory_order_relaxed) + 1, std::memory_order_relaxed); }
  void snapshot() {
    if (!eng_) return;
    std::unordered_map<std::string, double> m;
    for (auto& kv : eng_->stats()) m["qmx_engine_" + kv.first] = kv.second;
    if (heng_)
      for (auto& kv : heng_->kernel_stats()) m["qmx_kernel_" + kv.first] = kv.second;
    std::lock_guard<std::mutex> g(smu_);
    snap_.swap(m);
  }
  // exchange thread → this loop (thread-safe)
  void x_deliver(std::vector<XMsg>&& v) {
    {
      std::lock_guard<std::mutex> g(xmu_);
      for (auto& m : v) xin_.push_back(std::move(m));
    }
    uint64_t one = 1;
    ssize_t w = write(xfd_, &one, 8);
    (void)w;
  }
  ~Loop() {
    for (int fd : {lfd_, afd_})
      if (fd >= 0) close(fd);
    for (auto& kv : idle_ssl_) SSL_free(kv.second);  // before the run's SSL_CTX goes away
    for (auto& kv : ups_)
      if (kv.second->ssl) SSL_free(kv.second->ssl);
  }

  void run() {
    prof_thread();
    crash_thread();
    tid_.store((int)syscall(SYS_gettid));
    setup();
    if (++g_ready == cfg_.threads && !cfg_.ready_file.empty()) {
      FILE* f = fopen(cfg_.ready_file.c_str(), "w");  // supervisor: this generation is serving
      if (f) {
        fprintf(f, "%d\n", (int)getpid());
        if (cfg_.admin_port > 0) fprintf(f, "admin_port %d\n", cfg_.admin_port);
        fclose(f);
      }
    }
    std::vector<epoll_event> evs(512);
    double last_sweep = now_s();
    while (!g_stop.load()) {
      // read pacing (QMX_READ_PACE_US): a pass that read trickling upstreams — small reads of
      // responses still in progress, one SSE event each — is stretched to the pace, so the
      // events that arrive meanwhile come out of one receive per socket and one wait instead
      // of one each.  Whole-response reads never trigger it.
      if (pace_s_ > 0 && small_reads_ >= pace_min_reads_) {
        const double due = tnow_ + pace_s_, t = now_s();
        if (t < due) {
          timespec ts{0, (long)((due - t) * 1e9)};
          nanosleep(&ts, nullptr);
          c_paced++;
        }
      }
      small_reads_ = 0;
      // inline engine with work queued by the last iteration (e.g. a finalize submitted
      // while applying tick results): poll instead of sleeping
      int to = (!hub_ && !aeng_ && kick_) ? 0 : deferq_.empty() ? 50 : 1;
      if (lazy_wake_ && hub_) {
        in_wait_.store(true, std::memory_order_seq_cst);
        if (rq_pending_.load(std::memory_order_seq_cst)) to = 0;  // a batch came in: do not sleep
      }
      int n;
      if (jobs_live_) {
        // ticks of this loop are on the GPU: wake when the first is expected done, then poll
        // finely (results are published to host memory; nothing signals them)
        double exp_us = 1e9;
        bool ready = false;
        for (int k = 0; k < 2 && !ready; ++k) {
          double e = 0;
          if (!job_live_[k]) continue;
          ready = aeng_->job_ready(job_[k], &e);
          exp_us = std::min(exp_us, e);
        }
        if (ready || exp_us <= spin_us_) {
          // ready, or due within QMX_LOOP_SPIN_US: look again at once (no timer wake-up)
          n = epoll_wait(ep_, evs.data(), (int)evs.size(), 0);
        } else {
          // the timer ends where the spin window begins (a wake-up at the due time itself
          // would land a timer's latency after it, past the window)
          const double us = std::min(std::max(exp_us - spin_us_, (double)poll_us_), 1000.0 * std::max(to, 1));
          timespec ts{0, (long)(us * 1000.0)};
          n = epoll_pwait2(ep_, evs.data(), (int)evs.size(), &ts, nullptr);
          if (n < 0 && errno == ENOSYS) {  // a kernel before 5.11: sleep, then look
            nanosleep(&ts, nullptr);
            n = epoll_wait(ep_, evs.data(), (int)evs.size(), 0);
          }
        }
      } else {
        n = epoll_wait(ep_, evs.data(), (int)evs.size(), to);
      }
      tnow_ = now_s();  // this iteration's clock (lnow): stamps and timeouts, not hop timing
      if (stall_log_) pass_t0_.store(tnow_, std::memory_order_relaxed);
      double ph[7] = {0, 0, 0, 0, 0, 0, 0};  // QMX_LOOP_STALL_LOG: phase ends of this pass
      rusage ru0{};
      if (stall_log_) getrusage(RUSAGE_THREAD, &ru0);
      if (lazy_wake_ && hub_) {
        in_wait_.store(false, std::memory_order_seq_cst);
        if (rq_pending_.load(std::memory_order_acquire)) on_results(false);
      }
      cnt(SC_EPOLL_WAIT);
      // loop ticks: results published while this loop slept or worked are applied first, and
      // between every two events of the batch (a look at a few host-memory words): an io loop
      // is busy most of the time, and a tick's results waiting out a whole event batch were
      // most of its done -> taken time (tick_hops_us_avg)
      if (jobs_live_ && any_ready()) loop_tick();
      if (stall_log_) ph[0] = now_s();
      double ev_max = 0;
      int ev_kind = -1;
      for (int i = 0; i < n; ++i) {
        if (stall_log_) {
          const double e0 = now_s();
          dispatch(evs[i]);
          const double de = now_s() - e0;
          if (de > ev_max) {
            ev_max = de;
            ev_kind = (int)(evs[i].data.u64 >> 32);
          }
        } else {
          dispatch(evs[i]);
        }
        // QMX_EAGER_POST: upstream bytes go to a free door at once, not after the batch
        if (eager_post_ && aeng_ && !ops_.empty() && (evs[i].data.u64 >> 32) == 4 && aeng_->free_doors() > 0) {
          flush_ops();
          loop_tick();
        }
        // a long batch: tick results that arrived meanwhile are applied now, not after it
        if ((i & 7) == 7 && early_flush_ && rq_pending_.load(std::memory_order_acquire)) on_results(false);
        if ((i + 1) % check_every_ == 0 && jobs_live_ && any_ready()) loop_tick();
      }
      if (stall_log_) ph[1] = now_s();
      if (g_drain.load() && drain_step()) break;
      if ((hub_ || aeng_) && early_flush_) {
        // upstream bytes to the tick lanes and finished responses to their clients before
        // this iteration's new requests (whose parsing and upstream sends are the slow part)
        flush_ops();
        if (aeng_) {
          loop_tick();
        } else if (kick_) {
          kick_ = false;
          hub_->kick();
        }
        if (!flushq_.empty()) flush_queued();
      }
      if (stall_log_) ph[2] = now_s();
      if (!pending_requests_.empty()) {
        std::vector<int>& fds = scratch_fds_;  // swapped each iteration: both buffers keep their capacity
        fds.clear();
        fds.swap(pending_requests_);
        for (int fd : fds) {
          auto it = clients_.find(fd);
          if (it != clients_.end() && !it->second->sess && !it->second->dead) process_requests(it->second.get());
          if (req_check_ && jobs_live_ && any_ready()) loop_tick();
        }
      }
      double t = now_s();
      if (stall_log_) ph[3] = t;
      if (t - last_sweep > 0.1) {
        sweep_timeouts(t);
        last_sweep = t;
        snapshot();  // own CPU engine (the GPU hub snapshots the shared HIP engine)
        if (grid_) grid_->housekeep();  // the shared grid's heartbeat / idle stop
        // a tick that never completes: relaunch a grid that left on its own; after 10 s the
        // streams' bytes are in an unknown state — exit (the supervisor restarts the worker)
        for (int k = 0; k < 2 && jobs_live_; ++k) {
          if (!job_live_[k] || t - job_t_post_[k] < 0.2) continue;
          if (grid_) grid_->revive_if_exited();
          if (t - job_t_post_[k] > 10.0) {
            fprintf(stderr, "qmx: io loop %d: a tick posted %.1f s ago never completed — exiting\n", idx_,
                    t - job_t_post_[k]);
            fflush(stderr);
            _exit(70);
          }
        }
      }
      if (stall_log_) ph[4] = now_s();
      flush_ops();
      if (aeng_) {
        loop_tick();
      } else if (!hub_) {
        if (kick_ || eng_->has_work()) {
          kick_ = false;
          tick_inline();
          flush_ops();  // releases queued while applying the results
        }
      } else if (kick_) {
        kick_ = false;
        hub_->kick();
      }
      if (stall_log_) ph[5] = now_s();
      if (!deferq_.empty()) release_deferred(now_s());
      if (!flushq_.empty()) flush_queued();
      if (!pending_close_.empty()) reap_clients();
      flush_x();
      const double pass = now_s() - tnow_;
      if (stall_log_) pass_t0_.store(0.0, std::memory_order_relaxed);
      if (pass > 1e-3) {
        c_loop_pass_1ms++;
        if (pass > 5e-3) c_loop_pass_5ms++;
        if (pass > pass_max_.load(std::memory_order_relaxed)) pass_max_.store(pass, std::memory_order_relaxed);
        if (stall_log_ && pass > 5e-3 && stall_logs_++ < 50) {
          // on the CPU or blocked: this thread's CPU time, context switches (voluntary: it
          // slept on something; involuntary: preempted) and page faults over the pass
          rusage ru1{};
          getrusage(RUSAGE_THREAD, &ru1);
          auto tv = [](const timeval& t) { return 1e3 * t.tv_sec + 1e-3 * t.tv_usec; };
          fprintf(stderr, "qmx loop %d: stalled pass: cpu %.2f ms (user %.2f), vcsw %ld, ivcsw %ld, minflt %ld, majflt %ld\n",
                  idx_, tv(ru1.ru_utime) + tv(ru1.ru_stime) - tv(ru0.ru_utime) - tv(ru0.ru_stime),
                  tv(ru1.ru_utime) - tv(ru0.ru_utime), ru1.ru_nvcsw - ru0.ru_nvcsw, ru1.ru_nivcsw - ru0.ru_nivcsw,
                  ru1.ru_minflt - ru0.ru_minflt, ru1.ru_majflt - ru0.ru_majflt);
          ph[6] = tnow_ + pass;
          double prev = tnow_, d[7];
          for (int k = 0; k < 7; ++k) {
            d[k] = ph[k] > 0 ? 1e3 * (ph[k] - prev) : 0.0;
            if (ph[k] > 0) prev = ph[k];
          }
          fprintf(stderr, "qmx loop %d: %.2f ms pass (%d events): results %.2f, events %.2f, early flush %.2f, "
                  "requests %.2f, sweep %.2f, flush+tick %.2f, output %.2f ms; engine allocs %.0f (%.0f us); "
                  "grid launches %.0f stops %.0f; slowest event kind %d (%.2f ms)\n", idx_,
                  1e3 * pass, n, d[0], d[1], d[2], d[3], d[4], d[5], d[6],
                  heng_ ? heng_->kernel_stats()["runtime_allocs"] : 0.0,
                  heng_ ? heng_->kernel_stats()["runtime_alloc_us"] : 0.0,
                  grid_ ? grid_->stats()["grid_launches"] : 0.0, grid_ ? grid_->stats()["grid_stops"] : 0.0, ev_kind,
                  1e3 * ev_max);
        }
      }
    }
    // ticks still on the GPU complete before the engine (and its arenas) can go
    for (int w = 0; jobs_live_ && w < 200000; ++w) {
      for (int k = 0; k < 2; ++k)
        if (job_live_[k] && aeng_->job_ready(job_[k])) finish_job(k);
      if (jobs_live_) std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  }
  // deferred heads whose deadline passed are queued for this iteration's flush; entries whose
  // client was queued by later output (or closed) are dropped
  void release_deferred(double t) {
    size_t k = 0;
    for (size_t i = 0; i < deferq_.size(); ++i) {
      auto it = clients_.find(deferq_[i].fd);
      if (it == clients_.end()) continue;
      Client* c = it->second.get();
      if (c->serial != deferq_[i].serial) continue;  // fd closed and reused by a new connection
      if (c->queued || c->want_out || c->dead || c->out_off >= c->out.size()) {
        unhold(c);
        continue;
      }
      if (deferq_[i].deadline <= t || g_drain.load()) {
        if (c->held) c_hold_deadline++;
        unhold(c);
        c->queued = true;
        flushq_.push_back(c->fd);
        continue;
      }
      deferq_[k++] = deferq_[i];
    }
    deferq_.resize(k);
  }

 private:
  // ---------------------------------------------------------------- setup
  void setup() {
    ep_ = epoll_create1(0);
    lfd_ = socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK, 0);
    int one = 1;
    setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    setsockopt(lfd_, SOL_SOCKET, SO_REUSEPORT, &one, sizeof(one));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons(cfg_.port);
    inet_pton(AF_INET, cfg_.host.c_str(), &a.sin_addr);
    if (bind(lfd_, (sockaddr*)&a, sizeof(a)) != 0) throw std::runtime_error("bind failed: " + std::string(strerror(errno)));
    listen(lfd_, 4096);
    add(lfd_, EPOLLIN, tag_listen());
    if (idx_ == 0 && cfg_.admin_port > 0) {  // this process alone (per-rank /metrics, /health)
      afd_ = socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK, 0);
      setsockopt(afd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
      sockaddr_in b = a;
      b.sin_port = htons(cfg_.admin_port);
      if (bind(afd_, (sockaddr*)&b, sizeof(b)) != 0)
        throw std::runtime_error("admin port bind failed: " + std::string(strerror(errno)));
      listen(afd_, 256);
      add(afd_, EPOLLIN, tag(6, 0));
    }
    evfd_ = eventfd(0, EFD_NONBLOCK);
    add(evfd_, EPOLLIN, tag_event());
    add(xfd_, EPOLLIN, tag(5, 0));
    idle_.resize(cfg_.backends.size());
    if (!hub_) {  // own engine: the CPU engine ticked inline, or a HIP engine on the shared grid
      if (grid_) {
        prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);  // 1 us: the tick polls sleep a few us
        const int per = std::max(128, cfg_.max_slots / std::max(1, cfg_.threads));
        heng_ = new HipEngine(cfg_.tags, cfg_.device, cfg_.tile, per, cfg_.content_cap, 1, grid_,
                              idx_ * loop_doors_, loop_doors_);
        heng_->set_remote_hbm_direct(remote_hbm_direct(cfg_));
        eng_.reset(heng_);
        aeng_ = heng_;
        loop_slots_ = per;
      } else if (cfg_.tick_mode == "loops") {
        // the loop-tick protocol on the CPU: jobs run on the engine's worker thread while the
        // loop polls for them (tests / TSan of the io loops' asynchronous tick path)
        aeng_ = new AsyncCpuEngine(cfg_.tags);
        eng_.reset(aeng_);
      } else {
        eng_.reset(new CpuEngine(cfg_.tags));
      }
      if (cfg_.verify) ver_.reset(new Verifier(cfg_.tags));
    }
  }

  // epoll tags: fd in low 32 bits, kind in high bits
  static uint64_t tag(int kind, int fd) { return ((uint64_t)kind << 32) | (uint32_t)fd; }
  static uint64_t tag_listen() { return tag(1, 0); }
  static uint64_t tag_event() { return tag(2, 0); }
  void add(int fd, uint32_t ev, uint64_t t) {
    epoll_event e{};
    e.events = ev;
    e.data.u64 = t;
    epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &e);
    cnt(SC_EPOLL_CTL);
  }
  void mod(int fd, uint32_t ev, uint64_t t) {
    epoll_event e{};
    e.events = ev;
    e.data.u64 = t;
    epoll_ctl(ep_, EPOLL_CTL_MOD, fd, &e);
    cnt(SC_EPOLL_CTL);
  }

  void dispatch(const epoll_event& e) {
    int kind = (int)(e.data.u64 >> 32);
    int fd = (int)(uint32_t)e.data.u64;
    if (kind == 1) return on_accept(lfd_);
    if (kind == 6) return on_accept(afd_);
    if (kind == 2) return on_results();
    if (kind == 5) return on_xmsgs();
    if (kind == 7) return on_link(fd, e.events);
    if (kind == 3) {
      auto it = clients_.find(fd);
      if (it != clients_.end()) on_client(it->second.get(), e.events);
      return;
    }
    if (kind == 4) {
      auto it = ups_.find(fd);
      if (it != ups_.end()) on_up(it->second.get(), e.events);
      else on_parked(fd);
      return;
    }
  }

  // ---------------------------------------------------------------- engine plumbing
  // Loop ticks: this loop's ticks go straight from here to its doors of the shared grid, and
  // their results are applied here — no tick thread, no queue, no eventfd in between.  Up to
  // `loop_doors_` ticks in flight per loop (a door each): a stream that becomes dirty while
  // one runs goes out on the other at once (a stream in flight is busy in the engine until
  // its results are applied, so its own ticks stay in order).
  bool any_ready() {
    for (int k = 0; k < 2; ++k)
      if (job_live_[k] && aeng_->job_ready(job_[k])) return true;
    return false;
  }
  void loop_tick() {
    bool applied = false;
    for (int k = 0; k < 2; ++k)
      if (job_live_[k] && aeng_->job_ready(job_[k])) {
        finish_job(k);
        applied = true;
      }
    if (applied) flush_ops();  // releases queued while applying the results
    kick_ = false;
    if (aeng_->free_doors() == 0) return;
    const int k = job_live_[0] ? 1 : 0;
    // the finalize arenas are one set per engine: one tick with finalize work at a time
    const bool fin_ok = !(job_live_[k ^ 1] && !job_[k ^ 1].fin.empty());
    HostEngine::Job& j = job_[k];
    j.created = (int64_t)time(nullptr);
    j.lane = 0;
    if (!eng_->job_take(j, fin_ok)) return;
    job_t_post_[k] = now_s();
    eng_->job_prepare(j);
    eng_->job_post(j);
    job_live_[k] = true;
    ++jobs_live_;
    if (aeng_->job_ready(j)) finish_job(k);  // nothing went to the GPU (host-path streams only)
  }
  void finish_job(int k) {
    ResultBatch rb;
    taken_.clear();
    HostEngine::Job& j = job_[k];
    eng_->job_complete(j, rb.r, rb.f);
    eng_->job_finish(j, rb.r, taken_);
    job_live_[k] = false;
    --jobs_live_;
    eng_->settle(taken_);
    h_tick.observe(now_s() - job_t_post_[k]);
    if (ver_) ver_->check(j.created, rb.r, rb.f);
    c_ticks++;
    c_tick_slots += rb.r.size();
    apply(rb);
  }
  void tick_inline() {
    ResultBatch rb;
    const double tt = now_s();
    const int64_t created = (int64_t)time(nullptr);
    eng_->tick(created, rb.r, rb.f);
    h_tick.observe(now_s() - tt);
    if (ver_) ver_->check(created, rb.r, rb.f);
    c_ticks++;
    c_tick_slots += rb.r.size();
    apply(rb);
  }
  // read_fd = false: results picked up between the events of a busy iteration (the eventfd
  // stays readable and is drained when epoll reports it)
  void on_results(bool read_fd = true) {
    if (read_fd) {
      uint64_t v;
      ssize_t r = read(evfd_, &v, 8);
      cnt(SC_WAKE_READ);
      (void)r;
    }
    std::vector<ResultBatch>& q = scratch_rq_;
    q.clear();
    {
      std::lock_guard<std::mutex> g(rmu_);
      q.swap(rq_);
      rq_pending_.store(false, std::memory_order_relaxed);
    }
    const double t = now_s();
    for (auto& rb : q) {
      if (rb.t_routed > 0) {
        c_apply_ns += (uint64_t)((t - rb.t_routed) * 1e9);
        c_applies++;
      }
      apply(rb);
    }
    q.clear();  // now, not at the next call: an idle loop must not hold the batches (or their views)
  }
  void apply(ResultBatch& rb) {
    for (auto& r : rb.r) {
      auto it = slot_owner_.find(r.slot);
      // a result of an earlier session on this slot (ended while its tick was in flight; the
      // slot was freed and re-opened before this batch was applied) is dropped
      if (it == slot_owner_.end() || it->second.gen != r.gen) {
        r.hold = ViewRef();  // dropped: its bytes must not keep the lane's output arena pinned
        continue;
      }
      Session* s = it->second.s;
      int bi = it->second.bi;
      if (fault_drop_every_ > 0 && !r.empty() && ++fault_n_ % fault_drop_every_ == 0)
        r.clear_sse();  // QMX_FAULT_DROP_DELTA: fault injection (the bench's validator must notice)
      if (!r.empty()) {
        if (s->kind == K_REMOTE) {
          // framed from the view: one copy; XF_LAST: the owner may hold it for the session's
          // other streams (handle_x), never a stream's earlier deltas
          post_owner(s, X_DATA, (r.flags & (RF_DONE | RF_ABORTED)) ? XF_LAST : 0, 0, r.data(), r.size());
          s->data_sent++;
        } else if (s->cl) {
          // output coalescing across ticks: once the session's first content is out (TTFT),
          // a delta whose stream already has more bytes in the engine (fed, or in the other
          // tick in flight) waits for that output (<= one tick) instead of its own send — a
          // stream trickling in event by event otherwise costs a client send per tick.  A
          // stream with nothing pending (the steady-state LLM pace) is sent at once.
          // A stream's LAST output (its tick carried the end of the response) may also wait for
          // the rest of its session: another stream still running, or its final output (the
          // final event / the aggregator's answer) — one client send instead of one per tick.  A trickling
          // stream's earlier deltas never wait for other streams (per-token latency unchanged).
          const bool last = (r.flags & (RF_DONE | RF_ABORTED)) != 0;
          const bool hold = coalesce_s_ > 0 && s->first_content &&
                            (last ? session_hold(s, bi) : more_pending(r.slot, s->bs[bi].up));
          send_content(s, r.data(), r.size(), hold);
        }
      } else if (s->cl && s->cl->held && s->kind != K_REMOTE && !more_pending(r.slot, s->bs[bi].up))
        release_held(s->cl);  // its stream's held delta waited for this tick, which had nothing
      r.hold = ViewRef();  // the bytes were copied (or dropped): the lane may reuse its arena
      if ((r.flags & RF_ABORTED)) c_stream_aborts++;
      if ((r.flags & (RF_DONE | RF_ABORTED)) && s->bs[bi].state == 0) {
        s->bs[bi].state = 1;
        s->bs[bi].aborted = (r.flags & RF_ABORTED) != 0;
        if (s->bs[bi].t_fed > 0) h_engine.observe(lnow() - s->bs[bi].t_fed);
        s->finished++;
      }
      if (s->stage == 0 && s->finished == (int)s->bs.size()) begin_final(s);
    }
    for (auto& f : rb.f) {
      auto it = fin_owner_.find(f.id);
      if (it == fin_owner_.end()) continue;
      Session* s = it->second.first;
      const int bi = it->second.second;
      fin_owner_.erase(it);
      if (s->fin_id == f.id) s->fin_id = -1;
      on_finalized(s, f, bi);
    }
  }
  void kick() { kick_ = true; }
  HostEngine& eng() { return hub_ ? hub_->engine() : *eng_; }
  // engine calls, mirrored into the verify shadow when enabled
  // opens an engine slot for stream `bi` of session s and registers its owner
  // verify = false: a spread owner's shadow slot (its content comes from another rank)
  int e_open(Session* s, int bi, int index, bool f, bool e, bool verify = true) {
    uint32_t gen = 0;
    int slot;
    if (hub_) {
      slot = hub_->open(idx_, index, f, e, &gen, verify);
    } else {
      slot = eng_->open(index, f, e, &gen);
      if (heng_ && slot >= loop_slots_) c_host_path_opens++;  // beyond this loop's HBM slot state
      // latency mode (QMX_LIGHT_HOST=N, opt-in): a stream opened while this loop has no tick
      // on the GPU and has served at most N sessions at a time lately (an average over its
      // recent opens, so a momentary gap between two ticks under load does not count) runs on
      // the host path, byte-identical, without a GPU tick's fixed ~23 us (profiles/r6/lowload)
      else if (heng_ && light_host_ > 0) {
        sess_ema_ = 0.95 * sess_ema_ + 0.05 * (double)sessions_.size();
        if (jobs_live_ == 0 && sess_ema_ <= (double)light_host_) heng_->host_open(slot);
      }
      if (ver_ && verify) ver_->open(slot, gen, index, f, e);
    }
    slot_owner_[slot] = SlotOwner{s, bi, gen};
    return slot;
  }
  // feed / finish / release are queued in order and handed to the engine once per loop
  // iteration (flush_ops: one engine lock instead of one per upstream read — with the
  // shared engine, 8+ loops and the tick lanes otherwise contend on it per call)
  void e_feed_move(int slot, std::string& d) {
    if (ops_t0_ == 0) ops_t0_ = now_s();
    ops_.push_back(EngineOp{EngineOp::FEED, slot, std::move(d)});
  }
  void e_finish(int slot) { ops_.push_back(EngineOp{EngineOp::FINISH, slot, std::string()}); }
  void e_release(int slot) { ops_.push_back(EngineOp{EngineOp::RELEASE, slot, std::string()}); }
  void flush_ops() {
    if (ops_.empty()) return;
    if (ops_t0_ > 0) {
      c_flush_ns += (uint64_t)((now_s() - ops_t0_) * 1e9);
      c_flushes++;
      ops_t0_ = 0;
    }
    if (hub_) {
      hub_->apply_ops(ops_);
    } else {
      if (ver_) ver_->apply_ops(ops_);
      eng_->apply_ops(ops_, true);
    }
    ops_.clear();
    kick_ = true;
  }
  int e_submit(const std::vector<int>& slots, bool strip, bool texts, const std::string& joiner, int64_t created) {
    if (hub_) return hub_->submit(idx_, slots, strip, texts, joiner, created);
    int id = eng_->submit_finalize(slots, strip, texts, joiner, created);
    if (ver_) ver_->submit(id, slots, strip, texts, joiner, created);
    return id;
  }

  // Graceful drain: close the listener (SO_REUSEPORT peers / the next generation keep
  // accepting), close idle keep-alive connections, let in-flight sessions finish.
  // Returns true when this loop may exit.
  bool drain_step() {
    const double t = now_s();
    if (!draining_) {
      draining_ = true;
      drain_deadline_ = t + cfg_.drain_s;
      for (int* l : {&lfd_, &afd_}) {
        if (*l < 0) continue;
        on_accept(*l);  // connections already queued on this listener are served, not reset
        epoll_ctl(ep_, EPOLL_CTL_DEL, *l, nullptr);
        cnt(SC_EPOLL_CTL);
        close(*l);
        *l = -1;
      }
    }
    for (auto& kv : clients_) {
      Client* c = kv.second.get();
      // idle keep-alive connections close; a connection accepted but whose request has not
      // arrived yet gets a grace period (closing it would drop that request)
      const bool idle = !c->sess && c->in.empty() && c->out_off >= c->out.size();
      if (idle && (c->served > 0 || t - c->t_accept > 1.0)) mark_close(c);
    }
    if (!flushq_.empty()) flush_queued();
    if (!pending_close_.empty()) reap_clients();
    return (sessions_.empty() && clients_.empty()) || t > drain_deadline_;
  }

  // ---------------------------------------------------------------- clients
  void on_accept(int lfd) {
    while (true) {
      int fd = accept4(lfd, nullptr, nullptr, SOCK_NONBLOCK);
      if (fd < 0) break;
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      auto c = std::make_unique<Client>();
      c->fd = fd;
      c->serial = ++next_serial_;
      c->t_accept = lnow();
      add(fd, EPOLLIN, tag(3, fd));
      clients_[fd] = std::move(c);
      c_clients++;
    }
  }
  void reap_clients() {
    std::vector<int> fds;
    fds.swap(pending_close_);
    for (int fd : fds) {
      auto it = clients_.find(fd);
      if (it == clients_.end()) continue;
      Client* c = it->second.get();
      if (c->dead || (c->close_after && c->out_off >= c->out.size())) close_client(c);
    }
  }
  void mark_close(Client* c) {
    c->close_after = true;
    pending_close_.push_back(c->fd);
  }
  void on_client(Client* c, uint32_t ev) {
    if (ev & EPOLLOUT) flush_client(c);
    if (c->dead) return close_client(c);
    if (ev & (EPOLLIN | EPOLLHUP | EPOLLERR)) {
      char buf[65536];
      while (true) {
        ssize_t r = recv(c->fd, buf, sizeof(buf), 0);
        cnt(SC_RECV);
        if (r > 0) {
          c->in.append(buf, r);
          // a short read drained the socket: epoll is level-triggered, so skip the recv
          // that would only return EAGAIN (one syscall per request saved)
          if (r < (ssize_t)sizeof(buf)) break;
          continue;
        }
        if (r == 0 || (errno != EAGAIN && errno != EWOULDBLOCK)) c->dead = true;
        break;
      }
      if (!c->dead && !c->sess) process_requests(c);
      if (c->dead) return close_client(c);
    }
  }
  void close_client(Client* c) {
    if (c->sess) {
      c->sess->cl = nullptr;
      abort_session(c->sess);
    }
    epoll_ctl(ep_, EPOLL_CTL_DEL, c->fd, nullptr);
    cnt(SC_EPOLL_CTL);
    close(c->fd);
    clients_.erase(c->fd);
  }
  // Output is corked per loop iteration: everything written to a client while handling one
  // batch of epoll events and tick results (SSE headers + role event, several streams'
  // deltas, the last delta + [DONE]) leaves in ONE send at the end of the iteration.  A
  // loopback send runs the receiver's TCP input path in the sender's context, so sends —
  // not parsing — dominated the proxy's CPU profile (tools/cpuprof.py: __send 38%).
  void write_client(Client* c, const std::string& data) {
    if (c->dead) return;
    if (c->out.size() == c->out_off) {
      c->out.clear();
      c->out_off = 0;
    }
    c->out += data;
    if (!c->queued && !c->want_out) {
      c->queued = true;
      flushq_.push_back(c->fd);
    }
  }
  // HTTP chunk framing appended straight into the corked output (no temporary string)
  void write_chunk(Client* c, const std::string& data) { write_chunk(c, data.data(), data.size()); }
  void write_chunk(Client* c, const char* data, size_t len) {
    if (c->dead || len == 0) return;
    append_chunk(c, data, len);
    if (!c->queued && !c->want_out) {
      c->queued = true;
      flushq_.push_back(c->fd);
    }
  }
  void append_chunk(Client* c, const char* data, size_t len) {
    if (c->dead || len == 0) return;
    if (c->out.size() == c->out_off) {
      c->out.clear();
      c->out_off = 0;
    }
    char h[24];
    const int n = chunk_head(h, len);
    c->out.append(h, n);
    c->out.append(data, len);
    c->out.append("\r\n", 2);
  }
  void flush_queued() {
    std::vector<int>& fds = scratch_flush_;
    fds.clear();
    fds.swap(flushq_);
    for (int fd : fds) {
      auto it = clients_.find(fd);
      if (it == clients_.end()) continue;
      Client* c = it->second.get();
      c->queued = false;
      unhold(c);  // (held output leaves with this send; its deferral entry lapses)
      if (c->dead || c->want_out) continue;
      while (c->out_off < c->out.size()) {
        ssize_t w = send(c->fd, c->out.data() + c->out_off, c->out.size() - c->out_off, MSG_NOSIGNAL);
        cnt(SC_CLIENT_SEND);
        if (w > 0) {
          c->out_off += w;
          continue;
        }
        if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
          c->want_out = true;
          mod(c->fd, EPOLLIN | EPOLLOUT, tag(3, c->fd));
        } else {
          c->dead = true;
          pending_close_.push_back(c->fd);
        }
        break;
      }
      if (c->out_off >= c->out.size()) {
        c->out.clear();
        c->out_off = 0;
        if (c->close_after) pending_close_.push_back(c->fd);
      }
    }
  }
  void flush_client(Client* c) {
    while (c->out_off < c->out.size()) {
      ssize_t w = send(c->fd, c->out.data() + c->out_off, c->out.size() - c->out_off, MSG_NOSIGNAL);
      cnt(SC_CLIENT_SEND);
      if (w > 0) {
        c->out_off += w;
        continue;
      }
      if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) return;
      c->dead = true;
      return;
    }
    c->out.clear();
    c->out_off = 0;
    c->want_out = false;
    mod(c->fd, EPOLLIN, tag(3, c->fd));
    if (c->close_after) pending_close_.push_back(c->fd);
  }

  // parse as many complete requests as possible (one in flight at a time)
  void process_requests(Client* c) {
    while (!c->sess && !c->dead) {
      size_t he = c->in.find("\r\n\r\n");
      if (he == std::string::npos) {
        if (c->in.size() > (1 << 20)) c->dead = true;
        return;
      }
      // request line and headers parsed in place (no copy of the head)
      const char* head = c->in.data();
      const size_t le0 = c->in.find("\r\n");
      const size_t le = le0 == std::string::npos || le0 > he ? he : le0;
      const char* sp1p = (const char*)memchr(head, ' ', le);
      const char* sp2p = (const char*)memrchr(head, ' ', le);
      if (!sp1p || sp2p == sp1p) {
        c->dead = true;
        return;
      }
      const size_t sp1 = (size_t)(sp1p - head), sp2 = (size_t)(sp2p - head);
      thread_local std::string method, target;
      method.assign(head, sp1);
      target.assign(head + sp1 + 1, sp2 - sp1 - 1);
      const bool http10 = le - sp2 - 1 == 8 && memcmp(head + sp2 + 1, "HTTP/1.0", 8) == 0;
      std::vector<std::pair<std::string, std::string>> hdrs;
      hdrs.reserve(12);
      const size_t pos = le + 2;
      long clen = 0;
      bool chunked = false;
      bool keepalive = !http10;
      for_each_header(head + std::min(pos, he), he - std::min(pos, he), [&](std::string&& k, std::string&& v) {
        if (k == "content-length") clen = atol(v.c_str());
        if (k == "transfer-encoding" && icontains(v, "chunked")) chunked = true;
        if (k == "connection") {
          if (ieq(v, "close")) keepalive = false;
          if (ieq(v, "keep-alive")) keepalive = true;
        }
        hdrs.emplace_back(std::move(k), std::move(v));
      });
      std::string body;
      size_t used;
      if (chunked) {
        // decode a chunked request body
        size_t i = he + 4;
        bool complete = false;
        while (true) {
          size_t l2 = c->in.find("\r\n", i);
          if (l2 == std::string::npos) break;
          long sz = strtol(c->in.c_str() + i, nullptr, 16);
          if (sz == 0) {
            size_t t = c->in.find("\r\n\r\n", l2);
            if (t == std::string::npos) {
              if (c->in.size() >= l2 + 4 && c->in.compare(l2, 4, "\r\n\r\n") == 0) t = l2;
              else break;
            }
            i = t + 4;
            complete = true;
            break;
          }
          if (c->in.size() < l2 + 2 + sz + 2) break;
          body.append(c->in, l2 + 2, sz);
          i = l2 + 2 + sz + 2;
        }
        if (!complete) return;
        used = i;
      } else {
        if (c->in.size() < he + 4 + (size_t)clen) return;
        body = c->in.substr(he + 4, clen);
        used = he + 4 + clen;
      }
      c->in.erase(0, used);
      c->keepalive = keepalive && !draining_;
      handle_request(c, method, target, hdrs, body);
      if (!c->sess && !c->keepalive) {
        mark_close(c);
        return;
      }
    }
  }

  void respond(Client* c, int status, const std::string& ctype, const std::string& body,
               const std::vector<std::pair<std::string, std::string>>* extra = nullptr) {
    write_client(c, http_response(status, ctype, body, extra));
  }

  void handle_request(Client* c, const std::string& method, std::string target,
                      std::vector<std::pair<std::string, std::string>>& hdrs, std::string& body) {
    size_t q = target.find('?');
    if (q != std::string::npos) target.resize(q);
    if (method == "GET" && target == "/health") return respond(c, 200, "application/json", "{\"status\":\"healthy\"}");
    if (method == "GET" && target == "/metrics") return respond(c, 200, "text/plain; version=0.0.4", metrics_text());
    if (method == "GET" && target == "/openapi.json" && !cfg_.openapi_json.empty())
      return respond(c, 200, "application/json", cfg_.openapi_json);
    if (method == "GET" && target == "/docs" && !cfg_.docs_html.empty())
      return respond(c, 200, "text/html; charset=utf-8", cfg_.docs_html);
    if (method == "GET" && target == "/docs/oauth2-redirect" && !cfg_.oauth2_redirect_html.empty())
      return respond(c, 200, "text/html; charset=utf-8", cfg_.oauth2_redirect_html);
    if (method == "GET" && target == "/redoc" && !cfg_.redoc_html.empty())
      return respond(c, 200, "text/html; charset=utf-8", cfg_.redoc_html);
    if (target != "/chat/completions" && target != "/v1/chat/completions")
      return respond(c, 404, "application/json", "{\"detail\":\"Not Found\"}");
    if (method != "POST") return respond(c, 405, "application/json", "{\"detail\":\"Method Not Allowed\"}");
    c_requests++;
    c->served++;
    auto s = std::make_unique<Session>();
    s->t0 = lnow();
    std::string perr;
    if (!json_parse(body.data(), body.size(), s->body, &perr)) {
      c_errors++;
      return respond(c, 500, "application/json", err_json("Error processing request: " + perr, "proxy_error"));
    }
    if (s->body.t != JVal::OBJ) {
      c_errors++;
      const char* tn = s->body.t == JVal::ARR ? "list" : s->body.t == JVal::STR ? "str" : "int";
      return respond(c, 500, "application/json",
                     err_json(std::string("Error processing request: '") + tn + "' object has no attribute 'get'",
                              "proxy_error"));
    }
    const JVal* sv = s->body.get("stream");
    bool streaming = sv && sv->truthy();
    // forward all headers but host; auth fallback/normalisation; content-type default (quorum :972-1008)
    bool has_auth = false, has_ctype = false;
    s->fwd.reserve(hdrs.size() + 2);
    for (auto& h : hdrs) {
      if (h.first == "host") continue;
      if (h.first == "authorization") {
        has_auth = true;
        s->auth = h.second;
        continue;
      }
      if (h.first == "content-type") has_ctype = true;
      // hop-by-hop / entity headers are re-framed; accept-encoding dropped so upstream sends identity
      if (h.first == "content-length" || h.first == "transfer-encoding" || h.first == "connection" ||
          h.first == "keep-alive" || h.first == "te" || h.first == "upgrade" || h.first == "accept-encoding")
        continue;
      s->fwd.push_back(std::move(h));  // hdrs is not read again
    }
    if (!has_auth) {
      std::string env_key = cfg_.env_api_key;
      if (cfg_.api_key_from_env) {
        // per request, like os.environ.get (oai_proxy.py:981), from the environment snapshot
        // (qmx_env.h: getenv on an io thread can race a library's setenv and fault); a key
        // rotated inside this process applies once env_refresh() re-snapshots it
        const char* e = env_get("OPENAI_API_KEY");
        env_key = e ? e : "";
      }
      if (env_key.empty()) {
        c_errors++;
        return respond(c, 401, "application/json",
                       err_json("Authorization header is required and OPENAI_API_KEY environment variable is not set",
                                "auth_error"));
      }
      s->auth = "Bearer " + env_key;
    }
    s->fwd.emplace_back("Authorization", s->auth);
    if (!has_ctype) s->fwd.emplace_back("Content-Type", "application/json");
    if (!valid_init_) {
      valid_init_ = true;
      for (int i = 0; i < (int)cfg_.backends.size(); ++i)
        if (cfg_.backends[i].valid) valid_.push_back(i);
    }
    const std::vector<int>& valid = valid_;
    if (valid.empty())
      return respond(c, 500, "application/json", err_json("No valid backends configured", "configuration_error"));
    if (!s->body.get("model")) {
      bool any = false;
      for (int i : valid) any = any || !cfg_.backends[i].model.empty();
      if (!any)
        return respond(c, 400, "application/json",
                       err_json("Model must be specified when config.yaml model is blank", "invalid_request_error"));
    }
    bool parallel = cfg_.has_iterations_and_strategy && valid.size() > 1;
    s->raw = std::move(body);
    s->cl = c;
    Session* sp = s.get();
    sessions_[sp] = std::move(s);
    c->sess = sp;
    if (streaming && parallel) start_parallel(sp, valid);
    else if (streaming) start_single(sp, valid[0]);
    else start_nonstream(sp, valid, parallel);
  }

  // ---------------------------------------------------------------- upstream requests
  // call_backend body logic (quorum :157-180). Returns false with a synthetic result.
  bool upstream_body(Session* s, int b, std::string& out, int* st, std::string* msg, const char** etype) {
    const BackendCfg& be = cfg_.backends[b];
    if (!be.has_model_key) {
      *st = 500;
      *msg = "'model'";
      *etype = "proxy_error";
      return false;
    }
    if (!be.model.empty()) {
      // json.dumps of the body after body["model"] = model (quorum :161-163): the key keeps
      // its position, a new key goes last — serialised once per request around the value
      if (!s->msplit) {
        s->msplit = true;
        const auto& items = s->body.o;
        size_t k = 0;
        while (k < items.size() && items[k].first != "model") ++k;
        std::string& pre = s->mpre;
        pre.reserve(s->raw.size() + 32);
        pre.push_back('{');
        for (size_t i = 0; i < k; ++i) {
          if (i) pre += ", ";
          json_dump_str(items[i].first, pre);
          pre += ": ";
          json_dump(items[i].second, pre);
        }
        if (k > 0) pre += ", ";
        pre += "\"model\": ";
        for (size_t i = k + 1; i < items.size(); ++i) {
          s->mpost += ", ";
          json_dump_str(items[i].first, s->mpost);
          s->mpost += ": ";
          json_dump(items[i].second, s->mpost);
        }
        s->mpost.push_back('}');
      }
      out.reserve(s->mpre.size() + be.model.size() + s->mpost.size() + 8);
      out = s->mpre;
      json_dump_str(be.model, out);
      out += s->mpost;
      return true;
    }
    if (!s->body.get("model")) {
      *st = 400;
      *msg = "No model specified in config.yaml or request";
      *etype = "invalid_request_error";
      return false;
    }
    out = s->raw;
    return true;
  }
  std::string build_req(const BackendCfg& be, const std::vector<std::pair<std::string, std::string>>& hdrs,
                        const std::string& body) {
    // one reserved buffer, appended in place (the request line + headers were ~10 temporaries)
    size_t n = be.path.size() + be.host.size() + body.size() + 96;
    for (auto& h : hdrs) n += h.first.size() + h.second.size() + 4;
    std::string r;
    r.reserve(n);
    r.append("POST ").append(be.path).append("/chat/completions HTTP/1.1\r\nhost: ").append(be.host);
    char num[24];
    if (be.port != (be.https ? 443 : 80)) {
      r += ':';
      r.append(num, (size_t)dec_str(num, (size_t)be.port));
    }
    r.append("\r\n");
    for (auto& h : hdrs) r.append(h.first).append(": ").append(h.second).append("\r\n");
    r.append("content-length: ").append(num, (size_t)dec_str(num, body.size())).append("\r\n\r\n");
    r.append(body);
    return r;
  }
  Up* open_up(Session* s, int bi, int backend, UpMode mode, std::string req, double timeout) {
    const BackendCfg& be = cfg_.backends[backend];
    auto u = std::make_unique<Up>();
    u->backend = backend;
    u->sess = s;
    u->bi = bi;
    u->mode = mode;
    u->rp.keep_headers = mode != UP_ENGINE;
    u->req = std::move(req);
    u->timeout = timeout;
    u->last_io = lnow();
    u->t_open = u->last_io;
    u->deadline = cfg_.total_timeout > 0 ? u->last_io + cfg_.total_timeout : 0;
    if (!be.resolved || (be.https && !tls_)) return nullptr;
    int fd = -1;
    auto& pool = idle_[backend];
    while (!pool.empty() && fd < 0) {
      fd = pool.back();
      pool.pop_back();
      if (!parked_.count(fd)) {  // closed while parked (on_parked): stale entry
        fd = -1;
        continue;
      }
      u->reused = true;
      auto it = idle_ssl_.find(fd);
      if (it != idle_ssl_.end()) {
        u->ssl = it->second;
        idle_ssl_.erase(it);
      }
    }
    if (fd < 0) {
      fd = socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK, 0);
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      int r = connect(fd, (const sockaddr*)&be.addr, sizeof(be.addr));
      if (r != 0 && errno != EINPROGRESS) {
        close(fd);
        return nullptr;
      }
      u->connecting = r != 0;
      c_up_conns++;
      u->fd = fd;
      add(fd, EPOLLIN | EPOLLOUT, tag(4, fd));
      u->out_armed = true;
      if (be.https) {
        u->ssl = SSL_new(tls_);
        SSL_set_fd(u->ssl, fd);
        SSL_set_tlsext_host_name(u->ssl, be.host.c_str());
        X509_VERIFY_PARAM* vp = SSL_get0_param(u->ssl);
        in_addr ip4;
        if (inet_pton(AF_INET, be.host.c_str(), &ip4) == 1) X509_VERIFY_PARAM_set1_ip_asc(vp, be.host.c_str());
        else SSL_set1_host(u->ssl, be.host.c_str());
        u->tls_hs = true;
      }
    } else {
      u->fd = fd;  // pooled: still registered for EPOLLIN (no epoll_ctl on the reuse path)
      parked_.erase(fd);
    }
    Up* p = u.get();
    ups_[fd] = std::move(u);
    if (!p->connecting) {
      if (p->tls_hs) tls_step(p);
      else write_up(p);
    }
    return p;
  }
  // non-blocking TLS handshake step; on completion the request goes out
  void tls_step(Up* u) {
    ERR_clear_error();
    int r = SSL_connect(u->ssl);
    if (r == 1) {
      u->tls_hs = false;
      return write_up(u);
    }
    int e = SSL_get_error(u->ssl, r);
    if (e == SSL_ERROR_WANT_READ) return mod(u->fd, EPOLLIN, tag(4, u->fd));
    if (e == SSL_ERROR_WANT_WRITE) return mod(u->fd, EPOLLIN | EPOLLOUT, tag(4, u->fd));
    c_fail_connect++;
    up_error(u, "All connection attempts failed");
  }
  void write_up(Up* u) {
    while (u->req_off < u->req.size()) {
      if (u->ssl) {
        ERR_clear_error();
        int w = SSL_write(u->ssl, u->req.data() + u->req_off, (int)(u->req.size() - u->req_off));
        if (w > 0) {
          u->req_off += w;
          u->last_io = lnow();
          continue;
        }
        int e = SSL_get_error(u->ssl, w);
        if (e == SSL_ERROR_WANT_WRITE) {
          u->out_armed = true;
          return mod(u->fd, EPOLLIN | EPOLLOUT, tag(4, u->fd));
        }
        if (e == SSL_ERROR_WANT_READ) {
          u->out_armed = false;
          return mod(u->fd, EPOLLIN, tag(4, u->fd));
        }
        if (u->reused && !u->got_bytes) return retry_fresh(u);  // stale pooled TLS connection
        c_fail_connect++;
        return up_error(u, "All connection attempts failed");
      }
      ssize_t w = send(u->fd, u->req.data() + u->req_off, u->req.size() - u->req_off, MSG_NOSIGNAL);
      cnt(SC_UP_SEND);
      if (w > 0) {
        u->req_off += w;
        u->last_io = lnow();
        continue;
      }
      if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
        if (!u->out_armed) {
          u->out_armed = true;
          mod(u->fd, EPOLLIN | EPOLLOUT, tag(4, u->fd));
        }
        return;
      }
      c_fail_connect++;
      return up_error(u, "All connection attempts failed");
    }
    if (u->out_armed) {
      u->out_armed = false;
      mod(u->fd, EPOLLIN, tag(4, u->fd));
    }
  }
  // read what the socket (or the TLS layer) has: >0 bytes, 0 would block, -1 eof/error
  ssize_t up_read(Up* u, char* buf, size_t n) {
    if (!u->ssl) {
      ssize_t r = recv(u->fd, buf, n, 0);
      cnt(SC_RECV);
      if (r > 0) return r;
      if (r < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) return 0;
      return -1;
    }
    ERR_clear_error();
    int r = SSL_read(u->ssl, buf, (int)n);
    if (r > 0) return r;
    int e = SSL_get_error(u->ssl, r);
    if (e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE) return 0;
    return -1;
  }
  void on_up(Up* u, uint32_t ev) {
    if (u->connecting && (ev & (EPOLLOUT | EPOLLERR | EPOLLHUP))) {
      int err = 0;
      socklen_t len = sizeof(err);
      getsockopt(u->fd, SOL_SOCKET, SO_ERROR, &err, &len);
      if (err != 0) {
        c_fail_connect++;
        return up_error(u, "All connection attempts failed");
      }
      u->connecting = false;
    }
    const int fd = u->fd;
    if (u->tls_hs) {
      if (!u->connecting) tls_step(u);
      return;
    }
    if ((ev & (EPOLLOUT | (u->ssl ? EPOLLIN : 0))) && u->req_off < u->req.size()) {
      write_up(u);
      if (ups_.find(fd) == ups_.end()) return;
      if (u->req_off < u->req.size()) return;
    }
    if (ev & (EPOLLIN | EPOLLHUP | EPOLLERR)) {
      char buf[65536];
      bool eof = false;
      std::string body;
      while (true) {
        ssize_t r = up_read(u, buf, sizeof(buf));
        if (r > 0) {
          if (!u->got_bytes) h_upstream_ttfb.observe(lnow() - u->t_open);
          u->got_bytes = true;
          u->last_io = lnow();
          // a trickling upstream (read pacing): a short read of a response body already under
          // way — not the read that carried the headers (a whole response written after its
          // headers arrives as a header read and one body read, and never trickles)
          const bool in_body = u->rp.phase != 0;
          if (u->rp.feed(buf, r, body) < 0) {
            c_fail_protocol++;
            return up_error(u, "invalid HTTP response");
          }
          if (in_body && r < 2048 && !u->rp.done()) ++small_reads_;
          // plain TCP, short read: drained (level-triggered epoll reports more data); a
          // complete response needs no EAGAIN probe either.  TLS keeps reading: its
          // records can sit decrypted inside the SSL object with the socket empty.
          if (!u->ssl && (r < (ssize_t)sizeof(buf) || u->rp.done())) break;
          continue;
        }
        if (r < 0) eof = true;
        break;
      }
      if (!u->headers_seen && u->rp.phase > 0) {
        u->headers_seen = true;
        on_up_headers(u);
        if (ups_.find(fd) == ups_.end()) return;
      }
      if (!body.empty()) on_up_body(u, body);
      if (u->rp.done()) return up_complete(u, true);
      if (eof) {
        if (u->rp.phase == 6) return up_complete(u, false);
        if (!u->got_bytes && u->reused) return retry_fresh(u);
        c_fail_disconnect++;
        return up_error(u, "Server disconnected without sending a response.");
      }
    }
  }
  void retry_fresh(Up* u) {
    Session* s = u->sess;
    int bi = u->bi, backend = u->backend;
    UpMode mode = u->mode;
    std::string req = u->req;
    double to = u->timeout;
    drop_up(u, false);
    Up* nu = open_up(s, bi, backend, mode, req, to);
    if (!nu) return fail_backend(s, bi, 500, "All connection attempts failed", "proxy_error");
    if (bi >= 0) s->bs[bi].up = nu;
    else s->agg = nu;
  }
  void drop_up(Up* u, bool reuse) {
    int fd = u->fd;
    if (reuse && !u->rp.close && !u->tls_hs && !u->out_armed) {
      // parked, still registered for EPOLLIN: a keep-alive upstream sends nothing unasked,
      // so readiness while parked means it closed (on_parked); reuse needs no epoll_ctl
      idle_[u->backend].push_back(fd);
      parked_[fd] = u->backend;
      if (u->ssl) idle_ssl_[fd] = u->ssl;  // the TLS session stays with the pooled socket
    } else {
      epoll_ctl(ep_, EPOLL_CTL_DEL, fd, nullptr);
      cnt(SC_EPOLL_CTL);
      if (u->ssl) SSL_free(u->ssl);
      close(fd);
    }
    u->ssl = nullptr;
    ups_.erase(fd);
  }
  // readiness on a parked keep-alive socket: the upstream closed it (or broke protocol)
  void on_parked(int fd) {
    auto it = parked_.find(fd);
    if (it == parked_.end()) return;
    auto& pool = idle_[it->second];
    pool.erase(std::remove(pool.begin(), pool.end(), fd), pool.end());
    parked_.erase(it);
    auto s = idle_ssl_.find(fd);
    if (s != idle_ssl_.end()) {
      SSL_free(s->second);
      idle_ssl_.erase(s);
    }
    epoll_ctl(ep_, EPOLL_CTL_DEL, fd, nullptr);
    cnt(SC_EPOLL_CTL);
    close(fd);
  }
  void up_error(Up* u, const std::string& msg) {
    Session* s = u->sess;
    int bi = u->bi;
    c_up_fail++;
    drop_up(u, false);
    if (bi >= 0) s->bs[bi].up = nullptr;
    else s->agg = nullptr;
    fail_backend(s, bi, 500, msg, "proxy_error");
  }
  void sweep_timeouts(double t) {
    std::vector<int> expired;
    for (auto& kv : ups_) {
      Up* u = kv.second.get();
      if (t - u->last_io > u->timeout || (u->deadline > 0 && t > u->deadline)) expired.push_back(kv.first);
    }
    for (int fd : expired) {
      auto it = ups_.find(fd);
      if (it != ups_.end()) {
        c_fail_timeout++;
        up_error(it->second.get(), "");  // httpx timeouts stringify to ""
      }
    }
  }

  void on_up_headers(Up* u) {
    Session* s = u->sess;
    if (u->mode == UP_PASS && u->rp.status == 200) {
      // single-backend passthrough: upstream headers (minus entity/hop-by-hop) + own role event
      std::string h = "HTTP/1.1 200 OK\r\n";
      bool has_ct = false;
      for (auto& kv : u->rp.headers) {
        if (kv.first == "content-length" || kv.first == "transfer-encoding" || kv.first == "content-encoding" ||
            kv.first == "connection" || kv.first == "keep-alive")
          continue;
        if (kv.first == "content-type") has_ct = true;
        h += kv.first + ": " + kv.second + "\r\n";
      }
      if (!has_ct) h += "content-type: text/event-stream; charset=utf-8\r\n";
      h += "transfer-encoding: chunked\r\n\r\n";
      s->pass_started = true;
      if (s->cl) {
        write_client(s->cl, h);
        send_chunk(s, chunk_event_json("chatcmpl-role", (int64_t)time(nullptr), s->role_model_json,
                                       "{\"role\": \"assistant\"}", "null"));
      }
    }
  }
  // `body` is the caller's scratch: its bytes may be moved out
  void on_up_body(Up* u, std::string& body) {
    Session* s = u->sess;
    if (u->rp.status == 200 && u->mode == UP_ENGINE) {
      if (s->bs[u->bi].t_fed == 0) s->bs[u->bi].t_fed = lnow();
      e_feed_move(s->bs[u->bi].slot, body);  // the engine takes the buffer (no copy)
      kick();
      return;
    }
    if (u->rp.status == 200 && u->mode == UP_PASS) return pass_body(s, body);
    u->body += body;
  }
  void up_complete(Up* u, bool reusable) {
    Session* s = u->sess;
    int bi = u->bi;
    int status = u->rp.status;
    UpMode mode = u->mode;
    std::string body = std::move(u->body);
    auto rh = std::move(u->rp.headers);
    drop_up(u, reusable);
    if (bi >= 0) s->bs[bi].up = nullptr;
    else s->agg = nullptr;
    if (mode == UP_ENGINE && status == 200) {
      e_finish(s->bs[bi].slot);
      kick();
      return;
    }
    if (mode == UP_PASS && status == 200) return pass_end(s);
    // buffered result (call_backend classification)
    if (bi < 0) return on_aggregator_done(s, status, body);
    BState& b = s->bs[bi];
    b.status = status;
    b.rheaders = rh;
    JVal j;
    bool ok = utf8_valid((const uint8_t*)body.data(), 0, (int)body.size()) &&
              json_parse(body.data(), body.size(), j, nullptr);
    if (status == 200) {
      if (ok) {
        if (j.t == JVal::OBJ) j.set("backend", JVal::str(cfg_.backends[b.backend].name));
        else if (j.t == JVal::ARR) {
          return fail_backend(s, bi, 500, "list indices must be integers or slices, not str", "proxy_error");
        }
        b.is_json = true;
        b.js = std::move(j);
      } else {
        b.is_json = false;
        b.text = body;
      }
    } else {
      if (ok) {
        b.is_json = true;
        b.js = std::move(j);
      } else {
        JVal e;
        e.t = JVal::OBJ;
        JVal in;
        in.t = JVal::OBJ;
        in.set("message", JVal::str(body));
        in.set("type", JVal::str("backend_error"));
        e.set("error", in);
        b.is_json = true;
        b.js = std::move(e);
      }
      c_up_fail++; c_fail_status++;
    }
    if (mode == UP_ENGINE || mode == UP_PASS) {
      // non-200 on a streaming call
      return fail_backend(s, bi, status, error_message(b), nullptr, true);
    }
    b.state = 1;
    s->finished++;
    if (s->finished == (int)s->bs.size()) finish_nonstream(s);
  }
  static std::string error_message(const BState& b) {
    if (!b.is_json) return b.text;
    const JVal* e = b.js.get("error");
    if (e) {
      if (e->t == JVal::OBJ) {
        const JVal* m = e->get("message");
        return m ? py_str(*m) : "Unknown error";
      }
      return py_str(*e);
    }
    return py_str(b.js);
  }

  // record a failed backend (synthetic or transport) and advance the session
  void fail_backend(Session* s, int bi, int status, const std::string& msg, const char* etype, bool have_result = false) {
    if (bi < 0) return on_aggregator_done(s, 500, std::string());
    BState& b = s->bs[bi];
    if (b.state != 0) return;
    if (s->kind == K_REMOTE) {
      b.state = 2;
      post_owner(s, X_FINAL, XF_FAILED, status, have_result ? error_message(b) : msg, s->data_sent);
      return end_session(s);
    }
    if (!have_result) {
      b.status = status;
      JVal e;
      e.t = JVal::OBJ;
      JVal in;
      in.t = JVal::OBJ;
      in.set("message", JVal::str(msg));
      in.set("type", JVal::str(etype ? etype : "proxy_error"));
      e.set("error", in);
      b.is_json = true;
      b.js = std::move(e);
    }
    b.state = 2;
    s->finished++;
    if (s->kind == K_PAR) {
      if (s->stage == 0 && s->finished == (int)s->bs.size()) begin_final(s);
    } else if (s->kind == K_SINGLE) {
      if (s->cl) {
        if (s->pass_started) {
          write_client(s->cl, "0\r\n\r\n");
          s->cl->keepalive = false;
        } else {
          respond(s->cl, b.status, "application/json", err_json("Backend failed: " + error_message(b), "proxy_error"));
        }
      }
      end_session(s);
    } else if (s->finished == (int)s->bs.size()) {
      finish_nonstream(s);
    }
  }

  // ---------------------------------------------------------------- parallel streaming
  void send_chunk(Session* s, const std::string& data) {
    if (s->cl) write_chunk(s->cl, data);
  }
  // content-bearing events: the first one closes the session's TTFT span
  void send_content(Session* s, const std::string& data) { send_content(s, data.data(), data.size()); }
  void send_content(Session* s, const char* data, size_t len, bool hold = false) {
    if (!s->first_content) {
      s->first_content = true;
      h_ttft.observe(lnow() - s->t0);
    }
    if (!s->cl) return;
    Client* c = s->cl;
    if (!hold || c->queued || c->want_out || c->dead) return write_chunk(c, data, len);
    // held: corked without queueing the client, for as long as its stream keeps having more
    // bytes pending; the next unheld write to this client (the stream's last output, another
    // stream's, the final / [DONE]) sends it all, and the deferral deadline bounds the wait
    append_chunk(c, data, len);
    if (!c->held) {
      c->held = true;
      c->held_t0 = lnow();
      deferq_.push_back(Deferred{c->fd, c->serial, lnow() + coalesce_s_});
    }
    c_coalesced++;
  }
  // more output for this stream is on its way: bytes fed this iteration, in the engine (fed,
  // or in a tick in flight), or unread on its upstream socket.  The cheap look first; with
  // the shared engine (tick lanes) the FIONREAD before the engine lock the lanes also take
  bool more_pending(int slot, const Up* up) {
    if (ops_pending(slot)) return true;
    if (hub_) return up_readable(up) || eng().pending(slot);
    return eng().pending(slot) || up_readable(up);
  }
  // a finished stream's output may wait for the rest of its session: another of its streams
  // is still running, or (parallel sessions with a final output) the final event / the
  // aggregator's answer follows
  bool session_hold(const Session* s, int bi) const {
    if (s->stage == 0 && s->kind == K_PAR && final_follows_) return true;
    if (!session_hold_) return false;
    for (size_t k = 0; k < s->bs.size(); ++k)
      if ((int)k != bi && s->bs[k].state == 0) return true;
    return false;
  }
  void unhold(Client* c) {
    if (!c->held) return;
    c->held = false;
    c_hold_ns += (uint64_t)(1e9 * std::max(0.0, lnow() - c->held_t0));
    c_holds++;
  }
  // a held client's corked output goes out with this iteration's flush (as at its deadline)
  void release_held(Client* c) {
    if (!c->held || c->queued || c->dead) return;
    unhold(c);
    if (c->out_off >= c->out.size() || c->want_out) return;
    c->queued = true;
    flushq_.push_back(c->fd);
  }
  // the stream's upstream socket already holds unread bytes (its next events arrived while
  // this tick ran): one FIONREAD instead of a client send per tick of a trickling stream
  bool up_readable(const Up* u) const {
    if (!u || u->fd < 0 || u->ssl) return false;
    int n = 0;
    return ioctl(u->fd, FIONREAD, &n) == 0 && n > 0;
  }
  // a FEED for this slot is queued in this iteration's engine ops (not handed over yet)
  bool ops_pending(int slot) const {
    for (const EngineOp& o : ops_)
      if (o.slot == slot && o.kind == EngineOp::FEED) return true;
    return false;
  }
  void start_parallel(Session* s, const std::vector<int>& valid) {
    c_stream++;
    s->kind = K_PAR;
    s->filter = cfg_.hide_intermediate;
    s->emit = !cfg_.suppress;
    if (const JVal* sup = s->body.get("suppress_individual_responses")) s->emit = !sup->truthy();
    const bool defer = role_defer_s_ > 0 && s->cl && !s->cl->queued && !s->cl->want_out;
    // SSE head + chunked role event (quorum :530-541): identical within a second, cached
    const int64_t now_sec = (int64_t)time(nullptr);
    if (now_sec != role_sec_) {
      role_sec_ = now_sec;
      role_head_ = kSseHdr;
      role_head_ += chunk(chunk_event_json("chatcmpl-parallel", now_sec, "\"parallel-proxy\"",
                                           "{\"role\": \"assistant\"}", "null"));
    }
    write_client(s->cl, role_head_);
    if (defer && s->cl->queued && !flushq_.empty() && flushq_.back() == s->cl->fd) {
      flushq_.pop_back();  // un-queue: the first content (or the deadline) sends it
      s->cl->queued = false;
      deferq_.push_back(Deferred{s->cl->fd, s->cl->serial, now_s() + role_defer_s_});
    }
    s->bs.resize(valid.size());
    // spread placement (EP analog): backend i of a session owned by rank r runs on rank
    // (r + i) % world; its deltas and final text come back through the exchange (R1)
    const bool spread = xch_ && xch_->healthy() && (xch_->world() > 1 || self_spread_);
    if (spread) {
      s->skey = ((uint64_t)xch_->rank() << 56) | ((uint64_t)idx_ << 48) | next_skey_++;
      rsess_[s->skey] = s;
    }
    for (size_t i = 0; i < valid.size(); ++i) {
      s->bs[i].backend = valid[i];
      const int target = spread ? (xch_->rank() + (int)i) % xch_->world() : -1;
      // (self spread: every odd backend of a one-rank deployment goes through its own
      // exchange — opens, deltas and RCCL rounds to itself)
      if (spread && (target != xch_->rank() || (self_spread_ && (i & 1))) && xch_->peer_up(target)) {
        s->bs[i].remote = target;
        s->bs[i].via_link = link_up(target);  // the whole stream keeps one path (message order)
        s->remote_n++;
        // the owner's shadow slot: the remote stream's final text lands in its HBM content
        // area (RCCL, HBM to HBM), so this rank's fused finalize merges remote and local
        // streams alike; it is never fed upstream bytes
        s->bs[i].slot = e_open(s, (int)i, (int)i, false, false, false);
        size_t cap = 0;
        void* dev = eng().content_device_ptr(s->bs[i].slot, &cap);
        xch_->expect_bulk(s->skey, (int)i, dev, cap);
        continue;
      }
      s->bs[i].slot = e_open(s, (int)i, (int)i, s->filter, s->emit);
    }
    for (size_t i = 0; i < valid.size(); ++i) {
      std::string body, msg;
      int st = 0;
      const char* et = nullptr;
      if (!upstream_body(s, valid[i], body, &st, &msg, &et)) {
        fail_backend(s, (int)i, st, msg, et);
        continue;
      }
      if (s->bs[i].remote >= 0) {
        XMsg m;
        m.type = X_OPEN;
        m.flags = (uint8_t)((s->filter ? 1 : 0) | (s->emit ? 2 : 0));
        m.dst_rank = s->bs[i].remote;
        m.src_rank = xch_->rank();
        m.dst_loop = m.src_loop = (uint16_t)idx_;
        m.bi = (int)i;
        m.skey = s->skey;
        m.a = valid[i];
        m.b = (int)(cfg_.timeout * 1000.0);
        m.payload = build_req(cfg_.backends[valid[i]], s->fwd, body);
        xq(m, s->bs[i].via_link);
        s->bs[i].t_sp_open = now_s();
        continue;
      }
      Up* u = open_up(s, (int)i, valid[i], UP_ENGINE, build_req(cfg_.backends[valid[i]], s->fwd, body), cfg_.timeout);
      if (!u) fail_backend(s, (int)i, 500, "All connection attempts failed", "proxy_error");
      else s->bs[i].up = u;
    }
  }
  std::vector<int> good_slots(Session* s) {
    std::vector<int> g;
    for (auto& b : s->bs)
      if (b.state == 1 && !b.aborted) g.push_back(b.slot);
    return g;
  }
  void begin_final(Session* s) {
    s->stage = 1;
    if (s->kind == K_REMOTE) {  // worker: ship the stream's final text to the owner
      const BState& b = s->bs[0];
      const size_t len = b.aborted || cfg_.skip_final ? 0 : eng().content_size(b.slot);
      if (s->emit && !b.aborted && s->data_sent == 0 && eng().content_size(b.slot) > 0) {
        // content reached the engine but not one delta left for the owner: an emitting
        // stream's every non-empty filtered delta is an event (oai_proxy.py:629-652)
        c_sp_nodata++;
        if (g_sp_logs.fetch_add(1) < 20)
          fprintf(stderr, "qmx spread (rank %d loop %d): worker stream slot %d has %zu content bytes but sent no delta "
                  "(skey %llx bi %d filter %d)\n", cfg_.rank, idx_, b.slot, eng().content_size(b.slot),
                  (unsigned long long)s->owner_skey, s->shadow_bi, (int)s->filter);
      }
      if (len == 0) {
        post_owner(s, X_FINAL, b.aborted ? XF_ABORTED : 0, 0, std::string(), s->data_sent);
        return end_session(s);
      }
      const bool eager = (long long)len <= (long long)cfg_.xchg_eager_bytes;
      size_t cap0 = 0;
      // the text's bytes are needed on the host (eager, or a host transport: tcp mesh /
      // tcpbulk / RCCL not formed) and sit in HBM: the loop's next tick copies them out in a
      // texts-kind finalize item (on_finalized resumes here).  A synchronous hipMemcpy per
      // text on the io loop cost ~70 us of CPU each (4-rank spread profile, round 6)
      const bool host_bytes = eager || !(xch_->transport() == "rccl" && xch_->rccl_active());
      if (host_bytes && !s->fetched && eng().content_device_ptr(b.slot, &cap0) != nullptr) {
        s->fetching = true;  // (on_finalized runs begin_final again when the text is in)
        s->fin_id = e_submit({b.slot}, false, true, std::string(), (int64_t)time(nullptr));
        fin_owner_[s->fin_id] = {s, -1};
        kick();
        return;
      }
      if (eager) {
        // eager: a short text rides this loop's mesh frames right behind the stream's deltas
        // (one hop, no rank-0 manifest); the owner applies it as it would a round's delivery
        const std::string t = s->fetched ? std::move(s->fetched_text) : eng().text(b.slot);
        post_owner(s, X_BULK, XF_TEXT, (int)t.size(), t.data(), t.size(), s->data_sent);
        c_sp_eager++;
        return end_session(s);
      }
      // HBM content slot → the owner's shadow slot (RCCL p2p round), or its bytes over the
      // mesh; the slot stays ours until X_SENT says the transfer has left
      XMsg h;
      h.flags = XF_TEXT;
      h.dst_rank = s->owner_rank;
      h.src_rank = xch_->rank();
      h.dst_loop = (uint16_t)s->owner_loop;
      h.src_loop = (uint16_t)idx_;
      h.bi = s->shadow_bi;
      h.skey = s->owner_skey;
      h.b = s->data_sent;  // the owner applies the final after this many deltas
      size_t cap = 0;
      const void* dev = eng().content_device_ptr(b.slot, &cap);
      HostEngine* e = &eng();
      const int slot = b.slot;
      s->bulk_pending = true;
      flush_x();  // the stream's deltas go out ahead of its final text
      if (s->fetched) {  // host bytes already copied out by the tick: no device read on any thread
        std::string t = std::move(s->fetched_text);
        xch_->send_bulk(std::move(h), dev, len, [t] { return t; });
      } else {
        xch_->send_bulk(std::move(h), dev, len, [e, slot] { return e->text(slot); });
      }
      return;
    }
    if (cfg_.skip_final) return finish_stream(s);
    // (spread owners included: remote streams' texts sit in their shadow slots)
    std::vector<int> g = good_slots(s);
    bool texts = !cfg_.aggregator_name.empty();
    bool strip = cfg_.hide_final;
    if (texts && cfg_.documented) {
      // documented semantics: only the source backends feed the aggregator, stripped with
      // strip_intermediate_thinking; the finalize keeps the texts of slots with content, in
      // slot order, so their backends' names are known here (the prompt's source labels)
      g.clear();
      s->text_names.clear();
      for (auto& b : s->bs)
        if (b.state == 1 && !b.aborted && is_source(b.backend)) {
          g.push_back(b.slot);
          if (eng().content_size(b.slot) > 0) s->text_names.push_back(cfg_.backends[b.backend].name);
        }
      strip = strip || cfg_.strip_intermediate;
    }
    s->fin_texts = texts;
    s->fin_id = e_submit(g, strip, texts, "\n" + cfg_.separator, (int64_t)time(nullptr));
    fin_owner_[s->fin_id] = {s, -1};
    kick();
  }
  bool is_source(int backend) const {
    if (cfg_.sources_all) return true;
    for (const auto& n : cfg_.sources)
      if (n == cfg_.backends[backend].name) return true;
    return false;
  }
  void post_owner(Session* s, uint8_t type, uint8_t flags, int a, const std::string& payload, int b = 0) {
    post_owner(s, type, flags, a, payload.data(), payload.size(), b);
  }
  // mesh messages of this loop pass, framed per destination rank and handed to the exchange
  // once per pass (flush_x: one lock + one wake), not one locked post + wake per message
  // link: over this loop's own connection to the rank (a frame for a link that went down is
  // dropped, as the mesh drops frames for a peer that is down: its sessions were failed)
  void xq(const XMsg& hdr, const char* payload, size_t n, bool link) {
    if (!xch_) return;
    if (link) {
      if (hdr.dst_rank < 0 || hdr.dst_rank >= (int)xl_.size() || xl_[hdr.dst_rank].fd < 0) return;
      XLink& L = xl_[hdr.dst_rank];
      if (L.out_off == L.out.size()) {
        L.out.clear();
        L.out_off = 0;
      }
      Exchange::append_frame(L.out, hdr, payload, n);
      xlpending_ = true;
      c_link_msgs++;
      return;
    }
    if (xout_.size() < (size_t)xch_->world()) xout_.resize(xch_->world());
    Exchange::append_frame(xout_[hdr.dst_rank], hdr, payload, n);
    xpending_ = true;
  }
  void xq(const XMsg& m, bool link) { xq(m, m.payload.data(), m.payload.size(), link); }
  void flush_x() {
    if (xlpending_) {
      xlpending_ = false;
      for (int r = 0; r < (int)xl_.size(); ++r)
        if (xl_[r].fd >= 0 && !xl_[r].want_out && xl_[r].out_off < xl_[r].out.size()) flush_link(r);
    }
    if (!xpending_) return;
    xpending_ = false;
    for (int r = 0; r < (int)xout_.size(); ++r) xch_->post_frames(r, xout_[r]);
  }
  // ---- per-loop links (Exchange X_LINK): this loop's own socket to loop idx_ of each rank
  struct XLink {
    int fd = -1;
    std::string in, out;
    size_t out_off = 0;
    bool want_out = false;
  };
  bool link_up(int r) const { return r >= 0 && r < (int)xl_.size() && xl_[r].fd >= 0; }
  void on_link_msg(const XMsg& m) {  // X_LINK: adopt the socket (replacing a stale one)
    const int r = m.a, fd = m.b;
    if (!xch_ || r < 0 || r >= xch_->world()) {
      close(fd);
      return;
    }
    if (xl_.size() < (size_t)xch_->world()) xl_.resize(xch_->world());
    // a stale link (the pair's mesh connection re-formed): its unsent frames and unparsed bytes
    // go with it, so the streams that travelled on it are failed (as for a link that broke);
    // streams on the mesh are unaffected
    if (xl_[r].fd >= 0) link_down(r, true, true);
    xl_[r].fd = fd;
    xl_[r].in = m.payload;
    add(fd, EPOLLIN, tag(7, fd));
    if (!xl_[r].in.empty()) read_link(r, false);
  }
  int link_of(int fd) const {
    for (int r = 0; r < (int)xl_.size(); ++r)
      if (xl_[r].fd == fd) return r;
    return -1;
  }
  void on_link(int fd, uint32_t ev) {
    const int r = link_of(fd);
    if (r < 0) return;
    if (ev & EPOLLOUT) flush_link(r);
    if (xl_[r].fd >= 0 && (ev & (EPOLLIN | EPOLLHUP | EPOLLERR))) read_link(r, true);
  }
  void read_link(int r, bool do_recv) {
    XLink& L = xl_[r];
    bool dead = false;
    while (do_recv) {
      char buf[65536];
      ssize_t n = recv(L.fd, buf, sizeof(buf), 0);
      cnt(SC_RECV);
      if (n > 0) {
        L.in.append(buf, (size_t)n);
        if (n < (ssize_t)sizeof(buf)) break;
        continue;
      }
      if (n == 0 || (errno != EAGAIN && errno != EWOULDBLOCK)) dead = true;
      break;
    }
    std::vector<XMsg> msgs;
    const size_t used = Exchange::parse_frames(L.in, msgs);
    L.in.erase(0, used);
    if (!msgs.empty()) handle_x(msgs, true);
    if (dead) link_down(r, true);
  }
  void flush_link(int r) {
    XLink& L = xl_[r];
    while (L.fd >= 0 && L.out_off < L.out.size()) {
      ssize_t w = send(L.fd, L.out.data() + L.out_off, L.out.size() - L.out_off, MSG_NOSIGNAL);
      cnt(SC_UP_SEND);
      if (w > 0) {
        L.out_off += (size_t)w;
        continue;
      }
      if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
        if (!L.want_out) {
          L.want_out = true;
          mod(L.fd, EPOLLIN | EPOLLOUT, tag(7, L.fd));
        }
        return;
      }
      return link_down(r, true);
    }
    if (L.fd >= 0) {
      L.out.clear();
      L.out_off = 0;
      if (L.want_out) {
        L.want_out = false;
        mod(L.fd, EPOLLIN, tag(7, L.fd));
      }
    }
  }
  // a link closed: its streams end as for a peer that left this loop's reach (X_DOWN); new
  // sessions use the mesh until the exchange hands over a new link
  // link_only: fail only the streams that travelled on the link (their frames may be lost
  // with it); otherwise every stream shared with rank r, as for a rank that left
  void link_down(int r, bool fail_streams, bool link_only = false) {
    XLink& L = xl_[r];
    if (L.fd < 0) return;
    epoll_ctl(ep_, EPOLL_CTL_DEL, L.fd, nullptr);
    cnt(SC_EPOLL_CTL);
    close(L.fd);
    L = XLink();
    if (!fail_streams) return;
    std::vector<XMsg> v(1);
    v[0].type = X_DOWN;
    v[0].a = r;
    v[0].b = link_only ? 1 : 0;
    handle_x(v, true);
  }
  void post_owner(Session* s, uint8_t type, uint8_t flags, int a, const char* payload, size_t n, int b = 0) {
    if (!xch_) return;
    XMsg m;
    m.type = type;
    m.flags = flags;
    m.dst_rank = s->owner_rank;
    m.src_rank = xch_->rank();
    m.dst_loop = (uint16_t)s->owner_loop;
    m.src_loop = (uint16_t)idx_;
    m.bi = s->shadow_bi;
    m.skey = s->owner_skey;
    m.a = a;
    m.b = b;
    xq(m, payload, n, s->via_link);
  }
  // owner: a remote stream ends with `sent` deltas announced by its worker; anything else
  // than the count received means deltas were lost or are still missing
  bool delta_check(Session* s, int bi, int sent, const char* how) {
    const BState& b = s->bs[bi];
    if (b.rx_data == sent) return true;
    c_sp_delta_mismatch++;
    if (g_sp_logs.fetch_add(1) < 20)
      fprintf(stderr, "qmx spread (rank %d loop %d): remote stream %d of session %llx (rank %d) ended by %s after %d "
              "of its %d deltas\n", cfg_.rank, idx_, bi, (unsigned long long)s->skey, b.remote, how, b.rx_data, sent);
    return false;
  }
  void on_xmsgs() {
    uint64_t v;
    ssize_t r = read(xfd_, &v, 8);
    cnt(SC_WAKE_READ);
    (void)r;
    std::vector<XMsg> in;
    {
      std::lock_guard<std::mutex> g(xmu_);
      in.swap(xin_);
    }
    handle_x(in, false);
  }
  // exchange messages from the mesh thread (link = false) or this loop's own links
  void handle_x(std::vector<XMsg>& in, bool link) {
    for (auto& m : in) {
      if (m.type == X_UP) continue;  // a peer (re)joined: new sessions may place streams there
      if (m.type == X_RELEASE) {  // a deferred shadow-slot release: its round is over
        if (m.a >= 0) e_release(m.a);
        continue;
      }
      if (m.type == X_LINK) {
        on_link_msg(m);
        continue;
      }
      if (m.type == X_DOWN) {
        // peer m.a (or, a = -1, every peer) is unreachable: fail the streams it runs for
        // our sessions, drop the streams we run for its sessions (a worker whose final
        // text is in flight waits for X_SENT, which the exchange always sends)
        // (b = 1: a replaced link — only the streams that used it)
        const bool link_only = m.b == 1;
        std::vector<Session*> owners, shadows;
        for (auto& kv : rsess_) owners.push_back(kv.second);
        for (auto& kv : shadow_) shadows.push_back(kv.second);
        for (Session* s : shadows)
          if (sessions_.count(s) && (m.a < 0 || s->owner_rank == m.a) && !s->bulk_pending &&
              (!link_only || s->via_link))
            end_session(s);
        for (Session* s : owners) {
          for (int i = 0; i < (int)s->bs.size() && sessions_.count(s); ++i)
            if (s->bs[i].remote >= 0 && (m.a < 0 || s->bs[i].remote == m.a) && s->bs[i].state == 0 &&
                (!link_only || s->bs[i].via_link)) {
              c_sp_down++;
              fail_backend(s, i, 500, "rank exchange failed", "proxy_error");
            }
        }
        continue;
      }
      if (m.type == X_OPEN) {
        auto sp = std::make_unique<Session>();
        Session* s = sp.get();
        sessions_[s] = std::move(sp);
        s->kind = K_REMOTE;
        s->owner_rank = m.src_rank;
        s->owner_loop = m.src_loop;
        s->owner_skey = m.skey;
        s->shadow_bi = m.bi;
        s->via_link = link;
        s->filter = m.flags & 1;
        s->emit = (m.flags & 2) != 0;
        s->bs.resize(1);
        s->bs[0].backend = m.a;
        s->bs[0].slot = e_open(s, 0, m.bi, s->filter, s->emit);
        shadow_[{m.skey, m.bi}] = s;
        c_remote_streams++;
        Up* u = (m.a >= 0 && m.a < (int)cfg_.backends.size())
                    ? open_up(s, 0, m.a, UP_ENGINE, std::move(m.payload), m.b / 1000.0) : nullptr;
        if (!u) fail_backend(s, 0, 500, "All connection attempts failed", "proxy_error");
        else s->bs[0].up = u;
        continue;
      }
      if (m.type == X_CANCEL || m.type == X_SENT) {  // worker side
        auto it = shadow_.find({m.skey, m.bi});
        if (it == shadow_.end()) continue;
        Session* s = it->second;
        if (m.type == X_SENT) s->bulk_pending = false;
        if (!s->bulk_pending) end_session(s);  // a cancel during the transfer ends it at X_SENT
        continue;
      }
      auto it = rsess_.find(m.skey);
      if (it == rsess_.end()) continue;
      Session* s = it->second;
      if (m.bi < 0 || m.bi >= (int)s->bs.size()) continue;
      BState& b = s->bs[m.bi];
      if (m.type == X_DATA) {
        const double t = now_s();
        if (b.rx_data == 0 && b.t_sp_open > 0) h_sp_first.observe(t - b.t_sp_open);
        b.t_sp_last = t;
        b.rx_data++;
        if (s->cl) {
          // the session's other streams arrive from other ranks, each in a pass of its own: after
          // the first content (TTFT is not delayed), a remote stream's last deltas wait corked (at
          // most the coalescing deadline) while the rest of the session is still to come — the
          // last arrival's output sends them all, one client send instead of one per rank
          const bool hold = coalesce_s_ > 0 && s->first_content && (m.flags & XF_LAST) && session_hold(s, m.bi);
          send_content(s, m.payload.data(), m.payload.size(), hold);
        }
        if (b.bulk_waiting && b.rx_data >= b.bulk_msg.b) {
          b.bulk_waiting = false;
          XMsg bm = std::move(b.bulk_msg);
          remote_final(s, m.bi, bm);
        }
        continue;
      }
      if (m.type == X_BULK) {
        if (b.state != 0) continue;  // a duplicate (RCCL round failed after delivering)
        if (b.rx_data < m.b) {  // deltas still in flight on the mesh: apply it after them
          b.bulk_waiting = true;
          b.bulk_msg = std::move(m);
          continue;
        }
        remote_final(s, m.bi, m);
        continue;
      }
      if (m.type == X_FINAL) {
        if (b.state != 0) continue;
        delta_check(s, m.bi, m.b, (m.flags & XF_FAILED) ? "failure" : (m.flags & XF_ABORTED) ? "abort" : "empty final");
        if (m.flags & XF_FAILED) {
          c_sp_failed++;
          if (g_sp_logs.fetch_add(1) < 20)
            fprintf(stderr, "qmx spread (rank %d loop %d): remote stream %d of session %llx failed on rank %d: %d %s\n",
                    cfg_.rank, idx_, m.bi, (unsigned long long)s->skey, m.src_rank, m.a, m.payload.substr(0, 200).c_str());
          fail_backend(s, m.bi, m.a, m.payload, "proxy_error");
          continue;
        }
        if (m.flags & XF_ABORTED) c_sp_aborted++;
        else c_sp_empty++;
        sp_final_time(b);
        b.state = 1;
        b.aborted = (m.flags & XF_ABORTED) != 0;
        s->finished++;
        if (s->stage == 0 && s->finished == (int)s->bs.size()) begin_final(s);
      }
    }
  }
  static void sp_final_time(const BState& b) {
    const double t0 = b.t_sp_last > 0 ? b.t_sp_last : b.t_sp_open;
    if (t0 > 0) h_sp_final.observe(now_s() - t0);
  }
  // owner: a remote stream's final text is in (HBM already, or the mesh payload)
  void remote_final(Session* s, int bi, XMsg& m) {
    BState& b = s->bs[bi];
    if (b.state != 0) return;
    delta_check(s, bi, m.b, "final text");
    c_sp_text++;
    sp_final_time(b);
    // over the mesh the bytes are in the payload; an RCCL round already wrote them to HBM
    // (a final text is never empty: an empty one travels as X_FINAL)
    const bool bytes = !m.payload.empty();
    eng().set_remote_content(b.slot, bytes ? &m.payload : nullptr, bytes ? m.payload.size() : (size_t)m.a,
                             (m.flags & XF_HOSTCOPY) != 0);
    xch_->forget_bulk(s->skey, bi);
    b.state = 1;
    b.aborted = false;
    s->finished++;
    if (s->stage == 0 && s->finished == (int)s->bs.size()) begin_final(s);
  }
  void on_finalized(Session* s, FinalizeRes& f, int /*bi*/) {
    if (s->kind == K_REMOTE) {  // a worker's final text, fetched from HBM: ship it now
      if (!s->fetching) return;
      s->fetching = false;
      s->fetched = true;
      s->fetched_text = f.texts.empty() ? std::string() : std::move(f.texts[0]);
      c_sp_fetched++;
      return begin_final(s);
    }
    if (s->kind == K_NONSTREAM) return;  // not used
    if (!s->fin_texts) {
      if (f.kind == 1) send_chunk(s, f.event);
      else send_chunk(s, error_event());
      return finish_stream(s);
    }
    if (f.texts.empty()) {
      send_chunk(s, error_event());
      return finish_stream(s);
    }
    s->texts = std::move(f.texts);
    start_aggregator(s, "\n" + cfg_.separator);
  }
  std::string error_event() {
    return chunk_event_json("error", (int64_t)time(nullptr), "\"parallel-proxy\"",
                            "{\"content\": \"Error: All backends failed to provide content\"}", "\"error\"");
  }
  std::string joined(const std::vector<std::string>& t, const std::string& sep) {
    std::string o;
    for (size_t i = 0; i < t.size(); ++i) {
      if (i) o += sep;
      o += t[i];
    }
    return o;
  }
  void emit_final_value(Session* s, const JVal& content) {
    std::string delta = "{\"content\": " + json_dumps(content) + "}";
    send_chunk(s, chunk_event_json("chatcmpl-parallel-final", (int64_t)time(nullptr), "\"parallel-proxy\"", delta,
                                   "\"stop\""));
    finish_stream(s);
  }
  void finish_stream(Session* s) {
    send_chunk(s, kDone);
    if (s->cl) write_client(s->cl, "0\r\n\r\n");
    end_session(s);
  }

  // ---------------------------------------------------------------- aggregator
  // exc_joiner: join used when prompt building raises (quorum's outer except)
  void start_aggregator(Session* s, const std::string& exc_joiner) {
    s->stage = 2;
    int ab = -1;
    for (int i = 0; i < (int)cfg_.backends.size(); ++i)
      if (cfg_.backends[i].name == cfg_.aggregator_name) {
        ab = i;
        break;
      }
    if (ab < 0) return aggregate_result(s, JVal::str(joined(s->texts, exc_joiner)));
    // prompt (quorum :406-423)
    std::vector<std::string> parts;
    for (size_t i = 0; i < s->texts.size(); ++i) {
      if (cfg_.include_source_names) {
        std::string lab;
        const std::string name = cfg_.documented && i < s->text_names.size() ? s->text_names[i]
                                                                              : "LLM" + std::to_string(i + 1);
        if (!py_format(cfg_.source_label_format, "backend_name", name, lab))
          return aggregate_result(s, JVal::str(joined(s->texts, exc_joiner)));
        parts.push_back(lab + s->texts[i]);
      } else {
        parts.push_back(s->texts[i]);
      }
    }
    std::string prompt;
    if (cfg_.include_original_query) {
      std::string uq;
      const JVal* msgs = s->body.get("messages");
      if (msgs && msgs->truthy() && msgs->t == JVal::ARR) {
        for (auto& m : msgs->a) {
          const JVal* r = m.get("role");
          if (r && r->t == JVal::STR && r->s == "user") {
            const JVal* ct = m.get("content");
            uq = ct ? py_str(*ct) : "";
            break;
          }
        }
      }
      if (!py_format(cfg_.query_format, "query", uq, prompt))
        return aggregate_result(s, JVal::str(joined(s->texts, exc_joiner)));
    }
    std::string inter = joined(parts, cfg_.intermediate_separator);
    std::string tmpl = cfg_.prompt_template;
    std::string out;
    for (size_t i = 0; i < tmpl.size();) {
      if (tmpl.compare(i, 11, "{responses}") == 0) {
        out += inter;
        i += 11;
      } else {
        out.push_back(tmpl[i++]);
      }
    }
    prompt += out;
    const BackendCfg& be = cfg_.backends[ab];
    JVal req;
    req.t = JVal::OBJ;
    req.set("model", JVal::str(be.model));
    JVal msgs;
    msgs.t = JVal::ARR;
    JVal m;
    m.t = JVal::OBJ;
    m.set("role", JVal::str("user"));
    m.set("content", JVal::str(prompt));
    msgs.a.push_back(m);
    req.set("messages", msgs);
    req.set("stream", JVal::boolean(false));
    std::vector<std::pair<std::string, std::string>> h = {{"Authorization", s->auth},
                                                          {"Content-Type", "application/json"}};
    if (!be.valid || !be.has_model_key) return on_aggregator_done(s, 500, std::string());
    Up* u = open_up(s, -1, ab, UP_BUFFER, build_req(be, h, json_dumps(req)), 60.0);
    if (!u) return on_aggregator_done(s, 500, std::string());
    s->agg = u;
  }
  void on_aggregator_done(Session* s, int status, const std::string& body) {
    JVal j;
    if (status == 200 && json_parse(body.data(), body.size(), j, nullptr)) {
      const JVal* ch = j.get("choices");
      if (ch && ch->t == JVal::ARR && !ch->a.empty()) {
        const JVal* msg = ch->a[0].get("message");
        const JVal* ct = msg ? msg->get("content") : nullptr;
        if (ct && cfg_.documented && cfg_.hide_aggregator_think && ct->t == JVal::STR)
          return aggregate_result(s, JVal::str(strip_final(ts_, (const uint8_t*)ct->s.data(), ct->s.size())));
        if (ct) return aggregate_result(s, *ct);
      }
    }
    aggregate_result(s, JVal::str(joined(s->texts, cfg_.intermediate_separator)));
  }
  void aggregate_result(Session* s, const JVal& v) {
    if (s->kind == K_PAR) return emit_final_value(s, v);
    finish_nonstream_combined(s, v);
  }

  // ---------------------------------------------------------------- single-backend streaming
  void start_single(Session* s, int backend) {
    c_stream++;
    s->kind = K_SINGLE;
    s->bs.resize(1);
    s->bs[0].backend = backend;
    const JVal* m = s->body.get("model");
    if (m && m->truthy()) s->role_model_json = json_dumps(*m);
    else s->role_model_json = cfg_.backends[backend].has_model_key ? json_dumps(JVal::str(cfg_.backends[backend].model))
                                                                   : "\"unknown\"";
    std::string body, msg;
    int st = 0;
    const char* et = nullptr;
    if (!upstream_body(s, backend, body, &st, &msg, &et)) return fail_backend(s, 0, st, msg, et);
    Up* u = open_up(s, 0, backend, UP_PASS, build_req(cfg_.backends[backend], s->fwd, body), cfg_.timeout);
    if (!u) return fail_backend(s, 0, 500, "All connection attempts failed", "proxy_error");
    s->bs[0].up = u;
  }
  static bool bare_role(const std::string& ev) {
    std::string t = ev;
    if (t.compare(0, 6, "data: ") == 0) t = t.substr(6);
    JVal j;
    if (!json_parse(t.data(), t.size(), j, nullptr) || j.t != JVal::OBJ) return false;
    const JVal* ch = j.get("choices");
    if (!ch || ch->t != JVal::ARR || ch->a.empty() || ch->a[0].t != JVal::OBJ) return false;
    const JVal* d = ch->a[0].get("delta");
    if (!d || d->t != JVal::OBJ) return false;
    const JVal* r = d->get("role");
    const JVal* c = d->get("content");
    bool content_empty = !c || (c->t == JVal::STR && c->s.empty());
    return r && r->truthy() && content_empty;
  }
  void pass_forward(Session* s, const std::string& data) {
    bool all_ws = true;
    for (char ch : data)
      if (!(ch == ' ' || ch == '\n' || ch == '\r' || ch == '\t')) all_ws = false;
    if (all_ws) return;
    std::string w = s->done_tail + data;
    if (w.find("data: [DONE]") != std::string::npos) s->saw_done = true;
    s->done_tail = w.size() > 16 ? w.substr(w.size() - 16) : w;
    send_content(s, data);
  }
  void pass_body(Session* s, const std::string& body) {
    if (!s->first_decided) {
      s->first_buf += body;
      size_t j = s->first_buf.find("\n\n");
      if (j == std::string::npos) return;
      s->first_decided = true;
      std::string first = s->first_buf.substr(0, j + 2), rest = s->first_buf.substr(j + 2);
      s->first_buf.clear();
      if (!bare_role(first)) rest = first + rest;
      if (!rest.empty()) pass_forward(s, rest);
      return;
    }
    pass_forward(s, body);
  }
  void pass_end(Session* s) {
    if (!s->first_decided && !s->first_buf.empty() && !bare_role(s->first_buf)) pass_forward(s, s->first_buf);
    if (!s->saw_done) send_chunk(s, kDone);
    if (s->cl) write_client(s->cl, "0\r\n\r\n");
    s->bs[0].state = 1;
    end_session(s);
  }

  // ---------------------------------------------------------------- non-streaming
  void start_nonstream(Session* s, const std::vector<int>& valid, bool parallel) {
    c_nonstream++;
    s->kind = K_NONSTREAM;
    s->stage = parallel ? 10 : 11;
    s->bs.resize(valid.size());
    for (size_t i = 0; i < valid.size(); ++i) s->bs[i].backend = valid[i];
    for (size_t i = 0; i < valid.size(); ++i) {
      std::string body, msg;
      int st = 0;
      const char* et = nullptr;
      if (!upstream_body(s, valid[i], body, &st, &msg, &et)) {
        fail_backend(s, (int)i, st, msg, et);
        if (sessions_.find(s) == sessions_.end()) return;
        continue;
      }
      Up* u = open_up(s, (int)i, valid[i], UP_BUFFER, build_req(cfg_.backends[valid[i]], s->fwd, body), cfg_.timeout);
      if (!u) {
        fail_backend(s, (int)i, 500, "All connection attempts failed", "proxy_error");
        if (sessions_.find(s) == sessions_.end()) return;
      } else {
        s->bs[i].up = u;
      }
    }
  }
  void finish_nonstream(Session* s) {
    std::vector<BState*> ok;
    for (auto& b : s->bs)
      if (b.status == 200) ok.push_back(&b);
    if (ok.empty()) {
      if (s->cl)
        respond(s->cl, 500, "application/json",
                err_json("All backends failed. First error: " + error_message(s->bs[0]), "proxy_error"));
      return end_session(s);
    }
    if (s->stage == 11) {
      BState* f = ok[0];
      const std::string* ct = nullptr;
      for (auto& h : f->rheaders)
        if (h.first == "content-type") ct = &h.second;
      std::vector<std::pair<std::string, std::string>> extra;
      for (auto& h : f->rheaders)
        if (h.first != "content-length" && h.first != "content-type" && h.first != "transfer-encoding" &&
            h.first != "content-encoding" && h.first != "connection" && h.first != "keep-alive")
          extra.push_back(h);
      std::string body = f->is_json ? json_dumps(f->js) : f->text;
      if (s->cl) respond(s->cl, 200, ct ? *ct : "application/json", body, &extra);
      return end_session(s);
    }
    // parallel combine (quorum :1191-1341)
    const bool agg = !cfg_.aggregator_name.empty();
    const bool strip = cfg_.hide_final || (cfg_.documented && agg && cfg_.strip_intermediate);
    std::vector<std::string> processed;
    std::string err;
    for (BState* b : ok) {
      const JVal* content = nullptr;
      if (b->is_json) {
        const JVal* ch = b->js.get("choices");
        if (ch && ch->t == JVal::ARR && !ch->a.empty()) {
          const JVal* m = ch->a[0].get("message");
          if (m) content = m->get("content");
          else err = "'message'";
        } else {
          err = ch ? "list index out of range" : "'choices'";
        }
      } else {
        err = "string indices must be integers";
      }
      if (!content) {
        if (err.empty()) err = "'content'";
        break;
      }
      if (content->t != JVal::STR) {
        err = strip ? "expected string or bytes-like object" : "sequence item 0: expected str instance";
        break;
      }
      processed.push_back(strip ? strip_final(ts_, (const uint8_t*)content->s.data(),
                                                        content->s.size())
                                          : content->s);
    }
    if (!err.empty()) {
      if (s->cl) respond(s->cl, 500, "application/json", err_json("Error combining responses: " + err, "proxy_error"));
      return end_session(s);
    }
    if (cfg_.documented) {
      std::vector<std::string> names, kept;
      for (size_t i = 0; i < ok.size(); ++i)
        if (!agg || is_source(ok[i]->backend)) {
          names.push_back(cfg_.backends[ok[i]->backend].name);
          kept.push_back(std::move(processed[i]));
        }
      processed.swap(kept);
      if (processed.empty()) {
        if (s->cl) respond(s->cl, 500, "application/json", err_json("All source backends failed", "proxy_error"));
        return end_session(s);
      }
      bool sup = cfg_.suppress;
      if (const JVal* v = s->body.get("suppress_individual_responses")) sup = v->truthy();
      if (sup && !agg) return finish_nonstream_combined(s, JVal::str(processed[0]));  // "only the first"
      s->text_names = std::move(names);
    }
    s->texts = processed;
    s->fin_texts = true;
    if (agg) return start_aggregator(s, cfg_.separator);
    finish_nonstream_combined(s, JVal::str(joined(processed, cfg_.separator)));
  }
  void finish_nonstream_combined(Session* s, const JVal& combined) {
    std::vector<BState*> ok;
    for (auto& b : s->bs)
      if (b.status == 200) ok.push_back(&b);
    std::string err;
    JVal usage;
    usage.t = JVal::OBJ;
    for (const char* k : {"prompt_tokens", "completion_tokens", "total_tokens"}) {
      long long isum = 0;
      double fsum = 0;
      bool isf = false;
      for (BState* b : ok) {
        const JVal* u = b->is_json ? b->js.get("usage") : nullptr;
        const JVal* v = u ? u->get(k) : nullptr;
        if (!u) { err = "'usage'"; break; }
        if (!v) { err = std::string("'") + k + "'"; break; }
        if (v->t == JVal::INT) { isum += atoll(v->s.c_str()); fsum += atof(v->s.c_str()); }
        else if (v->t == JVal::FLOAT) { isf = true; fsum += v->d; }
        else { err = "unsupported operand type(s) for +"; break; }
      }
      if (!err.empty()) break;
      if (isf) {
        JVal f;
        f.t = JVal::FLOAT;
        f.d = fsum;
        usage.set(k, f);
      } else {
        usage.set(k, JVal::integer(isum));
      }
    }
    const JVal& first = ok[0]->js;
    for (const char* k : {"id", "created", "model"})
      if (err.empty() && !first.get(k)) err = std::string("'") + k + "'";
    if (!err.empty()) {
      if (s->cl) respond(s->cl, 500, "application/json", err_json("Error combining responses: " + err, "proxy_error"));
      return end_session(s);
    }
    JVal out;
    out.t = JVal::OBJ;
    out.set("id", *first.get("id"));
    out.set("object", JVal::str("chat.completion"));
    out.set("created", *first.get("created"));
    out.set("model", *first.get("model"));
    const JVal* fp = first.get("system_fingerprint");
    out.set("system_fingerprint", fp ? *fp : JVal::str(""));
    JVal choice;
    choice.t = JVal::OBJ;
    choice.set("index", JVal::integer(0));
    JVal msg;
    msg.t = JVal::OBJ;
    msg.set("role", JVal::str("assistant"));
    msg.set("content", combined);
    choice.set("message", msg);
    choice.set("logprobs", JVal());
    choice.set("finish_reason", JVal::str("stop"));
    JVal choices;
    choices.t = JVal::ARR;
    choices.a.push_back(choice);
    out.set("choices", choices);
    out.set("usage", usage);
    if (s->cl) respond(s->cl, 200, "application/json", json_dumps(out));
    end_session(s);
  }

  // ---------------------------------------------------------------- session lifecycle
  void end_session(Session* s) {
    if (s->stage == 3) return;
    s->stage = 3;
    if (s->kind != K_REMOTE && s->t0 > 0) h_latency.observe(now_s() - s->t0);
    if (s->kind == K_REMOTE) shadow_.erase({s->owner_skey, s->shadow_bi});
    if (s->skey) {
      rsess_.erase(s->skey);
      for (int i = 0; i < (int)s->bs.size(); ++i) {
        if (s->bs[i].remote < 0 || s->bs[i].state != 0 || !xch_) continue;
        XMsg m;  // client gone / session over before the worker finished: cancel it
        m.type = X_CANCEL;
        m.dst_rank = s->bs[i].remote;
        m.src_rank = xch_->rank();
        m.dst_loop = m.src_loop = (uint16_t)idx_;
        m.bi = i;
        m.skey = s->skey;
        xq(m, s->bs[i].via_link);
      }
    }
    for (int i = 0; i < (int)s->bs.size(); ++i) {
      BState& b = s->bs[i];
      if (b.up) {
        drop_up(b.up, false);
        b.up = nullptr;
      }
      // a shadow slot: no RCCL round may write into it once released.  A round receiving
      // into it right now keeps it: the exchange hands it back with X_RELEASE when that round
      // is over (never a wait here: a round stuck on a failed peer lasts up to its timeout)
      const bool reusable = !(b.remote >= 0 && xch_ && s->skey) || xch_->forget_bulk(s->skey, i, b.slot, idx_);
      if (b.slot >= 0) {
        slot_owner_.erase(b.slot);
        if (reusable) e_release(b.slot);
        else c_sp_release_deferred++;
        b.slot = -1;
      }
    }
    if (s->agg) {
      drop_up(s->agg, false);
      s->agg = nullptr;
    }
    if (s->fin_id >= 0) fin_owner_.erase(s->fin_id);
    Client* c = s->cl;
    sessions_.erase(s);
    if (c) {
      c->sess = nullptr;
      if (!c->keepalive || c->dead) mark_close(c);
      else if (!c->in.empty()) pending_requests_.push_back(c->fd);
    }
  }
  void abort_session(Session* s) { end_session(s); }

  std::string metrics_text() {
    std::string m;
    auto put = [&](const char* k, double v) { m += std::string(k) + " " + std::to_string(v) + "\n"; };
    put("qmx_requests_total", (double)c_requests.load());
    put("qmx_stream_requests_total", (double)c_stream.load());
    put("qmx_nonstream_requests_total", (double)c_nonstream.load());
    put("qmx_errors_total", (double)c_errors.load());
    put("qmx_upstream_failures_total", (double)c_up_fail.load());
    put("qmx_upstream_connections_total", (double)c_up_conns.load());
    put("qmx_client_connections_total", (double)c_clients.load());
    put("qmx_ticks_total", (double)c_ticks.load());
    put("qmx_output_coalesced_total", (double)c_coalesced.load());
    put("qmx_output_hold_seconds_sum", (double)c_hold_ns.load() * 1e-9);  // latency the holds added
    put("qmx_output_hold_seconds_count", (double)c_holds.load());
    put("qmx_output_hold_deadline_total", (double)c_hold_deadline.load());
    put("qmx_exchange_link_messages_total", (double)c_link_msgs.load());
    put("qmx_tick_slots_total", (double)c_tick_slots.load());
    put("qmx_tick_route_seconds_total", (double)c_route_ns.load() * 1e-9);
    put("qmx_flush_wait_seconds_total", (double)c_flush_ns.load() * 1e-9);
    put("qmx_flushes_total", (double)c_flushes.load());
    put("qmx_apply_wait_seconds_total", (double)c_apply_ns.load() * 1e-9);
    put("qmx_applies_total", (double)c_applies.load());
    put("qmx_remote_streams_total", (double)c_remote_streams.load());
    for (auto& kv : {std::make_pair("failed", &c_sp_failed), std::make_pair("aborted", &c_sp_aborted),
                     std::make_pair("empty", &c_sp_empty), std::make_pair("text", &c_sp_text),
                     std::make_pair("peer_down", &c_sp_down)})
      m += std::string("qmx_spread_remote_ends_total{how=\"") + kv.first + "\"} " + std::to_string(kv.second->load()) + "\n";
    put("qmx_spread_delta_mismatch_total", (double)c_sp_delta_mismatch.load());
    put("qmx_spread_worker_nodata_total", (double)c_sp_nodata.load());
    put("qmx_spread_eager_finals_total", (double)c_sp_eager.load());
    put("qmx_spread_release_deferred_total", (double)c_sp_release_deferred.load());
    put("qmx_spread_texts_fetched_total", (double)c_sp_fetched.load());
    put("qmx_loop_passes_over_1ms_total", (double)c_loop_pass_1ms.load());
    put("qmx_loop_passes_over_5ms_total", (double)c_loop_pass_5ms.load());
    put("qmx_loop_paced_total", (double)c_paced.load());
    {
      double mx = 0;
      for (Loop* l : *loops_) mx = std::max(mx, l->pass_max_.load(std::memory_order_relaxed));
      put("qmx_loop_pass_max_seconds", mx);
    }
    m += "qmx_upstream_failures_by_class_total{class=\"connect\"} " + std::to_string(c_fail_connect.load()) + "\n";
    m += "qmx_upstream_failures_by_class_total{class=\"timeout\"} " + std::to_string(c_fail_timeout.load()) + "\n";
    m += "qmx_upstream_failures_by_class_total{class=\"http_status\"} " + std::to_string(c_fail_status.load()) + "\n";
    m += "qmx_upstream_failures_by_class_total{class=\"disconnect\"} " + std::to_string(c_fail_disconnect.load()) + "\n";
    m += "qmx_upstream_failures_by_class_total{class=\"protocol\"} " + std::to_string(c_fail_protocol.load()) + "\n";
    put("qmx_stream_aborts_total", (double)c_stream_aborts.load());
    put("qmx_host_path_opens_total", (double)c_host_path_opens.load());
    put("qmx_verify_checked_total", (double)c_verify_checked.load());
    put("qmx_verify_mismatches_total", (double)c_verify_mismatch.load());
    h_ttft.render(m, "qmx_ttft_seconds");
    h_latency.render(m, "qmx_request_latency_seconds");
    h_tick.render(m, "qmx_tick_seconds");
    h_upstream_ttfb.render(m, "qmx_upstream_ttfb_seconds");
    h_engine.render(m, "qmx_engine_wait_seconds");
    h_sp_first.render(m, "qmx_spread_first_delta_seconds");
    h_sp_final.render(m, "qmx_spread_final_seconds");
    if (xch_) {
      put("qmx_exchange_rounds_total", (double)xch_->rounds());  // RCCL p2p rounds (final texts)
      put("qmx_exchange_bytes_total", (double)xch_->bytes());    // mesh payload bytes
      put("qmx_exchange_messages_total", (double)xch_->msgs());  // mesh messages (control + deltas)
      put("qmx_exchange_bulk_bytes_total", (double)xch_->bulk_bytes());  // final texts, HBM to HBM
      put("qmx_exchange_mesh_finals_total", (double)xch_->mesh_bulk());  // final texts over the mesh
      put("qmx_exchange_epochs_total", (double)xch_->epochs());
      put("qmx_exchange_rescued_total", (double)xch_->rescued());
      put("qmx_exchange_links_total", (double)xch_->links());  // per-loop links handed to the io loops  // resent on the receiver's report
      put("qmx_exchange_rejoins_total", (double)xch_->rejoins());
      put("qmx_exchange_peer_downs_total", (double)xch_->downs());
      put("qmx_exchange_busy_us_total", xch_->busy_us());
      put("qmx_exchange_healthy", xch_->healthy() ? 1.0 : 0.0);
      put("qmx_exchange_rccl_active", xch_->rccl_active() ? 1.0 : 0.0);
      put("qmx_exchange_host_copied_total", (double)xch_->host_copied());  // texts copied HBM -> host by the bulk thread
      put("qmx_exchange_deferred_releases_total", (double)xch_->deferred_releases());
      int up = 0;
      for (int r = 0; r < xch_->world(); ++r) up += xch_->peer_up(r);
      put("qmx_exchange_peers_up", (double)up);
    }
    // engine/kernel stats summed over every io loop's engine (snapshots taken by their tick threads)
    std::map<std::string, double> tot;
    for (Loop* l : *loops_) {
      std::lock_guard<std::mutex> g(l->smu_);
      for (auto& kv : l->snap_) tot[kv.first] += kv.second;
    }
    if (hub_)
      for (auto& kv : hub_->snapshot()) tot[kv.first] += kv.second;
    for (auto& kv : tot) put(kv.first.c_str(), kv.second);
    static const char* sc_names[SC_N] = {"client_send", "upstream_send", "recv", "epoll_wait", "epoll_ctl", "wake_read"};
    for (int i = 0; i < SC_N; ++i) {
      uint64_t v = 0;
      for (Loop* l : *loops_) v += l->sc_[i].load(std::memory_order_relaxed);
      m += std::string("qmx_syscalls_total{op=\"") + sc_names[i] + "\"} " + std::to_string(v) + "\n";
    }
    return m;
  }

  const ServerCfg& cfg_;
  int idx_;
  int ep_ = -1, lfd_ = -1, afd_ = -1, evfd_ = -1;
  // loop ticks: the ticks this loop has on the GPU.  Declared before eng_, so destroyed
  // after it: an AsyncCpuEngine's worker may still hold pointers to queued jobs until the
  // engine's destructor has joined it (a loop that leaves run() by an exception skips the
  // drain at its end)
  HostEngine::Job job_[2];
  std::unique_ptr<HostEngine> eng_;  // CPU engine (no GPU hub)
  std::unique_ptr<Verifier> ver_;
  GpuHub* hub_ = nullptr;            // shared HIP engine
  HipGrid* grid_ = nullptr;          // loop ticks: the shared multi-door grid
  HipEngine* heng_ = nullptr;        // loop ticks: eng_ as this loop's HIP engine
  HostEngine* aeng_ = nullptr;       // loop ticks: eng_, driven asynchronously (HIP grid / AsyncCpuEngine)
  int loop_slots_ = 0;
  bool job_live_[2] = {false, false};
  int jobs_live_ = 0;
  double job_t_post_[2] = {0, 0};
  const int loop_doors_ = [] {  // QMX_LOOP_INFLIGHT: ticks in flight per loop (1 or 2)
    const char* e = env_get("QMX_LOOP_INFLIGHT");
    return e ? std::min(std::max(atoi(e), 1), 2) : 2;
  }();
  std::vector<int> taken_;
  const int poll_us_ = [] {
    const char* e = env_get("QMX_LOOP_POLL_US");
    return e ? std::max(1, atoi(e)) : 3;
  }();
  // a tick due within this many us is waited for by looking again at once, not by a timer
  // (a timed wake-up of a sleeping thread lands ~2 us after its time); a longer wait sleeps
  // until the window begins.  4 us (MI355X, profiles/r6/spin): done -> taken 4.7-4.9 ->
  // 2.9-3.1 us with few connections (p50 TTFT 0.042 -> 0.039 ms at 1 connection, 0.050 ->
  // 0.044 ms and +19% req/s at 8), within noise at the headline's 64 (loops are busy there)
  const double spin_us_ = [] {
    const char* e = env_get("QMX_LOOP_SPIN_US");
    return e ? atof(e) : 4.0;
  }();
  // loop ticks: also look for results between the new requests an iteration parses (parsing
  // and the upstream sends are an iteration's longest stretch without a look);
  // QMX_LOOP_REQ_CHECK=0 turns it off (A/B)
  // loop ticks: results are looked for after every check_every_-th event of a batch
  // (QMX_LOOP_CHECK_EVERY, default 1: the look is a few host-memory loads, while an event's
  // handling — a request parse with its upstream sends, a client write — runs several us)
  const int check_every_ = [] {
    const char* e = env_get("QMX_LOOP_CHECK_EVERY");
    return e ? std::max(1, atoi(e)) : 1;
  }();
  double sess_ema_ = 0;  // latency mode: sessions on this loop, averaged over its recent opens
  const int light_host_ = [this] {  // runtime.light_host_sessions, else QMX_LIGHT_HOST, else off
    if (cfg_.light_host >= 0) return cfg_.light_host;
    const char* e = env_get("QMX_LIGHT_HOST");
    return e ? std::max(0, atoi(e)) : 0;
  }();
  const bool req_check_ = [] {
    const char* e = env_get("QMX_LOOP_REQ_CHECK");
    return !e || atoi(e) != 0;
  }();
  TagSet ts_ = make_tagset(cfg_.tags);
  bool kick_ = false;
  std::mutex rmu_;
  std::vector<ResultBatch> rq_;
  std::atomic<bool> rq_pending_{false};  // set by the tick lanes with each batch pushed
  std::unordered_map<int, std::unique_ptr<Client>> clients_;
  std::unordered_map<int, std::unique_ptr<Up>> ups_;
  std::unordered_map<Session*, std::unique_ptr<Session>> sessions_;
  struct SlotOwner {
    Session* s;
    int bi;
    uint32_t gen;  // open generation: results of an earlier owner of the slot are dropped
  };
  std::unordered_map<int, SlotOwner> slot_owner_;
  std::unordered_map<int, std::pair<Session*, int>> fin_owner_;  // fin id → (session, bs index | -1)
  // spread placement
  Exchange* xch_ = nullptr;
  bool draining_ = false;
  double drain_deadline_ = 0;
  const std::vector<Loop*>* loops_ = nullptr;
  double last_snap_ = 0;
  int xfd_ = -1;
  std::vector<int> valid_;  // backends with a URL (config order), computed once
  std::vector<int> scratch_fds_, scratch_flush_;  // per-iteration lists, capacity kept
  std::vector<ResultBatch> scratch_rq_;
  bool valid_init_ = false;
  std::mutex xmu_;
  std::vector<XMsg> xin_;
  std::vector<std::string> xout_;  // per destination rank: frames of this loop pass
  bool xpending_ = false;
  std::vector<XLink> xl_;  // per rank: this loop's link (fd -1: none yet / down)
  bool xlpending_ = false;
  uint64_t next_skey_ = 1;
  std::unordered_map<uint64_t, Session*> rsess_;            // owner sessions with remote streams
  std::map<std::pair<uint64_t, int>, Session*> shadow_;     // worker streams by (owner key, bi)
  std::vector<std::vector<int>> idle_;
  std::unordered_map<int, SSL*> idle_ssl_;  // pooled https connections
  std::unordered_map<int, int> parked_;     // pooled fd -> backend (registered, EPOLLIN)
  SSL_CTX* tls_ = nullptr;                  // https upstreams (peer + host verification, as httpx)
  std::vector<int> pending_close_, pending_requests_;
  std::vector<int> flushq_;  // clients with corked output (flushed at the end of each iteration)
  // parallel streams: the SSE head + role event wait (corked, not queued) for the first
  // content of the same session or this deadline, whichever comes first — one client send
  // per request instead of two when the tick answers within it (QMX_ROLE_DEFER_US, 0: off)
  struct Deferred {
    int fd;
    uint64_t serial;  // the connection the head belongs to (its fd may be reused after a close)
    double deadline;
  };
  std::vector<Deferred> deferq_;
  uint64_t next_serial_ = 0;
  const double role_defer_s_ = [] {
    const char* e = env_get("QMX_ROLE_DEFER_US");
    return (e ? atof(e) : 1000.0) * 1e-6;
  }();
  // output coalescing across ticks (apply): the longest a held delta waits for its stream's
  // next output (QMX_COALESCE_US, 0: off — every tick's output is sent on its own)
  const double coalesce_s_ = [] {
    const char* e = env_get("QMX_COALESCE_US");
    return (e ? atof(e) : 500.0) * 1e-6;
  }();
  // a finished stream's last output waits for its session's other streams (session_hold);
  // QMX_SESSION_HOLD=0 turns it off (A/B)
  const bool session_hold_ = env_flag("QMX_SESSION_HOLD", true);
  // a parallel session's streams are followed by its final output (the concatenated final
  // event, or the aggregator's answer): a stream's last deltas may wait for it (session_hold);
  // QMX_FINAL_HOLD=0 turns the hold off (A/B)
  const bool final_follows_ = env_flag("QMX_FINAL_HOLD", true) && !cfg_.skip_final;
  std::vector<EngineOp> ops_;  // engine feed / finish / release of this iteration (flush_ops)
  const bool early_flush_ = env_flag("QMX_EARLY_FLUSH", true);  // A/B knob
  // QMX_SPREAD_SELF=1 with placement spread at world 1 (rehearsal / GPU test): the odd
  // backends of every session run through this rank's own exchange, as if on a peer rank —
  // mesh frames to itself, worker sessions on this loop, final texts in RCCL rounds to itself
  // (the world > 1 path, HBM sinks and host copies included, on one GPU)
  const bool self_spread_ = env_flag("QMX_SPREAD_SELF", false);
  const bool stall_log_ = env_flag("QMX_LOOP_STALL_LOG", false);  // passes over 5 ms: phase split on stderr
  // A/B knob (see the event loop): measured within noise (profiles/r6/eager_post), so off
  const bool eager_post_ = env_flag("QMX_EAGER_POST", false);
  const double pace_s_ = [this] {
    const char* e = env_get("QMX_READ_PACE_US");
    return std::max(0.0, e ? atof(e) : (double)cfg_.read_pace_us) * 1e-6;
  }();
  const int pace_min_reads_ = [] {
    const char* e = env_get("QMX_READ_PACE_MIN");
    return e ? std::max(1, atoi(e)) : 2;
  }();
  int small_reads_ = 0;  // this pass: short reads of upstream responses still in progress
  int stall_logs_ = 0;
  const bool lazy_wake_ = env_flag("QMX_LAZY_WAKE", false);   // A/B knob (see attach_hub)
  std::atomic<bool> in_wait_{false};                          // in epoll_wait (lazy wake)
  double ops_t0_ = 0;  // the oldest unflushed FEED op (flush-wait timing)
  double tnow_ = now_s();  // refreshed after every epoll wait (lnow: stamps and timeouts)
  double lnow() const { return tnow_; }
  int64_t role_sec_ = -1;      // second of the cached SSE head + role event
  std::string role_head_;
  // fault injection (tests): drop every Nth stream result's SSE bytes before it is sent
  const long fault_drop_every_ = [] {
    const char* e = env_get("QMX_FAULT_DROP_DELTA");
    return e ? atol(e) : 0L;
  }();
  long fault_n_ = 0;
};

void on_signal(int sig) {
  if (sig == SIGTERM) g_drain.store(true);
  else g_stop.store(true);
}

}  // namespace

// The kernel grows a process's file-descriptor table by doubling it when a new fd does not
// fit, and in a multi-threaded process the growth waits for an RCU grace period
// (expand_files -> synchronize_rcu) while every other thread that allocates an fd waits for
// the resize.  Measured on the MI355X box (QMX_LOOP_STALL_LOG watchdog, /proc/<tid>/wchan):
// all 8 io loops parked in expand_files inside socket()/accept4() for 70-200 ms at a time as
// client and upstream connections grew the table — and the grid, with nothing posted for
// 50 ms, idled out meanwhile.  Growing the table once here, before any io loop runs, to the
// fd limit (at most 2^17 entries, ~1 MiB) leaves nothing to grow while serving.
// The soft fd limit is raised to the hard one first (capped the same way): a proxy holds a
// client socket, its upstream sockets and keep-alive pools, and 1024 is a common default.
static void presize_fd_table() {
  rlimit rl{};
  if (getrlimit(RLIMIT_NOFILE, &rl) != 0) return;
  if (rl.rlim_cur < rl.rlim_max && rl.rlim_cur < ((rlim_t)1 << 17)) {
    rlimit up = rl;
    up.rlim_cur = std::min<rlim_t>(rl.rlim_max, (rlim_t)1 << 17);
    if (setrlimit(RLIMIT_NOFILE, &up) == 0) rl = up;
  }
  const long want = (long)std::min<rlim_t>(rl.rlim_cur, (rlim_t)1 << 17);
  if (want <= 1024) return;
  // (dup3 onto an open descriptor would close it: the top slot must be free — it is, in a
  // process that has not opened ~1e5 files before the server starts)
  if (fcntl((int)want - 1, F_GETFD) != -1 || errno != EBADF) return;
  const int fd = open("/dev/null", O_RDONLY | O_CLOEXEC);
  if (fd < 0) return;
  const int hi = dup3(fd, (int)want - 1, O_CLOEXEC);  // the table now covers [0, want)
  if (hi >= 0) close(hi);
  close(fd);
}

int run_server(const ServerCfg& cfg0) {
  env_refresh();  // before any thread: the io loops, lanes and exchange read this snapshot
  ServerCfg cfg = cfg0;
  crash_handler_install();  // a native fault leaves a backtrace on stderr, not a silent exit
  prof_start();  // QMX_PROF=<path>: CPU sampling profile of this process (qmx_prof.h)
  bool any_https = false;
  for (auto& b : cfg.backends) {
    if (!b.valid || b.host.empty()) continue;
    any_https = any_https || b.https;
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(b.host.c_str(), std::to_string(b.port).c_str(), &hints, &res) == 0 && res) {
      std::memcpy(&b.addr, res->ai_addr, sizeof(sockaddr_in));
      b.resolved = true;
      freeaddrinfo(res);
    }
  }
  SSL_CTX* tls = nullptr;
  if (any_https) {
    tls = SSL_CTX_new(TLS_client_method());
    SSL_CTX_set_min_proto_version(tls, TLS1_2_VERSION);
    SSL_CTX_set_verify(tls, cfg.tls_verify ? SSL_VERIFY_PEER : SSL_VERIFY_NONE, nullptr);
    if (!cfg.ca_file.empty()) SSL_CTX_load_verify_locations(tls, cfg.ca_file.c_str(), nullptr);
    else SSL_CTX_set_default_verify_paths(tls);
    SSL_CTX_set_mode(tls, SSL_MODE_ENABLE_PARTIAL_WRITE | SSL_MODE_ACCEPT_MOVING_WRITE_BUFFER);
  }
  signal(SIGPIPE, SIG_IGN);
  presize_fd_table();
  if (cfg.install_signals) {
    struct sigaction sa {};
    sa.sa_handler = on_signal;
    sigaction(SIGTERM, &sa, nullptr);
    sigaction(SIGINT, &sa, nullptr);
  }
  g_stop.store(false);
  g_drain.store(false);
  g_ready.store(0);
  std::vector<std::unique_ptr<Loop>> loops;
  std::vector<std::thread> ts;
  for (int i = 0; i < std::max(1, cfg.threads); ++i) loops.emplace_back(new Loop(cfg, i));
  std::vector<Loop*> loop_ptrs;
  for (auto& l : loops) loop_ptrs.push_back(l.get());
  std::unique_ptr<GpuHub> hub;
  std::unique_ptr<HipGrid> grid;  // destroyed after the loops (their engines stop it first)
  const bool hip = cfg.engine == "hip";
  const bool spread = cfg.world > 1 && cfg.placement == "spread";
  // hip: loop ticks unless asked for lanes (tick_mode / an explicit shared engine).  Spread
  // placement included: a remote stream's final text lands in the owner's HBM shadow slot (an
  // RCCL round, synchronised before it is applied) or is staged into the finalize item that
  // reads it (the mesh), and the session finalizes in the grid like any other
  // (HipEngine::set_remote_content).  Ranks sharing one GPU
  // (rehearsals) split the grid budget: HipGrid sizes itself from QMX_GPU_SHARERS, and a grid
  // that does not fit falls back to lanes below.
  (void)spread;
  const bool loop_ticks = hip && cfg.tick_mode != "lanes" && cfg.shared_engine != 1;
  const bool shared = !loop_ticks && (cfg.shared_engine < 0 ? hip : cfg.shared_engine > 0);
  if (shared) hub.reset(new GpuHub(cfg, (int)loops.size()));
  if (loop_ticks) {
    const char* w = env_get("QMX_GRID_WPD");
    const char* im = env_get("QMX_PERSISTENT_IDLE_MS");
    const char* fl = env_get("QMX_LOOP_INFLIGHT");
    const int per_loop = fl ? std::min(std::max(atoi(fl), 1), 2) : 2;  // doors per loop (as Loop::loop_doors_)
    try {
      // (QMX_GRID_OCC=2: two workgroups per CU — twice the workgroups per door by default)
      const char* oc = env_get("QMX_GRID_OCC");
      const int wpd0 = oc && atoi(oc) == 2 ? 16 : 8;
      grid.reset(new HipGrid(cfg.device, (int)loops.size() * per_loop, w ? std::max(1, atoi(w)) : wpd0,
                             im ? atoi(im) : 50));
    } catch (const std::exception& e) {  // e.g. more io loops than a partitioned GPU has CUs
      fprintf(stderr, "qmx: loop ticks unavailable (%s) — tick lanes instead\n", e.what());
      hub.reset(new GpuHub(cfg, (int)loops.size()));
    }
  }
  for (auto& l : loops) {
    l->attach_loops(&loop_ptrs);
    l->attach_tls(tls);
    l->attach_hub(hub.get());
    l->attach_grid(grid.get());
  }
  if (hub) hub->start();
  std::unique_ptr<Exchange> xch;
  const bool self_spread = cfg.world == 1 && cfg.placement == "spread" && env_flag("QMX_SPREAD_SELF", false);
  if ((cfg.world > 1 || self_spread) && cfg.placement == "spread") {
    XOptions o;
    o.rank = cfg.rank;
    o.world = cfg.world;
    o.transport = cfg.xchg;
    o.addr = cfg.xchg_addr;
    o.port = cfg.xchg_port;
    o.bulk_port = cfg.xchg_bulk_port;
    o.device = cfg.device;
    o.batch_us = cfg.xchg_round_us;
    o.timeout_s = cfg.xchg_timeout;
    o.max_text = (size_t)cfg.content_cap;
    // RCCL texts a persistent grid must not read from HBM (a peer GPU wrote them): copied out
    // by the bulk thread after their round, never by an io loop
    o.host_copy = hip && o.transport == "rccl" && !remote_hbm_direct(cfg);
    // per-loop links (0: every session message via the mesh thread)
    o.links = cfg.xchg_links >= 0 ? cfg.xchg_links != 0 : env_flag("QMX_XCHG_LINKS", true);
    std::vector<Loop*> lp;
    for (auto& l : loops) lp.push_back(l.get());
    xch.reset(new Exchange(o, (int)lp.size(), [lp](int l, std::vector<XMsg>&& v) { lp[l]->x_deliver(std::move(v)); }));
    for (auto& l : loops) l->attach_exchange(xch.get());
  }
  // QMX_LOOP_STALL_LOG: a watchdog samples, for an io loop stuck in one pass for over 20 ms
  // (QMX_LOOP_STALL_WATCH_MS), what the kernel has that thread (and every other thread of the
  // process) waiting in: /proc/self/task/<tid>/wchan and .../syscall — the blocking call and
  // the lock behind it
  std::thread watchdog;
  std::atomic<bool> wd_stop{false};
  if (env_flag("QMX_LOOP_STALL_LOG", false)) {
    const char* wm = env_get("QMX_LOOP_STALL_WATCH_MS");
    const double watch_s = std::max(1.0, wm ? atof(wm) : 20.0) * 1e-3;
    watchdog = std::thread([&loops, &wd_stop, watch_s] {
      auto slurp = [](const std::string& path) {
        std::string out;
        if (FILE* f = fopen(path.c_str(), "r")) {
          char b[512];
          size_t n = fread(b, 1, sizeof(b) - 1, f);
          fclose(f);
          out.assign(b, n);
          while (!out.empty() && (out.back() == '\n' || out.back() == ' ')) out.pop_back();
        }
        return out;
      };
      int dumps = 0;
      std::vector<double> seen(loops.size(), 0.0);
      while (!wd_stop.load() && dumps < 60) {
        std::this_thread::sleep_for(std::chrono::microseconds(std::min(5000, (int)(watch_s * 2.5e5))));
        const double t = now_s();
        for (size_t i = 0; i < loops.size(); ++i) {
          const double t0 = loops[i]->pass_t0_.load(std::memory_order_relaxed);
          if (t0 <= 0 || t - t0 < watch_s || seen[i] == t0) continue;
          seen[i] = t0;
          ++dumps;
          std::string msg = "qmx watchdog: loop " + std::to_string(i) + " in one pass for " +
                            std::to_string((int)(1e3 * (t - t0))) + " ms; threads (tid comm wchan | syscall):";
          if (DIR* d = opendir("/proc/self/task")) {
            while (dirent* e = readdir(d)) {
              if (e->d_name[0] == '.') continue;
              const std::string base = std::string("/proc/self/task/") + e->d_name;
              const std::string w = slurp(base + "/wchan");
              if (w.empty() || w == "0") continue;  // running
              const std::string sc = slurp(base + "/syscall");
              msg += "\n   " + std::string(e->d_name) + " " + slurp(base + "/comm") + " " + w + " | " + sc.substr(0, 60);
            }
            closedir(d);
          }
          fprintf(stderr, "%s\n", msg.c_str());
          break;
        }
      }
    });
  }
  for (auto& l : loops) {
    Loop* lp = l.get();
    ts.emplace_back([lp] {
      char nm[16];  // "qmx-loop-N" in top -H, /proc/<pid>/task/*/comm and the stall watchdog
      snprintf(nm, sizeof(nm), "qmx-loop-%d", lp->index());
      pthread_setname_np(pthread_self(), nm);
      try {
        lp->run();
      } catch (const std::exception& e) {
        fprintf(stderr, "qmx_server loop error: %s\n", e.what());
        g_stop.store(true);
      }
    });
  }
  for (auto& t : ts) t.join();
  wd_stop.store(true);
  if (watchdog.joinable()) watchdog.join();
  prof_stop();
  if (xch) {
    xch->request_stop();  // keeps taking part in rounds until every rank has stopped
    xch->join();
    xch.reset();
  }
  hub.reset();  // tick thread joined before the loops (its result sinks) go away
  if (grid) grid->stop();  // before the loops' engines free what the grid may touch
  loops.clear();
  grid.reset();
  if (tls) SSL_CTX_free(tls);
  return 0;
}

void stop_server() { g_stop.store(true); }

std::unordered_map<std::string, double> server_counters() {
  return {{"requests", (double)c_requests.load()}, {"errors", (double)c_errors.load()},
          {"ticks", (double)c_ticks.load()}, {"upstream_failures", (double)c_up_fail.load()},
          {"verify_checked", (double)c_verify_checked.load()},
          {"verify_mismatches", (double)c_verify_mismatch.load()}};
}

}  // namespace qmx
