// qmx_loadgen — closed-loop HTTP/1.1 load generator for OpenAI-style streaming endpoints,
// with per-response validation.
//
// C keep-alive connections (spread over T epoll threads) each issue POST requests back to
// back until R requests have completed.  Per request it records TTFB (first SSE `data:`
// byte), TTFT (first SSE event carrying a non-empty "content") and total latency, parsing
// chunked or content-length bodies incrementally.  Prints one JSON line of statistics.
//
// Validation (--expect FILE): every completed response is checked against the expected
// event contract of the proxy (quorum's progress_streaming_aggregator, reference
// src/quorum/oai_proxy.py:530-885): status 200, the role event first, `data: [DONE]` last
// and exactly once, every event well-formed JSON-in-SSE with a known id, per-backend
// concatenated delta content equal to (or, for a stream allowed to fail, a prefix of) the
// text the mock backend streams, and the final event absent / one of the allowed texts.
// A response that fails any check counts in "invalid" (the first few are printed to
// stderr); completed = valid + invalid.  Spec file, one directive per line, texts hex:
//     role 1                       role event first (id chatcmpl-parallel)
//     done 1                       [DONE] last
//     stream <id> exact|prefix <hex>
//     final absent | final any <hex> [<hex> ...]
//     error allowed|absent         the all-failed "error" event
//     empty allowed                events without content are skipped (a backend's own role /
//                                  stop events: the direct harness-ceiling check, no proxy)
//     json 1                       non-streaming: the body is one JSON completion, checked by
//     message <hex>                  choices[0].message.content,
//     usage <p> <c> <t>              the usage totals,
//     field <key> <hex>              and top-level string fields (e.g. "backend")
//
// --abort-rate P: a request is abandoned (socket closed mid-stream, right after its first
// content event) with probability P — client-abort churn for the data plane's session
// teardown paths; abandoned requests are counted in "aborted", not "completed".
//
//   qmx_loadgen --port 8000 --conns 64 --requests 5000 [--threads 2] [--path /v1/chat/completions]
//               [--body-file req.json] [--stream 1] [--expect spec.txt] [--abort-rate 0]
#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <mutex>
#include <random>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

namespace {
using Clock = std::chrono::steady_clock;

struct StreamSpec {
  std::string id;
  bool exact = true;
  std::string text;
};
struct Spec {
  bool on = false;
  bool role = true, done = true;
  std::vector<StreamSpec> streams;
  bool final_absent = true;
  std::vector<std::string> final_any;
  bool error_allowed = false;
  // direct (no proxy: the harness ceiling): events with empty / no content are skipped (the
  // mock's own role and stop events), any event id accumulates into its stream's spec
  bool empty_allowed = false;
  // non-streaming JSON body (BASELINE config 1): choices[0].message.content, usage totals and
  // top-level string fields (the passthrough's "backend") must equal these
  bool json = false;
  bool have_message = false;
  std::string message;
  long usage[3] = {-1, -1, -1};
  std::vector<std::pair<std::string, std::string>> fields;
};

struct Opts {
  std::string host = "127.0.0.1";
  int port = 8000;
  int conns = 16;
  long requests = 1000;
  int threads = 1;
  std::string path = "/v1/chat/completions";
  std::string body;
  bool stream = true;
  double timeout_s = 60;
  double abort_rate = 0.0;
  Spec spec;
} g;

std::atomic<long> g_issued{0}, g_done{0}, g_errors{0}, g_non200{0}, g_no_content{0}, g_invalid{0},
    g_aborted{0}, g_validated{0};
std::mutex g_mu;
std::vector<double> g_ttft, g_ttfb, g_lat;

// receive buffer consumed from the front by offset (no memmove per HTTP chunk)
struct InBuf {
  std::string s;
  size_t off = 0;
  const char* data() const { return s.data() + off; }
  size_t size() const { return s.size() - off; }
  bool empty() const { return off >= s.size(); }
  void clear() {
    s.clear();
    off = 0;
  }
  void append(const char* p, size_t n) {
    if (off > 0 && off * 2 > s.size()) {
      s.erase(0, off);
      off = 0;
    }
    s.append(p, n);
  }
  void erase_front(size_t n) {
    off += n;
    if (off >= s.size()) clear();
  }
  size_t find(const char* pat) const {
    const size_t k = s.find(pat, off);
    return k == std::string::npos ? k : k - off;
  }
};

struct Conn {
  int fd = -1;
  std::string req;
  size_t req_off = 0;
  InBuf in;
  // response parse state
  int phase = 0;  // 0 idle, 1 headers, 2 body-chunked, 3 body-length
  bool chunked = false;
  long remaining = 0;
  long chunk_left = -1;
  int status = 0;
  bool got_data = false, got_content = false;
  bool abort_this = false;
  std::string tail;  // SSE scan carry
  std::string body;  // decoded body (validation)
  Clock::time_point t0, t_data, t_content;
  bool active = false;
};

int connect_to() {
  int fd = socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(g.port);
  inet_pton(AF_INET, g.host.c_str(), &a.sin_addr);
  if (connect(fd, (sockaddr*)&a, sizeof(a)) != 0) {
    close(fd);
    return -1;
  }
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) | O_NONBLOCK);
  return fd;
}

// ---------------------------------------------------------------------------------------
// validation: a small strict JSON reader for the proxy's SSE events
// ---------------------------------------------------------------------------------------
struct JR {
  const char* p;
  const char* e;
  bool ok = true;
  void ws() {
    while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
  }
  bool lit(const char* s) {
    size_t n = strlen(s);
    if ((size_t)(e - p) < n || memcmp(p, s, n) != 0) return ok = false;
    p += n;
    return true;
  }
  static int hexv(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  }
  static void put_utf8(uint32_t cp, std::string& o) {
    if (cp < 0x80) {
      o.push_back((char)cp);
    } else if (cp < 0x800) {
      o.push_back((char)(0xC0 | (cp >> 6)));
      o.push_back((char)(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      o.push_back((char)(0xE0 | (cp >> 12)));
      o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      o.push_back((char)(0x80 | (cp & 0x3F)));
    } else {
      o.push_back((char)(0xF0 | (cp >> 18)));
      o.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
      o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      o.push_back((char)(0x80 | (cp & 0x3F)));
    }
  }
  bool u4(uint32_t* v) {
    if (e - p < 4) return ok = false;
    uint32_t x = 0;
    for (int i = 0; i < 4; ++i) {
      int h = hexv(p[i]);
      if (h < 0) return ok = false;
      x = x * 16 + (uint32_t)h;
    }
    p += 4;
    *v = x;
    return true;
  }
  // string → UTF-8 (lone surrogates encoded as WTF-8, as the proxy's json.loads would keep them)
  bool str(std::string* out) {
    ws();
    if (p >= e || *p != '"') return ok = false;
    ++p;
    while (p < e) {
      const char* run = p;  // plain bytes are appended in one go
      while (p < e && *p != '"' && *p != '\\' && (unsigned char)*p >= 0x20) ++p;
      if (out && p > run) out->append(run, p - run);
      if (p >= e) break;
      const char c = *p++;
      if (c == '"') return true;
      if ((unsigned char)c < 0x20) return ok = false;
      if (c != '\\') {
        if (out) out->push_back(c);
        continue;
      }
      if (p >= e) return ok = false;
      const char d = *p++;
      char r = 0;
      switch (d) {
        case '"': r = '"'; break;
        case '\\': r = '\\'; break;
        case '/': r = '/'; break;
        case 'b': r = '\b'; break;
        case 'f': r = '\f'; break;
        case 'n': r = '\n'; break;
        case 'r': r = '\r'; break;
        case 't': r = '\t'; break;
        case 'u': {
          uint32_t cp;
          if (!u4(&cp)) return false;
          if (cp >= 0xD800 && cp < 0xDC00 && e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
            const char* save = p;
            p += 2;
            uint32_t lo;
            if (u4(&lo) && lo >= 0xDC00 && lo < 0xE000) {
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            } else {
              ok = true;
              p = save;
            }
          }
          if (out) put_utf8(cp, *out);
          continue;
        }
        default: return ok = false;
      }
      if (out) out->push_back(r);
    }
    return ok = false;
  }
  bool skip_value(int depth = 0) {
    ws();
    if (p >= e || depth > 32) return ok = false;
    if (*p == '"') return str(nullptr);
    if (*p == '{' || *p == '[') {
      const char close = *p == '{' ? '}' : ']';
      const bool obj = *p == '{';
      ++p;
      ws();
      if (p < e && *p == close) {
        ++p;
        return true;
      }
      while (true) {
        if (obj) {
          if (!str(nullptr)) return false;
          ws();
          if (p >= e || *p++ != ':') return ok = false;
        }
        if (!skip_value(depth + 1)) return false;
        ws();
        if (p < e && *p == ',') {
          ++p;
          continue;
        }
        if (p < e && *p == close) {
          ++p;
          return true;
        }
        return ok = false;
      }
    }
    const char* s = p;
    while (p < e && (isalnum((unsigned char)*p) || *p == '-' || *p == '+' || *p == '.')) ++p;
    return p > s ? true : (ok = false);
  }
};

struct Ev {
  std::string id, content, finish;
  bool has_content = false, has_role = false, content_null = false;
};

// {"id": ..., "choices": [{"delta": {"role"?, "content"?}, "finish_reason": ...}], ...}
bool parse_event(const char* p, const char* e, Ev& ev) {
  JR r{p, e};
  r.ws();
  if (!r.lit("{")) return false;
  bool have_choices = false;
  while (true) {
    std::string key;
    if (!r.str(&key)) return false;
    r.ws();
    if (!r.lit(":")) return false;
    r.ws();
    if (key == "id") {
      if (!r.str(&ev.id)) return false;
    } else if (key == "choices") {
      if (!r.lit("[")) return false;
      r.ws();
      if (!r.lit("{")) return false;
      while (true) {
        std::string k2;
        if (!r.str(&k2)) return false;
        r.ws();
        if (!r.lit(":")) return false;
        r.ws();
        if (k2 == "delta") {
          if (!r.lit("{")) return false;
          r.ws();
          if (r.p < r.e && *r.p == '}') {
            ++r.p;
          } else {
            while (true) {
              std::string k3;
              if (!r.str(&k3)) return false;
              r.ws();
              if (!r.lit(":")) return false;
              r.ws();
              if (k3 == "content") {
                if (r.p < r.e && *r.p == 'n') {
                  if (!r.lit("null")) return false;
                  ev.content_null = true;
                } else {
                  if (!r.str(&ev.content)) return false;
                  ev.has_content = true;
                }
              } else if (k3 == "role") {
                ev.has_role = true;
                if (!r.skip_value()) return false;
              } else if (!r.skip_value()) {
                return false;
              }
              r.ws();
              if (r.p < r.e && *r.p == ',') {
                ++r.p;
                continue;
              }
              if (!r.lit("}")) return false;
              break;
            }
          }
        } else if (k2 == "finish_reason") {
          if (r.p < r.e && *r.p == '"') {
            if (!r.str(&ev.finish)) return false;
          } else if (!r.lit("null")) {
            return false;
          }
        } else if (!r.skip_value()) {
          return false;
        }
        r.ws();
        if (r.p < r.e && *r.p == ',') {
          ++r.p;
          continue;
        }
        if (!r.lit("}")) return false;
        break;
      }
      r.ws();
      if (!r.lit("]")) return false;  // exactly one choice
      have_choices = true;
    } else if (!r.skip_value()) {
      return false;
    }
    r.ws();
    if (r.p < r.e && *r.p == ',') {
      ++r.p;
      continue;
    }
    if (!r.lit("}")) return false;
    break;
  }
  r.ws();
  return r.p == r.e && have_choices && !ev.id.empty();
}

// Fast path: the proxy's own envelope (json.dumps of quorum's event dicts, oai_proxy.py:530-541,
// 629-646, 847-860) matched literally around one strictly scanned JSON string — a strict
// subset of what parse_event accepts, with the same result; anything else takes the full
// parser.  Keeps validation off the load generator's critical CPU (it shares the box).
// kind: 1 role, 2 delta/final content (appended to *content), 0 no match.
int fast_event(const char* a, const char* b, std::string* id, std::string* content_out, bool* final_stop) {
  static const char kP0[] = "{\"id\": \"";
  static const char kP1[] = "\", \"object\": \"chat.completion.chunk\", \"created\": ";
  static const char kP2[] = ", \"model\": \"parallel-proxy\", \"choices\": [{\"index\": 0, \"delta\": {";
  static const char kP2m[] = ", \"model\": \"";
  static const char kP2c[] = "\", \"choices\": [{\"index\": 0, \"delta\": {";
  static const char kRole[] = "\"role\": \"assistant\"}, \"finish_reason\": null}]}";
  static const char kCont[] = "\"content\": ";
  static const char kEndNull[] = "}, \"finish_reason\": null}]}";
  static const char kEndStop[] = "}, \"finish_reason\": \"stop\"}]}";
  auto eat = [&](const char* lit, size_t n) {
    if ((size_t)(b - a) < n || memcmp(a, lit, n) != 0) return false;
    a += n;
    return true;
  };
  if (!eat(kP0, sizeof(kP0) - 1)) return 0;
  const char* q = (const char*)memchr(a, '"', b - a);
  if (!q) return 0;
  for (const char* x = a; x < q; ++x)
    if (*x == '\\' || (unsigned char)*x < 0x20) return 0;
  id->assign(a, q - a);
  a = q;
  if (!eat(kP1, sizeof(kP1) - 1)) return 0;
  const char* d = a;
  while (a < b && *a >= '0' && *a <= '9') ++a;
  if (a == d) return 0;
  if (!eat(kP2, sizeof(kP2) - 1)) {
    // another backend's envelope (the direct harness check: the mock's own "model"): the
    // same shape around any escape-free model string
    if (!eat(kP2m, sizeof(kP2m) - 1)) return 0;
    const char* mq = (const char*)memchr(a, '"', b - a);
    if (!mq) return 0;
    for (const char* x = a; x < mq; ++x)
      if (*x == '\\' || (unsigned char)*x < 0x20) return 0;
    a = mq;
    if (!eat(kP2c, sizeof(kP2c) - 1)) return 0;
  }
  if (eat(kRole, sizeof(kRole) - 1)) return a == b ? 1 : 0;
  if (!eat(kCont, sizeof(kCont) - 1)) return 0;
  const size_t n0 = content_out->size();
  {
    // escape-free string (the common case): one memchr, one check pass, one append
    const char* q2 = a < b && *a == '"' ? (const char*)memchr(a + 1, '"', b - a - 1) : nullptr;
    bool plain = q2 != nullptr;
    for (const char* x = a + 1; plain && x < q2; ++x) plain = *x != '\\' && (unsigned char)*x >= 0x20;
    if (plain) {
      content_out->append(a + 1, q2 - a - 1);
      a = q2 + 1;
    } else {
      JR r{a, b};
      if (!r.str(content_out) || !r.ok) {
        content_out->resize(n0);
        return 0;
      }
      a = r.p;
    }
  }
  const size_t left = (size_t)(b - a);
  if (left == sizeof(kEndNull) - 1 && memcmp(a, kEndNull, left) == 0) {
    *final_stop = false;
    return 2;
  }
  if (left == sizeof(kEndStop) - 1 && memcmp(a, kEndStop, left) == 0) {
    *final_stop = true;
    return 2;
  }
  content_out->resize(n0);
  return 0;
}

// Non-streaming body: {"choices": [{"message": {"content": "..."}, ...}], "usage": {...}, ...}
std::string validate_json(const std::string& body) {
  const Spec& S = g.spec;
  JR r{body.data(), body.data() + body.size()};
  r.ws();
  if (!r.lit("{")) return "body is not a JSON object";
  std::string content;
  bool have_content = false;
  long usage[3] = {-1, -1, -1};
  std::vector<std::pair<std::string, std::string>> strs;
  auto read_int = [&](long* v) {
    r.ws();
    const char* s0 = r.p;
    while (r.p < r.e && (*r.p == '-' || (*r.p >= '0' && *r.p <= '9'))) ++r.p;
    if (r.p == s0) return false;
    *v = strtol(std::string(s0, r.p - s0).c_str(), nullptr, 10);
    return true;
  };
  // generic object walk: f(key) consumes the value or returns false to skip it
  auto object = [&](auto&& self, auto&& f) -> bool {
    r.ws();
    if (!r.lit("{")) return false;
    r.ws();
    if (r.p < r.e && *r.p == '}') {
      ++r.p;
      return true;
    }
    while (true) {
      std::string key;
      if (!r.str(&key)) return false;
      r.ws();
      if (!r.lit(":")) return false;
      r.ws();
      int took = f(key);
      if (took < 0) return false;
      if (took == 0 && !r.skip_value()) return false;
      r.ws();
      if (r.p < r.e && *r.p == ',') {
        ++r.p;
        continue;
      }
      return r.lit("}");
    }
    (void)self;
  };
  r.p = body.data();
  bool ok = object(object, [&](const std::string& k) -> int {
    if (k == "choices") {
      if (!r.lit("[")) return -1;
      bool ok1 = object(object, [&](const std::string& k2) -> int {
        if (k2 != "message") return 0;
        return object(object, [&](const std::string& k3) -> int {
                 if (k3 != "content") return 0;
                 if (!r.str(&content)) return -1;
                 have_content = true;
                 return 1;
               }) ? 1 : -1;
      });
      if (!ok1) return -1;
      r.ws();
      return r.lit("]") ? 1 : -1;  // exactly one choice
    }
    if (k == "usage") {
      return object(object, [&](const std::string& k2) -> int {
               const int i = k2 == "prompt_tokens" ? 0 : k2 == "completion_tokens" ? 1 : k2 == "total_tokens" ? 2 : -1;
               if (i < 0) return 0;
               return read_int(&usage[i]) ? 1 : -1;
             }) ? 1 : -1;
    }
    for (auto& f : S.fields)
      if (f.first == k && r.p < r.e && *r.p == '"') {
        std::string v;
        if (!r.str(&v)) return -1;
        strs.emplace_back(k, v);
        return 1;
      }
    return 0;
  });
  r.ws();
  if (!ok || !r.ok || r.p != r.e) return "malformed JSON body";
  if (!have_content) return "no choices[0].message.content";
  if (S.have_message && content != S.message) return "message content differs (" + std::to_string(content.size()) + " B)";
  for (int i = 0; i < 3; ++i)
    if (S.usage[i] >= 0 && usage[i] != S.usage[i]) return "usage differs";
  for (auto& f : S.fields) {
    bool found = false;
    for (auto& x : strs) found = found || (x.first == f.first && x.second == f.second);
    if (!found) return "field " + f.first + " differs";
  }
  return std::string();
}

// returns "" when the response satisfies the spec, else a short reason
std::string validate(int status, const std::string& body) {
  const Spec& S = g.spec;
  if (status != 200) return "status " + std::to_string(status);
  if (S.json) return validate_json(body);
  std::vector<std::string> acc(S.streams.size());
  std::vector<int> nev(S.streams.size(), 0);
  bool saw_done = false, saw_final = false, saw_error = false;
  std::string final_text;
  std::string fid, fcontent;
  size_t pos = 0;
  int k = 0;
  while (pos < body.size()) {
    size_t j = body.find("\n\n", pos);
    if (j == std::string::npos) return "trailing bytes after the last event";
    const char* a = body.data() + pos;
    const char* b = body.data() + j;
    pos = j + 2;
    if (saw_done) return "event after [DONE]";
    if (b - a < 6 || memcmp(a, "data: ", 6) != 0) return "event without 'data: '";
    a += 6;
    if (b - a == 6 && memcmp(a, "[DONE]", 6) == 0) {
      saw_done = true;
      ++k;
      continue;
    }
    Ev ev;
    {
      // fast path: content goes straight into its stream's accumulator
      fcontent.clear();
      bool stop = false;
      const int kind = fast_event(a, b, &fid, &fcontent, &stop);
      if (kind == 1 && k == 0 && S.role && fid == "chatcmpl-parallel") {
        ++k;
        continue;
      }
      if (kind == 2 && !stop && !fcontent.empty() && !saw_final && k > 0) {
        size_t si = 0;
        while (si < S.streams.size() && S.streams[si].id != fid) ++si;
        if (si < S.streams.size()) {
          acc[si] += fcontent;
          ++nev[si];
          ++k;
          continue;
        }
      }
    }
    if (!parse_event(a, b, ev)) return "malformed event " + std::to_string(k);
    if (k == 0 && S.role) {
      if (ev.id != "chatcmpl-parallel" || !ev.has_role || ev.has_content) return "first event is not the role event";
      ++k;
      continue;
    }
    ++k;
    if (ev.id == "chatcmpl-parallel-final") {
      if (saw_final) return "two final events";
      if (ev.finish != "stop" || !ev.has_content) return "bad final event";
      saw_final = true;
      final_text = ev.content;
      continue;
    }
    if (ev.id == "error") {
      saw_error = true;
      continue;
    }
    size_t si = 0;
    while (si < S.streams.size() && S.streams[si].id != ev.id) ++si;
    if ((!ev.has_content || ev.content.empty()) && S.empty_allowed) continue;  // a backend's role / stop event
    if (si == S.streams.size()) return "unexpected event id " + ev.id;
    if (!ev.has_content || ev.content.empty()) return "delta event without content (" + ev.id + ")";
    if (saw_final) return "delta after the final event";
    acc[si] += ev.content;
    ++nev[si];
  }
  if (S.done && !saw_done) return "no [DONE]";
  if (S.role && k == 0) return "empty body";
  for (size_t si = 0; si < S.streams.size(); ++si) {
    const StreamSpec& ss = S.streams[si];
    if (ss.exact ? acc[si] != ss.text : ss.text.compare(0, acc[si].size(), acc[si]) != 0 ||
                                            acc[si].size() > ss.text.size())
      return "content of " + ss.id + " differs (" + std::to_string(acc[si].size()) + " B, " +
             std::to_string(nev[si]) + " events)";
  }
  if (saw_error && !S.error_allowed) return "unexpected error event";
  if (S.final_absent) {
    if (saw_final) return "unexpected final event";
  } else if (!saw_error || saw_final) {
    if (!saw_final) return "no final event";
    if (std::find(S.final_any.begin(), S.final_any.end(), final_text) == S.final_any.end())
      return "final content differs (" + std::to_string(final_text.size()) + " B)";
  }
  return std::string();
}

// scan decoded body bytes for SSE markers
void scan_sse(Conn& c, const char* p, size_t n, Clock::time_point now) {
  if (g.spec.on) c.body.append(p, n);
  if (c.got_data && c.got_content) return;
  std::string s = c.tail;
  s.append(p, n);
  if (!c.got_data && s.find("data:") != std::string::npos) {
    c.got_data = true;
    c.t_data = now;
  }
  if (!c.got_content) {
    // an event with non-empty content: "content": "<non-quote>  or "content":"<non-quote>
    for (const char* pat : {"\"content\": \"", "\"content\":\""}) {
      size_t k = 0;
      size_t L = strlen(pat);
      while ((k = s.find(pat, k)) != std::string::npos) {
        if (k + L < s.size() && s[k + L] != '"') {
          c.got_content = true;
          c.t_content = now;
          break;
        }
        k += L;
      }
      if (c.got_content) break;
    }
  }
  c.tail = s.size() > 16 ? s.substr(s.size() - 16) : s;
}

thread_local std::mt19937_64 t_rng(12345);

bool start_request(Conn& c) {
  long k = g_issued.fetch_add(1);
  if (k >= g.requests) {
    c.active = false;
    return false;
  }
  c.req_off = 0;
  c.phase = 1;
  c.chunked = false;
  c.remaining = 0;
  c.chunk_left = -1;
  c.status = 0;
  c.got_data = c.got_content = false;
  c.abort_this = g.abort_rate > 0 && std::uniform_real_distribution<double>(0, 1)(t_rng) < g.abort_rate;
  c.tail.clear();
  c.body.clear();
  if (g.spec.on) c.body.reserve(16384);
  c.t0 = Clock::now();
  c.active = true;
  return true;
}

void finish_request(Conn& c, std::vector<double>& ttft, std::vector<double>& ttfb, std::vector<double>& lat) {
  auto now = Clock::now();
  auto ms = [&](Clock::time_point t) { return std::chrono::duration<double, std::milli>(t - c.t0).count(); };
  if (c.status != 200) g_non200++;
  lat.push_back(ms(now));
  if (c.got_data) ttfb.push_back(ms(c.t_data));
  if (c.got_content) ttft.push_back(ms(c.t_content));
  else g_no_content++;
  if (g.spec.on) {
    g_validated++;
    std::string why = validate(c.status, c.body);
    if (!why.empty()) {
      const long n = g_invalid.fetch_add(1);
      if (n < 5) {
        fprintf(stderr, "qmx_loadgen: invalid response (%s): %.600s\n", why.c_str(),
                c.body.size() > 600 ? (c.body.substr(0, 300) + " ... " + c.body.substr(c.body.size() - 280)).c_str()
                                    : c.body.c_str());
        // QMX_LOADGEN_DUMP=FILE: the whole body of each of the first invalid responses
        if (const char* dp = getenv("QMX_LOADGEN_DUMP")) {
          static std::mutex mu;
          std::lock_guard<std::mutex> lk(mu);
          if (FILE* f = fopen(dp, "a")) {
            fprintf(f, "=== invalid response %ld (%s), status %d, %zu B\n", n, why.c_str(), c.status, c.body.size());
            fwrite(c.body.data(), 1, c.body.size(), f);
            fputs("\n=== end\n", f);
            fclose(f);
          }
        }
      }
    }
  }
  g_done++;
  c.phase = 0;
}

// returns false on protocol error; sets done when the response completed
bool parse(Conn& c, bool* done) {
  *done = false;
  auto now = Clock::now();
  while (true) {
    if (c.phase == 1) {
      size_t he = c.in.find("\r\n\r\n");
      if (he == std::string::npos) return true;
      std::string h(c.in.data(), he);
      c.status = atoi(h.c_str() + 9);
      for (auto& ch : h) ch = (char)tolower(ch);
      c.chunked = h.find("transfer-encoding: chunked") != std::string::npos;
      size_t p = h.find("content-length:");
      c.remaining = p != std::string::npos ? strtol(h.c_str() + p + 15, nullptr, 10) : 0;
      c.in.erase_front(he + 4);
      c.phase = c.chunked ? 2 : 3;
      c.chunk_left = -1;
      if (!c.chunked && c.remaining == 0) {
        *done = true;
        return true;
      }
      continue;
    }
    if (c.phase == 3) {
      size_t take = std::min((size_t)c.remaining, c.in.size());
      if (take) scan_sse(c, c.in.data(), take, now);
      c.in.erase_front(take);
      c.remaining -= take;
      if (c.remaining == 0) {
        *done = true;
        return true;
      }
      return true;
    }
    if (c.phase == 2) {
      if (c.chunk_left < 0 && c.chunk_left != -2) {
        size_t le = c.in.find("\r\n");
        if (le == std::string::npos) return true;
        long sz = strtol(c.in.data(), nullptr, 16);
        c.in.erase_front(le + 2);
        if (sz == 0) {
          c.chunk_left = -2;  // trailer: expect "\r\n"
        } else {
          c.chunk_left = sz;
        }
      }
      if (c.chunk_left == -2) {
        if (c.in.size() < 2) return true;
        c.in.erase_front(2);
        *done = true;
        return true;
      }
      size_t take = std::min((size_t)c.chunk_left, c.in.size());
      if (take) scan_sse(c, c.in.data(), take, now);
      c.in.erase_front(take);
      c.chunk_left -= take;
      if (c.chunk_left > 0) return true;
      if (c.in.size() < 2) return true;  // chunk_left == 0: its CRLF has not arrived yet
      c.in.erase_front(2);
      c.chunk_left = -1;
      continue;
    }
    return true;
  }
}

void worker(int tid, int nconns, Clock::time_point deadline) {
  t_rng.seed(12345 + 7919 * tid);
  int ep = epoll_create1(0);
  std::vector<Conn> cs(nconns);
  std::vector<double> ttft, ttfb, lat;
  std::string req = "POST " + g.path + " HTTP/1.1\r\nHost: " + g.host + "\r\ncontent-type: application/json\r\n"
                    "authorization: Bearer bench\r\ncontent-length: " + std::to_string(g.body.size()) + "\r\n\r\n" + g.body;
  int live = 0;
  // The request is written right away (a few hundred bytes into an empty socket buffer);
  // EPOLLOUT is armed only when that write comes up short, so a closed-loop request costs
  // one send and no epoll_ctl — the load generator shares the box with what it measures.
  auto send_now = [&](Conn& c, uint32_t idx) -> bool {
    while (c.req_off < c.req.size()) {
      ssize_t w = send(c.fd, c.req.data() + c.req_off, c.req.size() - c.req_off, MSG_NOSIGNAL);
      if (w > 0) {
        c.req_off += w;
        continue;
      }
      if (w < 0 && errno == EAGAIN) {
        epoll_event e{};
        e.events = EPOLLIN | EPOLLOUT;
        e.data.u32 = idx;
        epoll_ctl(ep, EPOLL_CTL_MOD, c.fd, &e);
        return true;
      }
      return false;
    }
    return true;
  };
  auto reconnect = [&](Conn& c, uint32_t idx) -> bool {
    epoll_ctl(ep, EPOLL_CTL_DEL, c.fd, nullptr);
    close(c.fd);
    c.in.clear();
    c.fd = connect_to();
    if (c.fd < 0) return false;
    epoll_event e{};
    e.events = EPOLLIN | EPOLLOUT;
    e.data.u32 = idx;
    epoll_ctl(ep, EPOLL_CTL_ADD, c.fd, &e);
    return true;
  };
  for (int i = 0; i < nconns; ++i) {
    cs[i].fd = connect_to();
    if (cs[i].fd < 0) {
      g_errors++;
      continue;
    }
    cs[i].req = req;
    epoll_event e{};
    e.events = EPOLLIN | EPOLLOUT;
    e.data.u32 = i;
    epoll_ctl(ep, EPOLL_CTL_ADD, cs[i].fd, &e);
    if (start_request(cs[i])) ++live;
  }
  std::vector<epoll_event> evs(256);
  char buf[65536];
  while (live > 0 && Clock::now() < deadline) {
    int n = epoll_wait(ep, evs.data(), (int)evs.size(), 100);
    for (int k = 0; k < n; ++k) {
      const uint32_t idx = evs[k].data.u32;
      Conn& c = cs[idx];
      if (!c.active) continue;
      bool dead = false;
      if (evs[k].events & EPOLLOUT) {
        while (c.req_off < c.req.size()) {
          ssize_t w = send(c.fd, c.req.data() + c.req_off, c.req.size() - c.req_off, MSG_NOSIGNAL);
          if (w > 0) c.req_off += w;
          else {
            if (errno != EAGAIN) dead = true;
            break;
          }
        }
        if (c.req_off >= c.req.size()) {
          epoll_event e{};
          e.events = EPOLLIN;
          e.data.u32 = idx;
          epoll_ctl(ep, EPOLL_CTL_MOD, c.fd, &e);
        }
      }
      if (!dead && (evs[k].events & (EPOLLIN | EPOLLHUP | EPOLLERR))) {
        while (true) {
          ssize_t r = recv(c.fd, buf, sizeof(buf), 0);
          if (r > 0) {
            c.in.append(buf, r);
            continue;
          }
          if (r == 0 || errno != EAGAIN) dead = true;
          break;
        }
        bool done = false;
        while (!c.in.empty() || done) {
          if (!parse(c, &done)) {
            dead = true;
            break;
          }
          if (!done && c.abort_this && c.got_content) {
            // client abort: hang up mid-stream, then carry on with a fresh connection
            g_aborted++;
            if (!reconnect(c, idx)) {
              c.active = false;
              --live;
            } else if (!start_request(c)) {
              --live;
            }
            dead = false;
            break;
          }
          if (!done) break;
          finish_request(c, ttft, ttfb, lat);
          done = false;
          if (!start_request(c)) {
            --live;
            break;
          }
          if (!send_now(c, idx)) {
            dead = true;
            break;
          }
          if (c.in.empty()) break;
        }
      }
      if (dead && c.active) {
        g_errors++;
        if (!reconnect(c, idx)) {
          c.active = false;
          --live;
          continue;
        }
        c.req_off = 0;
        c.phase = 1;
        c.t0 = Clock::now();
        c.got_data = c.got_content = false;
        c.tail.clear();
        c.body.clear();
      }
    }
  }
  for (auto& c : cs)
    if (c.fd >= 0) close(c.fd);
  std::lock_guard<std::mutex> lk(g_mu);
  g_ttft.insert(g_ttft.end(), ttft.begin(), ttft.end());
  g_ttfb.insert(g_ttfb.end(), ttfb.begin(), ttfb.end());
  g_lat.insert(g_lat.end(), lat.begin(), lat.end());
}

double pct(std::vector<double>& v, double p) {
  if (v.empty()) return -1;
  std::sort(v.begin(), v.end());
  size_t i = (size_t)std::min((double)v.size() - 1, p / 100.0 * (v.size() - 1) + 0.5);
  return v[i];
}

std::string unhex(const std::string& h) {
  std::string o;
  for (size_t i = 0; i + 1 < h.size(); i += 2) o.push_back((char)(JR::hexv(h[i]) * 16 + JR::hexv(h[i + 1])));
  return o;
}

bool load_spec(const std::string& path) {
  std::ifstream f(path);
  if (!f) return false;
  std::string line;
  Spec& S = g.spec;
  S.on = true;
  while (std::getline(f, line)) {
    std::istringstream ss(line);
    std::string kw;
    if (!(ss >> kw) || kw[0] == '#') continue;
    if (kw == "role") ss >> S.role;
    else if (kw == "done") ss >> S.done;
    else if (kw == "stream") {
      StreamSpec st;
      std::string mode, hex;
      ss >> st.id >> mode >> hex;
      st.exact = mode == "exact";
      st.text = unhex(hex);
      S.streams.push_back(st);
    } else if (kw == "final") {
      std::string mode, hex;
      ss >> mode;
      S.final_absent = mode == "absent";
      while (ss >> hex) S.final_any.push_back(hex == "-" ? std::string() : unhex(hex));
    } else if (kw == "error") {
      std::string m;
      ss >> m;
      S.error_allowed = m == "allowed";
    } else if (kw == "empty") {
      std::string m;
      ss >> m;
      S.empty_allowed = m == "allowed";
    } else if (kw == "json") {
      ss >> S.json;
    } else if (kw == "message") {
      std::string hex;
      ss >> hex;
      S.have_message = true;
      S.message = hex == "-" ? std::string() : unhex(hex);
    } else if (kw == "usage") {
      ss >> S.usage[0] >> S.usage[1] >> S.usage[2];
    } else if (kw == "field") {
      std::string k, hex;
      ss >> k >> hex;
      S.fields.emplace_back(k, unhex(hex));
    } else {
      fprintf(stderr, "qmx_loadgen: unknown spec directive %s\n", kw.c_str());
      return false;
    }
  }
  return true;
}

}  // namespace

int main(int argc, char** argv) {
  signal(SIGPIPE, SIG_IGN);
  std::string body_file, spec_file;
  for (int i = 1; i + 1 < argc; i += 2) {
    std::string k = argv[i], v = argv[i + 1];
    if (k == "--host") g.host = v;
    else if (k == "--port") g.port = atoi(v.c_str());
    else if (k == "--conns") g.conns = atoi(v.c_str());
    else if (k == "--requests") g.requests = atol(v.c_str());
    else if (k == "--threads") g.threads = atoi(v.c_str());
    else if (k == "--path") g.path = v;
    else if (k == "--body-file") body_file = v;
    else if (k == "--stream") g.stream = atoi(v.c_str()) != 0;
    else if (k == "--timeout") g.timeout_s = atof(v.c_str());
    else if (k == "--expect") spec_file = v;
    else if (k == "--abort-rate") g.abort_rate = atof(v.c_str());
  }
  if (!spec_file.empty() && !load_spec(spec_file)) {
    fprintf(stderr, "qmx_loadgen: cannot read spec %s\n", spec_file.c_str());
    return 2;
  }
  if (const char* vb = getenv("QMX_LOADGEN_VALIDATE_BENCH")) {  // FILE:N — validator cost per body
    std::string f(vb);
    const size_t c = f.rfind(':');
    std::ifstream in(f.substr(0, c));
    std::stringstream ss;
    ss << in.rdbuf();
    const std::string body = ss.str();
    const long n = atol(f.c_str() + c + 1);
    auto t0 = Clock::now();
    long bad = 0;
    for (long i = 0; i < n; ++i) bad += !validate(200, body).empty();
    const double us = std::chrono::duration<double, std::micro>(Clock::now() - t0).count() / n;
    printf("{\"validate_us\": %.3f, \"bytes\": %zu, \"invalid\": %ld, \"why\": \"%s\"}\n", us, body.size(), bad,
           validate(200, body).c_str());
    return 0;
  }
  if (!body_file.empty()) {
    std::ifstream f(body_file);
    std::stringstream ss;
    ss << f.rdbuf();
    g.body = ss.str();
  } else {
    g.body = std::string("{\"model\": \"bench\", \"messages\": [{\"role\": \"user\", \"content\": \"Hello!\"}], \"stream\": ") +
             (g.stream ? "true" : "false") + "}";
  }
  g.threads = std::max(1, std::min(g.threads, g.conns));
  auto t0 = Clock::now();
  auto deadline = t0 + std::chrono::milliseconds((long)(g.timeout_s * 1000));
  std::vector<std::thread> ts;
  for (int t = 0; t < g.threads; ++t) {
    int n = g.conns / g.threads + (t < g.conns % g.threads ? 1 : 0);
    ts.emplace_back(worker, t, n, deadline);
  }
  for (auto& t : ts) t.join();
  double el = std::chrono::duration<double>(Clock::now() - t0).count();
  printf("{\"completed\": %ld, \"errors\": %ld, \"non200\": %ld, \"no_content\": %ld, \"invalid\": %ld, "
         "\"validated\": %ld, \"aborted\": %ld, \"elapsed_s\": %.6f, "
         "\"rps\": %.3f, \"ttft_p50_ms\": %.3f, \"ttft_p90_ms\": %.3f, \"ttft_p99_ms\": %.3f, "
         "\"ttfb_p50_ms\": %.3f, \"lat_p50_ms\": %.3f, \"lat_p99_ms\": %.3f, \"conns\": %d}\n",
         g_done.load(), g_errors.load(), g_non200.load(), g_no_content.load(), g_invalid.load(), g_validated.load(),
         g_aborted.load(), el, g_done.load() / el, pct(g_ttft, 50), pct(g_ttft, 90), pct(g_ttft, 99), pct(g_ttfb, 50),
         pct(g_lat, 50), pct(g_lat, 99), g.conns);
  return 0;
}
