// qmx_mock — fast OpenAI-compatible mock LLM backend (epoll, SO_REUSEPORT, keep-alive).
//
// Serves POST /chat/completions and /v1/chat/completions.  Streaming responses are the
// survey's benchmark shape: role event, 4 split think fragments, N content
// tokens, stop, [DONE], sent with chunked transfer encoding; optional per-event delay.
// Fault knobs (BASELINE config 5): --fail-rate (HTTP 500), --stall-ms (never answer),
// --drop-rate (close mid-stream), --null-rate (content:null event); --trickle 1 writes a
// faulty response event by event instead of at once.
//
//   qmx_mock --port 9101 [--threads 2] [--tokens 20] [--think 1] [--delay-us 0]
//   qmx_mock --print-expected 1 [--tokens 20] [--think 1]   # JSON: what clients should see
//       {"stream_text": <content outside the think block>, "message": <non-stream content>,
//        "raw_text": <every streamed content byte>, "usage": [prompt, completion, total]}
#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <strings.h>
#include <map>
#include <queue>
#include <random>
#include <string>
#include <thread>
#include <vector>

namespace {

struct Opts {
  int port = 9101;
  int threads = 2;
  int tokens = 20;
  int think = 1;
  long delay_us = 0;
  double fail_rate = 0.0;
  double drop_rate = 0.0;
  double null_rate = 0.0;
  long stall_ms = 0;
  // faulty responses without a per-event delay: written at once like every other response
  // (0, the default) or event by event, each write a timer tick of its own (1: the round-4
  // behaviour, which made a faulty backend trickle; --delay-us paces events explicitly)
  int trickle = 0;
  std::string name = "mock";
} g;

std::string sse_event(const std::string& delta_json, const char* finish = "null") {
  std::string ev = "data: {\"id\": \"chatcmpl-mock\", \"object\": \"chat.completion.chunk\", \"created\": 1700000000, "
                   "\"model\": \"" + g.name + "\", \"choices\": [{\"index\": 0, \"delta\": " + delta_json +
                   ", \"finish_reason\": " + finish + "}]}\n\n";
  return ev;
}
std::string chunk(const std::string& s) {
  char hdr[32];
  snprintf(hdr, sizeof(hdr), "%zx\r\n", s.size());
  return std::string(hdr) + s + "\r\n";
}

std::vector<std::string> g_events;  // SSE events of one streamed response
std::string g_visible;              // concatenated content outside the think block
std::string g_raw;                  // every content byte of the stream (think block included)
std::string g_message;              // non-streaming message content
std::string g_stream_all;           // full chunked streamed response (no delay path)
std::string g_json_resp;            // non-streaming response
const char* kStreamHdr =
    "HTTP/1.1 200 OK\r\ncontent-type: text/event-stream\r\ncache-control: no-cache\r\n"
    "transfer-encoding: chunked\r\n\r\n";

void build_responses() {
  static const char* words[] = {"The", " quick", " brown", " fox", " jumps", " over", " the", " lazy", " dog", ".",
                                " Proxy", " tokens", " flow", " through", " MI355X", " kernels", " with", " low",
                                " latency", "!"};
  g_events.clear();
  g_events.push_back(sse_event("{\"role\": \"assistant\", \"content\": \"\"}"));
  if (g.think) {
    g_events.push_back(sse_event("{\"content\": \"<thi\"}"));
    g_events.push_back(sse_event("{\"content\": \"nk>let me reason about the request\"}"));
    g_events.push_back(sse_event("{\"content\": \" carefully before answering</th\"}"));
    g_events.push_back(sse_event("{\"content\": \"ink>\"}"));
  }
  std::string full;
  for (int i = 0; i < g.tokens; ++i) {
    std::string w = words[i % 20];
    full += w;
    g_events.push_back(sse_event("{\"content\": \"" + w + "\"}"));
  }
  g_visible = full;
  g_raw = std::string(g.think ? "<think>let me reason about the request carefully before answering</think>" : "") + full;
  g_message = std::string(g.think ? "<think>let me reason</think>" : "") + full;
  g_events.push_back(sse_event("{}", "\"stop\""));
  g_events.push_back("data: [DONE]\n\n");
  g_stream_all = kStreamHdr;
  for (auto& e : g_events) g_stream_all += chunk(e);
  g_stream_all += "0\r\n\r\n";
  std::string body = "{\"id\": \"chatcmpl-mock\", \"object\": \"chat.completion\", \"created\": 1700000000, "
                     "\"model\": \"" + g.name + "\", \"system_fingerprint\": \"fp_mock\", \"choices\": [{\"index\": 0, "
                     "\"message\": {\"role\": \"assistant\", \"content\": \"" +
                     std::string(g.think ? "<think>let me reason</think>" : "") + full +
                     "\"}, \"logprobs\": null, \"finish_reason\": \"stop\"}], \"usage\": {\"prompt_tokens\": 9, "
                     "\"completion_tokens\": " + std::to_string(g.tokens) + ", \"total_tokens\": " +
                     std::to_string(9 + g.tokens) + "}}";
  g_json_resp = "HTTP/1.1 200 OK\r\ncontent-type: application/json\r\ncontent-length: " +
                std::to_string(body.size()) + "\r\n\r\n" + body;
}

const std::string kFailBody = "{\"error\": {\"message\": \"injected failure\", \"type\": \"mock\"}}";
const std::string kFail = "HTTP/1.1 500 Internal Server Error\r\ncontent-type: application/json\r\ncontent-length: " +
                          std::to_string(kFailBody.size()) + "\r\n\r\n" + kFailBody;

struct Conn {
  int fd;
  std::string in;
  std::string out;
  size_t out_off = 0;
  // delayed streaming state
  int next_event = -1;
  bool drop_after = false;
  int drop_at = -1;
  bool stalled = false;
  bool close_after = false;  // a mid-stream drop written at once: close once it is out
};

using Clock = std::chrono::steady_clock;

void set_nb(int fd) { fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) | O_NONBLOCK); }

int make_listener(int port) {
  int fd = socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  setsockopt(fd, SOL_SOCKET, SO_REUSEPORT, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(port);
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  if (bind(fd, (sockaddr*)&a, sizeof(a)) != 0) {
    perror("bind");
    exit(1);
  }
  listen(fd, 4096);
  set_nb(fd);
  return fd;
}

void worker(int tid) {
  int lfd = make_listener(g.port);
  int ep = epoll_create1(0);
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.fd = lfd;
  epoll_ctl(ep, EPOLL_CTL_ADD, lfd, &ev);
  std::map<int, Conn> conns;
  std::mt19937_64 rng(1234 + tid);
  std::uniform_real_distribution<double> U(0, 1);
  // timer queue for delayed events: (time, fd)
  using TE = std::pair<Clock::time_point, int>;
  std::priority_queue<TE, std::vector<TE>, std::greater<TE>> timers;
  std::vector<epoll_event> evs(1024);

  auto flush = [&](Conn& c) -> bool {
    while (c.out_off < c.out.size()) {
      ssize_t n = send(c.fd, c.out.data() + c.out_off, c.out.size() - c.out_off, MSG_NOSIGNAL);
      if (n > 0) {
        c.out_off += n;
        continue;
      }
      if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
        epoll_event e{};
        e.events = EPOLLIN | EPOLLOUT;
        e.data.fd = c.fd;
        epoll_ctl(ep, EPOLL_CTL_MOD, c.fd, &e);
        return true;
      }
      return false;
    }
    c.out.clear();
    c.out_off = 0;
    return true;
  };
  auto close_conn = [&](int fd) {
    epoll_ctl(ep, EPOLL_CTL_DEL, fd, nullptr);
    close(fd);
    conns.erase(fd);
  };
  auto send_event = [&](Conn& c) -> bool {
    int i = c.next_event;
    if (i == c.drop_at) return false;
    if (i == (int)g_events.size()) {
      c.out += "0\r\n\r\n";
      c.next_event = -1;
    } else {
      const std::string& e = (i == 2 && g.null_rate > 0 && U(rng) < g.null_rate)
                                 ? sse_event("{\"content\": null}")
                                 : g_events[i];
      c.out += chunk(e);
      c.next_event = i + 1;
      timers.push({Clock::now() + std::chrono::microseconds(g.delay_us), c.fd});
    }
    return flush(c);
  };
  auto handle = [&](Conn& c) -> bool {
    while (true) {
      size_t he = c.in.find("\r\n\r\n");
      if (he == std::string::npos) return true;
      size_t cl = 0;
      {
        // case-insensitive content-length, found in place (no copy of the headers)
        static const char kCl[] = "content-length:";
        for (size_t i = 0; i + sizeof(kCl) - 1 <= he; ++i) {
          if ((c.in[i] | 0x20) != 'c' || strncasecmp(c.in.data() + i, kCl, sizeof(kCl) - 1) != 0) continue;
          cl = strtoul(c.in.data() + i + sizeof(kCl) - 1, nullptr, 10);
          break;
        }
      }
      if (c.in.size() < he + 4 + cl) return true;
      const char* body = c.in.data() + he + 4;
      const bool stream = memmem(body, cl, "\"stream\": true", 14) != nullptr ||
                          memmem(body, cl, "\"stream\":true", 13) != nullptr;
      c.in.erase(0, he + 4 + cl);
      if (g.stall_ms > 0) {
        c.stalled = true;
        continue;
      }
      if (g.fail_rate > 0 && U(rng) < g.fail_rate) {
        c.out += kFail;
        if (!flush(c)) return false;
        continue;
      }
      if (!stream) {
        c.out += g_json_resp;
        if (!flush(c)) return false;
        continue;
      }
      c.drop_at = (g.drop_rate > 0 && U(rng) < g.drop_rate) ? (int)(g_events.size() / 2) : -1;
      if (g.delay_us <= 0 && c.drop_at < 0 && g.null_rate <= 0 && !g.trickle) {
        c.out += g_stream_all;
        if (!flush(c)) return false;
        continue;
      }
      if (g.delay_us <= 0 && !g.trickle) {
        // faults drawn per response exactly as the event-by-event path draws them (null on
        // event 2, a drop at the middle event), the response written at once
        const bool null2 = g.null_rate > 0 && U(rng) < g.null_rate;
        c.out += kStreamHdr;
        const int end = c.drop_at >= 0 ? c.drop_at : (int)g_events.size();
        for (int i = 0; i < end; ++i) c.out += chunk(i == 2 && null2 ? sse_event("{\"content\": null}") : g_events[i]);
        if (c.drop_at >= 0) {  // mid-stream disconnect: the first half, then the connection closes
          c.close_after = true;
          if (!flush(c)) return false;
          return !c.out.empty();  // all out: close now; else once EPOLLOUT drained it
        }
        c.out += "0\r\n\r\n";
        if (!flush(c)) return false;
        continue;
      }
      c.out += kStreamHdr;
      c.next_event = 0;
      if (!send_event(c)) return false;
      return true;  // pipelined requests wait for this stream
    }
  };

  while (true) {
    int timeout = -1;
    if (!timers.empty()) {
      auto dt = std::chrono::duration_cast<std::chrono::microseconds>(timers.top().first - Clock::now()).count();
      timeout = dt <= 0 ? 0 : (int)((dt + 999) / 1000);
      if (dt > 0 && dt < 1000) timeout = 0;  // busy-poll sub-millisecond delays
    }
    int n = epoll_wait(ep, evs.data(), (int)evs.size(), timeout);
    for (int i = 0; i < n; ++i) {
      int fd = evs[i].data.fd;
      if (fd == lfd) {
        while (true) {
          int cfd = accept4(lfd, nullptr, nullptr, SOCK_NONBLOCK);
          if (cfd < 0) break;
          int one = 1;
          setsockopt(cfd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
          epoll_event e{};
          e.events = EPOLLIN;
          e.data.fd = cfd;
          epoll_ctl(ep, EPOLL_CTL_ADD, cfd, &e);
          conns[cfd] = Conn{cfd};
        }
        continue;
      }
      auto it = conns.find(fd);
      if (it == conns.end()) continue;
      Conn& c = it->second;
      bool ok = true;
      if (evs[i].events & EPOLLOUT) {
        ok = flush(c);
        if (ok && c.out.empty() && c.close_after) ok = false;  // a dropped stream's first half is out
        if (ok && c.out.empty()) {
          epoll_event e{};
          e.events = EPOLLIN;
          e.data.fd = fd;
          epoll_ctl(ep, EPOLL_CTL_MOD, fd, &e);
        }
      }
      if (ok && (evs[i].events & (EPOLLIN | EPOLLHUP | EPOLLERR))) {
        char buf[65536];
        while (true) {
          ssize_t r = recv(fd, buf, sizeof(buf), 0);
          if (r > 0) {
            c.in.append(buf, r);
            continue;
          }
          if (r == 0) ok = false;
          else if (errno != EAGAIN && errno != EWOULDBLOCK) ok = false;
          break;
        }
        if (ok && c.next_event < 0 && !c.stalled && !c.close_after) ok = handle(c);
      }
      if (!ok) close_conn(fd);
    }
    auto now = Clock::now();
    while (!timers.empty() && timers.top().first <= now) {
      int fd = timers.top().second;
      timers.pop();
      auto it = conns.find(fd);
      if (it == conns.end() || it->second.next_event < 0) continue;
      Conn& c = it->second;
      if (!send_event(c)) {
        close_conn(fd);
        continue;
      }
      if (c.next_event < 0 && !c.in.empty() && !handle(c)) close_conn(fd);
    }
  }
}

}  // namespace

int main(int argc, char** argv) {
  signal(SIGPIPE, SIG_IGN);
  bool print_expected = false;
  for (int i = 1; i + 1 < argc; i += 2) {
    std::string k = argv[i], v = argv[i + 1];
    if (k == "--port") g.port = atoi(v.c_str());
    else if (k == "--threads") g.threads = atoi(v.c_str());
    else if (k == "--tokens") g.tokens = atoi(v.c_str());
    else if (k == "--think") g.think = atoi(v.c_str());
    else if (k == "--delay-us") g.delay_us = atol(v.c_str());
    else if (k == "--fail-rate") g.fail_rate = atof(v.c_str());
    else if (k == "--drop-rate") g.drop_rate = atof(v.c_str());
    else if (k == "--null-rate") g.null_rate = atof(v.c_str());
    else if (k == "--stall-ms") g.stall_ms = atol(v.c_str());
    else if (k == "--trickle") g.trickle = atoi(v.c_str());
    else if (k == "--name") g.name = v;
    else if (k == "--print-expected") print_expected = atoi(v.c_str()) != 0;
  }
  build_responses();
  if (print_expected) {
    auto js = [](const std::string& x) {  // the texts are ASCII without quotes / backslashes
      return "\"" + x + "\"";
    };
    printf("{\"stream_text\": %s, \"message\": %s, \"raw_text\": %s, \"usage\": [9, %d, %d]}\n",
           js(g_visible).c_str(), js(g_message).c_str(), js(g_raw).c_str(), g.tokens, 9 + g.tokens);
    return 0;
  }
  std::vector<std::thread> ts;
  for (int t = 0; t < g.threads; ++t) ts.emplace_back(worker, t);
  fprintf(stderr, "qmx_mock listening on 127.0.0.1:%d (%d threads)\n", g.port, g.threads);
  for (auto& t : ts) t.join();
  return 0;
}
