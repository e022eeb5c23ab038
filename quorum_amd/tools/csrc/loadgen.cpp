// qmx_loadgen — closed-loop HTTP/1.1 load generator for OpenAI-style streaming endpoints.
//
// C keep-alive connections (spread over T epoll threads) each issue POST requests back to
// back until R requests have completed.  Per request it records TTFB (first SSE `data:`
// byte), TTFT (first SSE event carrying a non-empty "content") and total latency, parsing
// chunked or content-length bodies incrementally.  Prints one JSON line of statistics.
//
//   qmx_loadgen --port 8000 --conns 64 --requests 5000 [--threads 2] [--path /v1/chat/completions]
//               [--body-file req.json] [--stream 1]
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
#include <sstream>
#include <string>
#include <thread>
#include <vector>

namespace {
using Clock = std::chrono::steady_clock;

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
} g;

std::atomic<long> g_issued{0}, g_done{0}, g_errors{0}, g_non200{0}, g_no_content{0};
std::mutex g_mu;
std::vector<double> g_ttft, g_ttfb, g_lat;

struct Conn {
  int fd = -1;
  std::string req;
  size_t req_off = 0;
  std::string in;
  // response parse state
  int phase = 0;  // 0 idle, 1 headers, 2 body-chunked, 3 body-length
  bool chunked = false;
  long remaining = 0;
  long chunk_left = -1;
  int status = 0;
  bool got_data = false, got_content = false;
  std::string tail;  // SSE scan carry
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

// scan decoded body bytes for SSE markers
void scan_sse(Conn& c, const char* p, size_t n, Clock::time_point now) {
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
  c.tail.clear();
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
      std::string h = c.in.substr(0, he);
      c.status = atoi(h.c_str() + 9);
      for (auto& ch : h) ch = (char)tolower(ch);
      c.chunked = h.find("transfer-encoding: chunked") != std::string::npos;
      size_t p = h.find("content-length:");
      c.remaining = p != std::string::npos ? strtol(h.c_str() + p + 15, nullptr, 10) : 0;
      c.in.erase(0, he + 4);
      c.phase = c.chunked ? 2 : 3;
      c.chunk_left = -1;
      continue;
    }
    if (c.phase == 3) {
      size_t take = std::min((size_t)c.remaining, c.in.size());
      if (take) scan_sse(c, c.in.data(), take, now);
      c.in.erase(0, take);
      c.remaining -= take;
      if (c.remaining == 0) {
        *done = true;
        return true;
      }
      return true;
    }
    if (c.phase == 2) {
      if (c.chunk_left < 0) {
        size_t le = c.in.find("\r\n");
        if (le == std::string::npos) return true;
        long sz = strtol(c.in.c_str(), nullptr, 16);
        c.in.erase(0, le + 2);
        if (sz == 0) {
          // trailer: expect "\r\n"
          if (c.in.size() < 2) {
            c.chunk_left = -2;
            return true;
          }
          c.in.erase(0, 2);
          *done = true;
          return true;
        }
        c.chunk_left = sz;
      }
      if (c.chunk_left == -2) {
        if (c.in.size() < 2) return true;
        c.in.erase(0, 2);
        *done = true;
        return true;
      }
      size_t take = std::min((size_t)c.chunk_left, c.in.size());
      if (take) scan_sse(c, c.in.data(), take, now);
      c.in.erase(0, take);
      c.chunk_left -= take;
      if (c.chunk_left > 0) return true;
      if (c.in.size() < 2) {
        c.chunk_left = 0;
        if (c.in.empty()) return true;
      }
      if (c.chunk_left == 0) {
        if (c.in.size() < 2) return true;
        c.in.erase(0, 2);
        c.chunk_left = -1;
      }
      continue;
    }
    return true;
  }
}

void worker(int tid, int nconns, Clock::time_point deadline) {
  int ep = epoll_create1(0);
  std::vector<Conn> cs(nconns);
  std::vector<double> ttft, ttfb, lat;
  std::string req = "POST " + g.path + " HTTP/1.1\r\nHost: " + g.host + "\r\ncontent-type: application/json\r\n"
                    "authorization: Bearer bench\r\ncontent-length: " + std::to_string(g.body.size()) + "\r\n\r\n" + g.body;
  int live = 0;
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
      Conn& c = cs[evs[k].data.u32];
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
          e.data.u32 = evs[k].data.u32;
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
          if (!done) break;
          finish_request(c, ttft, ttfb, lat);
          done = false;
          if (!start_request(c)) {
            --live;
            break;
          }
          epoll_event e{};
          e.events = EPOLLIN | EPOLLOUT;
          e.data.u32 = evs[k].data.u32;
          epoll_ctl(ep, EPOLL_CTL_MOD, c.fd, &e);
          if (c.in.empty()) break;
        }
      }
      if (dead && c.active) {
        g_errors++;
        epoll_ctl(ep, EPOLL_CTL_DEL, c.fd, nullptr);
        close(c.fd);
        c.in.clear();
        c.fd = connect_to();
        if (c.fd < 0) {
          c.active = false;
          --live;
          continue;
        }
        epoll_event e{};
        e.events = EPOLLIN | EPOLLOUT;
        e.data.u32 = evs[k].data.u32;
        epoll_ctl(ep, EPOLL_CTL_ADD, c.fd, &e);
        c.req_off = 0;
        c.phase = 1;
        c.t0 = Clock::now();
        c.got_data = c.got_content = false;
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

}  // namespace

int main(int argc, char** argv) {
  signal(SIGPIPE, SIG_IGN);
  std::string body_file;
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
  printf("{\"completed\": %ld, \"errors\": %ld, \"non200\": %ld, \"no_content\": %ld, \"elapsed_s\": %.6f, "
         "\"rps\": %.3f, \"ttft_p50_ms\": %.3f, \"ttft_p90_ms\": %.3f, \"ttft_p99_ms\": %.3f, "
         "\"ttfb_p50_ms\": %.3f, \"lat_p50_ms\": %.3f, \"lat_p99_ms\": %.3f, \"conns\": %d}\n",
         g_done.load(), g_errors.load(), g_non200.load(), g_no_content.load(), el, g_done.load() / el,
         pct(g_ttft, 50), pct(g_ttft, 90), pct(g_ttft, 99), pct(g_ttfb, 50), pct(g_lat, 50), pct(g_lat, 99),
         g.conns);
  return 0;
}
