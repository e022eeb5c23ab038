// qmx_exchange.cpp — lock-step all-gather rounds over RCCL (xGMI) or a TCP hub.
#include "qmx_exchange.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <rccl/rccl.h>
#include <sys/socket.h>
#include <sched.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>

namespace qmx {

namespace {

using Clock = std::chrono::steady_clock;
double now_s() { return std::chrono::duration<double>(Clock::now().time_since_epoch()).count(); }

#pragma pack(push, 1)
struct WireHdr {
  uint8_t type, flags;
  uint16_t dst_loop, src_loop, pad;
  int32_t dst_rank, src_rank, bi;
  uint64_t skey;
  int32_t a, b;
  uint32_t len;
};
#pragma pack(pop)

void serialize(const std::vector<XMsg>& ms, std::string& out) {
  for (const XMsg& m : ms) {
    WireHdr h{m.type, m.flags, m.dst_loop, m.src_loop, 0, m.dst_rank, m.src_rank, m.bi, m.skey, m.a, m.b,
              (uint32_t)m.payload.size()};
    out.append((const char*)&h, sizeof(h));
    out += m.payload;
  }
}

bool parse_for(const std::string& buf, int rank, std::vector<XMsg>& out) {
  size_t p = 0;
  while (p + sizeof(WireHdr) <= buf.size()) {
    WireHdr h;
    std::memcpy(&h, buf.data() + p, sizeof(h));
    p += sizeof(h);
    if (p + h.len > buf.size()) return false;
    if (h.dst_rank == rank) {
      XMsg m;
      m.type = h.type;
      m.flags = h.flags;
      m.dst_loop = h.dst_loop;
      m.src_loop = h.src_loop;
      m.dst_rank = h.dst_rank;
      m.src_rank = h.src_rank;
      m.bi = h.bi;
      m.skey = h.skey;
      m.a = h.a;
      m.b = h.b;
      m.payload.assign(buf.data() + p, h.len);
      out.push_back(std::move(m));
    }
    p += h.len;
  }
  return p == buf.size();
}

// ------------------------------------------------------------------------------ TCP hub
bool send_all(int fd, const void* p, size_t n) {
  const char* c = (const char*)p;
  while (n) {
    ssize_t w = send(fd, c, n, MSG_NOSIGNAL);
    if (w <= 0) {
      if (w < 0 && errno == EINTR) continue;
      return false;
    }
    c += w;
    n -= (size_t)w;
  }
  return true;
}
bool recv_all(int fd, void* p, size_t n) {
  char* c = (char*)p;
  while (n) {
    ssize_t r = recv(fd, c, n, 0);
    if (r <= 0) {
      if (r < 0 && errno == EINTR) continue;
      return false;
    }
    c += r;
    n -= (size_t)r;
  }
  return true;
}
void set_timeouts(int fd, double s) {
  timeval tv{};
  tv.tv_sec = (time_t)s;
  tv.tv_usec = (suseconds_t)((s - (double)tv.tv_sec) * 1e6);
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

class TcpX : public XTransport {
 public:
  explicit TcpX(const XOptions& o) : o_(o), fds_(o.world, -1) {
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)o.port);
    inet_pton(AF_INET, o.addr.c_str(), &a.sin_addr);
    const double t_end = now_s() + o.timeout_s;
    if (o.rank == 0) {
      int l = socket(AF_INET, SOCK_STREAM, 0);
      int one = 1;
      setsockopt(l, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
      if (bind(l, (sockaddr*)&a, sizeof(a)) != 0 || listen(l, 64) != 0) {
        close(l);
        throw std::runtime_error("exchange: hub bind failed: " + std::string(strerror(errno)));
      }
      set_timeouts(l, o.timeout_s);
      for (int got = 1; got < o.world;) {
        int fd = accept(l, nullptr, nullptr);
        if (fd < 0) {
          if (errno == EINTR) continue;
          close(l);
          throw std::runtime_error("exchange: peers did not connect");
        }
        set_timeouts(fd, o.timeout_s);
        int32_t r = -1;
        if (!recv_all(fd, &r, 4) || r <= 0 || r >= o.world || fds_[r] >= 0) {
          close(fd);
          continue;
        }
        fds_[r] = fd;
        ++got;
      }
      close(l);
    } else {
      int fd = -1;
      while (true) {
        fd = socket(AF_INET, SOCK_STREAM, 0);
        if (connect(fd, (sockaddr*)&a, sizeof(a)) == 0) break;
        close(fd);
        fd = -1;
        if (now_s() > t_end) throw std::runtime_error("exchange: cannot reach hub");
        usleep(20000);
      }
      set_timeouts(fd, o.timeout_s);
      int32_t r = o.rank;
      if (!send_all(fd, &r, 4)) throw std::runtime_error("exchange: hub handshake failed");
      fds_[0] = fd;
    }
  }
  ~TcpX() override {
    for (int fd : fds_)
      if (fd >= 0) close(fd);
  }
  bool allgather(const std::string& mine, uint32_t flags, std::vector<std::string>& all,
                 std::vector<uint32_t>& all_flags) override {
    const int W = o_.world;
    all.assign(W, std::string());
    all_flags.assign(W, 0);
    if (o_.rank != 0) {
      uint32_t h[2] = {(uint32_t)mine.size(), flags};
      if (!send_all(fds_[0], h, 8) || !send_all(fds_[0], mine.data(), mine.size())) return false;
      std::vector<uint32_t> hs(2 * W);
      if (!recv_all(fds_[0], hs.data(), 8 * W)) return false;
      for (int r = 0; r < W; ++r) {
        all[r].resize(hs[2 * r]);
        all_flags[r] = hs[2 * r + 1];
        if (hs[2 * r] && !recv_all(fds_[0], &all[r][0], hs[2 * r])) return false;
      }
      return true;
    }
    all[0] = mine;
    all_flags[0] = flags;
    for (int r = 1; r < W; ++r) {
      uint32_t h[2];
      if (!recv_all(fds_[r], h, 8)) return false;
      all[r].resize(h[0]);
      all_flags[r] = h[1];
      if (h[0] && !recv_all(fds_[r], &all[r][0], h[0])) return false;
    }
    std::string blob;
    for (int r = 0; r < W; ++r) {
      uint32_t h[2] = {(uint32_t)all[r].size(), all_flags[r]};
      blob.append((const char*)h, 8);
    }
    for (int r = 0; r < W; ++r) blob += all[r];
    for (int r = 1; r < W; ++r)
      if (!send_all(fds_[r], blob.data(), blob.size())) return false;
    return true;
  }

 private:
  XOptions o_;
  std::vector<int> fds_;
};

// ------------------------------------------------------------------------------ RCCL
#define XHIP(x)                                                                            \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) throw std::runtime_error(std::string("exchange HIP: ") + hipGetErrorString(e_)); \
  } while (0)
#define XNCCL(x)                                                                           \
  do {                                                                                     \
    ncclResult_t r_ = (x);                                                                 \
    if (r_ != ncclSuccess) throw std::runtime_error(std::string("exchange RCCL: ") + ncclGetErrorString(r_)); \
  } while (0)

std::string to_hex(const ncclUniqueId& id) {
  static const char* d = "0123456789abcdef";
  std::string s;
  for (int i = 0; i < NCCL_UNIQUE_ID_BYTES; ++i) {
    uint8_t b = (uint8_t)id.internal[i];
    s.push_back(d[b >> 4]);
    s.push_back(d[b & 15]);
  }
  return s;
}
bool from_hex(const std::string& s, ncclUniqueId* id) {
  if (s.size() < 2 * NCCL_UNIQUE_ID_BYTES) return false;
  auto v = [](char c) { return c >= 'a' ? c - 'a' + 10 : c - '0'; };
  for (int i = 0; i < NCCL_UNIQUE_ID_BYTES; ++i) id->internal[i] = (char)((v(s[2 * i]) << 4) | v(s[2 * i + 1]));
  return true;
}

class RcclX : public XTransport {
 public:
  static constexpr size_t kSlot = 8192;  // fixed per-rank slot of the first all-gather

  explicit RcclX(const XOptions& o) : o_(o) {
    XHIP(hipSetDevice(o.device));
    ncclUniqueId id;
    if (o.rank == 0) {
      XNCCL(ncclGetUniqueId(&id));
      std::string tmp = o.id_file + ".tmp";
      {
        std::ofstream f(tmp);
        f << to_hex(id);
      }
      if (rename(tmp.c_str(), o.id_file.c_str()) != 0) throw std::runtime_error("exchange: cannot publish RCCL id");
    } else {
      const double t_end = now_s() + o.timeout_s;
      while (true) {
        std::ifstream f(o.id_file);
        std::string s;
        if (f && (f >> s) && from_hex(s, &id)) break;
        if (now_s() > t_end) throw std::runtime_error("exchange: RCCL id not published");
        usleep(20000);
      }
    }
    XHIP(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking));
    XNCCL(ncclCommInitRank(&comm_, o.world, id, o.rank));
    XHIP(hipMalloc(&d_s1_, kSlot));
    XHIP(hipMalloc(&d_r1_, kSlot * o.world));
    XHIP(hipHostMalloc((void**)&h_s1_, kSlot));
    XHIP(hipHostMalloc((void**)&h_r1_, kSlot * o.world));
  }
  ~RcclX() override {
    if (comm_) {
      if (aborted_) ncclCommAbort(comm_);
      else ncclCommDestroy(comm_);
    }
    if (st_) hipStreamDestroy(st_);
    hipFree(d_s1_);
    hipFree(d_r1_);
    hipFree(d_s2_);
    hipFree(d_r2_);
    hipHostFree(h_s1_);
    hipHostFree(h_r1_);
    hipHostFree(h_s2_);
    hipHostFree(h_r2_);
  }
  bool wait() {
    const double t_end = now_s() + o_.timeout_s;
    while (true) {
      hipError_t e = hipStreamQuery(st_);
      if (e == hipSuccess) return true;
      if (e != hipErrorNotReady || now_s() > t_end) {
        ncclCommAbort(comm_);  // a peer died or stalled: fail fast, survivors go local
        comm_ = nullptr;
        aborted_ = true;
        return false;
      }
      // yield while the round is young (collectives take tens of us), then back off
      if (now_s() - (t_end - o_.timeout_s) < 5e-4) sched_yield();
      else usleep(50);
    }
  }
  bool allgather(const std::string& mine, uint32_t flags, std::vector<std::string>& all,
                 std::vector<uint32_t>& all_flags) override {
    if (!comm_) return false;
    const int W = o_.world;
    const size_t cap = kSlot - 8;
    uint32_t h[2] = {(uint32_t)mine.size(), flags};
    std::memcpy(h_s1_, h, 8);
    const size_t n1 = std::min(mine.size(), cap);
    if (mine.size() <= cap) std::memcpy(h_s1_ + 8, mine.data(), n1);
    try {
      XHIP(hipMemcpyAsync(d_s1_, h_s1_, 8 + (mine.size() <= cap ? n1 : 0), hipMemcpyHostToDevice, st_));
      XNCCL(ncclAllGather(d_s1_, d_r1_, kSlot, ncclUint8, comm_, st_));
      XHIP(hipMemcpyAsync(h_r1_, d_r1_, kSlot * W, hipMemcpyDeviceToHost, st_));
    } catch (const std::exception& e) {
      fprintf(stderr, "%s\n", e.what());
      return false;
    }
    if (!wait()) return false;
    all.assign(W, std::string());
    all_flags.assign(W, 0);
    size_t M = 0;
    for (int r = 0; r < W; ++r) {
      uint32_t hr[2];
      std::memcpy(hr, h_r1_ + r * kSlot, 8);
      all_flags[r] = hr[1];
      if (hr[0] <= cap) all[r].assign((const char*)h_r1_ + r * kSlot + 8, hr[0]);
      else M = std::max(M, (size_t)hr[0]);
    }
    if (M == 0) return true;
    // phase 2: padded all-gather of the large buffers (every rank knows M from phase 1)
    try {
      if (M > cap2_) {
        hipFree(d_s2_);
        hipFree(d_r2_);
        hipHostFree(h_s2_);
        hipHostFree(h_r2_);
        cap2_ = std::max(M, cap2_ * 2);
        XHIP(hipMalloc(&d_s2_, cap2_));
        XHIP(hipMalloc(&d_r2_, cap2_ * W));
        XHIP(hipHostMalloc((void**)&h_s2_, cap2_));
        XHIP(hipHostMalloc((void**)&h_r2_, cap2_ * W));
      }
      if (mine.size() > cap) {
        std::memcpy(h_s2_, mine.data(), mine.size());
        XHIP(hipMemcpyAsync(d_s2_, h_s2_, mine.size(), hipMemcpyHostToDevice, st_));
      }
      XNCCL(ncclAllGather(d_s2_, d_r2_, M, ncclUint8, comm_, st_));
      XHIP(hipMemcpyAsync(h_r2_, d_r2_, M * W, hipMemcpyDeviceToHost, st_));
    } catch (const std::exception& e) {
      fprintf(stderr, "%s\n", e.what());
      return false;
    }
    if (!wait()) return false;
    for (int r = 0; r < W; ++r) {
      uint32_t hr[2];
      std::memcpy(hr, h_r1_ + r * kSlot, 8);
      if (hr[0] > cap) all[r].assign((const char*)h_r2_ + r * M, hr[0]);
    }
    return true;
  }

 private:
  XOptions o_;
  ncclComm_t comm_ = nullptr;
  hipStream_t st_ = nullptr;
  bool aborted_ = false;
  uint8_t *d_s1_ = nullptr, *d_r1_ = nullptr, *h_s1_ = nullptr, *h_r1_ = nullptr;
  uint8_t *d_s2_ = nullptr, *d_r2_ = nullptr, *h_s2_ = nullptr, *h_r2_ = nullptr;
  size_t cap2_ = 0;
};

}  // namespace

std::unique_ptr<XTransport> make_tcp_transport(const XOptions& o) { return std::unique_ptr<XTransport>(new TcpX(o)); }
std::unique_ptr<XTransport> make_rccl_transport(const XOptions& o) {
  return std::unique_ptr<XTransport>(new RcclX(o));
}
std::string rccl_unique_id_hex() {
  ncclUniqueId id;
  XNCCL(ncclGetUniqueId(&id));
  return to_hex(id);
}

// ------------------------------------------------------------------------------ Exchange
Exchange::Exchange(const XOptions& o, int nloops, Deliver deliver)
    : o_(o), nloops_(nloops), deliver_(std::move(deliver)) {
  th_ = std::thread([this] { run(); });
}
Exchange::~Exchange() {
  request_stop();
  join();
}
void Exchange::post(XMsg&& m) {
  if (stop_.load()) return;
  std::lock_guard<std::mutex> g(mu_);
  out_.push_back(std::move(m));
}
void Exchange::request_stop() {
  stop_.store(true);
  cv_.notify_all();
}
void Exchange::join() {
  if (th_.joinable()) th_.join();
}

void Exchange::run() {
  std::unique_ptr<XTransport> tr;
  auto down = [&]() {
    healthy_.store(false);
    for (int l = 0; l < nloops_; ++l) {
      std::vector<XMsg> v(1);
      v[0].type = X_DOWN;
      deliver_(l, std::move(v));
    }
  };
  try {
    tr = o_.transport == "rccl" ? make_rccl_transport(o_) : make_tcp_transport(o_);
  } catch (const std::exception& e) {
    fprintf(stderr, "qmx exchange (rank %d): %s — spread placement disabled\n", o_.rank, e.what());
    return down();
  }
  healthy_.store(true);  // sessions start placing streams on other ranks from now on
  int idle = 0;
  std::vector<std::string> all;
  std::vector<uint32_t> fl;
  while (true) {
    std::vector<XMsg> batch;
    bool stopping;
    {
      std::unique_lock<std::mutex> lk(mu_);
      // Every rank paces identically (idle is derived from the gathered totals), so the
      // lock-step collective is not held up by a sleeping peer for long.
      const int us = idle > 64 ? 1000 : o_.round_us;
      cv_.wait_for(lk, std::chrono::microseconds(us), [this] { return stop_.load(); });
      batch.swap(out_);
      stopping = stop_.load();
    }
    std::string mine;
    serialize(batch, mine);
    const double t0 = now_s();
    if (!tr->allgather(mine, stopping ? 1u : 0u, all, fl)) {
      fprintf(stderr, "qmx exchange (rank %d): round failed — falling back to local placement\n", o_.rank);
      return down();
    }
    busy_us_.store(busy_us_.load() + 1e6 * (now_s() - t0));
    rounds_++;
    size_t total = 0;
    bool all_stop = true;
    std::vector<std::vector<XMsg>> per(nloops_);
    for (int r = 0; r < (int)all.size(); ++r) {
      total += all[r].size();
      all_stop = all_stop && (fl[r] & 1);
      std::vector<XMsg> got;
      if (!parse_for(all[r], o_.rank, got)) continue;
      for (auto& m : got) per[m.dst_loop % nloops_].push_back(std::move(m));
    }
    bytes_ += total;
    for (int l = 0; l < nloops_; ++l)
      if (!per[l].empty()) deliver_(l, std::move(per[l]));
    idle = total ? 0 : idle + 1;
    if (all_stop) break;
  }
}

}  // namespace qmx
