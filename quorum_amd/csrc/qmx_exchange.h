// qmx_exchange.h — cross-rank message exchange for spread (EP-style) backend placement.
//
// One process per GPU.  With `placement: spread`, a session's N backend streams run on
// ranks owner, owner+1, ... (mod world): each worker rank opens the upstream connection
// from its own keep-alive pool and runs the stream through its own GPU tick kernel; the
// encoded SSE deltas and the stripped final text come back to the session owner.
//
// Transport = lock-step rounds of an all-gather: every rank contributes
// one buffer per round holding all its outgoing messages; receivers keep the messages
// addressed to them.  Round = ONE fixed-slot all-gather (header + up to kSlot bytes per
// rank) in the common case, plus a padded all-gather of max_len bytes when any rank has
// more (lengths travel in the first one).  Backends:
//   rccl — ncclAllGather on a dedicated HIP stream over xGMI (device buffers, pinned
//          staging); a round that does not complete within the timeout aborts the
//          communicator (rank death) and the survivors fall back to local placement.
//   tcp  — hub at rank 0 (CPU tests, no GPU).
// Messages are tiny (KB) and rounds are latency-bound, so the design batches every
// message of a round into one collective rather than issuing per-session operations.
#pragma once
#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace qmx {

enum XType : uint8_t { X_OPEN = 1, X_DATA = 2, X_FINAL = 3, X_CANCEL = 4, X_DOWN = 5 };
// X_FINAL flags
enum : uint8_t { XF_TEXT = 1, XF_ABORTED = 2, XF_FAILED = 4 };

struct XMsg {
  uint8_t type = 0, flags = 0;
  uint16_t dst_loop = 0, src_loop = 0;
  int32_t dst_rank = 0, src_rank = 0;
  int32_t bi = 0;     // backend slot within the owner's session
  uint64_t skey = 0;  // owner session key
  int32_t a = 0, b = 0;
  std::string payload;
};

struct XOptions {
  int rank = 0, world = 1;
  std::string transport = "tcp";  // tcp | rccl
  std::string addr = "127.0.0.1";
  int port = 0;                   // tcp hub port
  std::string id_file;            // rccl: rank 0 writes the unique id here, others read it
  int device = 0;
  int round_us = 200;             // pacing between rounds while traffic flows
  double timeout_s = 30.0;        // a round slower than this = peer failure
};

class XTransport {
 public:
  virtual ~XTransport() = default;
  // All-gather `mine` (+ flag bits); returns false on failure (peer death / timeout).
  virtual bool allgather(const std::string& mine, uint32_t flags, std::vector<std::string>& all,
                         std::vector<uint32_t>& all_flags) = 0;
};

std::unique_ptr<XTransport> make_tcp_transport(const XOptions& o);
std::unique_ptr<XTransport> make_rccl_transport(const XOptions& o);
std::string rccl_unique_id_hex();  // for launchers that distribute the id themselves

class Exchange {
 public:
  using Deliver = std::function<void(int loop, std::vector<XMsg>&&)>;
  Exchange(const XOptions& o, int nloops, Deliver deliver);
  ~Exchange();
  void post(XMsg&& m);       // thread-safe
  void request_stop();       // the thread exits once every rank has requested stop
  void join();
  bool healthy() const { return healthy_.load(); }  // false until connected and after a failure
  int rank() const { return o_.rank; }
  int world() const { return o_.world; }
  uint64_t rounds() const { return rounds_.load(); }
  uint64_t bytes() const { return bytes_.load(); }
  double busy_us() const { return busy_us_.load(); }

 private:
  void run();
  XOptions o_;
  int nloops_;
  Deliver deliver_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<XMsg> out_;
  std::atomic<bool> stop_{false}, healthy_{false};  // healthy once the transport is up
  std::atomic<uint64_t> rounds_{0}, bytes_{0};
  std::atomic<double> busy_us_{0};
  std::thread th_;
};

}  // namespace qmx
