// qmx_exchange.h — cross-rank messaging for spread (EP-style) backend placement.
//
// One process per GPU.  With `placement: spread`, a session's N backend streams run on
// ranks owner, owner+1, ... (mod world): each worker rank opens the upstream connection
// from its own keep-alive pool and runs the stream through its own GPU tick kernel.
//
// Two planes, both event-driven (nothing moves while every rank is idle):
//  * mesh — a TCP connection per rank pair (rank r listens on port + r; the higher rank
//    dials).  Control messages (open / cancel / final flags) and the encoded SSE deltas
//    travel point to point, owner <-> worker, never through a collective: they are on the
//    TTFT path (SURVEY §7.4 hard part 5).  A dropped connection marks the peer down (its
//    streams fail, new sessions stop placing streams there); the higher rank redials every
//    100 ms, so a restarted rank re-joins the mesh without any coordination.
//  * bulk — a stream's final text goes from the worker's HBM content arena straight into the
//    owner's HBM content arena (the owner's "shadow" slot for that stream) with ncclSend /
//    ncclRecv over xGMI, so the owner's own fused finalize kernel (K3 strip, K4 join, K5
//    encode) merges local and remote streams alike.  RCCL point-to-point
//    needs both ends to post matching operations in the same per-pair order: rank 0
//    coordinates — workers announce (owner, length) over the mesh, rank 0 batches the
//    announcements into numbered rounds and sends each involved rank its part of the round
//    manifest; every rank executes rounds in order, one ncclGroupStart/End per round with
//    only its own sends and receives.  A peer that never answers aborts the communicator
//    (a round timeout); bulk transfers then fall back to the mesh (host bytes) until rank 0
//    re-forms the communicator over the ranks that are up (a new "epoch").  transport=tcp
//    (CPU tests, no GPU) sends bulk bytes over the mesh only.
#pragma once
#include <atomic>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace qmx {

enum XType : uint8_t {
  X_OPEN = 1,    // owner → worker: run stream bi of session skey (payload: upstream request)
  X_DATA = 2,    // worker → owner: encoded SSE deltas of the stream
  X_FINAL = 3,   // worker → owner: stream over without a bulk text (flags below)
  X_CANCEL = 4,  // owner → worker: session gone, stop the stream
  X_DOWN = 5,    // exchange → loops: peer `a` is unreachable (a = -1: the whole exchange)
  X_BULK = 6,    // exchange → owner loop: the stream's final text arrived (a = length, b = data
                 //   messages sent before it; payload = the bytes when not written to HBM)
  X_SENT = 7,    // exchange → worker loop: the bulk left (flags XF_FAILED if it could not)
  X_UP = 8,      // exchange → loops: peer `a` (re)joined the mesh
  X_LINK = 9,    // exchange → loop: a connected per-loop link to peer `a` (fd `b`; payload: bytes
                 //   already read from it) — the loop owns the socket from here on
  X_RELEASE = 10,  // exchange → owner loop: the round that was writing into shadow slot `a` is
                   //   over — the slot whose release forget_bulk() deferred may be released now
};
// X_FINAL / X_BULK / X_SENT flags (XF_HOSTCOPY: an X_BULK whose bytes a bulk round put in HBM
// and the bulk thread copied out — XOptions::host_copy)
// XF_LAST (X_DATA): the stream's last deltas — its tick carried the end of the response
enum : uint8_t { XF_TEXT = 1, XF_ABORTED = 2, XF_FAILED = 4, XF_HOSTCOPY = 8, XF_LAST = 16 };

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
  // tcp: bulk bytes ride the mesh; rccl: RCCL rounds (HBM → HBM); tcpbulk: the same rounds
  // over a socket per rank pair (CPU / one-GPU rehearsals of the round protocol)
  std::string transport = "tcp";
  std::string addr = "127.0.0.1";
  int port = 0;                   // mesh: rank r listens on port + r
  int bulk_port = 0;              // tcpbulk: rank r listens on bulk_port + r (0: port + world)
  int device = 0;
  int batch_us = 50;              // rank 0: announcements arriving within this window share a round
  double timeout_s = 30.0;        // bulk round / epoch formation slower than this = peer failure
  // rccl: the longest final text a round can carry (the engines' per-slot content capacity):
  // the executor's discard / zero buffers are allocated once at this size, never in a round
  size_t max_text = 1u << 20;
  // per-loop links: io loop l of every rank pair gets a TCP connection of its own (dialled by
  // the higher rank once the pair's mesh connection forms), so a session's opens, deltas and
  // eager finals go io loop → socket → io loop with no mesh thread on the data path
  bool links = true;
  // device executors: every received text is copied HBM → host by the bulk thread as soon as
  // its round completes (one batch on the executor's stream) and X_BULK carries the bytes, so
  // the owner's io loop never issues a copy of its own.  For RCCL at world > 1, where a peer
  // GPU wrote the bytes and a persistent grid cannot be relied on to see them in HBM
  // (HipEngine::set_remote_hbm_direct)
  bool host_copy = false;
};

// the mesh's view of one peer
struct PeerStats {
  bool up = false;
  uint64_t msgs_out = 0, msgs_in = 0, bytes_out = 0, bytes_in = 0, connects = 0;
};

class Exchange {
 public:
  using Deliver = std::function<void(int loop, std::vector<XMsg>&&)>;
  Exchange(const XOptions& o, int nloops, Deliver deliver);
  ~Exchange();
  void post(XMsg&& m);  // thread-safe: control / delta message to m.dst_rank over the mesh
  // Batched posting (an io loop's messages of one event-loop pass): frames are encoded by the
  // caller straight into a per-destination buffer (append_frame: one copy of each payload),
  // then handed over with one lock and one mesh-thread wake (post_frames clears `frames`).
  static void append_frame(std::string& out, const XMsg& hdr, const char* payload, size_t n);
  // the complete frames at the front of `buf` → `out` (a link's receive side); returns the
  // bytes consumed.  Mesh-internal frame types never travel on a link.
  static size_t parse_frames(const std::string& buf, std::vector<XMsg>& out);
  void post_frames(int dst_rank, std::string& frames);
  // Worker: ship stream (hdr.skey, hdr.bi)'s final text to hdr.dst_rank.  `dev` points at
  // `len` bytes in HBM that stay valid until X_SENT comes back to hdr.src_loop; `host`
  // produces the bytes for the mesh fallback.  hdr.flags / hdr.b travel with it.
  void send_bulk(XMsg&& hdr, const void* dev, size_t len, std::function<std::string()> host);
  // Owner: a bulk for (skey, bi) lands at `dev` (HBM, capacity `cap`); nullptr / a mesh
  // transfer delivers the bytes in X_BULK's payload instead.
  void expect_bulk(uint64_t skey, int bi, void* dev, size_t cap);
  // The owner is done with (skey, bi)'s sink.  Never blocks.  true: no round writes into it,
  // the slot may be reused now.  false: a round is writing into it right now — the slot must
  // not be reused yet; when that round is over the exchange delivers X_RELEASE (a = `slot`) to
  // io loop `loop` (slot < 0: nothing is delivered, and a later forget_bulk decides).  Either
  // way no new round pins the sink.
  bool forget_bulk(uint64_t skey, int bi, int slot = -1, int loop = -1);
  void request_stop();
  void join();
  bool healthy() const { return healthy_.load(); }  // the mesh formed once and is running
  bool peer_up(int r) const;
  int rank() const { return o_.rank; }
  const std::string& transport() const { return o_.transport; }
  int world() const { return o_.world; }
  // the bulk communicator (RCCL or tcpbulk) of the current epoch is formed
  bool rccl_active() const { return rccl_epoch_.load() > 0 && rccl_ok_.load(); }
  bool bulk_transport() const { return o_.transport == "rccl" || o_.transport == "tcpbulk"; }
  // counters (/metrics)
  uint64_t rounds() const { return rounds_.load(); }        // RCCL bulk rounds executed here
  uint64_t bytes() const { return bytes_.load(); }          // mesh payload bytes sent + received
  uint64_t bulk_bytes() const { return bulk_bytes_.load(); }  // final-text bytes moved by RCCL
  uint64_t mesh_bulk() const { return mesh_bulk_.load(); }  // finals moved over the mesh
  uint64_t msgs() const { return msgs_.load(); }            // mesh messages sent + received
  uint64_t epochs() const { return rccl_epoch_.load(); }    // RCCL communicators formed
  uint64_t rejoins() const { return rejoins_.load(); }      // peer (re)connections after the first
  uint64_t downs() const { return downs_.load(); }          // live peer connections lost
  double busy_us() const { return busy_us_.load(); }        // time inside RCCL rounds
  // texts a round carried whose sender finished the round but whose receiver missed them
  // (it failed the round on another peer): resent over the mesh on the receiver's report
  uint64_t rescued() const { return rescued_.load(); }
  // carried sends whose receiver never reported, resent over the mesh after timeout_s
  uint64_t sweeps() const { return sweeps_.load(); }
  // receiver reports that arrived before their send was carried (kept until it is)
  uint64_t early_reports() const { return early_reports_.load(); }
  uint64_t links() const { return links_.load(); }  // per-loop links handed to the io loops
  uint64_t host_copied() const { return host_copied_.load(); }  // received texts copied HBM → host (host_copy)
  uint64_t deferred_releases() const { return deferred_releases_.load(); }  // forget_bulk → X_RELEASE

  struct Impl;

 private:
  XOptions o_;
  int nloops_;
  Deliver deliver_;
  std::unique_ptr<Impl> im_;
  std::atomic<bool> stop_{false}, healthy_{false}, rccl_ok_{false};
  std::atomic<uint64_t> rounds_{0}, bytes_{0}, bulk_bytes_{0}, mesh_bulk_{0}, msgs_{0}, rccl_epoch_{0}, rejoins_{0},
      downs_{0}, rescued_{0}, links_{0}, sweeps_{0}, early_reports_{0}, host_copied_{0}, deferred_releases_{0};
  std::atomic<double> busy_us_{0};
  std::thread mesh_th_, bulk_th_;
  void mesh_loop();
  void bulk_loop();
  friend struct Impl;
};

// RCCL point-to-point self-test over the same round machinery (bindings / GPU tests):
// every rank sends `rounds` payloads to every other rank and checks what it receives.
std::string rccl_unique_id_hex();

}  // namespace qmx
