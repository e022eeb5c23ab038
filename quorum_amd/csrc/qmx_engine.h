// qmx_engine.h — host-side stream engine core (slot table, batching, CPU algorithms).
//
// HostEngine owns the per-rank slot table and the tick protocol used by both engines:
//   open/feed/finish/release/submit_finalize  (event-loop thread, under mu_)
//   tick()                                    (ticker: inline or worker thread)
// CpuEngine runs the sequential oracle algorithm per slot; HipEngine (qmx_hip.hip)
// runs the fused CDNA4 tick kernel over all slots of the batch at once.
//
// Reference counterpart: the per-backend processing loop of progress_streaming_aggregator
// (src/quorum/oai_proxy.py:554-747) and the final combine (:759-881).
#pragma once
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <memory>
#include <thread>
#include <mutex>
#include <string>
#include <unordered_map>
#include <stdexcept>
#include <unordered_set>
#include <vector>

#include "qmx_text.h"

namespace qmx {

enum ResultFlags : int { RF_DONE = 1, RF_ABORTED = 2, RF_ESCALATED = 4 };

TagSet make_tagset(const std::vector<std::string>& tags);

struct FilterState {
  int depth = 0;
  int tail_len = 0;
  uint8_t tail[kMaxTail] = {0};
};

// Sequential streaming think filter: appends released bytes to `out`.
void filter_feed(const TagSet& ts, FilterState& fs, const uint8_t* text, size_t n, std::string& out);

// Final strip: same-tag leftmost non-greedy removal + Unicode strip.
std::string strip_final(const TagSet& ts, const uint8_t* x, size_t n);

// SSE envelopes (json.dumps(ensure_ascii=True) of quorum's event dicts, oai_proxy.py:629-646, 847-860)
void escape_append(const uint8_t* y, size_t n, std::string& out);
size_t escaped_size(const uint8_t* y, size_t n);
std::string delta_prefix(int index, int64_t created);
std::string final_prefix(int64_t created);
extern const char* kDeltaSuffix;
extern const char* kFinalSuffix;

// Host-side per-stream state.
struct SlotCore {
  bool filter = true, emit = true, started = false, aborted = false, done = false;
  int index = 0;
  std::string carry;  // unframed upstream bytes
  FilterState fs;
  std::string content;  // accumulated filtered content (host engine / fallback)
  // shape template: bytes around the content string of the last fully parsed content event
  // (an event identical outside a valid string body has the same parse — see qmx_lex.h)
  std::string tpl_pre, tpl_suf;
};

// Process newly arrived bytes of one stream (sequential algorithm); appends SSE to out.
void process_slot(const TagSet& ts, SlotCore& s, const uint8_t* data, size_t n, bool eof,
                  int64_t created, std::string& out);

// One deferred slot operation: io loops batch their feed / finish / release calls of an
// event-loop iteration and hand them over under ONE engine lock (apply_ops).
struct EngineOp {
  enum Kind : int { FEED = 0, FINISH = 1, RELEASE = 2 };
  int kind;
  int slot;
  std::string data;
};

// A result's SSE bytes may be a view into a tick lane's output arena instead of a copy
// (HipEngine: the lane turns a tick's result records into results without touching the
// bytes; the io loop copies them once, into the client's output).  The arena is reused only
// when no result viewing it is left: ViewRef counts them.
struct ViewRef {
  std::atomic<int>* r = nullptr;
  ViewRef() = default;
  explicit ViewRef(std::atomic<int>* p) : r(p) {
    if (r) r->fetch_add(1, std::memory_order_relaxed);
  }
  ViewRef(const ViewRef& o) : ViewRef(o.r) {}
  ViewRef(ViewRef&& o) noexcept : r(o.r) { o.r = nullptr; }
  ViewRef& operator=(ViewRef o) noexcept {
    std::swap(r, o.r);
    return *this;
  }
  ~ViewRef() {
    if (r) r->fetch_sub(1, std::memory_order_release);
  }
};

struct SlotResult {
  int slot;
  std::string sse;  // the SSE bytes, unless `view` is set
  int flags;
  // open() generation of the slot this result belongs to: a slot released while its tick
  // is in flight can be re-opened by another session before the result is applied; the
  // consumer drops results whose generation is not the one it opened (stamped by tick()).
  uint32_t gen = 0;
  const char* view = nullptr;  // set: the SSE bytes are view[0, view_len) (held by `hold`)
  uint32_t view_len = 0;
  ViewRef hold;
  const char* data() const { return view ? view : sse.data(); }
  size_t size() const { return view ? view_len : sse.size(); }
  bool empty() const { return size() == 0; }
  void clear_sse() {
    sse.clear();
    view = nullptr;
    view_len = 0;
    hold = ViewRef();
  }
};
struct FinalizeReq {
  int id;
  std::vector<int> slots;
  bool strip;
  bool texts;  // return stripped texts instead of the final event
  std::string joiner;
  int64_t created;
};
struct FinalizeRes {
  int id;
  int kind;  // 0 none (all empty), 1 event bytes, 2 texts
  std::string event;
  std::vector<std::string> texts;
};

// Append-only slot table with stable element addresses AND a never-moving index: chunks
// of 256 elements hang off a fixed pointer table, so a tick lane can index slot i
// (operator[]) while an io loop appends under the engine lock (a std::deque's block map
// may be reallocated by push_back underneath a concurrent reader).
template <class T>
class SlotTable {
 public:
  static constexpr int kShift = 8, kChunk = 1 << kShift, kMaxChunks = 4096;  // 1M slots
  SlotTable() : chunks_(new std::unique_ptr<T[]>[kMaxChunks]) {}
  T& operator[](size_t i) { return chunks_[i >> kShift][i & (kChunk - 1)]; }
  const T& operator[](size_t i) const { return chunks_[i >> kShift][i & (kChunk - 1)]; }
  size_t size() const { return n_.load(std::memory_order_acquire); }
  void emplace_back() {  // caller serialises appends
    const size_t n = n_.load(std::memory_order_relaxed);
    if ((n >> kShift) >= (size_t)kMaxChunks) throw std::length_error("slot table full");
    if ((n & (kChunk - 1)) == 0) chunks_[n >> kShift].reset(new T[kChunk]());
    n_.store(n + 1, std::memory_order_release);
  }

 private:
  std::unique_ptr<std::unique_ptr<T[]>[]> chunks_;
  std::atomic<size_t> n_{0};
};

class HostEngine {
 public:
  explicit HostEngine(const std::vector<std::string>& tags);
  virtual ~HostEngine() = default;

  // returns the slot; *gen (optional) receives the slot's open generation (SlotResult::gen)
  int open(int index, bool filter, bool emit, uint32_t* gen = nullptr);
  // A caller that opens many slots (an io loop) takes k free slots under ONE lock, then
  // opens them one by one without the lock: a reserved slot is in no list a tick lane reads,
  // and its first feed / finish / release goes through the lock (apply_ops) as usual.
  void reserve(int k, std::vector<int>& out);
  void open_reserved(int slot, int index, bool filter, bool emit, uint32_t* gen = nullptr);
  void feed(int slot, const std::string& data);
  void finish(int slot);
  void release(int slot);
  // in order, one lock; move_data: FEED payloads may be moved out of ops (the caller is done with them)
  void apply_ops(std::vector<EngineOp>& ops, bool move_data = false);
  int submit_finalize(const std::vector<int>& slots, bool strip, bool texts, const std::string& joiner,
                      int64_t created);
  bool has_work();
  // the slot has bytes the engine has not turned into results yet (fed and not taken by a
  // tick, or in a tick still in flight): more output for its stream is on the way
  bool pending(int slot);
  // One tick over every dirty slot that is not in flight on another lane.  `lane` picks the
  // engine's per-thread launch resources (HipEngine: stream + arenas), so several tick
  // threads can have kernels in flight at once over disjoint slot sets.  With `taken`, the
  // slots stay busy (excluded from other lanes' ticks) until settle(*taken) — the caller
  // routes the results first, so a stream's outputs are delivered in order.  Returns false
  // when there was nothing to do.
  bool tick(int64_t created, std::vector<SlotResult>& results, std::vector<FinalizeRes>& fres, int lane = 0,
            std::vector<int>* taken = nullptr);
  void settle(const std::vector<int>& taken);

  struct Work {
    int slot;
    std::string data;
    bool eof;
    bool fresh;
  };
  // Pipelined ticks (GpuHub lanes, engines with pipelined()): a job takes the lane's work
  // (job_take: the dirty streams no other tick holds, optionally the queued finalize
  // requests), is prepared while the lane's previous job still runs on the device, posted
  // the moment that one completes, and completed (results) while the next one runs.
  // job_finish stamps the results' generations and lists the taken slots for settle().
  struct Job {
    std::vector<Work> work;
    std::vector<FinalizeReq> fin;
    int64_t created = 0;
    int lane = 0;
    bool live = false;
    std::shared_ptr<void> impl;  // the engine's state between the phases
  };
  virtual bool pipelined() const { return false; }
  // QMX_PIPELINE=1: pipelined lanes.  Off by default: on MI355X they raise the tick rate
  // ~40% but not the closed-loop req/s (latency-bound), and cost ~3 us of proxy CPU per request
  bool pipeline_ = false;
  bool job_take(Job& j, bool allow_fin);
  virtual void job_prepare(Job&) {}
  virtual void job_post(Job&) {}
  virtual void job_wait_near(Job&) {}
  virtual void job_complete(Job&, std::vector<SlotResult>&, std::vector<FinalizeRes>&) {}
  void job_finish(Job& j, std::vector<SlotResult>& results, std::vector<int>& taken);
  // Loop ticks (an io loop drives its own jobs, at most free_doors() posted at once): has a
  // posted job completed?  Never blocks; expect_us: its expected remaining time.  Engines
  // that run jobs synchronously (in job_complete) are always ready.
  virtual bool async_jobs() const { return false; }
  virtual bool job_ready(Job&, double* expect_us = nullptr) {
    if (expect_us) *expect_us = 0;
    return true;
  }
  virtual int free_doors() const { return 1; }
  virtual std::string text(int slot);
  virtual std::unordered_map<std::string, double> stats();
  // Spread placement (qmx_exchange.h): a stream whose final text another rank produced.
  // content_device_ptr: the slot's HBM content area (nullptr: host engine / host path);
  // content_size: filtered content bytes so far; set_remote_content: the slot's content
  // becomes `len` bytes — *bytes if given, else already written into the HBM area;
  // host_copied: *bytes are a host copy of what a bulk round wrote into that area (counters).
  virtual void* content_device_ptr(int /*slot*/, size_t* cap) {
    *cap = 0;
    return nullptr;
  }
  virtual size_t content_size(int slot);
  virtual void set_remote_content(int slot, const std::string* bytes, size_t len, bool host_copied = false);

  const TagSet& tagset() const { return ts_; }

 protected:
  // engine-specific batch processing: the tick's stream work AND its finalize requests
  // (HipEngine: one fused launch for both; CpuEngine: sequentially)
  virtual void run_tick(std::vector<Work>& work, std::vector<FinalizeReq>& fin, int64_t created,
                        std::vector<SlotResult>& results, std::vector<FinalizeRes>& fres, int lane) = 0;
  virtual void on_free(int /*slot*/) {}

  void feed_locked(int slot, const std::string& data);
  void feed_locked_move(int slot, std::string& data);
  void finish_locked(int slot);
  void release_locked(int slot);

  struct Meta {
    bool live = false;
    bool dirty = false;
    bool eof = false;
    bool fresh = true;
    bool closed = false;  // DONE/ABORTED reported
    bool busy = false;    // taken by an unsettled tick (in flight on some lane)
    uint32_t gen = 0;     // bumped by every open()
    double t_dirty = 0;   // steady clock (s) when it last became dirty: take-wait timing
    std::string incoming;
  };

  TagSet ts_;
  std::mutex mu_;
  // open() appends under mu_ while tick lanes index other slots outside the lock
  SlotTable<Meta> meta_;
  SlotTable<SlotCore> core_;  // host state (CPU engine; HIP engine: flags + fallback)
  size_t nslots() const { return core_.size(); }
  std::vector<int> free_, pending_free_;
  std::vector<int> dirty_;
  std::vector<FinalizeReq> fin_;
  int next_fid_ = 0;
  uint64_t ticks_ = 0, bytes_in_ = 0, bytes_out_ = 0, takes_ = 0;
  double take_wait_s_ = 0;  // dirty -> taken by a tick, summed over takes
};

class CpuEngine : public HostEngine {
 public:
  explicit CpuEngine(const std::vector<std::string>& tags) : HostEngine(tags) {}
  // pipelined lanes on the CPU: the whole tick runs in job_complete (exercises GpuHub's
  // pipelined loop without a GPU)
  bool pipelined() const override { return pipeline_; }
  void job_complete(Job& j, std::vector<SlotResult>& results, std::vector<FinalizeRes>& fres) override {
    run_tick(j.work, j.fin, j.created, results, fres, j.lane);
  }

 protected:
  void run_tick(std::vector<Work>& work, std::vector<FinalizeReq>& fin, int64_t created,
                std::vector<SlotResult>& results, std::vector<FinalizeRes>& fres, int lane) override;
};

// The loop-tick protocol on the CPU (tick_mode "loops" with the cpu engine): a posted job
// runs on the engine's worker thread while the io loop keeps serving, which polls
// job_ready() exactly as with HipEngine's grid doors.  Exercises the io loops' asynchronous
// tick path (two jobs in flight, completion in any order, finalize on one of them) in the
// CPU and TSan suites, where no GPU is.
class AsyncCpuEngine : public CpuEngine {
 public:
  explicit AsyncCpuEngine(const std::vector<std::string>& tags);
  ~AsyncCpuEngine() override;
  bool async_jobs() const override { return true; }
  void job_post(Job& j) override;
  bool job_ready(Job& j, double* expect_us = nullptr) override;
  void job_complete(Job& j, std::vector<SlotResult>& results, std::vector<FinalizeRes>& fres) override;
  int free_doors() const override { return 2 - inflight_.load(std::memory_order_acquire); }

 private:
  struct Done;
  void run();
  std::mutex qmu_;
  std::condition_variable qcv_;
  std::vector<Job*> q_;
  bool stop_ = false;
  std::atomic<int> inflight_{0};
  std::thread th_;
};

// Shared by both engines' host-side finalisation.
void finalize_texts(const TagSet& ts, const std::vector<std::string>& texts, const FinalizeReq& r,
                    FinalizeRes& out);

}  // namespace qmx
