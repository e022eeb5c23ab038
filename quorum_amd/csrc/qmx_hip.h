// qmx_hip.h — HipEngine: the CDNA4 (gfx950) batched stream engine.
//
// One fused kernel launch per tick processes every slot with pending upstream bytes:
//   LDS-staged input tile → parallel SSE framing scan → per-event validating JSON delta
//   extraction → MFMA int8 think-tag matcher (mfma_i32_16x16x64_i8) → (a,b)-monoid depth
//   scan → holdback cuts per delta → compaction → device-resident content append →
//   ensure_ascii SSE encoding staged in LDS → coalesced 16-B stores to host-mapped output.
// Per-slot filter state and filtered content stay resident in HBM; input/output arenas
// are pinned host memory mapped into the GPU (zero-copy: no hipMemcpy per tick).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstddef>
#include <functional>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <vector>

#include "qmx_engine.h"
#include "qmx_streams.h"

namespace qmx {

struct WorkItem {
  uint32_t slot, in_off, in_len, out_off, out_cap, flags, index, content_len;
};
struct WorkResult {
  uint32_t consumed, out_len, status, content_len;
  uint32_t seq;  // written last (system-scope release): the lane's tick sequence number
  uint32_t pad;
  uint64_t t0, t1;  // s_memrealtime (100 MHz) at workgroup start / end: kernel span per tick
};
constexpr int kTplBytes = 320;  // per-stream event shape template (qmx_lex.h TPL_*)
struct DevSlot {
  alignas(16) uint8_t tpl[kTplBytes];  // prefix at [0, 256), suffix at [256, 320)
  int32_t depth;
  int32_t tail_len;
  uint16_t tpl_pre, tpl_suf;           // 0: no template yet
  uint8_t tail[kMaxTail];
};

// Per-event "hole" template (cross-stream, any event shape): a fully parsed event's bytes
// with its string-value bodies and numbers as holes.  An event that equals the literal
// runs between the holes and has a valid JSON string body / number in each hole lexes to
// the same token sequence, so it has the same parse: its kind (content / skip) and, for
// content, the target hole's bytes.  Covers what a prefix/suffix template cannot: a new
// stream's role, first-content and finish events, whose ids and timestamps differ per
// stream (qmx_lex.h wave_hole_match).
constexpr int kHoleMax = 16, kHoleTplBytes = 448, kHoleTpls = 4;
struct HoleTpl {
  alignas(16) uint8_t bytes[kHoleTplBytes];  // the source event (x[e0, e1))
  uint16_t len;                               // 0: none
  uint8_t nh, kind, target, tgt_bs;           // holes; EV_CONTENT / EV_SKIP; content hole; it has a '\\'
  uint16_t hs[kHoleMax], he[kHoleMax];        // hole i = bytes[hs[i], he[i])
  uint8_t num[kHoleMax];                      // 1: hole i is a number, 0: a string body
  uint8_t pad0[10];
  // the tick kernel's S3a test per 8-byte word of the first 256 bytes, bit per byte:
  // string-hole bytes (bits 0-7), number-hole bytes (8-15), first bytes of multi-digit
  // number holes (16-23) — built with the template (wave_hole_publish), copied with it
  uint32_t wmask[32];
  uint32_t claim;  // launch sequence number of the last writer (its own 16 B: a copy skips it)
  uint32_t pad1[3];
};

static_assert(offsetof(HoleTpl, claim) == sizeof(HoleTpl) - 16, "claim in the last 16 bytes");

// Per-backend event shape templates (cross-stream): written by the first workgroup of a
// launch that parses an event of that backend index, read by the lane's next launch
constexpr int kBackendTpl = 16;  // backend indices with a table entry
struct BackendTpl {
  alignas(16) uint8_t tpl[kTplBytes];
  uint16_t pre, suf;  // 0: none yet
  uint32_t claim;     // launch sequence number of the last writer
  uint32_t pad[2];
  HoleTpl hole[kHoleTpls];  // by shape class (hole count, kind): role / content / finish events
};

// WF_PUBLISH: the tick's first item of its backend index — the one workgroup that writes that
// backend's event-shape / hole templates for the lane's next launch
enum WorkFlags : uint32_t { WF_EOF = 1, WF_FILTER = 2, WF_EMIT = 4, WF_STARTED = 8, WF_FRESH = 16, WF_PUBLISH = 32 };
enum WorkStatus : uint32_t { WS_DONE = 1, WS_ABORTED = 2, WS_STARTED = 4, WS_ESCALATE = 8, WS_MORE = 16 };

struct KParams {
  TagSet ts;
  int npat;
  int32_t pat_E[2 * kMaxTags];  // Σ_j m(q0²+q1²) over the window part of each pattern (match iff dot == -E)
  int32_t plen[2 * kMaxTags];   // pattern_len(ts, t), 0 past npat (a load with no dependence on ts.n)
  // byte → matcher code: 1..94 for the bytes that occur in patterns (letters folded), 95 for
  // every other byte (never equal to a pattern byte), 0 past the end of the text
  alignas(16) uint8_t code[256];
  // MFMA B operand (patterns × window features) per lane, built once on the host, one
  // 16-pattern column block per MFMA: lane l = pattern 16·blk + (l & 15), feature group
  // (l >> 4): 0: -2·q0, 1: -2·q1, 2/3: mask (q = code, q0 = q & 7, q1 = q >> 3)
  alignas(16) int8_t bfrag[2][64 * 16];
  // each pattern's bytes as little-endian words (zero past its end): the holdback's prefix
  // test compares 8 bytes at a time (pattern_prefix_w) instead of byte by byte
  uint64_t pw[2 * kMaxTags][kMaxTail / 8];
  uint32_t content_cap;
  // single-wave fast paths of the common small tile (QMX_KFAST bit mask, default all):
  // 1 S2 framing, 2 S3a template prepass, 4 S4 filter, 8 S6 sizing, 16 S4's VALU matcher
  // for <= 4 candidates (else the MFMA matcher)
  uint32_t fast;
  int pre1_len, pre2_len, suf_len;
  char pre1[48];
  char pre2[176];
  char suf[48];
  unsigned long long* dbg;  // optional per-stage stamps [item][16] (QMX_STAGE_TIMING=1)
};

// Finalize (K3 strip + K4 join + K5 encode) work: one workgroup of the fused tick launch
// per session request.
struct FinItem {
  uint32_t first_text, n_texts;     // into the FinText array
  uint32_t flags;                   // 1 strip, 2 texts-kind (no join / encode)
  uint32_t join_off;                // device join buffer offset (16-B aligned)
  uint32_t out_off, out_cap;        // device + host output offset (16-B aligned), capacity
  uint32_t joiner_off, joiner_len;  // in the finalize input arena
  uint32_t pre_off, pre_len, suf_off, suf_len;
  uint32_t seg_off, seg_cap;        // kept-segment scratch (device), entries
  uint32_t tl_off;                  // texts-kind: per-text stripped lengths at text_len[tl_off..]
};
// in_off != kNoStage: the text arrived on the host (a spread worker's final over the mesh);
// its bytes are staged at fin_in[in_off] (host-mapped) and the item first copies them into
// the slot's HBM content area, then reads them from there like any other text
constexpr uint32_t kNoStage = 0xFFFFFFFFu;
struct FinText {
  uint32_t slot, len, in_off, pad;
};
struct FinResult {
  uint32_t out_len, status, n_kept;  // status 1: escalate to the host path
  uint32_t seq;                      // written last (system-scope release), as WorkResult::seq
  uint64_t t0, t1;                   // s_memrealtime at workgroup start / end
};

struct PDoor;  // persistent mode: host-mapped doorbell (qmx_hip.hip)
struct PCtl;   // persistent mode: device control block

// One persistent grid serving several doorbells ("loop ticks"): every io loop owns an engine
// (its own slots, arenas and templates) and posts its own ticks into door `d` of this grid —
// no tick-lane thread between an io loop and the GPU, no hand-off of results back.  The
// grid is `doors` sub-grids of `wg_per_door` workgroups; each sub-grid's first workgroup
// polls its door and relays the tick to its workers, exactly as a lane's grid does.
//
// Lifetime: a door's owner posts under post_guard() (a shared lock that launches the grid
// when it is not running).  housekeep(), from any io loop's periodic sweep, keeps the grid
// alive with a heartbeat every door sees, and stops it (stop ticks on every door, under the
// exclusive lock) once no door has posted for idle_ms.  The kernel's own exit — every relay
// idle, heartbeat included, for 2 s — only fires when the host stopped beating (a hung
// process), so every wave reaches an exit even if the host never stops the grid.
class HipGrid {
 public:
  HipGrid(int device, int doors, int wg_per_door, int idle_ms);
  ~HipGrid();
  int doors() const { return n_; }
  PDoor* door(int d) const;
  // held by a door's owner while it writes and posts a tick
  std::shared_lock<std::shared_mutex> post_guard();
  void note_post();
  void housekeep();
  // a tick that never completed: relaunch a grid that left on its own (its exit word names
  // the current generation); true when it did
  bool revive_if_exited();
  void stop();
  std::unordered_map<std::string, double> stats();
  // host steady clock (us) minus the device's s_memrealtime clock (us), from the quickest of
  // a few doorbell round trips; NaN before the first calibration
  double clock_offset_us() const { return clk_off_us_.load(std::memory_order_relaxed); }

 private:
  void launch_locked();
  void stop_locked();
  void calibrate_locked();
  std::atomic<double> clk_off_us_{__builtin_nan("")};
  bool interleave_ = true;  // doors' sub-grids XCD-local (blocks d, d + doors, ...)
  int occ_ = 1;             // workgroups per CU the kernel variant allows (QMX_GRID_OCC)
  // written by calibrate_locked (exclusive lock); read lock-free by housekeep() / stats()
  std::atomic<double> clk_rtt_us_{0.0}, last_cal_{0.0};
  int device_, n_, wpd_, idle_ms_;
  std::shared_mutex mu_;
  std::atomic<bool> running_{false};
  uint32_t gen_ = 0;
  std::atomic<double> last_post_{0.0};
  std::atomic<uint32_t> beat_{0};
  hipStream_t stream_ = nullptr;
  PDoor* h_doors_ = nullptr;  // host-mapped, n_ of them
  PCtl* d_ctls_ = nullptr;    // device, n_ of them
  std::atomic<uint64_t> launches_{0}, stops_{0}, revivals_{0};
  double launch_us_max_ = 0, launch_cal_us_max_ = 0, launch_us_sum_ = 0, stop_us_max_ = 0;  // under mu_ (exclusive)
};

// Launch resources of one tick lane: a tick thread owns a lane (HIP stream, events,
// host-mapped in/out arenas, work/result descriptors, counters), so several lanes can have
// tick kernels in flight at once over disjoint slot sets (HostEngine busy flags).
struct TickLane {
  std::mutex mu;  // held by the lane's tick for its whole process(); kernel_stats() reads under it
  hipStream_t stream = nullptr;  // none for a door of the shared grid (loop ticks)
  StreamKind skind = StreamKind::Shared;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, evb = nullptr;
  KParams params;
  uint64_t params_ver = 1;  // bumped whenever `params` changes (each Buf uploads its own copy)
  // [door sets][2][kBackendTpl]: per door set (loop ticks: a door of the engine's own; lanes:
  // one) a launch-parity double buffer — a tick reads its door set's last tick's half
  BackendTpl* d_btpl = nullptr;
  uint32_t tpl_launches[2] = {0, 0};  // completed ticks per door set (the parity)
  int64_t params_created = -1;
  // two buffer sets (tiles, work items, result records, stage stamps, kernel parameters), one
  // per tick in flight or in preparation (GpuHub's pipelined lanes; two doors of a loop)
  struct Buf {
    uint8_t* h_in = nullptr;
    size_t in_cap = 0;
    WorkItem* h_items = nullptr;
    WorkResult* h_res = nullptr;
    size_t items_cap = 0;
    unsigned long long* h_dbg = nullptr;
    size_t dbg_cap = 0;
    KParams* h_params = nullptr;  // pinned staging of this buffer's parameter upload
    KParams* d_params = nullptr;  // device copy read by this buffer's ticks
    uint64_t params_ver = 0;      // the TickLane::params version in d_params
    bool busy = false;            // a prepared tick holds it until complete()
  };
  Buf bufs[2];
  // output arenas (pinned, mapped): results view their SSE bytes in place (SlotResult::view),
  // so a tick writes into an arena no earlier result still views — a ring that grows while
  // every arena is held (OutArena objects are never freed: a late ViewRef may still count)
  struct OutArena {
    uint8_t* p = nullptr;
    size_t cap = 0;
    std::atomic<int> refs{0};
  };
  std::vector<OutArena*> outs;
  size_t out_i = 0;
  OutArena* out = nullptr;  // this tick's
  uint8_t* h_out = nullptr;  // == out->p
  size_t out_cap = 0;
  // counters (summed over lanes by kernel_stats)
  uint64_t launches = 0, items = 0, h2d_bytes = 0, d2h_bytes = 0;
  uint64_t s3_full = 0, s3_tpl = 0, s3_events = 0, stage_n = 0;  // QMX_STAGE_TIMING: S3 path counters
  uint64_t s3_cyc_full = 0, s3_cyc_tpl = 0, s3_cyc_lex = 0, s3_hole = 0, s3_cyc_hole = 0;  // S3 wave cycles: full parse / templates / lexer
  uint64_t s3a_unres = 0;  // stage timing: events S3a left to its loop
  double kernel_ms = 0.0, host_prep_us = 0, gpu_wait_us = 0, process_us = 0;  // host-side tick breakdown
  double first_result_us = 0;  // tick posted -> first result record seen by the host
  double item_us = 0, start_spread_us = 0;
  double items_host_us = 0;
  double relay_us = 0, pickup_us = 0, grid_span_us = 0, grid_ticks = 0;  // persistent: doorbell seen -> ...  // host: result records -> slot state + SSE strings (process_item)  // per tick: mean item run, last item start - first
  double stage_us[38] = {0};  // [20]: an item's system-scope release fence (stage timing)
  double clk_cycles = 0, clk_us = 0;
  // finalize arenas (fused into this lane's tick launches)
  FinItem* h_fin = nullptr;
  size_t fin_cap = 0;
  FinResult* h_finres = nullptr;
  size_t finres_cap = 0;
  FinText* h_fint = nullptr;
  size_t fint_cap = 0;
  uint8_t* h_fin_in = nullptr;
  size_t fin_in_cap = 0;
  uint8_t* h_fout = nullptr;
  size_t fout_cap = 0;
  uint32_t* h_tl = nullptr;
  size_t tl_cap = 0;
  uint8_t* d_join = nullptr;
  size_t join_cap = 0;
  uint8_t* d_fout = nullptr;
  size_t dfout_cap = 0;
  uint8_t* d_segs = nullptr;  // int2 entries
  size_t segs_cap = 0;        // bytes
  uint64_t fin_launches = 0, fin_items = 0, fin_host = 0;  // launches that carried finalize work
  uint64_t fin_staged = 0;  // mesh-delivered remote texts staged into finalize items
  // completion by polling the kernel-published sequence numbers (HipEngine::wait_results)
  uint32_t seq = 0;
  double ema_us = 40.0;  // launch-to-results time, smoothed
  double span_ema_us = 30.0;  // kernel span per tick (device clock), smoothed: pipelined lanes
  double lead_ema_us = 8.0;   // persistent: doorbell seen -> first item started (device clock), smoothed
  double post_seen_us = 0, done_host_us = 0, hop_ticks = 0;  // loop ticks: host <-> device hops (calibrated)
  // loop ticks: clock-offset bounds (host us − device us) from the ticks themselves, per 100 ms window
  double clo = -1e300, chi = 1e300, clo_prev = -1e300, cwin_t0 = 0, cwin_sum = 0, cwin_n = 0;
  bool timing_pending = false;
  uint64_t poll_fallbacks = 0;
  // persistent mode (QMX_PERSISTENT=1): the lane's long-lived grid and its doorbell
  PDoor* h_door = nullptr;
  PCtl* d_ctl = nullptr;
  bool p_running = false;
  uint32_t p_gen = 0;
  double p_last_post = 0;  // steady clock, seconds
  uint64_t p_revivals = 0;  // grids relaunched for a tick posted after they idled out
  uint64_t p_launches = 0, p_ticks = 0;
};

class HipEngine : public HostEngine {
 public:
  // grid: loop-tick mode — one lane whose ticks go to door `door` of a shared multi-door grid
  HipEngine(const std::vector<std::string>& tags, int device, int tile_bytes, int max_slots, int content_cap,
            int lanes = 1, HipGrid* grid = nullptr, int door = -1, int ndoors = 1);
  ~HipEngine() override;
  // loop-tick mode (the io loop drives its own ticks): has the posted job's every result been
  // published?  Never blocks.  expect_us: the job's expected remaining time (poll timing).
  bool job_ready(Job& j, double* expect_us = nullptr) override;
  bool async_jobs() const override { return grid_ != nullptr; }
  // loop-tick mode: doors of this engine with no tick on them (a job may be prepared + posted)
  int free_doors() const override;
  std::string text(int slot) override;
  void* content_device_ptr(int slot, size_t* cap) override;
  size_t content_size(int slot) override;
  void set_remote_content(int slot, const std::string* bytes, size_t len, bool host_copied = false) override;
  // An RCCL round's final text in this slot's HBM content area: read there by the next
  // finalize item (direct), or first copied to the host and staged like a mesh-delivered
  // text.  A peer GPU's writes into coarse-grained HBM are coherent with this device's L2
  // only at dispatch boundaries, which a persistent grid does not cross: the server keeps the
  // host copy at world > 1 unless QMX_REMOTE_HBM=1 (world 1: RCCL's own kernel on this
  // device wrote the bytes through this L2, direct is exact).
  void set_remote_hbm_direct(bool on) { remote_hbm_direct_ = on; }
  bool remote_hbm_direct() const { return remote_hbm_direct_; }
  std::unordered_map<std::string, double> kernel_stats();
  int lanes() const { return (int)lanes_.size(); }
  // Latency mode for one stream, at its open (loop-tick mode: the io loop's own engine): the
  // slot runs on the host path — the C++ engine inline in the loop's tick, byte-identical —
  // instead of the GPU.  For light load, where a GPU tick's fixed ~23 us (doorbell, relay,
  // one workgroup's 16 us kernel, publish) is most of a stream's TTFT (profiles/r6/lowload).
  void host_open(int slot);

 protected:
  void run_tick(std::vector<Work>& work, std::vector<FinalizeReq>& fin, int64_t created,
                std::vector<SlotResult>& results, std::vector<FinalizeRes>& fres, int lane) override;
  void on_free(int slot) override;

 public:
  // pipelined lanes (polled completion): the next tick is prepared while this one runs
  bool pipelined() const override { return poll_ && pipeline_; }
  void job_prepare(Job& j) override;
  void job_post(Job& j) override;
  void job_wait_near(Job& j) override;
  void job_complete(Job& j, std::vector<SlotResult>& results, std::vector<FinalizeRes>& fres) override;

 private:
  struct HipJob;
  HipJob& hjob(Job& j);
  void prepare(HipJob& J);
  void post(HipJob& J);
  void wait_near(HipJob& J);
  void complete(HipJob& J, std::vector<SlotResult>& results, std::vector<FinalizeRes>& fres);
  void escalate(int slot, bool fresh);
  void finalize_host(const FinalizeReq& r, std::vector<FinalizeRes>& out);
  // finalize items of this tick → the lane's arenas; returns the GPU ones (others: host path)
  std::vector<const FinalizeReq*> prep_finalize(TickLane& L, std::vector<FinalizeReq>& fin,
                                                std::vector<const FinalizeReq*>& host);
  void collect_finalize(TickLane& L, const std::vector<const FinalizeReq*>& gpu, std::vector<FinalizeRes>& out);
  void wait_stream(TickLane& L);
  // polls the tick's result records; on_item(i) as stream result i is seen published (in order)
  void wait_results(TickLane& L, int n, int m, uint32_t seq, const WorkResult* res,
                    std::chrono::steady_clock::time_point t0, const std::function<void(int)>& on_item);
  void collect_timing(TickLane& L);
  void ensure_in(TickLane::Buf& B, size_t bytes);
  void ensure_out(TickLane& L, size_t bytes);
  void build_params(TickLane& L, int64_t created);
  std::string device_content(int slot, uint32_t len);
  uint32_t next_seq(TickLane& L);
  void ensure_persistent(TickLane& L);
  void stop_persistent(TickLane& L);
  // arenas replaced by a larger one: freed at destruction (a free may wait for the device,
  // which a persistent grid would hold up)
  void retire_host(void* p);
  void retire_dev(void* p);
  void note_alloc(double t0, size_t bytes);
  std::atomic<uint64_t> allocs_{0}, alloc_bytes_{0};
  std::atomic<double> alloc_us_{0.0}, alloc_max_us_{0.0};

 public:
  void* halloc(size_t bytes);  // pinned + mapped host memory (timed: kernel_stats runtime_alloc_*)
  void* dalloc(size_t bytes);  // device memory (timed)

 private:
  std::vector<void*> grave_host_, grave_dev_;
  std::mutex grave_mu_;

  int device_;
  int tile_;
  int max_slots_;
  uint32_t content_cap_;
  KParams base_params_;  // tag patterns (each lane's copy also gets the tick's envelopes)
  std::vector<std::unique_ptr<TickLane>> lanes_;
  // device-resident
  DevSlot* d_state_ = nullptr;
  uint8_t* d_content_ = nullptr;
  // host mirrors (per slot; a slot is only touched by the lane it is busy on)
  std::vector<uint8_t> host_mode_;       // slot escalated to the host path
  // spread owner: a remote stream's final text that came over the mesh, held in the slot's
  // SlotCore::content and staged into the finalize item that reads it (fin_body copies it to
  // HBM) — no synchronous copy in the io loop, no host finalize
  std::vector<uint8_t> remote_host_;
  std::vector<uint32_t> content_len_;    // device content bytes per slot
  // stats
  std::atomic<uint64_t> escalations_{0}, fin_host_{0}, remote_dev_{0}, remote_staged_{0}, remote_copied_{0},
      remote_copied_inline_{0}, light_opens_{0};
  bool remote_hbm_direct_ = true;
  int spin_us_ = 0;  // QMX_WAIT_SPIN_US: yield-poll before the blocking wait
  bool poll_ = true;  // QMX_WAIT=event: wait on a blocking-sync HIP event instead of polling
  int poll_us_ = 1;   // QMX_POLL_US: poll period once the expected kernel time has passed (MI355X A/Bs: 2 beats 6, 1 beats 2)
  bool persistent_ = true;   // a long-lived grid per lane, ticks posted by doorbell (QMX_PERSISTENT=0: a launch per tick)
  bool views_ = true;         // QMX_VIEWS=0: results copy their SSE bytes on the lane thread
  bool keep_stale_records_ = false;  // QMX_DEBUG_STALE_RECORDS: no record clearing before a post (test control)
  bool stage_timing_ = false;  // QMX_STAGE_TIMING: per-item stage stamps (tools/kbench.py)
  int p_grid_ = 64;          // QMX_PERSISTENT_WG: workgroups per lane grid (1 per CU: 256 VGPRs)
  int p_idle_ms_ = 50;       // the grid exits after this long without a tick
  HipGrid* grid_ = nullptr;  // loop-tick mode: the shared grid and this engine's doors
  int door_ = -1;            // the first of them
  int ndoors_ = 1;           // doors [door_, door_ + ndoors_): ticks in flight at once (<= 2)
  std::vector<char> door_busy_;

 public:
  bool persistent() const { return persistent_; }
  void set_persistent(bool on);
  // Test hook: fill every result record of every buffer set (and the finalize records) as
  // pinned pages recycled from an earlier engine would be — records that claim the sequence
  // number of the `ahead`-th next post with done/empty results.  An engine that trusted its
  // records' initial contents would complete that tick at once with wrong results
  // (tests/test_gpu_engine.py::test_hip_stale_result_records).  Call with no tick in flight.
  void debug_poison_results(int ahead);
};

}  // namespace qmx
