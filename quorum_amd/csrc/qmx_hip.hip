// qmx_hip.hip — CDNA4 (gfx950) fused tick kernel + HipEngine host runtime.
//
// One workgroup (256 threads = 4 wave64) per stream slot with pending bytes; everything
// between the input tile load and the output store happens in LDS:
//
//   S0 load      host-mapped input tile → LDS (16-B vector loads, zero-copy)
//   S1 start     leading Unicode-whitespace strip at stream start (quorum's body.strip())
//   S2 framing   "\n\n" separators with Python split() pairing: newline-run lengths via a
//                block scan over the map monoid x ↦ (all-newline ? x+len : trailing)
//   S3 extract   one thread per event: strict UTF-8 + validating JSON scan with quorum's
//                exception semantics (qmx_text.h classify_event); ordered compaction of
//                content deltas; JSON unescape into Z = tail ++ deltas
//   S4 filter    '<' candidates → MFMA int8 matcher (v_mfma_i32_16x16x64_i8: 16 candidate
//                windows × 16 patterns per instruction, exact via digit-split squared
//                distance) → token list → depth scan over the (a,b) monoid
//                f(x)=max(x+a,b) → per-delta holdback cuts → kept-byte compaction
//   S5 content   filtered bytes appended to the slot's HBM-resident content arena
//   S6 encode    json.dumps(ensure_ascii) SSE events staged in an LDS window, stored with
//                coalesced 16-B stores to host-mapped output
//
// Semantics: SURVEY §2.7 (reference src/quorum/oai_proxy.py:262-371, 578-673).
#include "qmx_env.h"
#include "qmx_hip.h"
#include "qmx_streams.h"

#include <rocprofiler-sdk-roctx/roctx.h>

#include <sched.h>
#include <sys/prctl.h>
#include <time.h>

#include <chrono>
#include <thread>

#include "qmx_lex.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

namespace qmx {

#define HIP_CHECK(x)                                                                       \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess)                                                                  \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e_) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__));                 \
  } while (0)

constexpr int BS = 512;  // 8 waves: S3 spreads events over 8 waves; 2 waves per SIMD hide LDS latency (16 waves measured slower: S3 13.3 -> 15.6 us)
constexpr int TILE_MAX = 16384;
constexpr int MAX_EV = 512;  // events per tile (more → WS_MORE requeue); keeps LDS < 80 KiB (two fit a CU's 160 KB: the QMX_GRID_OCC=2 variant)
constexpr int MAX_CAND = 1024;
constexpr int PAD = 16;
constexpr int kSpecTile = BS * 16;  // tile bytes loaded before the work item is known (16 B per thread: a whole headline stream, ~4.9 KB, in the same PCIe round trip as the item)
constexpr int TOK_CAP = 512;
// QMX_STAGE_TIMING record per work item: stamps 0-12, S3 counters 13-20, sub-stage stamps
// 21 (S3a done), 22 (S3 loop done), 23 (s4_wave: matched), 24 (s4_wave: cuts), 25 (s4_wave:
// token list + depth scan done), 26 (S6 write: output window filled, host stores next),
// 27 (the item's system-scope release fence done: its cost is 27 minus the result's t1)
constexpr int kDbg = 40;

typedef int v4i __attribute__((ext_vector_type(4)));

// optional per-stage wall-clock stamps (s_memrealtime, 100 MHz) written by thread 0
// (reads the LDS copy P of the kernel parameters: a persistent grid's parameters are not
// launch-invariant, so reading them from memory at every use would cost vector registers)
// Stamps are stored through the global address space: a flat store also counts against
// lgkmcnt, so the stage's next LDS wait would wait for the host-memory write too and the
// stamp would bill its own PCIe store to the stage after it.
__device__ __forceinline__ void dbg_put(unsigned long long* p, unsigned long long v) {
  *(__attribute__((address_space(1))) unsigned long long*)p = v;
}
// s_waitcnt vmcnt(0) (expcnt and lgkmcnt left alone): this wave's vector memory accesses,
// stores included, have completed; a compiler barrier too, so no store is moved past it
// bit i of m (i < 8) -> byte i of the result 0xff
// (shifts and masks per 32-bit half, no 64-bit multiply: v_mul_lo_u32 is quarter rate)
__device__ __forceinline__ uint32_t byte_mask4(uint32_t n) {  // bits 0-3 -> bytes 0-3
  const uint32_t t = (n | (n << 7) | (n << 14) | (n << 21)) & 0x01010101u;
  return (t << 8) - t;  // each byte 0 or 1 -> 0x00 or 0xff (mod 2^32)
}
__device__ __forceinline__ uint64_t byte_mask8(uint32_t m) {
  return ((uint64_t)byte_mask4((m >> 4) & 0xfu) << 32) | byte_mask4(m & 0xfu);
}
__device__ __forceinline__ void wave_stores_done() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// Publish a sequence number: the release fence (buffer_wbl2: this XCD's L2 written back to
// memory), a HARD wait for that write-back, then the store.  The memory legalizer follows
// buffer_wbl2 with a wait of its own, but the waitcnt pass may drop it when it believes no
// vector memory access is outstanding (it does not count the write-back): with a flag load
// waited just before, the persistent kernel's item publish was emitted as wbl2 + store with
// no wait between, and the host read the previous tick's output bytes behind a new sequence
// number (1-7 mislabelled deltas per 2.6M responses).  tests/test_isa.py checks the built
// code object for any write-back not waited before the next store.
__device__ __forceinline__ void publish_system(uint32_t* p, uint32_t v) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void publish_agent(uint32_t* p, uint32_t v) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
#define QMX_STAMP(k)                                               \
  do {                                                             \
    if (P.dbg != nullptr && threadIdx.x == 0)                      \
      dbg_put(&P.dbg[bi * kDbg + (k)], __builtin_amdgcn_s_memrealtime()); \
  } while (0)

struct Smem {
  alignas(16) uint8_t A[TILE_MAX + 64];  // X (input) → W (kept bytes) / output window
  alignas(16) uint8_t B[TILE_MAX + 128];  // Z = tail (<= 63) ++ decoded deltas (at B+PAD) → output window
  uint16_t ev_a[MAX_EV], ev_b[MAX_EV], ev_sa[MAX_EV], ev_sb[MAX_EV], ev_dl[MAX_EV];
  uint8_t ev_kind[MAX_EV];
  uint16_t dl_end[MAX_EV];
  uint16_t cut[MAX_EV];
  uint16_t wpos[MAX_EV];
  uint32_t epos[MAX_EV];
  uint16_t eidx[MAX_EV];
  uint16_t ejx[MAX_EV];  // emitted event k -> delta j
  uint16_t cand[MAX_CAND];
  int8_t cand_tok[MAX_CAND];
  uint16_t tok_pos[MAX_CAND];
  uint8_t tok_len[MAX_CAND];
  int8_t tok_id[MAX_CAND];
  int16_t tok_dep[MAX_CAND + 1];
  int32_t chunk_base[BS + 1];
  int32_t scr[2 * (BS / 64)];  // block scans: one (pair) partial per wave
  int32_t scr2[2 * (BS / 64)];  // a second scan's partials (no barrier between the two)
  int32_t v[40];
  alignas(16) uint8_t tpl[TPL_BYTES];  // this stream's event shape template
  // this item's SSE envelope (prefix with the index digits at 0, suffix at 256), written by
  // waves 1-7 while wave 0 runs the one-wave filter: S6's fill then loads its bytes without
  // the digit / envelope-part selection in its path
  alignas(16) uint8_t env[256 + 64];
};
static_assert(TPL_BYTES == kTplBytes, "template size");

enum : int {
  V_START = 0, V_NSEP, V_LASTSEP, V_ABORT, V_NEV, V_CONSUMED, V_STATUS, V_NDELTA, V_YLEN, V_NCAND,
  V_NTOK, V_BAIL, V_DEPTH0, V_TAILLEN, V_NEWTAIL, V_NEWDEPTH, V_WLEN, V_NEMIT, V_ETOT, V_OUTLEN,
  V_TPLPRE, V_TPLSUF, V_TPLK, V_NEXTEV, V_NFULL, V_NTPL, V_CFULL, V_CTPL, V_CLEX, V_NHOLE, V_CHOLE, V_S4W,
  V_HCLAIM,  // hole-template slots this workgroup wrote (bit per slot): one writer per slot
  V_S6W      // the sizing ran on wave 0 right after s4_wave
};

// LDS byte reader that fetches one aligned 64-bit word per 8 sequential bytes: a byte-serial
// scanner otherwise pays a dependent ds_read_u8 latency per character.
struct LdsWords {
  const uint64_t* base;  // 8-byte aligned LDS array
  mutable int wb;
  mutable uint64_t w;
  __device__ explicit LdsWords(const uint8_t* b) : base((const uint64_t*)b), wb(-1), w(0) {}
  QMX_HD uint8_t operator[](int i) const {
    int b = i >> 3;
    if (b != wb) {
      wb = b;
      w = base[b];
    }
    return (uint8_t)(w >> ((i & 7) << 3));
  }
};

// ------------------------------------------------------------------------------------
// block-level scans: wave64 inclusive scans on DPP (row_shr 1/2/4/8 inside each 16-lane
// row, then row_bcast15 / row_bcast31 across rows — GFX9-family DPP, a few cycles per step
// instead of a ds_bpermute round trip per __shfl_up), then a cross-wave combine in LDS
// ------------------------------------------------------------------------------------
#define QMX_DPP(old, v, ctrl, rm) __builtin_amdgcn_update_dpp((old), (v), (ctrl), (rm), 0xf, false)
enum : int { DPP_SHR1 = 0x111, DPP_SHR2 = 0x112, DPP_SHR4 = 0x114, DPP_SHR8 = 0x118, DPP_BC15 = 0x142, DPP_BC31 = 0x143,
             DPP_WSHR1 = 0x138 };

// Wave-wide moves without an LDS round trip (HIP's __shfl / __shfl_up are ds_bpermute: an
// LDS instruction and a wait on a dependent chain).  Every lane of the wave must be active.
// lane 63's value in every lane (v_readlane into a scalar register)
__device__ __forceinline__ int wave_last(int x) { return __builtin_amdgcn_readlane(x, 63); }
// lane - 1's value (DPP wave_shr:1); lane 0 gets `first`
__device__ __forceinline__ int wave_prev(int x, int first) { return QMX_DPP(first, x, DPP_WSHR1, 0xf); }

__device__ inline int wave_incl_sum(int x) {
  x += QMX_DPP(0, x, DPP_SHR1, 0xf);  // lanes whose source is outside the row / a masked row get 0
  x += QMX_DPP(0, x, DPP_SHR2, 0xf);
  x += QMX_DPP(0, x, DPP_SHR4, 0xf);
  x += QMX_DPP(0, x, DPP_SHR8, 0xf);
  x += QMX_DPP(0, x, DPP_BC15, 0xa);  // rows 1, 3 += lane 15 of the row below
  x += QMX_DPP(0, x, DPP_BC31, 0xc);  // rows 2, 3 += lane 31
  return x;
}

// inclusive scan of a (non-commutative) pair monoid, lane order; a lane combines only when
// its DPP source is valid (exactly the lanes the shuffle scan combined)
template <class Op>
__device__ inline int2 wave_incl_pair(int2 x, Op op) {
  const int lane = threadIdx.x & 63, r = lane & 15;
  int2 y;
#define QMX_PAIR_STEP(ctrl, rm, valid) \
  y.x = QMX_DPP(x.x, x.x, ctrl, rm);   \
  y.y = QMX_DPP(x.y, x.y, ctrl, rm);   \
  if (valid) x = op(y, x);
  QMX_PAIR_STEP(DPP_SHR1, 0xf, r >= 1)
  QMX_PAIR_STEP(DPP_SHR2, 0xf, r >= 2)
  QMX_PAIR_STEP(DPP_SHR4, 0xf, r >= 4)
  QMX_PAIR_STEP(DPP_SHR8, 0xf, r >= 8)
  QMX_PAIR_STEP(DPP_BC15, 0xa, (lane >> 4) & 1)
  QMX_PAIR_STEP(DPP_BC31, 0xc, lane >= 32)
#undef QMX_PAIR_STEP
  return x;
}

// tail_barrier = false: the caller guarantees a block barrier before anything writes `scr`
// again (its own later barrier, or the next scan uses another scratch array)
template <bool tail_barrier = true>
__device__ inline int block_excl_sum(int v, int32_t* scr, int* total) {
  int w = threadIdx.x >> 6;
  const int x = wave_incl_sum(v);
  if ((threadIdx.x & 63) == 63) scr[w] = x;
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < BS / 64; ++i) {
    int s = scr[i];
    if (i < w) base += s;
    tot += s;
  }
  if (tail_barrier) __syncthreads();
  *total = tot;
  return base + x - v;
}

// generic pair monoid scan: T = int2 {a, b}
template <class Op, bool tail_barrier = true>
__device__ inline int2 block_excl_pair(int2 v, int2 ident, Op op, int32_t* scr, int2* total) {
  int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int2 x = wave_incl_pair(v, op);
  if (lane == 63) {
    scr[2 * w] = x.x;
    scr[2 * w + 1] = x.y;
  }
  __syncthreads();
  int2 base = ident, tot = ident;
#pragma unroll
  for (int i = 0; i < BS / 64; ++i) {
    int2 s = make_int2(scr[2 * i], scr[2 * i + 1]);
    if (i < w) base = op(base, s);
    tot = op(tot, s);
  }
  if (tail_barrier) __syncthreads();
  const int2 ex = make_int2(wave_prev(x.x, ident.x), wave_prev(x.y, ident.y));
  *total = tot;
  return op(base, ex);
}

// newline-run map x ↦ (x.x ? x + x.y : x.y); compose (first f then g)
struct RunOp {
  __device__ int2 operator()(int2 f, int2 g) const { return g.x ? make_int2(f.x, f.y + g.y) : g; }
};
// depth map x ↦ max(x + a, b); compose (first f then g)
struct DepthOp {
  __device__ int2 operator()(int2 f, int2 g) const { return make_int2(f.x + g.x, max(f.y + g.x, g.y)); }
};

// ------------------------------------------------------------------------------------
// MFMA tag matcher
// ------------------------------------------------------------------------------------
// ASCII upper → lower case on 8 bytes at once (other bytes unchanged)
__device__ inline uint64_t lower8(uint64_t x) {
  constexpr uint64_t ones = 0x0101010101010101ull, hi = 0x8080808080808080ull;
  const uint64_t lo7 = x & ~hi;
  const uint64_t ge_a = lo7 + (0x80 - 'A') * ones;      // bit 7 set: byte >= 'A'
  const uint64_t gt_z = lo7 + (0x80 - 'Z' - 1) * ones;  // bit 7 set: byte > 'Z'
  return x | (((ge_a & ~gt_z & ~x) & hi) >> 2);
}

// B operand (patterns × window features) of column block `blk`: host-built per lane
// (KParams::bfrag), one 16-byte LDS read per lane instead of per-byte pattern decoding.
__device__ inline v4i build_pattern_frag(const KParams& P, int blk) {
  v4i b;
  __builtin_memcpy(&b, &P.bfrag[blk][(threadIdx.x & 63) * 16], 16);
  return b;
}

// pattern t's bytes past the 16-byte window at Z[p ...) (patterns longer than the window)
__device__ inline bool pattern_tail_ok(const uint8_t* Z, int Zn, int p, int t, const KParams& P) {
  const int L = pattern_len(P.ts, t);
  if (p + L > Zn) return false;
  for (int j = kWindow; j < L; ++j)
    if (lower_ascii(Z[p + j]) != pattern_byte(P.ts, t, j)) return false;
  return true;
}

// 16 candidate windows per MFMA and 16 patterns per column block; result[row][pat] ==
// Σ_j mask·(w_j²) − 2·w_j·p_j (per base-8 digit) == −E[pat]  <=>  Σ_j (w_j − p_j)² == 0 over
// the pattern's first 16 bytes  <=>  the window equals them (all of a tag up to 13 bytes;
// longer patterns then compare their tail).  Distinct tags never both match at
// one '<' (make_tagset), so at most one column of a row survives.
// PatCol: this lane's pattern column of each block (t = 16·blk + lane % 16) — its match value
// −E and length — read from KParams once per tile, ahead of the candidate scan
struct PatCol {
  int negE[2], plen[2];
};
__device__ inline PatCol pattern_cols(const KParams& P) {
  PatCol c;
#pragma unroll
  for (int blk = 0; blk < 2; ++blk) {
    // (no dependence on P.npat: entries past it are zero, and the match tests t < npat)
    const int t = 16 * blk + (threadIdx.x & 15);
    c.negE[blk] = -P.pat_E[t];
    c.plen[blk] = P.plen[t];
  }
  return c;
}
__device__ inline void mfma_match_group(const uint8_t* Z, int Zn, const uint16_t* cand, int ncand, int g,
                                        const KParams& P, v4i bf0, v4i bf1, const PatCol& pc, int npat, int nts,
                                        int8_t* cand_tok);
__device__ inline void mfma_match_group(const uint8_t* Z, int Zn, const uint16_t* cand, int ncand, int g,
                                        const KParams& P, v4i bf0, v4i bf1, int8_t* cand_tok) {
  mfma_match_group(Z, Zn, cand, ncand, g, P, bf0, bf1, pattern_cols(P), P.npat, P.ts.n, cand_tok);
}
__device__ inline void mfma_match_group(const uint8_t* Z, int Zn, const uint16_t* cand, int ncand, int g,
                                        const KParams& P, v4i bf0, v4i bf1, const PatCol& pc, int npat, int nts,
                                        int8_t* cand_tok) {
  int l = threadIdx.x & 63, r = l & 15, kg = l >> 4;
  int c = g * 16 + r;
  int p = c < ncand ? (int)cand[c] : -1;
  // the 16-byte window from two aligned-word LDS reads (Z is 8-byte aligned with >= 24
  // readable bytes past Zn), bytes past Zn get code 0
  uint64_t w0 = 0, w1 = 0;
  const int nv = p >= 0 ? min(16, Zn - p) : 0;
  if (nv > 0) {  // (zero past Zn: 0 is no pattern byte)
    w0 = lower8(lds_window8(Z, p, Zn));
    w1 = lower8(lds_window8(Z, p + 8, Zn));
  }
  // the window's bytes themselves (ASCII-lowercased, the tags' IGNORECASE) as base-8 digits
  // d0, d1 (0..7) and d2 (0..3), and d0² + d1² + d2² (<= 107: int8) — feature group kg of the
  // A operand.  Four bytes per 32-bit word at once: digits by shift-and-mask, squares by a
  // v_perm_b32 byte lookup (the 8-entry table {0,1,4,...,49} as two words), the group's
  // feature by a per-lane select — a per-byte loop with a per-lane branch on kg compiled to
  // ~1,000 masked instructions per group (2 us of the filter stage, r4/i)
  v4i a;
  {
    const uint32_t sq_lo = 0x09040100u, sq_hi = 0x31241910u;  // d² for d = 0..7
    const uint32_t h[4] = {(uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32)};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t d0 = h[q] & 0x07070707u, d1 = (h[q] >> 3) & 0x07070707u, d2 = (h[q] >> 6) & 0x03030303u;
      const uint32_t sq = __builtin_amdgcn_perm(sq_hi, sq_lo, d0) + __builtin_amdgcn_perm(sq_hi, sq_lo, d1) +
                          __builtin_amdgcn_perm(sq_hi, sq_lo, d2);  // bytewise: <= 107, no carries
      a[q] = (int)(kg == 0 ? d0 : kg == 1 ? d1 : kg == 2 ? d2 : sq);
    }
  }
  const int nblk = npat > 16 ? 2 : 1;
  for (int blk = 0; blk < nblk; ++blk) {
    // this lane's pattern column: its match value, length (pc: read ahead) and token id
    const int t = 16 * blk + (l & 15);
    const bool tv = t < npat;
    const int negE = blk ? pc.negE[1] : pc.negE[0], plen = blk ? pc.plen[1] : pc.plen[0];  // (no dynamic index)
    const int8_t tok = (int8_t)(t < nts ? t + 1 : -(t - nts + 1));
    v4i acc = {0, 0, 0, 0};
    acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, blk ? bf1 : bf0, acc, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int row = 4 * (l >> 4) + i;
      int cc = g * 16 + row;
      if (tv && cc < ncand && acc[i] == negE && (plen <= kWindow || pattern_tail_ok(Z, Zn, (int)cand[cc], t, P)))
        cand_tok[cc] = tok;
    }
  }
}

// The same match for a handful of candidates (<= 4) and tags whose patterns fit the 16-byte
// window (every default tag): lane (c, t) = (lane >> 4, lane & 15) compares candidate c's
// lowercased window with pattern t on VALU, 8 bytes at a time under the pattern's length
// mask — one step for all 64 pairs.  Measured (tools/probes/s3a_mfma_probe.hip): against one
// or a few patterns VALU SWAR is several times cheaper than building the MFMA operands; the
// MFMA matcher keeps the tiles with many '<' (16 candidate windows × 16 patterns per MFMA).
// Bytes past Zn read as 0 (no pattern byte), as in mfma_match_group.  Pattern words and
// lengths from the item's LDS copy of the parameters.
__device__ inline void swar_match_small(const uint8_t* Z, int Zn, const uint16_t* cand, int ncand, int npat, int nts,
                                        const KParams& P, int8_t* cand_tok) {
  const int lane = threadIdx.x & 63, c = lane >> 4, t = lane & 15;
  const uint64_t p0 = P.pw[t][0], p1 = P.pw[t][1];
  const int L = P.plen[t];
  const bool v = c < ncand && t < npat;
  const int p = v ? (int)cand[c] : 0;
  bool hit = false;
  if (v) {
    const uint64_t w0 = lower8(lds_window8(Z, p, Zn)), w1 = lower8(lds_window8(Z, p + 8, Zn));
    const uint64_t m0 = L >= 8 ? ~0ull : ((1ull << (8 * L)) - 1ull);
    const uint64_t m1 = L >= 16 ? ~0ull : L > 8 ? ((1ull << (8 * (L - 8))) - 1ull) : 0ull;
    hit = L > 0 && ((w0 ^ p0) & m0) == 0 && ((w1 ^ p1) & m1) == 0;
  }
  // distinct tags never both match at one '<' (make_tagset): one writer per candidate
  if (hit) cand_tok[c] = (int8_t)(t < nts ? t + 1 : -(t - nts + 1));
}

__device__ inline int tok_plen(const KParams& P, int id) {
  return id > 0 ? P.ts.len[id - 1] + 2 : P.ts.len[-id - 1] + 3;
}

// number of tokens with pos < x  /  <= x
__device__ inline int tok_lower(const Smem& s, int ntok, int x) {
  int lo = 0, hi = ntok;
  while (lo < hi) {
    int m = (lo + hi) >> 1;
    if (s.tok_pos[m] < x) lo = m + 1;
    else hi = m;
  }
  return lo;
}
__device__ inline int tok_upper(const Smem& s, int ntok, int x) {
  int lo = 0, hi = ntok;
  while (lo < hi) {
    int m = (lo + hi) >> 1;
    if (s.tok_pos[m] <= x) lo = m + 1;
    else hi = m;
  }
  return lo;
}
// kept(x) given k = #tokens with pos <= x
__device__ inline bool kept_at(const Smem& s, int k, int x) {
  if (k > 0 && x < (int)s.tok_pos[k - 1] + (int)s.tok_len[k - 1])
    return s.tok_id[k - 1] < 0 && s.tok_dep[k - 1] == 0;
  return s.tok_dep[k] == 0;
}

// Is Z[q, e) (lowercased) a prefix of some pattern (opens only: open patterns)?  The device
// form of qmx_text.h pattern_prefix: 8-byte words against KParams::pw.
__device__ inline bool pattern_prefix_w(const uint8_t* Z, int q, int e, const KParams& P, bool opens_only) {
  const int m = e - q;
  if (m <= 0 || m > kMaxTail) return m <= 0;
  const int npat = opens_only ? P.ts.n : 2 * P.ts.n;
  // the first 16 bytes stay in registers (every default tag's pattern fits); longer partial
  // tags read their further words per pattern
  const uint64_t z0 = lower8(lds_window8(Z, q, e)), z1 = m > 8 ? lower8(lds_window8(Z, q + 8, e)) : 0ull;
  auto word_mask = [m](int w) {
    const int nb = min(8, m - 8 * w);
    return nb >= 8 ? ~0ull : ((1ull << (8 * nb)) - 1);
  };
  for (int t = 0; t < npat; ++t) {
    if (m > pattern_len(P.ts, t)) continue;
    bool ok = z0 == (P.pw[t][0] & word_mask(0)) && (m <= 8 || z1 == (P.pw[t][1] & word_mask(1)));
    for (int w = 2; ok && 8 * w < m; ++w) ok = lower8(lds_window8(Z, q + 8 * w, e)) == (P.pw[t][w] & word_mask(w));
    if (ok) return true;
  }
  return false;
}

// holdback test at stream position e (Z coords): returns cut (q when held, else e).
// opens_only=false also reports any-pattern prefixes at depth > 0 (tail carry).
__device__ inline int hold_cut(const Smem& s, const uint8_t* Z, int ncand, int ntok, int e, const KParams& P,
                               bool for_tail, int* q_out) {
  int lo = 0, hi = ncand;  // last candidate index with cand < e
  while (lo < hi) {
    int m = (lo + hi) >> 1;
    if ((int)s.cand[m] < e) lo = m + 1;
    else hi = m;
  }
  int idx = lo - 1;
  *q_out = -1;
  if (idx < 0) return e;
  int q = s.cand[idx];
  int tk = s.cand_tok[idx];
  if (tk != 0 && q + tok_plen(P, tk) <= e) return e;  // completed token
  int dq = s.tok_dep[tok_lower(s, ntok, q)];
  bool pre = pattern_prefix_w(Z, q, e, P, dq == 0);
  if (!pre) return e;
  if (dq == 0 || for_tail) {
    *q_out = q;
    return dq == 0 ? q : e;
  }
  return e;
}

// ------------------------------------------------------------------------------------
// hole templates (qmx_hip.h HoleTpl): match and publish, one wave per event
// ------------------------------------------------------------------------------------
// Does the event x[e0, e1) equal T's literal runs with a valid string body / number in each
// hole?  Then it has T's parse: kind T.kind and, for content, the target hole (*sa, *sb,
// *body: 1 when it holds a backslash).  Wave-uniform (T is in LDS).
__device__ inline bool wave_hole_exact(const uint8_t* x, int e0, int e1, const HoleTpl& T, int* sa, int* sb,
                                       int* body) {
  const int n = T.len;
  if (n == 0 || e1 - e0 != n || !wave_lit_eq(x, e0, T.bytes, 0, n)) return false;  // the very same bytes
  if (T.kind == EV_CONTENT) {
    *sa = e0 + T.hs[T.target];
    *sb = e0 + T.he[T.target];
    *body = T.tgt_bs;
  }
  return true;
}

// Same-length fast path: an event as long as T whose holes are as long as T's (ids,
// timestamps and counters of one backend usually are) has every literal run at T's offsets,
// so one wave-parallel pass decides it — literal bytes equal, string-hole bytes printable
// ASCII other than '"' and '\\', number-hole bytes digits without a leading zero.  What passes
// is exactly what wave_hole_match accepts with the same holes (each string body ends at T's
// closing quote, each number at T's next literal); anything else (escapes, UTF-8, DEL, signs,
// fractions, other lengths) is left to the walk.  T in LDS; the hole bounds sit one per lane.
__device__ inline bool wave_hole_samelen(const uint8_t* x, int e0, int e1, const HoleTpl& T, int* sa, int* sb,
                                         int* body) {
  const int n = T.len, nh = T.nh;
  if (n == 0 || nh == 0 || e1 - e0 != n) return false;
  const int lane = threadIdx.x & 63;
  const int hs_l = lane < nh ? (int)T.hs[lane] : 0, he_l = lane < nh ? (int)T.he[lane] : 0;
  const int num_l = lane < nh ? (int)T.num[lane] : 0;
  bool bad = false;
  for (int c0 = 0; c0 < n; c0 += 64) {
    const int i = c0 + lane;
    const bool v = i < n;
    const uint32_t c = v ? x[e0 + i] : 0u;
    int h = -1, hs = 0, he = 0, num = 0;
    for (int k = 0; k < nh; ++k) {  // (uniform: the bounds come from lane k)
      const int a = __builtin_amdgcn_readlane(hs_l, k), b = __builtin_amdgcn_readlane(he_l, k);
      if (i >= a && i < b) {
        h = k;
        hs = a;
        he = b;
        num = __builtin_amdgcn_readlane(num_l, k);
      }
    }
    if (!v) continue;
    if (h < 0) bad = bad || c != T.bytes[i];
    else if (num) bad = bad || c - '0' > 9u || (i == hs && c == '0' && he - hs > 1);
    else bad = bad || c < 0x20u || c > 0x7eu || c == '"' || c == '\\';
  }
  if (__ballot(bad) != 0) return false;
  if (T.kind == EV_CONTENT) {
    *sa = e0 + T.hs[T.target];
    *sb = e0 + T.he[T.target];
    *body = 0;
  }
  return true;
}

// One step that rejects most other shapes: the event's head / tail against T's first / last
// literal run (up to 256 bytes each, a half wave each).
__device__ inline bool wave_hole_quick(const uint8_t* x, int e0, int e1, const HoleTpl& T) {
  const int n = T.len, nh = T.nh;
  if (n == 0 || nh == 0) return false;  // no holes: only the exact compare applies
  const int L0 = T.hs[0], Lm = n - (int)T.he[nh - 1];
  if (e1 - e0 < L0 + Lm) return false;
  const int lane = threadIdx.x & 63;
  bool bad = false;
  if (lane < 32) {
    const int o = lane * 8, L = min(L0, 256);
    if (o < L) bad = lds_window8(x, e0 + o, e0 + L) != lds_window8(T.bytes, o, L);
  } else {
    const int o = (lane - 32) * 8, L = min(Lm, 256);
    if (o < L) bad = lds_window8(x, e1 - Lm + o, e1 - Lm + L) != lds_window8(T.bytes, n - Lm + o, n - Lm + L);
  }
  return __ballot(bad) == 0;
}

// The walk: literal run, hole, literal run, ... — every hole's bytes validated.
__device__ inline bool wave_hole_match(const uint8_t* x, int e0, int e1, const HoleTpl& T, int* sa, int* sb,
                                       int* body) {
  const int n = T.len, nh = T.nh;
  int p = e0, q = 0;
  for (int i = 0; i < nh; ++i) {
    const int L = (int)T.hs[i] - q;
    if (p + L > e1 || !wave_lit_eq(x, p, T.bytes, q, L)) return false;
    p += L;
    q = T.he[i];
    int end;
    bool bs = false;
    if (T.num[i]) {
      int r = -1;
      if ((threadIdx.x & 63) == 0) r = num_hole_end(x, p, e1);
      end = __builtin_amdgcn_readfirstlane(r);
    } else {
      end = wave_str_end(x, p, e1, &bs);
    }
    if (end < 0) return false;
    if (i == T.target && T.kind == EV_CONTENT) {
      *sa = p;
      *sb = end;
      *body = bs ? 1 : 0;
    }
    p = end;
  }
  const int L = n - q;
  return p + L == e1 && wave_lit_eq(x, p, T.bytes, q, L);
}

// After a full parse of x[e0, e1) (tokens tpos/ttype[0, nt), string-value opens `vopen`,
// result kind / content body start str_a): its hole template into the launch's write table,
// entry by shape class, if no other workgroup of this launch claimed that entry.
__device__ inline void wave_hole_publish(const uint8_t* x, int e0, int e1, const uint16_t* tpos,
                                         const uint8_t* ttype, int nt, uint64_t vopen, int kind, int str_a,
                                         bool tgt_bs, HoleTpl* table, int* claims) {
  const int lane = threadIdx.x & 63;
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  const bool v = lane < nt;
  const int pos = v ? (int)tpos[lane] : 0;
  const int ty = v ? (ttype[lane] & TK_TYPE) : 0;
  const int nxt = __shfl_down(pos, 1, 64);  // a string value's closing quote (its SCLOSE token)
  const bool hstr = (vopen >> lane) & 1;
  int nend = -1;
  if (v && ty == TK_SCALAR) {
    const uint32_t c = x[pos];
    if (c == '-' || c - '0' < 10u) nend = num_hole_end(x, pos, e1);
  }
  const bool hnum = nend > 0;
  const uint64_t H = __ballot(hstr || hnum);
  const int nh = __popcll(H);
  if (nh > kHoleMax) return;
  int target = 0;
  if (kind == EV_CONTENT) {
    const uint64_t Tm = __ballot(hstr && pos + 1 == str_a);
    if (Tm == 0) return;
    target = __popcll(H & ((1ull << (__ffsll((unsigned long long)Tm) - 1)) - 1));
  }
  const int slot = (nh * 2 + (kind == EV_CONTENT ? 1 : 0)) % kHoleTpls;
  HoleTpl& D = table[slot];
  // the launch's only writer of this backend's table is its publishing workgroup (WF_PUBLISH);
  // within it one wave per slot (an LDS claim — no global atomic round trip on the path)
  int won = 0;
  if (lane == 0) won = (atomicOr(claims, 1 << slot) & (1 << slot)) == 0;
  if (!__builtin_amdgcn_readfirstlane(won)) return;
  const int len = e1 - e0;
  for (int i = lane; i < len; i += 64) D.bytes[i] = x[e0 + i];
  if ((H >> lane) & 1) {
    const int k = __popcll(H & below);
    D.hs[k] = (uint16_t)((hstr ? pos + 1 : pos) - e0);
    D.he[k] = (uint16_t)((hstr ? nxt : nend) - e0);
    D.num[k] = hnum ? 1 : 0;
  }
  // S3a's byte classes of word `lane` (< 32): the holes' bounds from their owner lanes
  {
    const int ha = (hstr ? pos + 1 : pos) - e0, hb = (hstr ? nxt : nend) - e0;
    const int o = lane * 8;
    uint32_t sm = 0, nm = 0, zm = 0;
    for (uint64_t m = H; m; m &= m - 1) {
      const int L = __ffsll((unsigned long long)m) - 1;
      const int a = __builtin_amdgcn_readlane(ha, L), e = __builtin_amdgcn_readlane(hb, L);
      const bool isnum = (__builtin_amdgcn_readlane((int)hnum, L)) != 0;
      const int lo = max(a, o) - o, up = min(e, o + 8) - o;
      if (lo < up) {
        const uint32_t m8 = ((1u << up) - 1u) & ~((1u << lo) - 1u);
        if (isnum) {
          nm |= m8;
          if (a >= o && e - a > 1) zm |= 1u << (a - o);
        } else {
          sm |= m8;
        }
      }
    }
    if (lane < 32) D.wmask[lane] = sm | (nm << 8) | (zm << 16);
  }
  if (lane == 0) {
    D.nh = (uint8_t)nh;
    D.kind = (uint8_t)kind;
    D.target = (uint8_t)target;
    D.tgt_bs = tgt_bs ? 1 : 0;
    D.len = (uint16_t)len;
  }
}

// A hole template that matched in this launch is carried into the launch's write table
// (the tables alternate per launch: a shape that only ever matches would otherwise vanish
// from every other launch).  Everything but the claim word is copied.
__device__ inline void wave_hole_carry(const HoleTpl& T, HoleTpl* dst, int slot, int* claims) {
  const int lane = threadIdx.x & 63;
  int won = 0;
  if (lane == 0) won = (atomicOr(claims, 1 << slot) & (1 << slot)) == 0;
  if (!__builtin_amdgcn_readfirstlane(won)) return;
  constexpr int kW = (int)(sizeof(HoleTpl) / 16) - 1;
  if (lane < kW) ((uint4*)dst)[lane] = ((const uint4*)&T)[lane];
}

// ------------------------------------------------------------------------------------
// the fused tick kernel
// ------------------------------------------------------------------------------------
// LDS of a tick workgroup (the fused kernel overlays it with the finalize workgroup's)
// ------------------------------------------------------------------------------------
// S4 on one wave (the common tile: Z <= 2048 bytes, <= 64 deltas, <= 63 '<' candidates)
// ------------------------------------------------------------------------------------
// The block-wide S4 spends ten block barriers and four block scans on what is, in a
// streaming tile, a few hundred bytes with a handful of '<': wave 0 alone runs the same
// stages wave-synchronously — ballot candidate scan in 64-byte strides, the MFMA matcher,
// the (a,b) depth scan on DPP, a hold_cut per delta lane, ballot compaction of the kept
// bytes with each delta's kept-prefix count — and the other waves wait at one barrier.
// Returns false (nothing written that the block path does not rewrite) when the tile has
// more than 63 candidates.
__device__ inline void wave_fence() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront"); }

// (a call, not inlined: inlined, the persistent kernel spills 16 B per lane and its span
// grows 28.0 -> 29.7 us, r3/loops/s3tune/; the call's entry wait for the wave's outstanding
// stores is the cheaper cost)
__device__ bool s4_wave(Smem& s, const uint8_t* Z, int Zn, int ndelta, int depth0, const KParams& P,
                        unsigned long long* dbg) {
  const int lane = threadIdx.x & 63;
  if (dbg != nullptr && lane == 0) dbg_put(&dbg[28], __builtin_amdgcn_s_memrealtime());
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  // the filter's KParams reads (the item's LDS copy), issued together before the candidate
  // scan and none depending on another (no P.npat / P.ts.n first): their latency overlaps
  // the scan instead of heading the MFMA match and the holdback cuts
  const v4i bf0 = build_pattern_frag(P, 0), bf1 = build_pattern_frag(P, 1);  // (block 1 unused when npat <= 16)
  const PatCol pc = pattern_cols(P);
  // pattern_prefix_w from registers: lane t holds pattern t's length and first two 8-byte
  // words (every default tag's pattern fits 16 bytes; longer ones read further words from P)
  // (lanes past 2·ts.n read zero entries: no dependence on P.ts.n)
  const int pl_l = lane < 2 * kMaxTags ? P.plen[lane] : 0;
  const uint64_t pw0_l = lane < 2 * kMaxTags ? P.pw[lane][0] : 0ull, pw1_l = lane < 2 * kMaxTags ? P.pw[lane][1] : 0ull;
  // candidates: every '<' of Z, in position order — 8 bytes per lane (SWAR compare on one
  // ds_read_b64; Z is 8-byte aligned with readable bytes past Zn), 512 bytes per step
  int nc = 0;
  for (int base = 0; base < Zn; base += 512) {
    const int x0 = base + lane * 8;
    uint32_t lm = 0;
    if (x0 < Zn) {
      const uint64_t w = *(const uint64_t*)&Z[x0];
      const uint64_t v = w ^ 0x3c3c3c3c3c3c3c3cull;
      const uint64_t y = (((v & 0x7f7f7f7f7f7f7f7full) + 0x7f7f7f7f7f7f7f7full) | v) & 0x8080808080808080ull;
      lm = (uint32_t)((((~y & 0x8080808080808080ull) >> 7) * 0x0102040810204080ull) >> 56);
      const int nb = Zn - x0;
      if (nb < 8) lm &= (1u << nb) - 1u;
    }
    const int cnt = __popc(lm);
    const int incl = wave_incl_sum(cnt);
    int k = nc + incl - cnt;
    for (uint32_t m = lm; m; m &= m - 1, ++k)
      if (k < 64) s.cand[k] = (uint16_t)(x0 + __ffs(m) - 1);
    nc += wave_last(incl);
    if (nc > 63) return false;  // (lane k owns token k AND the gap after it: ntok <= 63)
  }
  if (nc == 0) {
    // no '<' anywhere in Z (the block path's no-candidate case; a held tail starts with '<', so
    // none is pending): outside a think block every byte is kept in place (W = Z: the caller
    // sees V_S4W = 2), inside one every byte is dropped — the usual streaming tick
    const bool keep = depth0 == 0;
    if (lane < ndelta) {
      s.cut[lane] = s.dl_end[lane];
      s.wpos[lane] = keep ? s.dl_end[lane] : 0;
    }
    if (lane == 0) {
      s.v[V_WLEN] = keep ? Zn : 0;
      s.v[V_NEWTAIL] = -1;
      s.v[V_NEWDEPTH] = depth0;
      s.v[V_S4W] = 2;
    }
    return true;
  }
  // (read after the scan: only the match and the cuts use them)
  const int npat = P.npat, nts = P.ts.n;
  const int npw = 2 * nts;  // (<= 2 * kMaxTags <= 64 lanes)
  if (lane < nc) s.cand_tok[lane] = 0;
  wave_fence();
  if (dbg != nullptr && lane == 0) dbg_put(&dbg[29], __builtin_amdgcn_s_memrealtime());
  // a few candidates and window-sized patterns (QMX_KFAST bit 16): VALU pairs; else MFMA
  const bool small = (P.fast & 16) && nc <= 4 && npat <= 16 && __ballot(lane < npat && pl_l > kWindow) == 0;
  if (small) {
    swar_match_small(Z, Zn, s.cand, nc, npat, nts, P, s.cand_tok);
  } else {
    for (int g = 0; g * 16 < nc; ++g) mfma_match_group(Z, Zn, s.cand, nc, g, P, bf0, bf1, pc, npat, nts, s.cand_tok);
  }
  wave_fence();
  if (dbg != nullptr && lane == 0) dbg_put(&dbg[23], __builtin_amdgcn_s_memrealtime());
  // tokens and the depth before each (candidates in order, non-tokens the scan identity);
  // candidate lane c also keeps, in registers, its position, token id / length and the depth
  // before it — the holdback cuts below read them with v_readlane, not LDS searches
  int cpos = 0, ctok = 0, cplen = 0, cdep = 0, fdep, ntok;
  {
    const int id = lane < nc ? (int)s.cand_tok[lane] : 0;
    const uint64_t m = __ballot(id != 0);
    ntok = __popcll(m);  // (from the ballot: no LDS round trip through V_NTOK)
    const int k = __popcll(m & below);
    DepthOp op;
    int2 x = id > 0 ? make_int2(1, 1) : id < 0 ? make_int2(-1, 0) : make_int2(0, 0);
    x = wave_incl_pair(x, op);
    const int2 ex = make_int2(wave_prev(x.x, 0), wave_prev(x.y, 0));
    cpos = lane < nc ? (int)s.cand[lane] : 0;
    ctok = id;
    // the token's pattern length from lane (pattern index)'s pl_l: no KParams read here
    const int pidx = id > 0 ? id - 1 : id < 0 ? nts - id - 1 : 0;
    const int plx = __shfl(pl_l, pidx, 64);
    cplen = id != 0 ? plx : 0;
    cdep = max(depth0 + ex.x, ex.y);
    fdep = __builtin_amdgcn_readlane(max(depth0 + x.x, x.y), 63);
    if (id != 0) {
      s.tok_pos[k] = (uint16_t)cpos;
      s.tok_id[k] = (int8_t)id;
      s.tok_len[k] = (uint8_t)cplen;
      s.tok_dep[k] = (int16_t)cdep;
    }
    if (lane == 63) {
      s.v[V_NTOK] = ntok;
      s.tok_dep[ntok] = (int16_t)fdep;
    }
  }
  // hold_cut, wave-wide (every lane calls it; `active` lanes get an answer): the last
  // candidate before e from the candidate registers (positions ascend), its token / length and
  // the depth before it; then, for each lane whose candidate could still open a tag, the
  // tag-prefix test runs lane-parallel over the patterns — lane t tests pattern t against that
  // lane's window and a ballot answers (a loop over the patterns on each lane, with v_readlane
  // of every pattern word, cost ~1.4 us per headline tile); then the same decisions as hold_cut
  auto hold_cut_w = [&](int e, bool active, bool for_tail, int* q_out) -> int {
    int q = -1, tk = 0, pl = 0, dq = 0;
    for (int k = 0; k < nc; ++k) {  // (uniform bound, nc <= 63)
      const int ck = __builtin_amdgcn_readlane(cpos, k), tkk = __builtin_amdgcn_readlane(ctok, k);
      const int plk = __builtin_amdgcn_readlane(cplen, k), dqk = __builtin_amdgcn_readlane(cdep, k);
      const bool b = ck < e;
      q = b ? ck : q;
      tk = b ? tkk : tk;
      pl = b ? plk : pl;
      dq = b ? dqk : dq;
    }
    if (dbg != nullptr && lane == 0) dbg_put(&dbg[30], __builtin_amdgcn_s_memrealtime());
    // (q < e, so the window is never empty; longer than kMaxTail bytes it is no tag prefix)
    const bool need = active && q >= 0 && !(tk != 0 && q + pl <= e) && e - q <= kMaxTail;
    // a token that completes later in Z (the cut falls inside it: q + pl > e) answers its own
    // test — Z[q, e) is a proper prefix of its pattern, which counts for an open tag always
    // and for a close tag inside a block (np = npw).  Only a '<' that is no complete token
    // (tk == 0: a tag cut off at the end of Z, or no tag) and a close tag at depth 0 (a prefix
    // of some open tag?) take the lane-parallel pattern test (a tag split across deltas — the
    // usual "<thi" | "nk>" — cost ~0.35 us of dependent LDS reads and ballots per delta)
    const bool implied = tk > 0 || (tk < 0 && dq != 0);
    bool pref = implied;
    for (uint64_t bm = __ballot(need && !implied); bm; bm &= bm - 1) {
      const int j = __ffsll((unsigned long long)bm) - 1;
      const int qj = __builtin_amdgcn_readlane(q, j), m = __builtin_amdgcn_readlane(e, j) - qj;
      const int np = __builtin_amdgcn_readlane(dq, j) == 0 ? nts : npw;  // (opens only at depth 0)
      const uint64_t z0 = lower8(lds_window8(Z, qj, qj + m)), z1 = m > 8 ? lower8(lds_window8(Z, qj + 8, qj + m)) : 0ull;
      const uint64_t m0 = m >= 8 ? ~0ull : ((1ull << (8 * m)) - 1);
      const uint64_t m1 = m >= 16 ? ~0ull : m <= 8 ? 0ull : ((1ull << (8 * (m - 8))) - 1);
      bool ok = lane < np && m <= pl_l && z0 == (pw0_l & m0) && (m <= 8 || z1 == (pw1_l & m1));
      for (int w = 2; 8 * w < m; ++w) {  // (uniform: windows longer than 16 bytes)
        const int nb = min(8, m - 8 * w);
        const uint64_t mw = nb >= 8 ? ~0ull : ((1ull << (8 * nb)) - 1);
        const uint64_t zw = lower8(lds_window8(Z, qj + 8 * w, qj + m));
        if (ok) ok = zw == (P.pw[lane][w] & mw);
      }
      const bool f = __ballot(ok) != 0;
      if (lane == j) pref = f;
    }
    if (dbg != nullptr && lane == 0) dbg_put(&dbg[31], __builtin_amdgcn_s_memrealtime());
    *q_out = -1;
    if (!need || !pref) return e;  // no candidate, a completed token, or no tag prefix
    if (dq == 0 || for_tail) {
      *q_out = q;
      return dq == 0 ? q : e;
    }
    return e;
  };
  wave_fence();
  if (dbg != nullptr && lane == 0) dbg_put(&dbg[25], __builtin_amdgcn_s_memrealtime());
  // a cut per delta (lane j) and the new holdback tail (lane ndelta, in the same pass)
  int cut = 0;
  const bool tail_here = ndelta < 64;  // a free lane for the tail: lane ndelta
  {
    const bool is_tail = tail_here && lane == ndelta;
    const int e = is_tail ? Zn : lane < ndelta ? (int)s.dl_end[lane] : 0;
    int q;
    const int c = hold_cut_w(e, lane < ndelta || is_tail, is_tail, &q);
    if (is_tail) {
      s.v[V_NEWTAIL] = q;
      s.v[V_NEWDEPTH] = fdep;
    } else if (lane < ndelta) {
      cut = c;
      s.cut[lane] = (uint16_t)cut;
    }
  }
  if (!tail_here) {  // 64 deltas: the tail after them, on lane 0
    int q;
    hold_cut_w(Zn, lane == 0, true, &q);
    if (lane == 0) {
      s.v[V_NEWTAIL] = q;
      s.v[V_NEWDEPTH] = fdep;
    }
  }
  const int cutN = __builtin_amdgcn_readlane(cut, max(ndelta - 1, 0));
  if (dbg != nullptr && lane == 0) dbg_put(&dbg[24], __builtin_amdgcn_s_memrealtime());
  // compaction of the kept bytes of [0, cutN) into A, by segments (kept_at's cases): lane k
  // owns the gap before token k (kept at depth 0) and token k itself (kept when it is a
  // close tag at depth 0: literal text); a DPP scan gives each segment its output offset,
  // the kept segments are copied 64 bytes per step, and each delta's kept prefix is one
  // segment lookup — no per-byte token search
  const bool seg = lane <= ntok;
  int gs = 0, ge = 0, ts0 = 0, te = 0;
  bool gk = false, tk = false;
  if (seg) {
    gs = lane == 0 ? 0 : min((int)s.tok_pos[lane - 1] + (int)s.tok_len[lane - 1], cutN);
    ge = lane < ntok ? min((int)s.tok_pos[lane], cutN) : cutN;
    ge = max(ge, gs);
    const int dep = s.tok_dep[lane];
    gk = dep == 0;
    if (lane < ntok) {
      ts0 = min((int)s.tok_pos[lane], cutN);
      te = min((int)s.tok_pos[lane] + (int)s.tok_len[lane], cutN);
      tk = s.tok_id[lane] < 0 && dep == 0;
    }
  }
  const int gl = gk ? ge - gs : 0, tl = tk ? te - ts0 : 0;
  const int incl = wave_incl_sum(gl + tl);
  const int ob = incl - gl - tl;  // output offset of this lane's gap (its token follows it)
  const int out = wave_last(incl);
  for (uint64_t m = __ballot(gl > 0); m; m &= m - 1) {
    const int k = __ffsll((unsigned long long)m) - 1;
    const int a = __builtin_amdgcn_readlane(gs, k), n = __builtin_amdgcn_readlane(gl, k),
              o = __builtin_amdgcn_readlane(ob, k);
    for (int x = lane; x < n; x += 64) s.A[o + x] = Z[a + x];
  }
  for (uint64_t m = __ballot(tl > 0); m; m &= m - 1) {
    const int k = __ffsll((unsigned long long)m) - 1;
    const int a = __builtin_amdgcn_readlane(ts0, k), n = __builtin_amdgcn_readlane(tl, k),
              o = __builtin_amdgcn_readlane(ob, k) + __builtin_amdgcn_readlane(gl, k);
    for (int x = lane; x < n; x += 64) s.A[o + x] = Z[a + x];
  }
  // kept bytes before each delta's cut: the segment that holds cut - 1
  const int c = lane < ndelta ? cut : 0;
  // tokens starting before c: a walk over the token lanes' positions (ts0: tok_pos clamped to
  // cutN, the same answer for c - 1 < cutN) — the binary search's dependent LDS reads only
  // for token-dense tiles
  int kk = 0;
  if (ntok <= 16) {
    for (int k = 0; k < ntok; ++k) kk += __builtin_amdgcn_readlane(ts0, k) <= c - 1 ? 1 : 0;
    kk = c > 0 && c < cutN ? kk : 0;
  } else {
    kk = c > 0 && c < cutN ? tok_upper(s, ntok, c - 1) : 0;
  }
  const int pk = kk > 0 ? kk - 1 : 0;
  const int p_gs = __shfl(gs, kk, 64), p_ob = __shfl(ob, kk, 64), p_gk = __shfl((int)gk, kk, 64);
  const int q_ts = __shfl(ts0, pk, 64), q_te = __shfl(te, pk, 64), q_ob = __shfl(ob, pk, 64),
            q_gl = __shfl(gl, pk, 64), q_tk = __shfl((int)tk, pk, 64);
  if (lane < ndelta) {
    int wp;
    if (c >= cutN) wp = out;
    else if (c == 0) wp = 0;
    else if (kk > 0 && c < q_te) wp = q_ob + q_gl + (q_tk ? c - q_ts : 0);  // inside token kk-1
    else wp = p_ob + (p_gk ? c - p_gs : 0);                                   // in gap kk
    s.wpos[lane] = (uint16_t)wp;
  }
  if (lane == 0) s.v[V_WLEN] = out;
  if (dbg != nullptr && lane == 0) dbg_put(&dbg[32], __builtin_amdgcn_s_memrealtime());
  return true;
}

// S2's last step (one thread): events of the tile from the separators, what it consumed,
// and whether the stream is done / has more events than one tile holds
// owner = false: only the event list (identical writes from every wave's lane 0), not the
// result's consumed count and status bits (thread 0's)
__device__ inline void s2_finalize(Smem& s, int start, int in_len, bool eof, bool owner = true) {
  int nsep = s.v[V_NSEP];
  int nev, consumed;
  bool done = false, more = false;
  if (nsep > MAX_EV) {
    nev = MAX_EV;
    consumed = s.ev_b[MAX_EV - 1] + 2;
    more = true;
  } else {
    nev = nsep;
    int rem = nsep > 0 ? s.v[V_LASTSEP] + 2 : start;
    consumed = rem;
    if (eof) {
      if (rem < in_len) {
        if (nev < MAX_EV) {
          s.ev_a[nev] = (uint16_t)rem;
          s.ev_b[nev] = (uint16_t)in_len;
          ++nev;
          consumed = in_len;
          done = true;
        } else {
          more = true;
        }
      } else {
        consumed = in_len;
        done = true;
      }
    }
  }
  s.v[V_NEV] = nev;
  if (!owner) return;
  s.v[V_CONSUMED] = consumed;
  if (done) s.v[V_STATUS] |= WS_DONE;
  if (more) s.v[V_STATUS] |= WS_MORE;
}

// newline mask of x[lo, lo + len) (len <= 64, 8-byte aligned lo, 64 B readable past it):
// SWAR byte compares on ds_read_b64 words
__device__ inline uint64_t nl_mask64(const uint8_t* x, int lo, int len) {
  uint64_t nm = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    if (q * 8 < len) {
      const uint64_t w = *(const uint64_t*)&x[lo + 8 * q];
      const uint64_t v = w ^ 0x0a0a0a0a0a0a0a0aull;
      const uint64_t y = (((v & 0x7f7f7f7f7f7f7f7full) + 0x7f7f7f7f7f7f7f7full) | v) & 0x8080808080808080ull;
      const uint64_t zb = ~y & 0x8080808080808080ull;  // high bit of every '\n' byte
      nm |= (uint64_t)(((zb >> 7) * 0x0102040810204080ull) >> 56) << (8 * q);
    }
  }
  return nm & (len >= 64 ? ~0ull : ((1ull << len) - 1ull));
}

// S2 on wave 0 (tiles up to 4 KiB past the leading whitespace: a streaming tick, or a whole
// short response): the block path's newline-run framing with DPP wave scans instead of block
// scans and the finalize on lane 0 — one block barrier instead of five.  4 KiB per pass (64
// lanes x <= 64 bytes, one 64-bit newline mask per lane); the newline-run state, the
// separator count and the last separator carry from pass to pass.
__device__ inline void s2_wave(Smem& s, int start, int in_len, bool eof) {
  const int lane = threadIdx.x & 63;
  int2 carry = make_int2(1, 0);  // newline run ending at the pass's start (none before `start`)
  int kb = 0, lastsep = -1;      // separators of earlier passes / the last one
  for (int base = start; base < in_len; base += 64 * 64) {
    const int end = min(base + 64 * 64, in_len);
    const int C8 = ((((end - base) + 63) / 64) + 7) & ~7;  // <= 64
    const int lo = min(base + lane * C8, end), hi = min(lo + C8, end), len = hi - lo;
    const uint64_t nm = nl_mask64(s.A, lo, len);
    const uint64_t valid = len >= 64 ? ~0ull : ((1ull << len) - 1ull);
    const uint64_t inv = ~nm & valid;
    const bool all_nl = inv == 0;
    const int trail = all_nl ? len : len - 64 + __clzll(inv);
    const bool next_nl = hi < in_len && s.A[hi] == '\n';
    const int2 run = all_nl ? make_int2(1, len) : make_int2(0, trail);
    const int2 incl = wave_incl_pair(run, RunOp());
    int2 ex = make_int2(wave_prev(incl.x, 0), wave_prev(incl.y, 0));
    ex = lane == 0 ? carry : RunOp()(carry, ex);
    // separators: "\n" at an even position of its newline run, followed by a "\n"
    auto each_sep = [&](auto&& f) {
      uint64_t m = nm;
      while (m) {
        const int r0 = __ffsll((unsigned long long)m) - 1;
        const uint64_t rest = ~(m >> r0);
        const int L = rest == 0 ? 64 - r0 : __ffsll((unsigned long long)rest) - 1;
        const int c = r0 == 0 ? ex.y : 0;
        const bool ext = r0 + L == len && next_nl;
        for (int i = 0; i < L; ++i)
          if (!((c + i) & 1) && (i + 1 < L || ext)) f(lo + r0 + i);
        m &= ~(L >= 64 ? ~0ull : (((1ull << L) - 1ull) << r0));
      }
    };
    int cnt = 0, last = -1;
    each_sep([&](int p) {
      ++cnt;
      last = p;
    });
    const int ci = wave_incl_sum(cnt);
    int k = kb + ci - cnt;
    each_sep([&](int p) {
      if (k < MAX_EV) s.ev_b[k] = (uint16_t)p;
      if (k + 1 < MAX_EV) s.ev_a[k + 1] = (uint16_t)(p + 2);
      ++k;
    });
    // the pass's last separator: the highest lane that has one (lanes own ascending ranges)
    const uint64_t lm = __ballot(last >= 0);
    if (lm != 0) lastsep = __builtin_amdgcn_readlane(last, 63 - __clzll(lm));
    kb += wave_last(ci);
    carry = RunOp()(carry, make_int2(wave_last(incl.x), wave_last(incl.y)));
  }
  if (lane == 0) {
    s.ev_a[0] = (uint16_t)start;
    s.v[V_NSEP] = kb;
    s.v[V_LASTSEP] = lastsep;
  }
  wave_fence();
  if (lane == 0) s2_finalize(s, start, in_len, eof);
}

struct TickShared {
  Smem s;
  KParams P;                                   // kernel args staged in LDS: lane-divergent reads
  uint16_t TKP[BS / 64][TOK_CAP];              // per-wave token buffers (positions)
  alignas(8) uint8_t TKT[BS / 64][TOK_CAP];    // token bytes (type | key id | flags)
  int wtpl[BS / 64][4];  // S3: per-wave in-tile templates {p0, tp, s0, ts} (p0 < 0: none)
  int s3w[BS / 64][4];   // S3a per wave: events left for the loop, hole templates matched, newest content event
  HoleTpl htpl[kHoleTpls];  // S3: this item's backend hole templates (previous launch's)
};

// threadIdx.x as an opaque value: in the persistent grid the tick body sits inside a loop,
// and the compiler hoists every `tid < k` mask it derives out of that loop — dozens of 64-bit
// masks live across the whole body, more than the SGPR file holds, spilled into VGPR lanes
// (v_writelane / v_readlane) and scratch.  Re-deriving a mask costs one v_cmp.
__device__ __forceinline__ int opaque_tid() {
  int t;
  asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"((int)threadIdx.x));
  return t;
}

// S6 sizing on one wave (the common tile: <= 64 deltas, W <= 2048 bytes): emitted-delta
// ballot, per-lane chunks of escaped lengths with a DPP scan, each delta's escaped prefix.
// Called by wave 0 — right after s4_wave when the filter ran on one wave (no barrier between
// the two), else after the filter's barrier.
__device__ inline void s6_size_wave(Smem& s, const uint8_t* W, int Wlen, int ndelta) {
    const int lane = threadIdx.x & 63;
    const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
    const int wp = lane < ndelta ? (int)s.wpos[lane] : 0;
    const int prev = wave_prev(wp, 0);
    const bool f = lane < ndelta && wp > prev;
    const uint64_t m = __ballot(f);
    if (lane < ndelta) s.eidx[lane] = (uint16_t)__popcll(m & below);
    if (f) s.ejx[__popcll(m & below)] = (uint16_t)lane;
    const int C = (Wlen + 63) / 64;
    const int lo = min(lane * C, Wlen), hi = min(lo + C, Wlen);
    // clean content (printable ASCII without '"' or '\\': every byte escapes to itself) —
    // escaped offsets are raw offsets, no decode walk: 8 bytes per lane per step (SWAR, the
    // zero / less-than tricks only err towards "not clean")
    bool dirty = false;
    {
      const uint64_t hb = 0x8080808080808080ull, one = 0x0101010101010101ull;
      for (int x0 = lane * 8; x0 < Wlen; x0 += 64 * 8) {
        const int nb = min(8, Wlen - x0);
        const uint64_t w = lds_window8(W, x0, Wlen), vm = nb >= 8 ? ~0ull : ((1ull << (8 * nb)) - 1);
        const uint64_t q = w ^ 0x2222222222222222ull, b = w ^ 0x5c5c5c5c5c5c5c5cull, d = w ^ 0x7f7f7f7f7f7f7f7full;
        const uint64_t odd = (((q - one) & ~q) | ((b - one) & ~b) | ((d - one) & ~d) | ((w - 0x20 * one) & ~w) | w) & hb;
        dirty = dirty || (odd & vm) != 0;
      }
    }
    int tot;
    if (__ballot(dirty) == 0) {
      tot = Wlen;
      s.chunk_base[lane] = lo;
      if (lane < ndelta) s.epos[lane] = (uint32_t)min(wp, Wlen);
    } else {
      int x = lo, e = 0;
      while (x < hi && is_cont(W[x])) ++x;
      while (x < hi) {
        uint32_t cp;
        x += wtf8_decode(W, x, Wlen, &cp);
        e += escaped_len_cp(cp);
      }
      const int incl = wave_incl_sum(e);
      const int excl = incl - e;
      tot = wave_last(incl);
      s.chunk_base[lane] = excl;  // the write phase's escaped-content chunks (64 of them here)
      // (shuffles with every lane active: a lane's chunk base for its delta's escaped prefix)
      const int t = (lane < ndelta && wp < Wlen && C > 0) ? wp / C : 0;
      const int tbase = __shfl(excl, t, 64);
      if (lane < ndelta) {
        uint32_t ep = (uint32_t)tot;
        if (wp < Wlen) {
          int xx = min(t * C, Wlen), ee = tbase;
          while (xx < wp && is_cont(W[xx])) ++xx;
          while (xx < wp) {
            uint32_t cp;
            xx += wtf8_decode(W, xx, Wlen, &cp);
            ee += escaped_len_cp(cp);
          }
          ep = (uint32_t)ee;
        }
        s.epos[lane] = ep;
      }
    }
  if (lane == 0) {
    s.v[V_NEMIT] = __popcll(m);
    s.v[V_ETOT] = tot;
  }
}

__device__ __forceinline__ void tick_body(const WorkItem* __restrict__ items, const uint8_t* __restrict__ in,
                                          uint8_t* __restrict__ out, WorkResult* __restrict__ res,
                                          DevSlot* __restrict__ state, uint8_t* __restrict__ content,
                                          const KParams& Pk, TickShared& U, const BackendTpl* __restrict__ btpl_rd,
                                          BackendTpl* __restrict__ btpl_wr, uint32_t seq, const int bi) {
  Smem& s = U.s;
  KParams& P = U.P;
  auto& TKP = U.TKP;
  auto& TKT = U.TKT;
  auto& wtpl = U.wtpl;
  const int tid = opaque_tid();
  // Tiles sit at a fixed stride (item bi at bi x TILE_MAX, HipEngine::prepare), so the first
  // 4 KiB of this item's tile — all of it for a streaming tick or a short response — is
  // requested from host memory together with the work item itself: one PCIe round trip
  // before the tile is in registers, not item → offset → tile (two)
  const uint8_t* tile = in + (size_t)bi * TILE_MAX;
  uint4 spec = make_uint4(0, 0, 0, 0);
  if (tid * 16 < kSpecTile) spec = *(const uint4*)&tile[tid * 16];
  WorkItem it = items[bi];
  for (int i = tid; i < (int)(sizeof(KParams) / 4); i += BS) ((uint32_t*)&P)[i] = ((const uint32_t*)&Pk)[i];
  if (Pk.dbg != nullptr && threadIdx.x == 0) dbg_put(&Pk.dbg[bi * kDbg + 0], __builtin_amdgcn_s_memrealtime());
  if (Pk.dbg != nullptr && threadIdx.x == 0) dbg_put(&Pk.dbg[bi * kDbg + 11], __builtin_amdgcn_s_memtime());
  // the work item is wave-uniform: keep its fields in scalar registers (a one-shot launch
  // reads it through the scalar cache anyway; a persistent grid loads it per tick with
  // vector loads, and every address derived from VGPR copies would cost vector registers)
  it.slot = __builtin_amdgcn_readfirstlane(it.slot);
  it.in_off = __builtin_amdgcn_readfirstlane(it.in_off);
  it.in_len = __builtin_amdgcn_readfirstlane(it.in_len);
  it.out_off = __builtin_amdgcn_readfirstlane(it.out_off);
  it.out_cap = __builtin_amdgcn_readfirstlane(it.out_cap);
  it.flags = __builtin_amdgcn_readfirstlane(it.flags);
  it.index = __builtin_amdgcn_readfirstlane(it.index);
  it.content_len = __builtin_amdgcn_readfirstlane(it.content_len);
  const int in_len = (int)it.in_len;
  const bool eof = it.flags & WF_EOF;
  const bool filt = it.flags & WF_FILTER;
  const bool emit = it.flags & WF_EMIT;
  const bool fresh = it.flags & WF_FRESH;
  // this workgroup writes the launch's backend templates of its index (first item of it)
  const bool pub = (it.flags & WF_PUBLISH) && btpl_wr != nullptr && it.index < (uint32_t)kBackendTpl;

  // ---- S0: load tile (16-B vector loads from host-mapped memory) -----------------
  if (tid * 16 < kSpecTile && tid * 16 < in_len) *(uint4*)&s.A[tid * 16] = spec;
  for (int i = kSpecTile + tid * 16; i < in_len; i += BS * 16) *(uint4*)&s.A[i] = *(const uint4*)&tile[i];
  if (tid == 0) {
    s.v[V_ABORT] = MAX_EV;
    s.v[V_LASTSEP] = -1;
    s.v[V_BAIL] = 0;
    s.v[V_STATUS] = 0;
    s.v[V_TPLK] = -1;
    s.v[V_NEXTEV] = 0;
    s.v[V_NFULL] = s.v[V_NTPL] = s.v[V_CFULL] = s.v[V_CTPL] = s.v[V_CLEX] = s.v[V_NHOLE] = s.v[V_CHOLE] = 0;
    s.v[V_HCLAIM] = 0;
    s.v[V_S4W] = 0;  // (s4_wave's "no candidates" mark: LDS outlives the previous item)
    s.v[V_S6W] = 0;
    for (int q = 0; q < BS / 64; ++q) wtpl[q][0] = -1;
    if (fresh) {
      s.v[V_DEPTH0] = 0;
      s.v[V_TAILLEN] = 0;
    } else {
      s.v[V_DEPTH0] = state[it.slot].depth;
      s.v[V_TAILLEN] = state[it.slot].tail_len;
    }
  }
  // Event shape template: the stream's own (earlier ticks), else its backend's — published
  // by any stream of the same backend index in this lane's previous launch (a fresh burst
  // of a new session then matches its content events at once instead of lexing the first
  // ones; a template is only ever a real parsed event's bytes around its content string,
  // and a match re-validates the string, so whose it is never changes a result)
  // Both candidates' lengths and bytes are requested at once, right after the work item: the
  // choice (own, else the backend's) is made when they are in registers — one dependent
  // round trip to device memory instead of three (lengths, then the other lengths, then bytes)
  const BackendTpl* bt = (btpl_rd != nullptr && it.index < (uint32_t)kBackendTpl) ? &btpl_rd[it.index] : nullptr;
  uint32_t st_pre = 0, st_suf = 0, b_pre = 0, b_suf = 0;
  uint4 st_w = make_uint4(0, 0, 0, 0), b_w = make_uint4(0, 0, 0, 0);
  if (!fresh) {
    st_pre = state[it.slot].tpl_pre;
    st_suf = state[it.slot].tpl_suf;
    if (tid < TPL_BYTES / 16) st_w = ((const uint4*)state[it.slot].tpl)[tid];
  }
  if (bt != nullptr) {
    b_pre = bt->pre;
    b_suf = bt->suf;
    if (tid < TPL_BYTES / 16) b_w = ((const uint4*)bt->tpl)[tid];
  }
  const bool own_tpl = !fresh && st_pre != 0;
  const bool borrow = !own_tpl && bt != nullptr && b_pre != 0;
  if (tid == 0) {
    s.v[V_TPLPRE] = own_tpl ? st_pre : borrow ? b_pre : 0;
    s.v[V_TPLSUF] = own_tpl ? st_suf : borrow ? b_suf : 0;
  }
  if (tid < TPL_BYTES / 16) {
    if (own_tpl) ((uint4*)s.tpl)[tid] = st_w;
    else if (borrow) ((uint4*)s.tpl)[tid] = b_w;
  }
  {  // the backend's hole templates (role / content / finish shapes of other streams)
    constexpr int kHW = (int)(sizeof(HoleTpl) * kHoleTpls / 16);
    static_assert(sizeof(HoleTpl) % 16 == 0, "HoleTpl copies as uint4");
    const bool have = btpl_rd != nullptr && it.index < (uint32_t)kBackendTpl;
    if (have) {
      for (int i = tid; i < kHW; i += BS) ((uint4*)U.htpl)[i] = ((const uint4*)btpl_rd[it.index].hole)[i];
    } else if (tid < kHoleTpls) {
      U.htpl[tid].len = 0;
    }
  }
  __syncthreads();
  QMX_STAMP(1);
  const int tail_len = filt ? s.v[V_TAILLEN] : 0;
  uint8_t* Z = s.B + PAD;
  {  // the holdback tail (<= kMaxTail = 64 bytes) by the last wave: wave 0 frames the tile next
    static_assert(kMaxTail <= 64, "one wave copies the tail");
    const int tt = tid - (BS - 64);
    if (tt >= 0 && tt < tail_len) Z[tt] = state[it.slot].tail[tt];
  }

  // ---- S1: leading whitespace at stream start ---------------------------------------
  // Every thread decides it from the tile's first bytes (broadcast LDS reads): no barrier to
  // publish one thread's answer.  (Fusing S1 into S2's one-wave framing measured no faster, r4/d.)
  int start = 0;
  bool wait = false;
  if (!(it.flags & WF_STARTED)) {
    while (start < in_len) {
      const int w = ws_at(s.A, start, in_len);
      if (w <= 0) break;
      start += w;
    }
    const bool undecided = start < in_len && ws_at(s.A, start, in_len) < 0;
    wait = start >= in_len || (undecided && !eof);
    if (!wait && tid == 0) s.v[V_STATUS] |= WS_STARTED;
  }
  if (wait) {  // (block-uniform)
    if (tid == 0) {
      if (fresh) {
        state[it.slot].depth = 0;
        state[it.slot].tail_len = 0;
        state[it.slot].tpl_pre = state[it.slot].tpl_suf = 0;
      }
      s.v[V_CONSUMED] = start;
      if (eof) s.v[V_STATUS] |= WS_DONE;
      WorkResult r{(uint32_t)start, 0u, (uint32_t)s.v[V_STATUS], it.content_len};
      res[bi] = r;
    }
    return;
  }
  QMX_STAMP(2);

  // ---- S2: framing -----------------------------------------------------------------
  // Common case (8-byte aligned start): each thread takes an 8-byte-multiple chunk with
  // ds_read_b64 loads and works on a 32-bit newline mask (SWAR byte compare) — byte loops
  // over stride-C chunks were bank-conflicted LDS reads, three passes over every byte.
  const int flen0 = in_len - start;
  const int C8 = (((flen0 + BS - 1) / BS) + 7) & ~7;
  const bool s2_wave_ok = (P.fast & 1) && (start & 7) == 0 && flen0 <= 4096;  // (two passes, 4.9 KB: 3.7 us vs the block path's 2.7, r4/i)
  if (s2_wave_ok) {
    if (tid < 64) s2_wave(s, start, in_len, eof);
  } else if ((start & 7) == 0 && C8 <= 32) {
    const int lo = min(start + tid * C8, in_len), hi = min(lo + C8, in_len);
    const int len = hi - lo;
    uint32_t nm = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q * 8 < len) {
        const uint64_t w = *(const uint64_t*)&s.A[lo + 8 * q];  // A has 64 B of padding
        const uint64_t x = w ^ 0x0a0a0a0a0a0a0a0aull;
        const uint64_t y = (((x & 0x7f7f7f7f7f7f7f7full) + 0x7f7f7f7f7f7f7f7full) | x) & 0x8080808080808080ull;
        const uint64_t zb = ~y & 0x8080808080808080ull;  // high bit of every '\n' byte
        nm |= (uint32_t)(((zb >> 7) * 0x0102040810204080ull) >> 56) << (8 * q);
      }
    }
    const uint32_t valid = len >= 32 ? 0xffffffffu : ((1u << len) - 1u);
    nm &= valid;
    // one-scan path: with no run of three or more newlines in the frame (SSE separates events
    // with exactly "\n\n"), a separator is a "\n\n" not preceded by '\n' — decided from the
    // chunk's mask and its neighbour bytes, no run scan.  Any triple newline (each is seen by
    // the thread whose chunk holds its first byte: two bytes of look-ahead) rides in the count
    // scan's total and sends the whole block down the run-scan path below (block-uniform).
    {
      const bool n1 = hi < in_len && s.A[hi] == '\n', n2 = hi + 1 < in_len && s.A[hi + 1] == '\n';
      const bool pnl = lo > start && s.A[lo - 1] == '\n';
      const uint64_t vm = len >= 32 ? 0xffffffffull : ((1ull << len) - 1ull);
      const uint64_t ext = (uint64_t)nm | ((uint64_t)n1 << len) | ((uint64_t)n2 << (len + 1));
      const uint64_t prevm = (ext << 1) | (pnl ? 1ull : 0ull);  // bit i: byte lo + i - 1 is '\n'
      const bool triple = (ext & (ext >> 1) & (ext >> 2) & vm) != 0;
      const uint64_t seps = ext & (ext >> 1) & ~prevm & vm;
      int tot1;
      int k = block_excl_sum<false>(__popcll(seps) + (triple ? (1 << 20) : 0), s.scr2, &tot1);
      if (tot1 < (1 << 20)) {  // (block-uniform)
        for (uint64_t m = seps; m; m &= m - 1) {
          const int p = lo + __ffsll((unsigned long long)m) - 1;
          if (k < MAX_EV) s.ev_b[k] = (uint16_t)p;
          if (k + 1 < MAX_EV) s.ev_a[k + 1] = (uint16_t)(p + 2);
          if (k == tot1 - 1) s.v[V_LASTSEP] = p;
          ++k;
        }
        if (tid == 0) {
          s.ev_a[0] = (uint16_t)start;
          s.v[V_NSEP] = tot1;
        }
        goto s2_framed;
      }
    }
    {
    const uint32_t inv = ~nm & valid;
    const bool all_nl = inv == 0;
    const int trail = all_nl ? len : len - 32 + __clz(inv);  // newlines at the chunk's end
    const bool next_nl = hi < in_len && s.A[hi] == '\n';
    int2 run = all_nl ? make_int2(1, len) : make_int2(0, trail);
    int2 tot2;
    // (no tail barriers: the count scan below uses scr2, and S2's barrier follows it)
    int2 ex = block_excl_pair<RunOp, false>(run, make_int2(1, 0), RunOp(), s.scr, &tot2);
    // separators: "\n" at an even position of its newline run, followed by a "\n"
    auto each_sep = [&](auto&& f) {
      uint32_t m = nm;
      while (m) {
        const int r0 = __ffs(m) - 1;
        const uint32_t rest = ~(m >> r0);
        const int L = rest == 0 ? 32 - r0 : __ffs(rest) - 1;  // run length in the chunk
        const int c = r0 == 0 ? ex.y : 0;                     // newlines just before it
        const bool ext = r0 + L == len && next_nl;            // the run continues past lo + len
        for (int i = 0; i < L; ++i)
          if (!((c + i) & 1) && (i + 1 < L || ext)) f(lo + r0 + i);
        m &= ~(L >= 32 ? 0xffffffffu : (((1u << L) - 1u) << r0));
      }
    };
    int cnt = 0;
    each_sep([&](int) { ++cnt; });
    int nsep;
    int k = block_excl_sum<false>(cnt, s.scr2, &nsep);
    each_sep([&](int p) {
      if (k < MAX_EV) s.ev_b[k] = (uint16_t)p;
      if (k + 1 < MAX_EV) s.ev_a[k + 1] = (uint16_t)(p + 2);
      if (k == nsep - 1) s.v[V_LASTSEP] = p;  // the last separator's writer (no LDS atomics)
      ++k;
    });
    if (tid == 0) {
      s.ev_a[0] = (uint16_t)start;
      s.v[V_NSEP] = nsep;
    }
    }
  s2_framed:;
  } else {
    int flen = in_len - start;
    int C = (flen + BS - 1) / BS;
    int lo = min(start + tid * C, in_len), hi = min(lo + C, in_len);
    const uint8_t* rd = s.A;  // independent byte reads pipeline (a cached-word reader measured slower)
    bool all_nl = true;
    int trail = 0;
    for (int p = lo; p < hi; ++p) {
      if (rd[p] == '\n') ++trail;
      else { trail = 0; all_nl = false; }
    }
    int2 run = all_nl ? make_int2(1, hi - lo) : make_int2(0, trail);
    int2 tot2;
    int2 ex = block_excl_pair(run, make_int2(1, 0), RunOp(), s.scr, &tot2);
    int r = ex.y;
    int cnt = 0;
    for (int p = lo; p < hi; ++p) {
      if (rd[p] == '\n') {
        if (!(r & 1) && p + 1 < in_len && rd[p + 1] == '\n') ++cnt;
        ++r;
      } else {
        r = 0;
      }
    }
    int nsep;
    int k = block_excl_sum(cnt, s.scr, &nsep);
    r = ex.y;
    for (int p = lo; p < hi; ++p) {
      if (rd[p] == '\n') {
        if (!(r & 1) && p + 1 < in_len && rd[p + 1] == '\n') {
          if (k < MAX_EV) s.ev_b[k] = (uint16_t)p;
          if (k + 1 < MAX_EV) s.ev_a[k + 1] = (uint16_t)(p + 2);
          if (k == nsep - 1) s.v[V_LASTSEP] = p;
          ++k;
        }
        ++r;
      } else {
        r = 0;
      }
    }
    if (tid == 0) {
      s.ev_a[0] = (uint16_t)start;
      s.v[V_NSEP] = nsep;
    }
  }
  __syncthreads();
  if (!s2_wave_ok) {  // (s2_wave finalises on its own lane 0)
    // every wave's lane 0 finalises (the same event list) and its wave reads it after a wave
    // fence — no second block barrier to publish one thread's answer
    if ((tid & 63) == 0) s2_finalize(s, start, in_len, eof, tid == 0);
    wave_fence();
  }
  QMX_STAMP(3);
  const int nev = s.v[V_NEV];

  // ---- S3: per-event extraction --------------------------------------------------------
  // Waves pull events from a shared counter (load balance: a few events need a full parse,
  // most only a template compare).  Per event, wave-wide: compare against the stream's shape
  // template (device state from earlier ticks) or any template published by a wave in this
  // tile; else the wave-cooperative lexer + wave grammar (publishing a template on success).
  // Lane 0 writes the result.  > 64 tokens → per-token walk; exotic → validating scalar
  // scanner (both by lane 0, rare) — exact either way.
  int packed_local[4];
  // S3a: content events of the stream's known shape (its own or its backend's template),
  // half a wave per event by static assignment, one 8-byte word per lane: the prefix and suffix
  // words compared with the template, the body bytes tested with SWAR for anything that would
  // need a real string scan ('"', '\\', control bytes, non-ASCII).  An event that passes has
  // the template's parse with an escape-free body — exactly wave_tpl_match + wave_str_body's
  // answer for it — at ~4 dependent LDS round trips instead of an atomic claim, two ballot
  // passes and LDS atomics per event.
  // S3a (b): in the same layout, the other shapes of a burst — "data: [DONE]" and the
  // backend's hole templates (role / finish events; wave_hole_exact + wave_hole_samelen's
  // test: literal bytes equal, string-hole bytes printable ASCII other than '"' and '\\',
  // number-hole bytes digits without a leading zero).  Everything else (0xFE / 0xFF) goes
  // through the loop below, which is skipped when nothing is left (V_UNRES).
  {
    // half a wave per event (32 lanes x 8 bytes: events up to 256 bytes), two per wave
    const int hw = tid >> 5, lane = tid & 31;
    const bool upper = (tid >> 5) & 1;
    const int tp = s.v[V_TPLPRE], ts = s.v[V_TPLSUF];
    const bool fast = (P.fast & 2) != 0;
    const uint64_t hi = 0x8080808080808080ull, one = 0x0101010101010101ull;
    auto half_clear = [upper](uint64_t m) { return (upper ? (m >> 32) : (m & 0xffffffffull)) == 0; };
    int newest = -1, nm = 0, nhole = 0, unres = 0;
    uint32_t hmatch = 0;
    // the hole templates' lengths, 0 for none / a kind S3a does not resolve (item-invariant)
    int hl[kHoleTpls];
#pragma unroll
    for (int qi = 0; qi < kHoleTpls; ++qi) {
      const HoleTpl& T = U.htpl[qi];
      hl[qi] = (T.kind == EV_CONTENT || T.kind == EV_SKIP) ? (int)T.len : 0;
    }
    // loop-invariant: this lane's template prefix word; the next round's event bounds are
    // read while this round's event is examined (one LDS round trip less per round)
    const uint64_t tw0 = ((const uint64_t*)s.tpl)[lane];  // (lane < 32: o < 256)
    int ne0 = hw < nev ? s.ev_a[hw] : 0, ne1 = hw < nev ? s.ev_b[hw] : 0;
    if (P.dbg != nullptr && tid == 0) dbg_put(&P.dbg[bi * kDbg + 35], __builtin_amdgcn_s_memrealtime());
    for (int kb = 0; kb < nev; kb += BS / 32) {
      if (P.dbg != nullptr && tid == 0 && kb == BS / 32) dbg_put(&P.dbg[bi * kDbg + 36], __builtin_amdgcn_s_memrealtime());
      const int k = kb + hw;
      const bool have = k < nev;
      const int e0 = ne0, e1 = ne1, L = e1 - e0;
      {
        const int kn = k + BS / 32;
        ne0 = kn < nev ? s.ev_a[kn] : 0;
        ne1 = kn < nev ? s.ev_b[kn] : 0;
      }
      const int o = lane * 8;
      const bool word = have && fast && L <= 256 && o < L;
      const int nb = min(8, L - o);
      const uint64_t valid = !word ? 0ull : nb == 8 ? ~0ull : ((1ull << (8 * nb)) - 1);
      const uint64_t ev = word ? lds_window8(s.A, e0 + o, e1) : 0ull;
      const uint64_t q = ev ^ 0x2222222222222222ull, b = ev ^ 0x5c5c5c5c5c5c5c5cull;
      // any '"', '\\', byte < 0x20 or >= 0x80 (the zero / less-than tricks only ever err
      // towards "bad", which just sends the event down the exact path)
      const uint64_t odd = (((q - one) & ~q) | ((b - one) & ~b) | ((ev - 0x20 * one) & ~ev) | ev) & hi;
      bool ok = have && fast && tp > 0 && L >= tp + ts && L <= 256;
      bool shape_bad = false;  // the prefix / suffix words differ (not just an odd body byte)
      {
        bool bad = false, sbad = false;
        if (ok && o < L) {
          const int pe = min(max(tp - o, 0), 8);  // prefix bytes of this word
          const uint64_t pmask = pe == 8 ? ~0ull : ((1ull << (8 * pe)) - 1);
          const int ss = (L - ts) - o;  // the suffix starts at byte ss of this word
          uint64_t smask = 0, sw = 0;
          if (ts > 0 && ss < 8) {
            const int s0 = max(ss, 0);
            smask = valid & ~(s0 == 0 ? 0ull : ((1ull << (8 * s0)) - 1));
            sw = ss >= 0 ? lds_window8(s.tpl + TPL_PRE_MAX, 0, ts) << (8 * ss)
                         : lds_window8(s.tpl + TPL_PRE_MAX, -ss, ts);
          }
          const uint64_t tw = pe > 0 ? tw0 : 0ull;
          const uint64_t bmask = valid & ~pmask & ~smask;
          sbad = ((ev ^ tw) & pmask) != 0 || ((ev ^ sw) & smask) != 0;
          bad = sbad || (odd & bmask) != 0;
        }
        const uint64_t bm = __ballot(bad), sm = __ballot(sbad);
        ok = ok && half_clear(bm);  // this half's lanes
        shape_bad = !half_clear(sm) || L < tp + ts;
      }
      // (b) the event's other possible shapes (block-uniform fast flag; ballots wave-wide)
      if (P.dbg != nullptr && tid == 0 && kb == 0) dbg_put(&P.dbg[bi * kDbg + 38], __builtin_amdgcn_s_memrealtime());
      const bool try_b = have && !ok && fast && L <= 256;
      bool done_ev = false;
      int hq = -1;
      // (wave-uniform: a wave whose two events both matched the content template — the bulk
      // of a burst — skips the whole section; S3a is VALU-bound with 8 waves on 4 SIMDs)
      if (fast && __ballot(try_b) != 0) {
        // each test only when some lane of the wave needs it (wave-uniform skips)
        if (__ballot(try_b && L == 12) != 0) {
          const bool dbad = !(try_b && L == 12) || (lane == 0 && ev != 0x445b203a61746164ull) ||  // "data: [D"
                            (lane == 1 && ev != 0x5d454e4full);                                    // "ONE]"
          done_ev = try_b && half_clear(__ballot(dbad));
        }
        // the templates are independent tests (no chain through the first match); the first
        // one whose half-wave is clear wins.  Usually one template has the event's length.
        uint32_t okm = 0;
#pragma unroll
        for (int qi = 0; qi < kHoleTpls; ++qi) {
          const bool cand = try_b && !done_ev && L > 0 && hl[qi] == L;
          if (__ballot(cand) == 0) continue;
          const HoleTpl& T = U.htpl[qi];
          bool bad = !cand;
          if (cand && o < L) {
            const uint32_t hm = T.wmask[lane];  // (lane < 32)
            const uint64_t tw = ((const uint64_t*)T.bytes)[lane];
            // DEL (0x7f) and number-hole digits, SWAR like `odd`; a byte '0' (the first byte of
            // a multi-digit number hole may not be one)
            const uint64_t dl = ev ^ 0x7f7f7f7f7f7f7f7full, x7 = ev & 0x7f7f7f7f7f7f7f7full;
            const uint64_t strbad = odd | (((dl - one) & ~dl) & hi);
            const uint64_t digit = ((x7 + 0x5050505050505050ull) & ~(x7 + 0x4646464646464646ull) & ~ev) & hi;
            const uint64_t z0 = ev ^ 0x3030303030303030ull, zero = ((z0 - one) & ~z0) & hi;
            const uint64_t smask = byte_mask8(hm & 0xffu), nmask = byte_mask8((hm >> 8) & 0xffu),
                           zmask = byte_mask8((hm >> 16) & 0xffu);
            const uint64_t lit = valid & ~(smask | nmask);
            bad = ((ev ^ tw) & lit) != 0 || (strbad & smask) != 0 || ((~digit & hi) & nmask) != 0 ||
                  (zero & zmask) != 0;
          }
          if (half_clear(__ballot(bad)) && cand) okm |= 1u << qi;
        }
        hq = done_ev || okm == 0 ? -1 : __ffs(okm) - 1;
      }
      if (P.dbg != nullptr && tid == 0 && kb == 0) dbg_put(&P.dbg[bi * kDbg + 39], __builtin_amdgcn_s_memrealtime());
      // unresolved: 0xFE when the stream template cannot match (its prefix / suffix differ:
      // the loop skips its own template compare), 0xFF otherwise (an escaped or non-ASCII
      // body the loop's exact string check may still accept, or no check ran)
      const bool examined = fast && tp > 0 && L <= 256 && shape_bad;
      int kind = -1, sa = 0, sb = 0;
      if (ok) {
        kind = EV_CONTENT;
        sa = e0 + tp;
        sb = e1 - ts;
      } else if (done_ev) {
        kind = EV_SKIP;
      } else if (hq >= 0) {
        const HoleTpl& T = U.htpl[hq];
        kind = T.kind;
        if (kind == EV_CONTENT) {
          sa = e0 + T.hs[T.target];
          sb = e0 + T.he[T.target];
        }
      }
      if (lane == 0 && have) {
        s.ev_kind[k] = kind >= 0 ? (uint8_t)kind : examined ? (uint8_t)0xFE : (uint8_t)0xFF;
        if (kind == EV_CONTENT) {
          s.ev_sa[k] = (uint16_t)sa;
          s.ev_sb[k] = (uint16_t)sb;
          s.ev_dl[k] = (uint16_t)(sb - sa);  // escape-free body (checked above)
        }
      }
      if (have && kind < 0) ++unres;
      if (hq >= 0 && !ok && !done_ev) {
        ++nhole;
        hmatch |= 1u << hq;
      }
      if (ok) ++nm;
      // the tile's newest content event (template or hole match) becomes the template
      if (kind == EV_CONTENT && sa - e0 <= TPL_PRE_MAX && e1 - sb <= TPL_SUF_MAX) newest = k;
    }
    if (P.dbg != nullptr && tid == 0) dbg_put(&P.dbg[bi * kDbg + 34], __builtin_amdgcn_s_memrealtime());
    // per wave, not per half-wave LDS atomics on shared words (32 of them serialised at the
    // LDS): the upper half's values come over by readlane, lane 0 stores the wave's slot
    {
      const int w = tid >> 6;
      const int unres2 = unres + __builtin_amdgcn_readlane(unres, 32);
      const int newest2 = max(newest, __builtin_amdgcn_readlane(newest, 32));
      const uint32_t hm2 = hmatch | (uint32_t)__builtin_amdgcn_readlane((int)hmatch, 32);
      if ((tid & 63) == 0) {
        U.s3w[w][0] = unres2;
        U.s3w[w][1] = (int)hm2;
        U.s3w[w][2] = newest2;
        if (P.dbg != nullptr) {  // (stage-timing counters)
          atomicAdd(&s.v[V_NTPL], nm + __builtin_amdgcn_readlane(nm, 32));
          atomicAdd(&s.v[V_NHOLE], nhole + __builtin_amdgcn_readlane(nhole, 32));
        }
      }
    }
  }
  __syncthreads();
  QMX_STAMP(21);
  // S3a's per-wave results: events left for the loop, hole templates matched, the newest
  // content event (block-uniform: read after the barrier)
  int unres_all = 0, newest_all = -1;
  {
    const int w = tid >> 6, lane = tid & 63;
    uint32_t hm_all = 0;
#pragma unroll
    for (int q = 0; q < BS / 64; ++q) {
      unres_all += U.s3w[q][0];
      hm_all |= (uint32_t)U.s3w[q][1];
      newest_all = max(newest_all, U.s3w[q][2]);
    }
    if (tid == 0 && newest_all >= 0) atomicMax(&s.v[V_TPLK], newest_all);
    if (P.dbg != nullptr && tid == 0) P.dbg[bi * kDbg + 37] = (unsigned long long)unres_all;  // (stage timing)
    // a hole template S3a matched is carried into the launch's write table (as the loop's
    // matches are, wave_hole_carry): wave w carries template w
    if (pub && w < kHoleTpls && ((hm_all >> w) & 1))
      wave_hole_carry(U.htpl[w], &btpl_wr[it.index].hole[w], w, &s.v[V_HCLAIM]);
    const bool loop = unres_all > 0;
    const LdsWords rd(s.A);
    const int tp = s.v[V_TPLPRE], ts = s.v[V_TPLSUF];
    bool published = false;
    int hint = w;  // template that matched last (tried first)
    int hhint = 0;  // hole template that matched last
    while (loop) {
      int g = 0;
      if (lane == 0) g = atomicAdd(&s.v[V_NEXTEV], 1);
      g = __builtin_amdgcn_readfirstlane(g);
      if (g >= nev) break;
      // pull order: the first 4 events, then the last 4 (a stream's closing events — finish
      // reason, usage, [DONE] — usually have their own shape and need a full parse), then the
      // middle, which by then matches a published template: the few full parses overlap.
      // (A compacted list of the events S3a left unresolved measured no faster: the claims
      // are not what this loop waits on.)
      const int k = nev <= 8 ? g : g < 4 ? g : g < 8 ? nev - 1 - (g - 4) : g - 4;
      const int k0 = s.ev_kind[k];
      if (k0 < 0xFE) continue;  // resolved by S3a
      const int e0 = s.ev_a[k], e1 = s.ev_b[k];
      int kind = EV_SKIP, sa = 0, sb = 0, body = -1;
      bool slow = false, lexed = false;
      int nt = 0;
      const bool probe = P.dbg != nullptr;
      const uint64_t c0 = probe ? __builtin_amdgcn_s_memtime() : 0;
      uint64_t c1 = 0;
      if (k0 == 0xFF && tp > 0 && e1 - e0 >= tp + ts && wave_tpl_match(s.A, e0, e1, s.tpl, tp, ts) &&
          (body = wave_str_body(s.A, e0 + tp, e1 - ts)) >= 0) {
        kind = EV_CONTENT;  // same shape as this stream's last parsed content event
        sa = e0 + tp;
        sb = e1 - ts;
        if (lane == 0) {
          atomicAdd(&s.v[V_NTPL], 1);
          // a matched event is as good a template as a parsed one: the tile's NEWEST content
          // event (parsed or matched) becomes the stream's and the backend's template — not
          // the newest parsed one, which in a burst is the odd-shaped first event (role +
          // empty content) and would make the next stream of this backend parse again
          atomicMax(&s.v[V_TPLK], k);
        }
      } else {
        // in-tile templates (this tile's parsed content shapes) — not for an event S3a already
        // found to differ from the stream's content shape (0xFE: a role / finish / usage
        // event, which the hole templates below resolve); skipping a try never changes a result
        for (int q = 0; q < BS / 64 && kind != EV_CONTENT && k0 == 0xFF; ++q) {
          const int qi = (hint + q) & (BS / 64 - 1);
          const int p0 = __atomic_load_n(&wtpl[qi][0], __ATOMIC_ACQUIRE);  // published last
          if (p0 < 0) continue;
          const int ttp = wtpl[qi][1], s0 = wtpl[qi][2], tts = wtpl[qi][3];
          if (e1 - e0 >= ttp + tts && wave_tpl_match_tile(s.A, e0, e1, p0, ttp, s0, tts) &&
              (body = wave_str_body(s.A, e0 + ttp, e1 - tts)) >= 0) {
            kind = EV_CONTENT;  // same shape as an event parsed earlier in this tile
            sa = e0 + ttp;
            sb = e1 - tts;
            hint = qi;
            if (lane == 0) {
              atomicAdd(&s.v[V_NTPL], 1);
              atomicMax(&s.v[V_TPLK], k);
            }
          }
        }
        if (probe) c1 = __builtin_amdgcn_s_memtime();
        if (kind != EV_CONTENT && lit_at(s.A, e0, e1, QMX_LIT("data: "))) {
          int a = e0 + 6, b = e1;
          ustrip(s.A, &a, &b);
          if (!(b - a == 6 && lit_at(s.A, a, b, QMX_LIT("[DONE]")))) {
            // a hole template of this backend (another stream's event of the same shape)?
            bool hm = false;
            const uint64_t ch0 = probe ? __builtin_amdgcn_s_memtime() : 0;
            // exact bytes first (one compare per same-length template), then the walks of
            // templates whose first / last literal runs fit
            for (int q = 0; q < 2 * kHoleTpls && !hm; ++q) {
              const int qi = (hhint + q) & (kHoleTpls - 1);
              const HoleTpl& T = U.htpl[qi];
              if (T.len == 0) continue;
              int ha = 0, hb = 0, hbody = 0;
              if (q < kHoleTpls ? !(wave_hole_exact(s.A, e0, e1, T, &ha, &hb, &hbody) ||
                                    wave_hole_samelen(s.A, e0, e1, T, &ha, &hb, &hbody))
                                : !(wave_hole_quick(s.A, e0, e1, T) && wave_hole_match(s.A, e0, e1, T, &ha, &hb, &hbody)))
                continue;
              hm = true;
              hhint = qi;
              kind = T.kind;
              if (pub) wave_hole_carry(T, &btpl_wr[it.index].hole[qi], qi, &s.v[V_HCLAIM]);
              if (kind == EV_CONTENT) {
                sa = ha;
                sb = hb;
                body = hbody;
              }
              if (lane == 0) atomicAdd(&s.v[V_NHOLE], 1);
              if (kind == EV_CONTENT && sa - e0 <= TPL_PRE_MAX && e1 - sb <= TPL_SUF_MAX) {
                if (lane == 0) {
                  if (!published) {  // as a parsed event: later events compare against this one
                    wtpl[w][1] = sa - e0;
                    wtpl[w][2] = sb;
                    wtpl[w][3] = e1 - sb;
                    __atomic_store_n(&wtpl[w][0], e0, __ATOMIC_RELEASE);
                  }
                  atomicMax(&s.v[V_TPLK], k);
                }
                published = true;
              }
            }
            if (probe && lane == 0) atomicAdd(&s.v[V_CHOLE], (int)(__builtin_amdgcn_s_memtime() - ch0));
            if (!hm) {
              const uint64_t cl0 = probe ? __builtin_amdgcn_s_memtime() : 0;
              nt = wave_lex(s.A, a, b, TKP[w], TKT[w], 0, TOK_CAP);
              if (probe && lane == 0) atomicAdd(&s.v[V_CLEX], (int)(__builtin_amdgcn_s_memtime() - cl0));
              if (lane == 0) atomicAdd(&s.v[V_NFULL], 1);
              if (nt == -LEX_COMPLEX) {
                slow = true;
              } else if (nt > 64) {
                lexed = true;
              } else if (nt >= 0) {
                EvResult r;
                bool esc = true;
                uint64_t vopen = 0;
                const int g = wave_grammar(TKP[w], TKT[w], 0, nt, r, &esc, &vopen);
                if (g == LEX_COMPLEX) {
                  slow = true;
                } else if (g == LEX_OK) {
                  kind = r.kind;
                  sa = r.str_a;
                  sb = r.str_b;
                  body = esc ? 1 : 0;
                  if (kind == EV_CONTENT && sa - e0 <= TPL_PRE_MAX && e1 - sb <= TPL_SUF_MAX && lane == 0) {
                    if (!published) {  // later events (any wave) compare against this one
                      wtpl[w][1] = sa - e0;
                      wtpl[w][2] = sb;
                      wtpl[w][3] = e1 - sb;
                      __atomic_store_n(&wtpl[w][0], e0, __ATOMIC_RELEASE);
                    }
                    atomicMax(&s.v[V_TPLK], k);  // newest parsed content → device template
                  }
                  if (kind == EV_CONTENT && sa - e0 <= TPL_PRE_MAX && e1 - sb <= TPL_SUF_MAX) published = true;
                  // its hole template for the next launch: other streams' events of this shape
                  // (ids / timestamps / text differ) then skip the full parse
                  if ((kind == EV_CONTENT || kind == EV_SKIP) && e1 - e0 <= kHoleTplBytes && pub)
                    wave_hole_publish(s.A, e0, e1, TKP[w], TKT[w], nt, vopen, kind, sa, esc, btpl_wr[it.index].hole,
                                      &s.v[V_HCLAIM]);
                }
              }
            }
          }
        }
      }
      if (probe && lane == 0) {
        const uint64_t c2 = __builtin_amdgcn_s_memtime();
        if (c1) {
          atomicAdd(&s.v[V_CTPL], (int)(c1 - c0));
          atomicAdd(&s.v[V_CFULL], (int)(c2 - c1));
        } else {
          atomicAdd(&s.v[V_CTPL], (int)(c2 - c0));
        }
      }
      if (lane == 0) {
        EvResult r;
        r.kind = kind;
        r.str_a = sa;
        r.str_b = sb;
        if (lexed) {  // long token list: the per-token walk
          const int g = token_grammar(TKP[w], TKT[w], 0, nt, r);
          if (g == LEX_INVALID) r.kind = EV_SKIP;
          else if (g == LEX_COMPLEX) slow = true;
          body = 1;
        }
        if (slow) {  // rare shapes: the validating scalar scanner
          r = classify_event_at(rd, e0, e1 - e0);
          r.str_a += e0;
          r.str_b += e0;
          body = 1;
        }
        if ((lexed || slow) && r.kind == EV_CONTENT && r.str_a - e0 <= TPL_PRE_MAX && e1 - r.str_b <= TPL_SUF_MAX)
          atomicMax(&s.v[V_TPLK], k);
        s.ev_kind[k] = (uint8_t)r.kind;
        if (r.kind == EV_CONTENT) {
          s.ev_sa[k] = (uint16_t)r.str_a;
          s.ev_sb[k] = (uint16_t)r.str_b;
          s.ev_dl[k] = (uint16_t)(body == 0 ? r.str_b - r.str_a : json_unescape(rd, r.str_a, r.str_b, nullptr));
        } else if (r.kind == EV_ABORT) {
          atomicMin(&s.v[V_ABORT], k);
        }
      }
    }
  }
  // the loop's results (event kinds, V_TPLK) need a barrier; without the loop every thread
  // already has the newest content event, and S3a's writes were published by its barrier
  if (unres_all > 0) __syncthreads();
  QMX_STAMP(22);
  // persist the newest template now (S4 reuses the input tile) — on waves 4-7: wave 0 goes on
  // to the content placement (its reads of ev_a / ev_sa / ev_b / ev_sb and of A are not
  // written before the placement's barrier, which every wave passes after this)
  if (tid >= BS - TPL_PRE_MAX) {
    static_assert(TPL_PRE_MAX <= BS && TPL_BYTES / 16 <= TPL_PRE_MAX, "template persist threads");
    const int pt = tid - (BS - TPL_PRE_MAX);
    const int tk = unres_all > 0 ? s.v[V_TPLK] : newest_all;
    if (tk >= 0) {
      const int e0 = s.ev_a[tk], pre = s.ev_sa[tk] - e0, e1 = s.ev_b[tk], suf = e1 - s.ev_sb[tk];
      DevSlot& ds = state[it.slot];
      if (pt < pre) ds.tpl[pt] = s.A[e0 + pt];
      if (pt < suf) ds.tpl[TPL_PRE_MAX + pt] = s.A[e1 - suf + pt];
      if (pt == 0) {
        ds.tpl_pre = (uint16_t)pre;
        ds.tpl_suf = (uint16_t)suf;
      }
      // publish it for this backend index: the launch's publishing workgroup of that index
      // (WF_PUBLISH, picked by the host) writes it; the lane's next launch reads it (a kernel
      // boundary in between).  No claim: a global atomic here cost every item a round trip.
      if (pub) {
        BackendTpl& bw = btpl_wr[it.index];
        if (pt < pre) bw.tpl[pt] = s.A[e0 + pt];
        if (pt < suf) bw.tpl[TPL_PRE_MAX + pt] = s.A[e1 - suf + pt];
        if (pt == 0) {
          bw.pre = (uint16_t)pre;
          bw.suf = (uint16_t)suf;
        }
      }
    } else if (borrow) {  // keep the backend's template as the stream's own
      DevSlot& ds = state[it.slot];
      if (pt < TPL_BYTES / 16) ((uint4*)ds.tpl)[pt] = ((const uint4*)s.tpl)[pt];
      if (pt == 0) {
        ds.tpl_pre = (uint16_t)s.v[V_TPLPRE];
        ds.tpl_suf = (uint16_t)s.v[V_TPLSUF];
      }
    } else if (fresh && pt == 0) {
      state[it.slot].tpl_pre = state[it.slot].tpl_suf = 0;
    }
  }
  QMX_STAMP(4);
  const int kab = s.v[V_ABORT];
  {
    // each content event's delta index and offset in Z (a prefix sum of (1, escaped length)
    // pairs); unescaped bodies are written here, escape-free ones copied below by waves.  The
    // copy offset replaces the event's ev_dl (read here by the same thread, by nobody after),
    // not its ev_a: other waves may still be reading ev_a in the template persist above
    // (the one-wave path has no block barrier in between)
    auto place = [&](int k, int pre) {
      const int j = pre >> 16, doff = pre & 0xFFFF;
      const int dl = s.ev_dl[k];
      s.dl_end[j] = (uint16_t)(tail_len + doff + dl);
      if (dl == s.ev_sb[k] - s.ev_sa[k]) {  // escape-free (every escape shrinks): copied below
        s.ev_dl[k] = (uint16_t)doff;
      } else {
        json_unescape(LdsWords(s.A), s.ev_sa[k], s.ev_sb[k], Z + tail_len + doff);
        s.ev_dl[k] = 0xFFFF;
      }
    };
    int tot = 0;
    if (nev <= 64) {
      // the common tile: wave 0, an event per lane, one DPP scan — no block scan barrier
      if (tid < 64) {
        const int k = tid;
        const bool c = k < nev && k < kab && s.ev_kind[k] == EV_CONTENT;
        const int pk = c ? ((1 << 16) | (int)s.ev_dl[k]) : 0;
        const int incl = wave_incl_sum(pk);
        tot = wave_last(incl);
        if (c) place(k, incl - pk);
        else if (k < nev) s.ev_dl[k] = 0xFFFF;
      }
    } else {
      int loc = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int k = tid * 4 + i;
        int pk = 0;
        if (k < nev && k < kab && s.ev_kind[k] == EV_CONTENT) pk = (1 << 16) | s.ev_dl[k];
        packed_local[i] = loc;
        loc += pk;
      }
      int base = block_excl_sum<false>(loc, s.scr, &tot);  // (the barrier below follows)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int k = tid * 4 + i;
        if (k < nev && k < kab && s.ev_kind[k] == EV_CONTENT) place(k, base + packed_local[i]);
        else if (k < nev) s.ev_dl[k] = 0xFFFF;
      }
    }
    __syncthreads();
    {  // escape-free contents: one wave per event, 64 bytes per step; each lane fetches one
       // of its wave's events' (offset, start, length) up front (nev <= MAX_EV = 8 x 64), so
       // an event costs no dependent LDS read but its bytes'
      const int w = tid >> 6, lane = tid & 63;
      const int kl = w + (BS / 64) * lane;
      int off_l = 0xFFFF, sa_l = 0, n_l = 0;
      if (kl < nev) {
        off_l = s.ev_dl[kl];
        if (off_l != 0xFFFF) {
          sa_l = s.ev_sa[kl];
          n_l = s.ev_sb[kl] - sa_l;
        }
      }
      for (int i = 0; w + (BS / 64) * i < nev; ++i) {
        const int off = __builtin_amdgcn_readlane(off_l, i);
        if (off == 0xFFFF) continue;
        const int sa = __builtin_amdgcn_readlane(sa_l, i), n = __builtin_amdgcn_readlane(n_l, i);
        for (int x = lane; x < n; x += 64) Z[tail_len + off + x] = s.A[sa + x];
      }
    }
    if (tid == 0) {
      s.v[V_NDELTA] = tot >> 16;
      s.v[V_YLEN] = tot & 0xFFFF;
      if (kab < MAX_EV && kab < nev) {
        s.v[V_STATUS] = (s.v[V_STATUS] | WS_ABORTED) & ~(WS_DONE | WS_MORE);
        s.v[V_CONSUMED] = in_len;
      }
    }
  }
  __syncthreads();
  const int ndelta = s.v[V_NDELTA];
  const int Zn = tail_len + s.v[V_YLEN];
  const int depth0 = s.v[V_DEPTH0];
  QMX_STAMP(5);

  // ---- S4: think filter ----------------------------------------------------------------
  const uint8_t* W = Z;  // identity when not filtering
  int ncand = 0, ntok = 0;
  bool s4_done = false;
  const bool env_ready = (P.fast & 4) && filt && ndelta > 0 && Zn <= 2048 && ndelta <= 64 && emit;
  if ((P.fast & 4) && filt && ndelta > 0 && Zn <= 2048 && ndelta <= 64) {  // the common tile: one wave (s4_wave)
    if (tid >= 64 && env_ready) {
      // the idle waves: the item's envelope bytes, assembled off the fill's path
      const int b = tid - 64, ix = (int)it.index, p1 = P.pre1_len;
      const int nd = ix >= 100 ? 3 : ix >= 10 ? 2 : 1, pre = p1 + nd + P.pre2_len;
      if (b < pre) {
        const int d = b - p1, q = nd - 1 - d;  // index digit, most significant first
        const int dv = q == 2 ? ix / 100 : q == 1 ? (ix / 10) % 10 : ix % 10;
        s.env[b] = b < p1 ? (uint8_t)P.pre1[b] : d < nd ? (uint8_t)('0' + dv) : (uint8_t)P.pre2[d - nd];
      }
      if (b < P.suf_len) s.env[256 + b] = (uint8_t)P.suf[b];
    }
    if (tid < 64) {
      const bool ok = s4_wave(s, Z, Zn, ndelta, depth0, P, P.dbg != nullptr ? P.dbg + bi * kDbg : nullptr);
      if (tid == 0 && s.v[V_S4W] != 2) s.v[V_S4W] = ok ? 1 : 0;  // (2: no candidates, W = Z)
      // the sizing on the same wave at once (the filter's own results: no barrier between)
      wave_fence();
      const int wl = __builtin_amdgcn_readfirstlane(s.v[V_WLEN]);
      if (ok && (P.fast & 8) && emit && wl <= 2048) {
        s6_size_wave(s, s.v[V_S4W] == 2 ? Z : s.A, wl, ndelta);
        if (tid == 0) s.v[V_S6W] = 1;
        if (P.dbg != nullptr && tid == 0) dbg_put(&P.dbg[bi * kDbg + 33], __builtin_amdgcn_s_memrealtime());
      }
    }
    __syncthreads();
    if (s.v[V_S4W]) {
      s4_done = true;
      W = s.v[V_S4W] == 2 ? Z : s.A;
    }
  }
  if (filt && ndelta > 0 && !s4_done) {
    // candidates: per-thread 8-byte-multiple chunks of Z (16-B aligned) as ds_read_b64
    // words, a 32-bit '<' mask per thread (SWAR compare), popcount + ordered compaction
    {
      const int C8 = (((Zn + BS - 1) / BS) + 7) & ~7;
      int cnt = 0, tot;
      if (C8 <= 32) {
        const int lo = min(tid * C8, Zn), hi = min(lo + C8, Zn), len = hi - lo;
        uint32_t lm = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (q * 8 < len) {
            const uint64_t w = *(const uint64_t*)&Z[lo + 8 * q];  // B has >= 48 B past Zn
            const uint64_t x = w ^ 0x3c3c3c3c3c3c3c3cull;
            const uint64_t y = (((x & 0x7f7f7f7f7f7f7f7full) + 0x7f7f7f7f7f7f7f7full) | x) & 0x8080808080808080ull;
            const uint64_t zb = ~y & 0x8080808080808080ull;
            lm |= (uint32_t)(((zb >> 7) * 0x0102040810204080ull) >> 56) << (8 * q);
          }
        }
        lm &= len >= 32 ? 0xffffffffu : ((1u << len) - 1u);
        cnt = __popc(lm);
        int k = block_excl_sum(cnt, s.scr, &tot);
        if (tot <= MAX_CAND)
          for (uint32_t m = lm; m; m &= m - 1) s.cand[k++] = (uint16_t)(lo + __ffs(m) - 1);
      } else {
        const int C = (Zn + BS - 1) / BS;
        const int lo = min(tid * C, Zn), hi = min(lo + C, Zn);
        for (int p = lo; p < hi; ++p) cnt += Z[p] == '<';
        int k = block_excl_sum(cnt, s.scr, &tot);
        if (tot <= MAX_CAND)
          for (int p = lo; p < hi; ++p)
            if (Z[p] == '<') s.cand[k++] = (uint16_t)p;
      }
      ncand = tot;
    }
  }
  if (s4_done) {
    // s4_wave wrote cut / wpos / V_WLEN / V_NEWTAIL / V_NEWDEPTH
  } else if (filt && ndelta > 0 && ncand == 0) {  // no '<' anywhere in Z (old holdback tail + new deltas)
    // no tag can start in these bytes (and no holdback is pending: a held tail starts with
    // '<'): outside a think block every byte is kept, inside one every byte is dropped
    const bool keep = depth0 == 0;
    for (int j = tid; j < ndelta; j += BS) {
      s.cut[j] = s.dl_end[j];
      s.wpos[j] = keep ? s.dl_end[j] : 0;
    }
    if (tid == 0) {
      s.v[V_WLEN] = keep ? Zn : 0;
      s.v[V_NEWTAIL] = -1;
      s.v[V_NEWDEPTH] = depth0;
    }
  } else if (filt && ndelta > 0) {
    if (ncand > MAX_CAND) {
      if (tid == 0) {
        WorkResult r{0u, 0u, (uint32_t)WS_ESCALATE, it.content_len};
        res[bi] = r;
      }
      return;  // uniform: every thread saw the same total
    }
    for (int c = tid; c < ncand; c += BS) s.cand_tok[c] = 0;
    __syncthreads();
    {
      const v4i bf0 = build_pattern_frag(P, 0), bf1 = build_pattern_frag(P, P.npat > 16 ? 1 : 0);
      int w = tid >> 6;
      for (int g = w; g * 16 < ncand; g += BS / 64) mfma_match_group(Z, Zn, s.cand, ncand, g, P, bf0, bf1, s.cand_tok);
    }
    __syncthreads();
    QMX_STAMP(6);
    if (ncand <= 64) {
      // common case (a few '<' in the tile): wave 0 alone compacts the tokens by ballot and
      // runs the depth scan with wave shuffles — one barrier instead of five.  Candidates
      // are in position order and non-tokens are the scan identity (0,0), so the lane-order
      // exclusive prefix at a token lane is its depth before the token.
      if (tid < 64) {
        const int lane = tid;
        const int id = lane < ncand ? (int)s.cand_tok[lane] : 0;
        const uint64_t m = __ballot(id != 0);
        const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
        const int k = __popcll(m & below);
        DepthOp op;
        int2 x = id > 0 ? make_int2(1, 1) : id < 0 ? make_int2(-1, 0) : make_int2(0, 0);
        x = wave_incl_pair(x, op);
        const int2 ex = make_int2(wave_prev(x.x, 0), wave_prev(x.y, 0));
        if (id != 0) {
          s.tok_pos[k] = s.cand[lane];
          s.tok_id[k] = (int8_t)id;
          s.tok_len[k] = (uint8_t)tok_plen(P, id);
          s.tok_dep[k] = (int16_t)max(depth0 + ex.x, ex.y);
        }
        if (lane == 63) {
          const int nt = __popcll(m);
          s.v[V_NTOK] = nt;
          s.tok_dep[nt] = (int16_t)max(depth0 + x.x, x.y);
        }
      }
      __syncthreads();
      ntok = s.v[V_NTOK];
    } else {
      // token compaction (4 candidates per thread)
      {
        int loc = 0, flags[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          int c = tid * 4 + i;
          flags[i] = loc;
          loc += (c < ncand && s.cand_tok[c] != 0) ? 1 : 0;
        }
        int tot;
        int base = block_excl_sum(loc, s.scr, &tot);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          int c = tid * 4 + i;
          if (c < ncand && s.cand_tok[c] != 0) {
            int k = base + flags[i];
            int id = s.cand_tok[c];
            s.tok_pos[k] = s.cand[c];
            s.tok_id[k] = (int8_t)id;
            s.tok_len[k] = (uint8_t)tok_plen(P, id);
          }
        }
        ntok = tot;
      }
      __syncthreads();
      // depth scan over tokens: open (1,1), close (-1,0)
      {
        int2 loc = make_int2(0, 0);
        int2 pre[4];
        DepthOp op;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          int k = tid * 4 + i;
          pre[i] = loc;
          if (k < ntok) loc = op(loc, s.tok_id[k] > 0 ? make_int2(1, 1) : make_int2(-1, 0));
        }
        int2 tot;
        int2 base = block_excl_pair(loc, make_int2(0, 0), op, s.scr, &tot);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          int k = tid * 4 + i;
          if (k < ntok) {
            int2 f = op(base, pre[i]);
            s.tok_dep[k] = (int16_t)max(depth0 + f.x, f.y);
          }
        }
        if (tid == 0) s.tok_dep[ntok] = (int16_t)max(depth0 + tot.x, tot.y);
      }
      __syncthreads();
    }
    // cuts per delta + new tail
    for (int j = tid; j < ndelta; j += BS) {
      int q;
      s.cut[j] = (uint16_t)hold_cut(s, Z, ncand, ntok, s.dl_end[j], P, false, &q);
    }
    if (tid == 0) {
      int q;
      hold_cut(s, Z, ncand, ntok, Zn, P, true, &q);
      s.v[V_NEWTAIL] = q;
      s.v[V_NEWDEPTH] = s.tok_dep[ntok];
    }
    __syncthreads();
    // compaction of kept bytes in [0, cutN) into W (= A; input tile no longer needed)
    {
      const int cutN = s.cut[ndelta - 1];
      int C = (cutN + BS - 1) / BS;
      int lo = min(tid * C, cutN), hi = min(lo + C, cutN);
      int k = tok_upper(s, ntok, lo);
      int cnt = 0;
      for (int x = lo; x < hi; ++x) {
        while (k < ntok && (int)s.tok_pos[k] <= x) ++k;
        cnt += kept_at(s, k, x);
      }
      int tot;
      int base = block_excl_sum(cnt, s.scr, &tot);
      s.chunk_base[tid] = base;
      if (tid == 0) {
        s.chunk_base[BS] = tot;
        s.v[V_WLEN] = tot;
      }
      k = tok_upper(s, ntok, lo);
      int o = base;
      for (int x = lo; x < hi; ++x) {
        while (k < ntok && (int)s.tok_pos[k] <= x) ++k;
        if (kept_at(s, k, x)) s.A[o++] = Z[x];
      }
      __syncthreads();
      for (int j = tid; j < ndelta; j += BS) {
        int c = s.cut[j];
        if (c >= cutN) {
          s.wpos[j] = (uint16_t)s.chunk_base[BS];
          continue;
        }
        int t = C > 0 ? c / C : 0;
        int tlo = min(t * C, cutN);
        int kk = tok_upper(s, ntok, tlo);
        int cc = s.chunk_base[t];
        for (int x = tlo; x < c; ++x) {
          while (kk < ntok && (int)s.tok_pos[kk] <= x) ++kk;
          cc += kept_at(s, kk, x);
        }
        s.wpos[j] = (uint16_t)cc;
      }
    }
    W = s.A;
  } else {
    for (int j = tid; j < ndelta; j += BS) {
      s.cut[j] = s.dl_end[j];
      s.wpos[j] = s.dl_end[j];  // tail_len == 0 when not filtering
    }
    if (tid == 0) {
      s.v[V_WLEN] = ndelta > 0 ? Zn : 0;
      s.v[V_NEWTAIL] = -1;
      s.v[V_NEWDEPTH] = depth0;
    }
  }
  __syncthreads();
  QMX_STAMP(7);
  const int Wlen = s.v[V_WLEN];

  // ---- S6 (sizing): emitted deltas, escaped lengths -------------------------------------
  int n_emit = 0, etot = 0;
  bool s6_wave = false;  // sizing ran on wave 0: 64 escaped-content chunks instead of BS
  const int ndig = it.index >= 100 ? 3 : it.index >= 10 ? 2 : 1;
  const int PRE = P.pre1_len + ndig + P.pre2_len, SUF = P.suf_len, EVL = PRE + SUF;
  if (s.v[V_S6W]) {  // sized by wave 0 right after the one-wave filter
    n_emit = s.v[V_NEMIT];
    etot = s.v[V_ETOT];
    s6_wave = true;
  } else if ((P.fast & 8) && emit && ndelta > 0 && ndelta <= 64 && Wlen <= 2048) {
    // the common tile on wave 0 alone (s6_size_wave), then one barrier for the block
    if (tid < 64 && !s.v[V_S6W]) s6_size_wave(s, W, Wlen, ndelta);
    __syncthreads();
    n_emit = s.v[V_NEMIT];
    etot = s.v[V_ETOT];
    s6_wave = true;
  } else if (emit && ndelta > 0) {
    {
      int loc = 0, pre[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int j = tid * 4 + i;
        pre[i] = loc;
        if (j < ndelta) loc += (s.wpos[j] > (j ? s.wpos[j - 1] : 0)) ? 1 : 0;
      }
      int tot;
      int base = block_excl_sum(loc, s.scr, &tot);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int j = tid * 4 + i;
        if (j < ndelta) {
          s.eidx[j] = (uint16_t)(base + pre[i]);
          if (s.wpos[j] > (j ? s.wpos[j - 1] : 0)) s.ejx[base + pre[i]] = (uint16_t)j;
        }
      }
      n_emit = tot;
    }
    {
      int C = (Wlen + BS - 1) / BS;
      int lo = min(tid * C, Wlen), hi = min(lo + C, Wlen);
      int x = lo;
      while (x < hi && is_cont(W[x])) ++x;
      int e = 0;
      while (x < hi) {
        uint32_t cp;
        x += wtf8_decode(W, x, Wlen, &cp);
        e += escaped_len_cp(cp);
      }
      int base = block_excl_sum(e, s.scr, &etot);
      s.chunk_base[tid] = base;
      __syncthreads();
      for (int j = tid; j < ndelta; j += BS) {
        int wp = s.wpos[j];
        if (wp >= Wlen) {
          s.epos[j] = (uint32_t)etot;
          continue;
        }
        int t = C > 0 ? wp / C : 0;
        int tlo = min(t * C, Wlen);
        int xx = tlo;
        while (xx < wp && is_cont(W[xx])) ++xx;
        int ee = s.chunk_base[t];
        while (xx < wp) {
          uint32_t cp;
          xx += wtf8_decode(W, xx, Wlen, &cp);
          ee += escaped_len_cp(cp);
        }
        s.epos[j] = (uint32_t)ee;
      }
    }
    __syncthreads();
  }
  QMX_STAMP(8);
  const int out_len = emit ? n_emit * EVL + etot : 0;
  const uint32_t new_clen = it.content_len + (uint32_t)Wlen;
  if ((uint32_t)out_len > it.out_cap || new_clen > P.content_cap) {
    if (tid == 0) {
      WorkResult r{0u, 0u, (uint32_t)WS_ESCALATE, it.content_len};
      res[bi] = r;
    }
    return;
  }

  // ---- S5: commit content + state ---------------------------------------------------
  {
    uint8_t* dst = content + (size_t)it.slot * P.content_cap + it.content_len;
    for (int x = tid; x < Wlen; x += BS) dst[x] = W[x];
  }
  if (filt) {
    int q = s.v[V_NEWTAIL];
    int tl = (ndelta > 0) ? (q >= 0 ? Zn - q : 0) : tail_len;
    if (tid < tl) state[it.slot].tail[tid] = ndelta > 0 ? Z[q + tid] : Z[tid];
    if (tid == 0) {
      state[it.slot].tail_len = tl;
      state[it.slot].depth = ndelta > 0 ? s.v[V_NEWDEPTH] : depth0;
    }
  } else if (fresh && tid == 0) {
    state[it.slot].tail_len = 0;
    state[it.slot].depth = 0;
  }
  __syncthreads();
  QMX_STAMP(9);

  // ---- S6 (write): SSE events through an LDS window, 16-B stores to host memory ------
  if (out_len > 0) {
    // output window: whichever tile buffer does not hold W (Z's tail is already committed)
    uint8_t* O = (W == s.A) ? s.B : s.A;
    const int WIN = TILE_MAX;
    // the sizing's chunking (chunk_base): per thread, or per lane of wave 0 (s6_wave; the
    // other threads' chunks then start at Wlen and are empty)
    const int C = s6_wave ? (Wlen + 63) / 64 : (Wlen + BS - 1) / BS;
    // clean content (every code point escapes to itself, so etot == Wlen): escaped offsets
    // are raw offsets, and one wave per emitted event writes its envelope prefix, its content
    // bytes and its suffix, 64 bytes per store instruction (no division, no per-byte branch
    // or search, all waves busy; the general path below runs the content on wave 0 alone)
    const bool clean = etot == Wlen && out_len <= WIN;
    for (int w0 = 0; w0 < out_len; w0 += WIN) {
      const int w1 = min(w0 + WIN, out_len);
      if (clean) {
        const int ix = (int)it.index;
        const int p1 = P.pre1_len, wave = tid >> 6, lane = tid & 63;
        // the envelope bytes are the same for every event of the item (one backend index):
        // each lane holds its prefix bytes lane + 64r (PRE <= 227: r < 4) and suffix byte
        // (SUF <= 48) in registers, read once — the per-event copies then store without
        // reading P; and each lane fetches one event's (start, length) for its wave up front
        // (n_emit <= MAX_EV = 8 waves x 64 lanes), so an event costs no dependent LDS read
        // but its content bytes'
        static_assert(sizeof(P.pre1) + 3 + sizeof(P.pre2) <= 256 && sizeof(P.suf) <= 64 && MAX_EV <= BS,
                      "envelope bytes per lane / events per wave lane");
        uint32_t pw = 0;
        uint8_t sch = 0;
        if (env_ready) {  // staged in LDS during the filter
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (lane + 64 * r < PRE) pw |= (uint32_t)s.env[lane + 64 * r] << (8 * r);
          sch = lane < SUF ? s.env[256 + lane] : 0;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int b = lane + 64 * r;
            if (b < PRE) {
              const int d = b - p1, q = ndig - 1 - d;  // index digit, most significant first
              const int dv = q == 2 ? ix / 100 : q == 1 ? (ix / 10) % 10 : ix % 10;
              const uint32_t ch = b < p1 ? (uint8_t)P.pre1[b] : d < ndig ? (uint8_t)('0' + dv) : (uint8_t)P.pre2[d - ndig];
              pw |= ch << (8 * r);
            }
          }
          sch = lane < SUF ? (uint8_t)P.suf[lane] : 0;
        }
        const int kl = wave + (BS / 64) * lane;
        int cs_l = 0, cl_l = 0;
        if (kl < n_emit) {
          const int j = s.ejx[kl];
          cs_l = j ? (int)s.wpos[j - 1] : 0;
          cl_l = (int)s.wpos[j] - cs_l;
        }
        for (int i = 0; wave + (BS / 64) * i < n_emit; ++i) {
          const int k = wave + (BS / 64) * i;
          const int cs = __builtin_amdgcn_readlane(cs_l, i), cl = __builtin_amdgcn_readlane(cl_l, i);
          uint8_t* ev = O + k * EVL + cs;  // the event's start: k envelopes + earlier content
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (lane + 64 * r < PRE) ev[lane + 64 * r] = (uint8_t)(pw >> (8 * r));
          for (int b = lane; b < cl; b += 64) ev[PRE + b] = W[cs + b];
          if (lane < SUF) ev[PRE + cl + lane] = sch;
        }
      } else {
      // envelopes: fully parallel over (emitted event, envelope byte)
      {
        // the index digits, most significant first, as registers (a local array indexed by
        // a loop variable lands in scratch)
        const int ix = (int)it.index;
        const uint32_t dg_packed = ndig == 1 ? (uint32_t)('0' + ix)
                                 : ndig == 2 ? (uint32_t)('0' + ix / 10) | ((uint32_t)('0' + ix % 10) << 8)
                                             : (uint32_t)('0' + ix / 100) | ((uint32_t)('0' + (ix / 10) % 10) << 8) |
                                                   ((uint32_t)('0' + ix % 10) << 16);
        // 8 envelope bytes per thread: one division, one ejx / epos lookup per 8 bytes
        const int CPE = (EVL + 7) >> 3;  // chunks per event
        for (int idx = tid; idx < n_emit * CPE; idx += BS) {
          const int k = idx / CPE, b0 = (idx - k * CPE) * 8;
          const int j = s.ejx[k];
          const int opre = k * EVL + (j ? (int)s.epos[j - 1] : 0);  // the event's start
          const int osuf = k * EVL + PRE + (int)s.epos[j] - PRE;    // + bpos for suffix bytes
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const int bpos = b0 + q;
            if (bpos >= EVL) break;
            int o;
            uint8_t ch;
            if (bpos < PRE) {
              o = opre + bpos;
              ch = bpos < P.pre1_len ? (uint8_t)P.pre1[bpos]
                   : bpos < P.pre1_len + ndig ? (uint8_t)(dg_packed >> (8 * (bpos - P.pre1_len)))
                                              : (uint8_t)P.pre2[bpos - P.pre1_len - ndig];
            } else {
              o = osuf + bpos;
              ch = (uint8_t)P.suf[bpos - PRE];
            }
            if (o >= w0 && o < w1) O[o - w0] = ch;
          }
        }
      }
      // escaped content
      {
        int lo = min(tid * C, Wlen), hi = min(lo + C, Wlen);
        int x = lo;
        while (x < hi && is_cont(W[x])) ++x;
        // delta containing x: first j with wpos[j] > x
        int j = 0;
        {
          int a = 0, b = ndelta;
          while (a < b) {
            int m = (a + b) >> 1;
            if ((int)s.wpos[m] <= x) a = m + 1;
            else b = m;
          }
          j = a;
        }
        int e = s.chunk_base[tid];
        uint8_t buf[12];
        while (x < hi) {
          while (j < ndelta && (int)s.wpos[j] <= x) ++j;
          uint32_t cp;
          x += wtf8_decode(W, x, Wlen, &cp);
          int n = escape_cp(cp, buf);
          int o = (int)s.eidx[j] * EVL + PRE + e;
          for (int i = 0; i < n; ++i)
            if (o + i >= w0 && o + i < w1) O[o + i - w0] = buf[i];
          e += n;
        }
      }
      }  // general path
      __syncthreads();
      if (w0 == 0) QMX_STAMP(26);
      const int wl = w1 - w0;
      for (int i = tid * 16; i < wl; i += BS * 16) *(uint4*)&out[it.out_off + w0 + i] = *(const uint4*)&O[i];
      if (w1 < out_len) __syncthreads();  // O is refilled by the next window (the last one: the
                                          // item's publish barrier follows)
    }
  }
  QMX_STAMP(10);
  if (P.dbg != nullptr && threadIdx.x == 0) {
    P.dbg[bi * kDbg + 12] = __builtin_amdgcn_s_memtime();
    P.dbg[bi * kDbg + 13] = (unsigned long long)s.v[V_NFULL];  // S3: events fully parsed
    P.dbg[bi * kDbg + 14] = (unsigned long long)s.v[V_NTPL];   // S3: template hits
    P.dbg[bi * kDbg + 15] = (unsigned long long)nev;
    P.dbg[bi * kDbg + 16] = (unsigned long long)s.v[V_CFULL];  // S3 cycles: full parses (sum over waves)
    P.dbg[bi * kDbg + 17] = (unsigned long long)s.v[V_CTPL];   // S3 cycles: template checks
    P.dbg[bi * kDbg + 18] = (unsigned long long)s.v[V_CLEX];   // S3 cycles: wave_lex part of full
    P.dbg[bi * kDbg + 19] = (unsigned long long)s.v[V_NHOLE];  // S3: hole-template hits
    P.dbg[bi * kDbg + 20] = (unsigned long long)s.v[V_CHOLE];  // S3 cycles: hole-template tries
  }
  if (tid == 0) {
    WorkResult r{(uint32_t)s.v[V_CONSUMED], (uint32_t)out_len, (uint32_t)s.v[V_STATUS], new_clen};
    res[bi] = r;
  }
}

// ------------------------------------------------------------------------------------
// finalize body: K3 think_strip_final + K4 join_pack + K5 sse_encode for one session
// request, texts read straight from the HBM-resident content arena (reference
// oai_proxy.py:120-139 strip, :834-860 join + final event, :406-423 texts for the aggregator)
// ------------------------------------------------------------------------------------
constexpr int FIN_TOK = 4096;   // tag tokens of one tokenisation window staged in LDS
constexpr int FIN_WIN = 8192;   // window bytes: a token is >= 3 bytes, so <= 2731 tokens per window
constexpr int FIN_BIG = 256;    // kept segments at least this long are copied by the whole workgroup

struct FinShared {
  int32_t tpos[FIN_TOK];
  int8_t tkid[FIN_TOK];  // +(t+1) open, -(t+1) close
  uint8_t tlen[FIN_TOK];
  int32_t scr[2 * (BS / 64)];
  int32_t v[16];
  int32_t last_close[kMaxTags];  // start of the last close token of each tag in the text
  TagSet ts;                     // the tag set, staged from the kernel parameters
};
enum : int { FV_CUR = 0, FV_PEND, FV_SEGA, FV_NSEG, FV_NTOK, FV_S0, FV_S1, FV_NBIG, FV_OVF };

// Interval selection of re.sub("<(t)>.*?</\1>", "", IGNORECASE|DOTALL): leftmost open whose
// tag closes later (re tries every start position, so an open that never closes is just
// skipped), its interval ends at the FIRST close of the same tag after it, the scan resumes
// there.  Blockwise over tokenisation windows with the (cursor, pending-tag) state carried
// between them; within a window wave 0 walks 64 tokens per step by ballot: each selection is
// one ballot + find-first + shuffle (no per-token thread-serial loop, no token-count cap).
// Kept segments (text between selected intervals) go to segs[]; returns their count, -1 if
// more than cap (host path).  Block-uniform.
__device__ __forceinline__ int fin_select(const uint8_t* __restrict__ src, int n, const TagSet& ts, int2* __restrict__ segs, int cap,
                          FinShared& F) {
  const int tid = threadIdx.x;
  if (tid < kMaxTags) F.last_close[tid] = -1;
  if (tid == 0) {
    F.v[FV_CUR] = 0;
    F.v[FV_PEND] = 0;
    F.v[FV_SEGA] = 0;
    F.v[FV_NSEG] = 0;
    F.v[FV_OVF] = 0;
  }
  __syncthreads();
  for (int p = tid; p < n; p += BS) {  // pass 0: which opens can close at all
    if (src[p] != '<' || p + 1 >= n || src[p + 1] != '/') continue;
    int L = 0;
    const int id = match_at(src, n, p, ts, &L);
    if (id < 0) atomicMax(&F.last_close[-id - 1], p);
  }
  __syncthreads();
  for (int w0 = 0; w0 < n; w0 += FIN_WIN) {
    const int w1 = min(n, w0 + FIN_WIN);
    {  // tokens starting in [w0, w1), compacted in position order
      const int C = (w1 - w0 + BS - 1) / BS;
      const int lo = min(w0 + tid * C, w1), hi = min(lo + C, w1);
      int cnt = 0;
      for (int p = lo; p < hi; ++p) {
        if (src[p] != '<') continue;
        int L = 0;
        cnt += match_at(src, n, p, ts, &L) != 0;
      }
      int tot;
      int k = block_excl_sum(cnt, F.scr, &tot);
      for (int p = lo; p < hi && cnt > 0; ++p) {
        if (src[p] != '<') continue;
        int L = 0;
        const int id = match_at(src, n, p, ts, &L);
        if (id == 0) continue;
        F.tpos[k] = p;
        F.tkid[k] = (int8_t)id;
        F.tlen[k] = (uint8_t)L;
        ++k;
      }
      if (tid == 0) F.v[FV_NTOK] = tot;
    }
    __syncthreads();
    if (tid < 64) {
      const int lane = tid;
      const int ntok = F.v[FV_NTOK];
      int cur = F.v[FV_CUR], pend = F.v[FV_PEND], sega = F.v[FV_SEGA], nseg = F.v[FV_NSEG];
      for (int c0 = 0; c0 < ntok; c0 += 64) {
        const int k = c0 + lane;
        const bool valid = k < ntok;
        const int pos = valid ? F.tpos[k] : 0x7fffffff;
        const int id = valid ? (int)F.tkid[k] : 0;
        const int end = pos + (valid ? (int)F.tlen[k] : 0);
        const bool can_open = id > 0 && F.last_close[id - 1] >= end;
        while (true) {
          uint64_t m;
          if (pend != 0) {
            m = __ballot(valid && id == -pend && pos >= cur);
            if (m == 0) break;
            const int L = __ffsll((unsigned long long)m) - 1;
            cur = __shfl(end, L, 64);
            pend = 0;
            sega = cur;
          } else {
            m = __ballot(can_open && pos >= cur);
            if (m == 0) break;
            const int L = __ffsll((unsigned long long)m) - 1;
            const int po = __shfl(pos, L, 64);
            if (po > sega) {
              if (lane == 0 && nseg < cap) segs[nseg] = make_int2(sega, po);
              ++nseg;
            }
            pend = __shfl(id, L, 64);
            cur = __shfl(end, L, 64);
          }
        }
      }
      if (lane == 0) {
        F.v[FV_CUR] = cur;
        F.v[FV_PEND] = pend;
        F.v[FV_SEGA] = sega;
        F.v[FV_NSEG] = nseg;
      }
    }
    __syncthreads();
  }
  // an open is only taken when its tag closes later, so no interval is left pending
  if (tid == 0) {
    int nseg = F.v[FV_NSEG];
    const int sega = F.v[FV_SEGA];
    if (n > sega) {
      if (nseg < cap) segs[nseg] = make_int2(sega, n);
      ++nseg;
    }
    F.v[FV_NSEG] = nseg;
  }
  __syncthreads();
  const int nseg = F.v[FV_NSEG];
  return nseg > cap ? -1 : nseg;
}

struct FinArgs {
  const FinItem* items;
  const FinText* texts;
  const uint8_t* fin_in;   // joiners + final-event envelopes (host-mapped)
  uint8_t* join;           // device join buffer
  uint8_t* out_dev;        // device encode buffer
  uint8_t* out_host;       // host-mapped output
  FinResult* res;          // host-mapped result records
  uint32_t* text_len;      // host-mapped per-text stripped lengths (texts-kind)
  int2* segs;              // device kept-segment scratch
};

// Spread owner: final texts that came over the mesh are staged in the host-mapped finalize
// input (FinText::in_off).  Copy them into their shadow slots' HBM content areas first —
// coalesced 16-B loads, one pass over PCIe — so fin_body reads every text from HBM alike.
// (The writes are this workgroup's own, read back by it after the barrier: one CU, one L1.)
__device__ __forceinline__ void fin_stage(const FinArgs& fa, int j, uint8_t* __restrict__ content,
                                          uint32_t content_cap) {
  const int tid = opaque_tid();
  const FinItem it = fa.items[j];
  bool any = false;
  for (uint32_t i = 0; i < it.n_texts; ++i) {
    const FinText ft = fa.texts[it.first_text + i];
    if (ft.in_off == kNoStage || ft.len == 0) continue;
    any = true;
    const uint8_t* src = fa.fin_in + ft.in_off;
    uint8_t* dst = content + (size_t)ft.slot * content_cap;
    const int nv = ((uintptr_t)dst & 15) == 0 ? (int)(ft.len / 16) : 0;
    for (int k = tid; k < nv; k += BS) ((uint4*)dst)[k] = ((const uint4*)src)[k];
    for (int k = nv * 16 + tid; k < (int)ft.len; k += BS) dst[k] = src[k];
  }
  if (any) __syncthreads();  // (any is block-uniform)
}

__device__ __forceinline__ void fin_body(const FinArgs& fa, int j, const uint8_t* __restrict__ content, uint32_t content_cap,
                         const TagSet& ts_mem, FinShared& F) {
  const int tid = opaque_tid();
  for (int i = tid; i < (int)(sizeof(TagSet) / 4); i += BS) ((uint32_t*)&F.ts)[i] = ((const uint32_t*)&ts_mem)[i];
  __syncthreads();
  const TagSet& ts = F.ts;
  const FinItem it = fa.items[j];
  const bool strip = it.flags & 1, as_texts = it.flags & 2;
  uint8_t* J = fa.join + it.join_off;
  int2* segs = fa.segs + it.seg_off;
  int jl = 0, nk = 0;
  auto bail = [&]() {
    if (tid == 0) {
      FinResult r{};
      r.status = 1;
      fa.res[j] = r;
    }
  };
  for (uint32_t i = 0; i < it.n_texts; ++i) {
    const FinText ft = fa.texts[it.first_text + i];
    const int n = (int)ft.len;
    if (n == 0) continue;  // empty texts are not kept (nor joined)
    const uint8_t* src = content + (size_t)ft.slot * content_cap;
    if (nk > 0 && !as_texts) {
      for (uint32_t k = tid; k < it.joiner_len; k += BS) J[jl + k] = fa.fin_in[it.joiner_off + k];
      jl += (int)it.joiner_len;
    }
    int nseg = 1;
    if (strip) {
      nseg = fin_select(src, n, ts, segs, (int)it.seg_cap, F);
      if (nseg < 0) {
        bail();
        return;
      }
    } else if (tid == 0) {
      segs[0] = make_int2(0, n);
    }
    __syncthreads();
    if (tid == 0) {  // str.strip() over the kept text: whitespace at the outer segment ends
      int s0 = 0, s1 = nseg - 1;
      if (strip) {
        for (; s0 < nseg; ++s0) {
          int2 g = segs[s0];
          while (g.x < g.y) {
            const int w = ws_at(src, g.x, g.y);
            if (w <= 0) break;
            g.x += w;
          }
          segs[s0] = g;
          if (g.x < g.y) break;
        }
        for (; s1 >= s0; --s1) {
          int2 g = segs[s1];
          while (g.y > g.x) {
            const int w = ws_before(src, g.x, g.y);
            if (w <= 0) break;
            g.y -= w;
          }
          segs[s1] = g;
          if (g.y > g.x) break;
        }
      }
      F.v[FV_S0] = s0;
      F.v[FV_S1] = s1;
    }
    __syncthreads();
    // K4: kept segments → join buffer (short ones by one thread each, long ones by all)
    const int s0 = F.v[FV_S0], s1 = F.v[FV_S1];
    int run = 0;
    for (int c0 = s0; c0 <= s1; c0 += BS) {
      const int q = c0 + tid;
      const int2 g = q <= s1 ? segs[q] : make_int2(0, 0);
      const int len = g.y - g.x;
      if (tid == 0) F.v[FV_NBIG] = 0;
      int tot;
      const int dst = jl + run + block_excl_sum(len, F.scr, &tot);  // (its barriers order the reset)
      if (len >= FIN_BIG) {
        const int b = atomicAdd(&F.v[FV_NBIG], 1);
        F.tpos[3 * b] = g.x;  // tokens are dead by now: reuse as the big-segment list
        F.tpos[3 * b + 1] = len;
        F.tpos[3 * b + 2] = dst;
      } else {
        for (int x = 0; x < len; ++x) J[dst + x] = src[g.x + x];
      }
      __syncthreads();
      const int nbig = F.v[FV_NBIG];
      for (int b = 0; b < nbig; ++b) {
        const int a = F.tpos[3 * b], l = F.tpos[3 * b + 1], d = F.tpos[3 * b + 2];
        for (int x = tid; x < l; x += BS) J[d + x] = src[a + x];
      }
      __syncthreads();
      run += tot;
    }
    if (as_texts && tid == 0) fa.text_len[it.tl_off + nk] = (uint32_t)run;
    jl += run;
    ++nk;
    __syncthreads();  // LDS token / state arrays are reused by the next text
  }
  __syncthreads();
  uint8_t* O = fa.out_dev + it.out_off;
  int out_len = 0;
  const uint8_t* src_out = J;
  if (as_texts) {
    out_len = jl;
  } else if (nk > 0) {
    // K5: ensure_ascii JSON escape of the joined text inside the final-event envelope
    for (uint32_t k = tid; k < it.pre_len; k += BS) O[k] = fa.fin_in[it.pre_off + k];
    const int C = (jl + BS - 1) / BS;
    int lo = min(tid * C, jl), hi = min(lo + C, jl);
    while (lo < jl && is_cont(J[lo])) ++lo;  // code points starting in [lo, hi): both bounds
    while (hi < jl && is_cont(J[hi])) ++hi;  // move to the next code-point start
    hi = max(hi, lo);
    int el = 0;
    for (int p = lo; p < hi;) {
      uint32_t cpv;
      p += wtf8_decode(J, p, jl, &cpv);
      el += escaped_len_cp(cpv);
    }
    int tot;
    int o = (int)it.pre_len + block_excl_sum(el, F.scr, &tot);
    out_len = (int)it.pre_len + tot + (int)it.suf_len;
    if ((uint32_t)out_len > it.out_cap) {
      bail();
      return;
    }
    for (int p = lo; p < hi;) {
      uint32_t cpv;
      p += wtf8_decode(J, p, jl, &cpv);
      o += escape_cp(cpv, O + o);
    }
    for (uint32_t k = tid; k < it.suf_len; k += BS) O[it.pre_len + tot + k] = fa.fin_in[it.suf_off + k];
    src_out = O;
  }
  __syncthreads();
  // coalesced 16-B stores into the host-mapped output arena
  uint4* dst = (uint4*)(fa.out_host + it.out_off);
  const uint4* sv = (const uint4*)src_out;
  for (int k = tid; k * 16 < out_len; k += BS) dst[k] = sv[k];
  if (tid == 0) {
    FinResult r{};
    r.out_len = (uint32_t)out_len;
    r.status = 0;
    r.n_kept = (uint32_t)nk;
    fa.res[j] = r;
  }
}

// ------------------------------------------------------------------------------------
// the fused kernel: workgroups [0, n_tick) run one stream tile each, [n_tick, grid) one
// finalize request each — one launch per tick for both (their LDS overlays: a workgroup is
// one or the other).  Every workgroup publishes its result record last: every wave waits for
// its own stores (output, content, state, result record), a barrier, then thread 0 stores the
// tick's sequence number with a system-scope release (one L2 write-back per item).  The host
// polls these sequence numbers instead of waiting on a HIP event (no interrupt round trip, no
// HSA spin-wait per tick).  Every early exit of tick_body / fin_body is block-uniform, so
// every thread reaches the barrier.
// ------------------------------------------------------------------------------------
union TickLds {
  TickShared t;
  FinShared f;
};

template <class T>
__device__ __forceinline__ T* uni(T* p) {
  typedef __attribute__((address_space(1))) T GT;
  const uint64_t v = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (T*)(GT*)(((uint64_t)hi << 32) | lo);
}

// A finalize item's arguments as wave-uniform scalars, made where they are used: held in
// registers across the whole item loop they add to the persistent kernel's SGPR spills
__device__ __forceinline__ FinArgs fin_uni(const FinArgs& a) {
  FinArgs f;
  f.items = uni(a.items);
  f.texts = uni(a.texts);
  f.fin_in = uni(a.fin_in);
  f.join = uni(a.join);
  f.out_dev = uni(a.out_dev);
  f.out_host = uni(a.out_host);
  f.res = uni(a.res);
  f.text_len = uni(a.text_len);
  f.segs = uni(a.segs);
  return f;
}

// One work item of a tick: k < n_tick a stream tile, else finalize request k - n_tick.
// Publishes the item's result record last (fence + sequence number).
__device__ __forceinline__ void run_item(int k, const WorkItem* __restrict__ items, const uint8_t* __restrict__ in,
                                         uint8_t* __restrict__ out, WorkResult* __restrict__ res,
                                         DevSlot* __restrict__ state, uint8_t* __restrict__ content,
                                         const KParams& Pk, uint32_t seq, uint32_t n_tick, const FinArgs& fa_src,
                                         const BackendTpl* __restrict__ btpl_rd, BackendTpl* __restrict__ btpl_wr,
                                         TickLds& U) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  if ((uint32_t)k < n_tick) {
    tick_body(items, in, out, res, state, content, Pk, U.t, btpl_rd, btpl_wr, seq, k);
    if (threadIdx.x == 0) {
      res[k].t0 = t0;
      res[k].t1 = __builtin_amdgcn_s_memrealtime();
    }
    // publish: every wave waits for its OWN stores (output, content, slot state, the record),
    // then the barrier, then ONE system-scope release by thread 0 (one L2 write-back per
    // item; a __threadfence_system() per thread was one per wave, nine per item)
    wave_stores_done();
    __syncthreads();
    if (Pk.dbg != nullptr && threadIdx.x == 0) dbg_put(&Pk.dbg[k * kDbg + 27], __builtin_amdgcn_s_memrealtime());
    if (threadIdx.x == 0) publish_system(&res[k].seq, seq);
  } else {
    const int j = (int)(k - n_tick);
    const FinArgs fa = fin_uni(fa_src);
    fin_stage(fa, j, content, Pk.content_cap);
    fin_body(fa, j, content, Pk.content_cap, Pk.ts, U.f);
    if (threadIdx.x == 0) {
      fa.res[j].t0 = t0;
      fa.res[j].t1 = __builtin_amdgcn_s_memrealtime();
    }
    wave_stores_done();
    __syncthreads();
    if (threadIdx.x == 0) publish_system(&fa.res[j].seq, seq);
  }
}

__global__ __launch_bounds__(BS) void qmx_tick_kernel(const WorkItem* __restrict__ items,
                                                      const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                      WorkResult* __restrict__ res, DevSlot* __restrict__ state,
                                                      uint8_t* __restrict__ content, const KParams* __restrict__ Pkp,
                                                      uint32_t seq, uint32_t n_tick, FinArgs fa,
                                                      const BackendTpl* __restrict__ btpl_rd,
                                                      BackendTpl* __restrict__ btpl_wr) {
  __shared__ TickLds U;
  // tag patterns, MFMA B operand and SSE envelopes: in device memory (uploaded by the lane
  // when they change, ~once a second), not a 1.5 KB by-value kernel argument per launch
  run_item((int)blockIdx.x, items, in, out, res, state, content, *Pkp, seq, n_tick, fa, btpl_rd, btpl_wr, U);
}

// ------------------------------------------------------------------------------------
// Persistent mode (QMX_PERSISTENT=1): one long-lived grid per tick lane replaces the launch
// per tick.  The host posts a tick by writing its arguments (TickDesc) into a host-mapped
// doorbell and then its sequence number; workgroup 0 polls the doorbell (relaxed system-
// scope loads with s_sleep, one PCIe read in flight) and relays the tick into a device-
// memory control block, which the other workgroups poll (relaxed agent-scope loads: no cache
// invalidation per poll).  On a new tick every workgroup takes one acquire fence (system
// scope: host-written items / tile bytes and other XCDs' slot state become visible), then
// runs items blockIdx.x, blockIdx.x + grid, ... exactly like the one-shot kernel, result
// records included, so the host's completion polling is unchanged.
// Exit conditions every wave reaches: a posted tick with stop set; or workgroup 0 idle for
// idle_ticks (s_memrealtime, 100 MHz) — it then raises the control block's exit word for
// this launch generation; or (safety net) any workgroup idle for 2 x idle_ticks.  The host
// never posts to a grid that may be idling out (HipEngine::ensure_persistent), and stops it
// before anything that would wait for the device.
// Multi-door grids (HipGrid, loop ticks): the grid is doors x wpd workgroups, sub-grid
// blockIdx.x / wpd serving door blockIdx.x / wpd with its own control block — one launch,
// one hardware queue, every io loop's ticks.  The host bumps each door's heartbeat word
// (read with `posted` in one 8-byte load) while it wants the grid; a change resets the idle
// clock of the relay and, through the control block, of its workers, so a door with no
// traffic keeps its sub-grid while the others are busy.  Idle time counts from the last
// post or heartbeat, so the 2 s limit HipGrid passes fires only for a host that stopped.
// ------------------------------------------------------------------------------------
// A wave-uniform pointer held in SGPRs, into the global address space (device or host-mapped
// memory, never LDS).  Saying so lets the compiler emit global_* instead of flat_* accesses
// through the descriptor's pointers, as it does for kernel arguments: a flat access also
// counts against lgkmcnt, so every LDS wait after it would wait for the memory access too.

struct TickDesc {
  const WorkItem* items;
  const uint8_t* in;
  uint8_t* out;
  WorkResult* res;
  KParams* params;            // device copy read by the items
  const KParams* params_src;  // non-null: host-mapped new parameters, copied into `params` first
  const BackendTpl* btpl_rd;
  BackendTpl* btpl_wr;
  FinArgs fa;
  DevSlot* state;  // the posting engine's slot state and content arena
  uint8_t* content;
  uint32_t seq, n_tick, n_fin, stop;
};
struct PDoor {  // host-mapped: written by the host, polled by the door's relay workgroup
  TickDesc d;
  alignas(64) uint32_t posted;
  uint32_t beat;  // host keep-alive (multi-door grid): a change resets the relay's idle clock
  uint32_t base;  // the last tick relayed before this launch (the launch's starting point)
  // written by the relay (diagnostics: the host reports them when a tick goes missing)
  alignas(64) uint32_t relayed;  // last tick relayed
  uint32_t exits;                // last grid exit: reason << 16 | launch generation (1 idle, 2 stop)
  uint32_t idle_limit_hit_us;    // the idle time that triggered the last idle exit, us
  uint64_t t_seen, t_relayed;    // s_memrealtime: the last tick's doorbell seen / relayed (timing)
};
struct PCtl {  // device memory: written by the relay, polled by the door's other workgroups
  TickDesc d;
  alignas(64) uint32_t seq;
  uint32_t exit_gen;
  uint32_t beat;                 // the door's heartbeat, mirrored by the relay (workers' idle clock)
  alignas(64) uint32_t next[4];  // item counters, tick seq & 3 (reset by the relay before publishing)
};
static_assert(offsetof(PDoor, beat) == offsetof(PDoor, posted) + 4, "posted + beat: one 8-byte load");

// `door` / `ctl` are neither const nor __restrict__ and their words are read with atomic
// loads: a readonly noalias kernel argument may be read through the scalar cache, which no
// acquire fence invalidates — the next tick's descriptor would come back stale.
//
// WPE: waves per SIMD the register allocation must allow.  2 (the default): one 512-thread
// workgroup per CU (8 waves on 4 SIMDs), up to 256 VGPRs.  4: two workgroups per CU — at most
// 128 VGPRs (some live values go to scratch) and 2 x 79 KB of the CU's 160 KB LDS; the grid
// then counts its budget in workgroup slots (HipGrid, QMX_GRID_OCC=2).
template <int WPE>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void qmx_tick_persistent(
    PDoor* doors, PCtl* ctls, int wpd, uint32_t gen, uint32_t idle_ticks, int interleave) {
  __shared__ TickLds U;
  __shared__ TickDesc D;
  __shared__ uint32_t cmd;  // new tick's sequence number, 0: exit
  __shared__ uint32_t pre_k;  // a worker's first item of the tick, claimed with the descriptor read
  // door of this workgroup: blocks [d·wpd, (d+1)·wpd) — or, interleaved, blocks d, d + ndoors,
  // d + 2·ndoors, ...: the dispatcher deals block b to XCD b % 8, so with a multiple of 8
  // doors every door's sub-grid (and, tick after tick, its io loop's slot state, templates and
  // content tails) stays in ONE XCD's L2.  The door's first workgroup is its relay.
  const int ndoors = (int)gridDim.x / wpd;
  const int di = interleave ? (int)blockIdx.x % ndoors : (int)blockIdx.x / wpd;
  PDoor* const door = doors + di;
  PCtl* const ctl = ctls + di;
  const bool relay = interleave ? (int)blockIdx.x < ndoors : blockIdx.x % wpd == 0;
  constexpr int kWords = (int)(sizeof(TickDesc) / 4);
  static_assert(kWords <= 64, "the descriptor is copied by one wave, a word per lane");
  const int tid = threadIdx.x;
  // the last tick relayed before this launch (written by the host before it launched)
  if (tid == 0) cmd = __hip_atomic_load(&door->base, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __syncthreads();
  uint32_t last = cmd;
  uint32_t beat = 0;  // thread 0's view of the door's heartbeat
  __syncthreads();
  for (;;) {
    if (tid == 0) {
      uint64_t t_idle = __builtin_amdgcn_s_memrealtime();
      const uint64_t limit = relay ? (uint64_t)idle_ticks : 2ull * idle_ticks;
      uint32_t c = 0;
      for (;;) {
        if (relay) {
          // posted and beat in one 8-byte load: one PCIe read in flight per poll
          const uint64_t pb = __hip_atomic_load((uint64_t*)&door->posted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          const uint32_t v = (uint32_t)pb;
          if ((int32_t)(v - last) > 0) {  // newer only: a control word left by an earlier launch is older
            c = v;
            __hip_atomic_store(&door->t_seen, (uint64_t)__builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
            break;
          }
          if ((uint32_t)(pb >> 32) != beat) {  // the host is alive: idle time starts over
            beat = (uint32_t)(pb >> 32);
            t_idle = __builtin_amdgcn_s_memrealtime();
            __hip_atomic_store(&ctl->beat, beat, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        } else {
          const uint32_t v = __hip_atomic_load(&ctl->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((int32_t)(v - last) > 0) {
            c = v;
            break;
          }
          if (__hip_atomic_load(&ctl->exit_gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen) break;
          const uint32_t b = __hip_atomic_load(&ctl->beat, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (b != beat) {
            beat = b;
            t_idle = __builtin_amdgcn_s_memrealtime();
          }
        }
        const uint64_t idle = __builtin_amdgcn_s_memrealtime() - t_idle;
        if (idle > limit) {
          if (relay) {
            __hip_atomic_store(&ctl->exit_gen, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&door->idle_limit_hit_us, (uint32_t)(idle / 100), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&door->exits, (1u << 16) | (gen & 0xffffu), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          }
          break;
        }
        __builtin_amdgcn_s_sleep(8);
      }
      cmd = c;
    }
    __syncthreads();
    const uint32_t c = cmd;
    if (c == 0) return;
    // the descriptor: a word per lane of wave 0, all loads in flight at once (one round trip
    // to host memory / the coherence point, not one per word)
    if (tid < kWords) {
      uint32_t w;
      if (relay) {
        // written by the host before `posted`, which thread 0 saw before the barrier: these
        // system-scope loads bypass the caches and are issued after that load returned.  The
        // acquire (for the tick's host-written items and tiles) follows them, so its wait for
        // thread 0's t_seen store — a PCIe write — overlaps the descriptor's round trip
        // instead of preceding it
        w = __hip_atomic_load((uint32_t*)&door->d + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      } else {
        // system scope (not just agent): this is also the workgroup's acquire of the tick's
        // host-written items / tile bytes and of other XCDs' slot state — one cache
        // invalidation per workgroup (the caches are per CU / per XCD), not one per wave
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        w = __hip_atomic_load((uint32_t*)&ctl->d + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // the first claim rides with the descriptor read (after the same acquire: the relay
        // reset the counter before publishing the tick) — one round trip to the L2 before
        // this workgroup's first item instead of two (r5: start spread 1.3 us per tick)
        if (tid == 0) pre_k = __hip_atomic_fetch_add(&ctl->next[c & 3], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      ((uint32_t*)&D)[tid] = w;
    }
    __syncthreads();
    if (relay) {
      // new kernel parameters (about once a second): copied by this workgroup's threads, then
      // the tick is published to the other workgroups (agent-scope release)
      if (D.params_src != nullptr && !D.stop)
        for (int i = tid; i < (int)(sizeof(KParams) / 4); i += BS)
          ((uint32_t*)D.params)[i] =
              __hip_atomic_load((uint32_t*)D.params_src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (tid < kWords)
        __hip_atomic_store((uint32_t*)&ctl->d + tid, ((const uint32_t*)&D)[tid], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      // item 0 is the relay's own (no claim round trip on the first item's path): the
      // others claim from 1
      if (tid == 0) __hip_atomic_store(&ctl->next[c & 3], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // each wave's own stores done (descriptor words, counter, parameters), then the barrier:
      // thread 0's agent-scope release of ctl->seq below is the one L2 write-back (a
      // __threadfence() per thread was one per wave)
      wave_stores_done();
      __syncthreads();
      // the host-visible stamp and diagnostics (PCIe writes) from wave 1: a wave waits on its
      // own counter, so wave 0's publish below does not wait for these writes to complete
      // (they preceded it in wave 0 through r6).  The relay's item 0 publishes its result only
      // after every wave's stores are done, so the host — which reads these after every result
      // of the tick — sees this tick's values
      if (tid == 64) {
        __hip_atomic_store(&door->t_relayed, (uint64_t)__builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&door->relayed, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (D.stop) __hip_atomic_store(&door->exits, (2u << 16) | (gen & 0xffffu), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      if (tid == 0) publish_agent(&ctl->seq, c);
    }
    if (D.stop) return;  // D is block-uniform (LDS, written before the barrier)
    last = c;  // (the tick's acquire: wave 0's fence above, ordered before every wave by the barrier)
    // descriptor fields read from LDS land in VGPRs: make them wave-uniform scalars again
    // (as kernel arguments are), or every address derived from them costs vector registers
    const uint32_t n_tick = __builtin_amdgcn_readfirstlane(D.n_tick);
    const int total = (int)(n_tick + __builtin_amdgcn_readfirstlane(D.n_fin));
    const uint32_t seq = __builtin_amdgcn_readfirstlane(D.seq);
    // items are claimed from the tick's counter, not dealt by workgroup index: a workgroup
    // that is not resident (the CUs are shared with other grids / kernels) holds up nothing.
    // The relay runs item 0 without a claim (it reset the counter to 1 before publishing).
    // A worker's first item was claimed with the descriptor read (pre_k).  Every claim of the
    // tick — that first one, the relay's reset and the loop below — uses the counter of the
    // relayed command c, never the descriptor's seq: one index, whatever the host numbers
    // (the host posts D.seq == c today; a claim on another counter would skip or repeat items)
    bool first = true;
    for (;;) {
      if (tid == 0)
        cmd = first ? (relay ? 0u : pre_k)
                    : __hip_atomic_fetch_add(&ctl->next[c & 3], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      first = false;
      __syncthreads();
      const int k = (int)cmd;
      __syncthreads();  // cmd is rewritten by the next claim
      if (k >= total) break;
      // a visible clobber: the host rewrites items, tile bytes and finalize descriptors
      // between ticks, so none of them may be read through the scalar cache as
      // launch-invariant data (which the compiler does for uniform addresses it proves
      // unclobbered within the kernel)
      asm volatile("" ::: "memory");
      run_item(k, uni(D.items), uni(D.in), uni(D.out), uni(D.res), uni(D.state), uni(D.content), *uni(D.params), seq,
               n_tick, D.fa, uni(D.btpl_rd), uni(D.btpl_wr), U);
      __syncthreads();  // LDS is reused by the next item
    }
    __syncthreads();  // D / cmd are rewritten by thread 0 for the next tick
  }
}

// ------------------------------------------------------------------------------------
// HipEngine host runtime
// ------------------------------------------------------------------------------------
static void put(char* dst, int cap, int* len, const std::string& s) {
  if ((int)s.size() > cap) throw std::runtime_error("envelope too long");
  std::memcpy(dst, s.data(), s.size());
  *len = (int)s.size();
}

static double steady_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ---- stream registry (qmx_streams.h) -----------------------------------------------------
namespace {
std::atomic<int> g_streams_shared{0}, g_streams_excl{0};
std::atomic<uint64_t> g_streams_created{0};
}  // namespace

bool exclusive_queues() {
  const char* q = env_get("QMX_GRID_QUEUE");
  if (q && std::string(q) == "shared") return false;
  int least = 0, greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) return false;
  return least != greatest;
}

hipStream_t stream_create(StreamKind kind) {
  hipStream_t s = nullptr;
  if (kind == StreamKind::Exclusive && exclusive_queues()) {
    int least = 0, greatest = 0;
    HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    HIP_CHECK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, greatest));
  } else {
    HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  }
  (kind == StreamKind::Exclusive ? g_streams_excl : g_streams_shared).fetch_add(1);
  g_streams_created.fetch_add(1);
  return s;
}

void stream_destroy(hipStream_t s, StreamKind kind) {
  if (!s) return;
  hipStreamDestroy(s);
  (kind == StreamKind::Exclusive ? g_streams_excl : g_streams_shared).fetch_sub(1);
}

__global__ void qmx_touch(uint32_t* mark) {
  // (relaxed: the mark carries no data to order — and a release store is emitted as an L2
  // write-back the store does not wait for, which tests/test_isa.py rejects anywhere)
  if (threadIdx.x == 0) __hip_atomic_store(mark, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

std::unordered_map<std::string, double> stream_probe(int n, double wait_ms) {
  n = std::max(1, std::min(n, 64));
  uint32_t* marks = nullptr;
  HIP_CHECK(hipHostMalloc((void**)&marks, 4 * (size_t)(n + 1), hipHostMallocMapped));
  std::memset(marks, 0, 4 * (size_t)(n + 1));
  uint8_t* dsrc = nullptr;
  HIP_CHECK(hipMalloc((void**)&dsrc, 4096));
  std::vector<uint8_t> host(4096);
  std::vector<hipStream_t> st;
  for (int i = 0; i < n; ++i) st.push_back(stream_create(StreamKind::Shared));
  const double t0 = steady_s();
  for (int i = 0; i < n; ++i) {
    hipLaunchKernelGGL(qmx_touch, dim3(1), dim3(64), 0, st[i], marks + i);
    HIP_CHECK(hipGetLastError());
  }
  hipEvent_t ev;
  HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  HIP_CHECK(hipMemcpyAsync(host.data(), dsrc, 4096, hipMemcpyDeviceToHost, 0));
  HIP_CHECK(hipEventRecord(ev, 0));
  auto done = [&](int i) { return __atomic_load_n(marks + i, __ATOMIC_ACQUIRE) != 0; };
  double last = 0;
  int ndone = 0;
  bool null_done = false;
  while (steady_s() - t0 < 1e-3 * wait_ms) {
    ndone = 0;
    for (int i = 0; i < n; ++i) ndone += done(i);
    null_done = hipEventQuery(ev) == hipSuccess;
    if (ndone == n && null_done) {
      last = 1e3 * (steady_s() - t0);
      break;
    }
    sched_yield();
  }
  // drain before the streams go (a blocked one completes once whatever holds its queue leaves)
  const double t1 = steady_s();
  bool drained = false;
  while (steady_s() - t1 < 5.0) {
    bool all = hipEventQuery(ev) == hipSuccess;
    for (int i = 0; i < n && all; ++i) all = done(i);
    if (all) {
      drained = true;
      break;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
  if (drained) {
    for (hipStream_t s : st) stream_destroy(s, StreamKind::Shared);
    hipEventDestroy(ev);
    hipFree(dsrc);
    hipHostFree(marks);
  }  // (else leaked: destroying a stream with work queued would wait for it)
  return {{"streams", (double)n}, {"completed", (double)ndone}, {"null_stream_copy_done", null_done ? 1.0 : 0.0},
          {"all_done_ms", last}, {"drained", drained ? 1.0 : 0.0}};
}

std::unordered_map<std::string, double> stream_stats() {
  const char* hq = env_get("GPU_MAX_HW_QUEUES");
  const int queues = hq ? std::max(1, atoi(hq)) : 4;  // HIP's default
  const int ex = g_streams_excl.load(), sh = g_streams_shared.load();
  const bool own = exclusive_queues();
  return {{"streams_shared", (double)sh},
          {"streams_exclusive", (double)ex},
          {"streams_created", (double)g_streams_created.load()},
          {"hw_queues_per_priority", (double)queues},
          {"grid_queue_exclusive", own ? 1.0 : 0.0},
          // every persistent grid alone on a queue: exclusive streams have a priority level of
          // their own and fit its pool
          {"grid_queue_ok", own && ex <= queues ? 1.0 : 0.0}};
}

// Wait for a lane's stream without pinning a core: the io loops share the CPU with the tick
// threads.  A blocking-sync event sleeps on the completion interrupt: measured on MI355X
// (tools/probes/launch_bench.hip) launch+wait = 11 us, vs 18 us spinning
// hipStreamSynchronize (one core burnt per engine) and 77 us polling with sleep_for.
void HipEngine::wait_stream(TickLane& L) {
  HIP_CHECK(hipEventRecord(L.evb, L.stream));
  if (spin_us_ > 0) {  // optional: yield-poll for the expected kernel time before sleeping
    const auto t0 = std::chrono::steady_clock::now();
    while (hipEventQuery(L.evb) == hipErrorNotReady) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us_)) break;
      sched_yield();
    }
  }
  HIP_CHECK(hipEventSynchronize(L.evb));
}

// Results published by the tick kernel itself (qmx_tick_kernel's sequence numbers): sleep
// most of the expected kernel time (EMA), then poll every poll_us_ with a 1 us timer slack.
// A launch that has not published after 4x the EMA + 2 ms synchronises its stream (surfaces a
// fault; correct even if host-mapped visibility misbehaved: counted in poll_fallbacks).
void HipEngine::wait_results(TickLane& L, int n, int m, uint32_t seq, const WorkResult* res,
                             std::chrono::steady_clock::time_point t0, const std::function<void(int)>& on_item) {
  using HC = std::chrono::steady_clock;
  static thread_local bool slack = (prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0), true);
  (void)slack;
  // t0: when the tick was posted (a pipelined lane prepares its next tick before waiting)
  auto nap = [](double us) {
    if (us < 1) return;
    timespec ts{0, (long)(us * 1000)};
    nanosleep(&ts, nullptr);
  };
  auto done = [&](int& i) {
    while (i < n && __atomic_load_n(&res[i].seq, __ATOMIC_ACQUIRE) == seq) on_item(i++);
    while (i >= n && i < n + m && __atomic_load_n(&L.h_finres[i - n].seq, __ATOMIC_ACQUIRE) == seq) ++i;
    return i == n + m;
  };
  int i = 0;
  bool revived = false;
  double revive_at = 2e5;  // loop-tick mode: us after the post
  nap(0.6 * L.ema_us - 6.0 - std::chrono::duration<double, std::micro>(HC::now() - t0).count());
  while (!done(i)) {
    const double el = std::chrono::duration<double, std::micro>(HC::now() - t0).count();
    if (grid_) {
      // loop-tick mode: a grid that left on its own (the host's heartbeat stopped for 2 s) is
      // relaunched from the last tick it relayed; a grid that runs but never answers is fatal
      if (el > revive_at) {
        revive_at = el + 1e5;
        grid_->revive_if_exited();
      }
      if (el > 1e7)
        throw std::runtime_error("tick results missing after 10 s (door " + std::to_string(door_) + ", seq " +
                                 std::to_string(seq) + ", relayed " +
                                 std::to_string(__atomic_load_n(&L.h_door->relayed, __ATOMIC_ACQUIRE)) + ")");
      nap(el < 2e3 ? poll_us_ : 50.0);
      continue;
    }
    // the persistent grid idled out between ensure_persistent() and this tick's doorbell (the
    // lane thread was descheduled for longer than the margin): it reported an idle exit for
    // its generation and never relayed the tick.  Relaunch it from just before this tick's
    // sequence number — the doorbell still holds the descriptor — instead of losing the tick.
    if (L.p_running && !revived && el > 2.0 * L.ema_us + 500.0) {
      const uint32_t ex = __atomic_load_n(&L.h_door->exits, __ATOMIC_ACQUIRE);
      const uint32_t rl = __atomic_load_n(&L.h_door->relayed, __ATOMIC_ACQUIRE);
      if ((ex >> 16) == 1 && (ex & 0xffffu) == (L.p_gen & 0xffffu) && rl != seq) {
        uint32_t seq0 = seq - 1;
        if (seq0 == 0) seq0 = (uint32_t)-1;  // (0 never names a tick)
        HIP_CHECK(hipStreamSynchronize(L.stream));  // the idle grid has left
        L.h_door->base = seq0;
        hipLaunchKernelGGL(qmx_tick_persistent<2>, dim3(p_grid_), dim3(BS), 0, L.stream, L.h_door, L.d_ctl, p_grid_,
                           ++L.p_gen, (uint32_t)p_idle_ms_ * 100000u, 0);
        HIP_CHECK(hipGetLastError());
        L.p_last_post = steady_s();
        ++L.p_launches;
        ++L.p_revivals;
        revived = true;
        continue;
      }
    }
    // a persistent grid is only stopped to surface a fault: a tick it has not reached yet
    // (first launch loading the code object, a long finalize) would be lost to the stop
    if (el > (L.p_running ? 1e6 : 4.0 * L.ema_us + 2000.0)) {
      if (L.p_running) stop_persistent(L);  // the grid leaves after this tick; throws on a fault
      else HIP_CHECK(hipStreamSynchronize(L.stream));  // throws on a kernel fault
      ++L.poll_fallbacks;
      // the stream has drained: every result is final — or the tick was never run
      if (!done(i)) {
        std::string why = "tick results missing after the lane drained (seq " + std::to_string(seq) + ", " +
                          std::to_string(i) + "/" + std::to_string(n + m) + " published";
        if (L.h_door)
          why += "; grid: relayed " + std::to_string(__atomic_load_n(&L.h_door->relayed, __ATOMIC_ACQUIRE)) +
                 ", exits " + std::to_string(L.h_door->exits) + ", last idle exit after " +
                 std::to_string(L.h_door->idle_limit_hit_us) + " us, launches " + std::to_string(L.p_launches) +
                 ", posted " + std::to_string(L.h_door->posted);
        throw std::runtime_error(why + ")");
      }
      break;
    }
    if (el < spin_us_) {
      sched_yield();
      continue;
    }
    nap(poll_us_);
  }
  const double tot = std::chrono::duration<double, std::micro>(HC::now() - t0).count();
  L.ema_us = 0.85 * L.ema_us + 0.15 * std::min(tot, 2000.0);
}

void HipEngine::collect_timing(TickLane& L) {
  if (!L.timing_pending) return;
  L.timing_pending = false;
  HIP_CHECK(hipEventSynchronize(L.ev1));  // long complete when called for the previous launch
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, L.ev0, L.ev1) == hipSuccess) L.kernel_ms += ms;
}

HipEngine::HipEngine(const std::vector<std::string>& tags, int device, int tile_bytes, int max_slots,
                     int content_cap, int lanes, HipGrid* grid, int door, int ndoors)
    : HostEngine(tags),
      device_(device),
      tile_(std::min(std::max(tile_bytes, 1024), TILE_MAX) & ~15),
      max_slots_(max_slots),
      content_cap_((uint32_t)content_cap),
      grid_(grid),
      door_(door),
      ndoors_(grid ? std::min(std::max(ndoors, 1), 2) : 1) {
  HIP_CHECK(hipSetDevice(device_));
  if (grid_ && (door_ < 0 || door_ + ndoors_ > grid_->doors())) throw std::invalid_argument("HipEngine: door out of range");
  if (grid_) lanes = 1;
  door_busy_.assign(ndoors_, 0);
  if (const char* sp = env_get("QMX_WAIT_SPIN_US")) spin_us_ = atoi(sp);
  if (const char* w = env_get("QMX_WAIT")) poll_ = std::string(w) != "event";
  if (const char* pu = env_get("QMX_POLL_US")) poll_us_ = std::max(1, atoi(pu));
  // a persistent grid assumes its process owns the GPU: grids of several processes on one
  // device (a rehearsal with more ranks than GPUs) need not all be resident at once
  if (const char* gs = env_get("QMX_GPU_SHARERS")) persistent_ = atoi(gs) <= 1;
  if (const char* pe = env_get("QMX_PERSISTENT")) persistent_ = atoi(pe) != 0;
  if (const char* va = env_get("QMX_VIEWS")) views_ = atoi(va) != 0;
  keep_stale_records_ = env_get("QMX_DEBUG_STALE_RECORDS") != nullptr;
  stage_timing_ = env_get("QMX_STAGE_TIMING") != nullptr;  // read once: getenv scans the environment
  if (const char* pw = env_get("QMX_PERSISTENT_WG")) p_grid_ = std::min(std::max(8, atoi(pw)), 1024);
  if (const char* pi = env_get("QMX_PERSISTENT_IDLE_MS")) p_idle_ms_ = std::min(std::max(5, atoi(pi)), 1000);
  {
    // HIP streams share GPU_MAX_HW_QUEUES hardware queues round-robin, and a persistent grid
    // holds its queue: a second lane's grid on the same queue would wait for the first to
    // idle out (MI355X, 4 lanes / 4 queues: the first result of a tick came 100 us late).
    // Persistent lanes need a queue each: on exclusive (highest-priority) streams that level's
    // pool holds only them; on shared streams one queue stays for everything else.
    const char* hq = env_get("GPU_MAX_HW_QUEUES");
    const int queues = hq ? std::max(1, atoi(hq)) : 4;
    if (persistent_ && lanes > (exclusive_queues() ? queues : queues - 1)) persistent_ = false;
  }
  if (grid_) {  // the shared grid is the only way this engine's ticks run
    persistent_ = false;
    poll_ = true;
  }
  HIP_CHECK(hipMalloc(&d_state_, sizeof(DevSlot) * (size_t)max_slots_));
  HIP_CHECK(hipMemset(d_state_, 0, sizeof(DevSlot) * (size_t)max_slots_));
  HIP_CHECK(hipMalloc(&d_content_, (size_t)content_cap_ * (size_t)max_slots_));

  std::memset(&base_params_, 0, sizeof(base_params_));
  base_params_.ts = ts_;
  base_params_.npat = 2 * ts_.n;
  // matcher codes: every byte that occurs in a pattern gets its own code (letters: one code
  // for both cases, the tags' IGNORECASE), everything else shares code 95
  {
    int next = 1;
    for (int b = 0; b < 256; ++b) base_params_.code[b] = 95;
    for (int p = 0; p < base_params_.npat; ++p)
      for (int j = 0; j < pattern_len(ts_, p); ++j) {
        const uint8_t b = pattern_byte(ts_, p, j);
        if (base_params_.code[b] != 95) continue;
        if (next > 94) throw std::invalid_argument("thinking tags use more than 94 distinct characters");
        base_params_.code[b] = (uint8_t)next;
        if (b >= 'a' && b <= 'z') base_params_.code[b - 32] = (uint8_t)next;
        ++next;
      }
  }
  // the matcher works on the bytes themselves as base-8 digits (mfma_match_group): E is the
  // squared digit sum of the pattern's window part
  auto digits = [](int b, int k) { return k == 0 ? (b & 7) : k == 1 ? ((b >> 3) & 7) : (b >> 6); };
  for (int p = 0; p < base_params_.npat; ++p) {
    int E = 0;
    for (int j = 0; j < std::min(kWindow, pattern_len(ts_, p)); ++j) {
      const int b = pattern_byte(ts_, p, j);
      for (int k = 0; k < 3; ++k) E += digits(b, k) * digits(b, k);
    }
    base_params_.pat_E[p] = E;
    base_params_.plen[p] = pattern_len(ts_, p);
  }
  base_params_.content_cap = content_cap_;
  for (int p = 0; p < base_params_.npat; ++p)
    for (int j = 0; j < pattern_len(ts_, p); ++j)
      base_params_.pw[p][j >> 3] |= (uint64_t)pattern_byte(ts_, p, j) << (8 * (j & 7));
  base_params_.fast = 31;
  if (const char* kf = env_get("QMX_KFAST")) base_params_.fast = (uint32_t)strtoul(kf, nullptr, 0);
  for (int blk = 0; blk < 2; ++blk)
    for (int l = 0; l < 64; ++l) {
      const int t = 16 * blk + (l & 15), kg = l >> 4;
      for (int j = 0; j < 16; ++j) {
        int v = 0;
        if (t < base_params_.npat && j < pattern_len(ts_, t)) {
          const int b = pattern_byte(ts_, t, j);
          v = kg < 3 ? -2 * digits(b, kg) : 1;  // -2·p digit, or the mask of the squares
        }
        base_params_.bfrag[blk][l * 16 + j] = (int8_t)v;
      }
    }
  for (int i = 0; i < std::max(1, lanes); ++i) {
    std::unique_ptr<TickLane> L(new TickLane());
    if (!grid_) {
      // loop ticks (a door of the shared grid) launch nothing of their own: no stream, no
      // events.  A lane whose ticks may run on a persistent grid holds its queue: exclusive
      L->skind = persistent_ ? StreamKind::Exclusive : StreamKind::Shared;
      L->stream = stream_create(L->skind);
      HIP_CHECK(hipEventCreate(&L->ev0));
      HIP_CHECK(hipEventCreate(&L->ev1));
      HIP_CHECK(hipEventCreateWithFlags(&L->evb, hipEventBlockingSync | hipEventDisableTiming));
    }
    L->params = base_params_;
    HIP_CHECK(hipMalloc((void**)&L->d_btpl, sizeof(BackendTpl) * 2 * kBackendTpl * ndoors_));
    HIP_CHECK(hipMemset(L->d_btpl, 0, sizeof(BackendTpl) * 2 * kBackendTpl * ndoors_));
    if (grid_) {
      L->h_door = grid_->door(door_);  // the grid's (not freed here)
    } else {
      HIP_CHECK(hipHostMalloc((void**)&L->h_door, sizeof(PDoor), hipHostMallocMapped));
      std::memset((void*)L->h_door, 0, sizeof(PDoor));
      HIP_CHECK(hipMalloc((void**)&L->d_ctl, sizeof(PCtl)));
      HIP_CHECK(hipMemset(L->d_ctl, 0, sizeof(PCtl)));
    }
    // an io loop's engine (loop ticks) carries a few streams per tick: arenas start small
    const size_t arena0 = grid_ ? (1u << 20) : (4u << 20);
    for (TickLane::Buf& B : L->bufs) {
      HIP_CHECK(hipMalloc((void**)&B.d_params, sizeof(KParams)));
      HIP_CHECK(hipHostMalloc((void**)&B.h_params, sizeof(KParams), hipHostMallocMapped));
      ensure_in(B, arena0);
      B.items_cap = 1024;
      HIP_CHECK(hipHostMalloc((void**)&B.h_items, sizeof(WorkItem) * B.items_cap, hipHostMallocMapped));
      HIP_CHECK(hipHostMalloc((void**)&B.h_res, sizeof(WorkResult) * B.items_cap, hipHostMallocMapped));
      std::memset((void*)B.h_res, 0, sizeof(WorkResult) * B.items_cap);  // (pages may be recycled)
    }
    for (int a = 0; a < 3; ++a) L->outs.push_back(new TickLane::OutArena());
    ensure_out(*L, arena0);
    lanes_.push_back(std::move(L));
  }
  host_mode_.assign(max_slots_, 0);
  remote_host_.assign(max_slots_, 0);
  content_len_.assign(max_slots_, 0);
}

HipEngine::~HipEngine() {
  if (grid_) {  // frees below wait for the device: the shared grid must have left
    try {
      grid_->stop();
    } catch (const std::exception&) {
    }
  }
  for (auto& L : lanes_) {
    try {
      stop_persistent(*L);
    } catch (const std::exception&) {
    }
    if (L->stream) hipStreamSynchronize(L->stream);
    if (L->h_door && !grid_) hipHostFree(L->h_door);
    if (L->d_ctl) hipFree(L->d_ctl);
    for (TickLane::Buf& B : L->bufs) {
      if (B.h_in) hipHostFree(B.h_in);
      if (B.h_items) hipHostFree(B.h_items);
      if (B.h_res) hipHostFree(B.h_res);
      if (B.h_dbg) hipHostFree(B.h_dbg);
      if (B.h_params) hipHostFree(B.h_params);
      if (B.d_params) hipFree(B.d_params);
    }
    for (TickLane::OutArena* a : L->outs)
      if (a->p) hipHostFree(a->p);  // the OutArena objects stay (see TickLane::outs)
    if (L->d_btpl) hipFree(L->d_btpl);
    if (L->h_fin) hipHostFree(L->h_fin);
    if (L->h_finres) hipHostFree(L->h_finres);
    if (L->h_fint) hipHostFree(L->h_fint);
    if (L->h_fin_in) hipHostFree(L->h_fin_in);
    if (L->h_fout) hipHostFree(L->h_fout);
    if (L->h_tl) hipHostFree(L->h_tl);
    if (L->d_join) hipFree(L->d_join);
    if (L->d_fout) hipFree(L->d_fout);
    if (L->d_segs) hipFree(L->d_segs);
    if (L->ev0) hipEventDestroy(L->ev0);
    if (L->ev1) hipEventDestroy(L->ev1);
    if (L->evb) hipEventDestroy(L->evb);
    stream_destroy(L->stream, L->skind);
  }
  for (void* p : grave_host_) hipHostFree(p);
  for (void* p : grave_dev_) hipFree(p);
  if (d_state_) hipFree(d_state_);
  if (d_content_) hipFree(d_content_);
}

// Arena growth while serving (the io loop's or lane's thread): timed, because a pinned
// allocation can take milliseconds and the thread serves sockets (kernel_stats: runtime_allocs)
void* HipEngine::halloc(size_t bytes) {
  const double t0 = steady_s();
  void* p = nullptr;
  HIP_CHECK(hipHostMalloc(&p, bytes, hipHostMallocMapped));
  note_alloc(t0, bytes);
  return p;
}
void* HipEngine::dalloc(size_t bytes) {
  const double t0 = steady_s();
  void* p = nullptr;
  HIP_CHECK(hipMalloc(&p, bytes));
  note_alloc(t0, bytes);
  return p;
}
void HipEngine::note_alloc(double t0, size_t bytes) {
  const double us = 1e6 * (steady_s() - t0);
  allocs_.fetch_add(1, std::memory_order_relaxed);
  alloc_bytes_.fetch_add(bytes, std::memory_order_relaxed);
  alloc_us_.store(alloc_us_.load(std::memory_order_relaxed) + us, std::memory_order_relaxed);
  if (us > alloc_max_us_.load(std::memory_order_relaxed)) alloc_max_us_.store(us, std::memory_order_relaxed);
}

void HipEngine::retire_host(void* p) {
  std::lock_guard<std::mutex> g(grave_mu_);
  grave_host_.push_back(p);
}
void HipEngine::retire_dev(void* p) {
  std::lock_guard<std::mutex> g(grave_mu_);
  grave_dev_.push_back(p);
}

void HipEngine::set_persistent(bool on) {
  if (!on)
    for (auto& L : lanes_) {
      std::lock_guard<std::mutex> lg(L->mu);
      stop_persistent(*L);
    }
  persistent_ = on;
}

void HipEngine::debug_poison_results(int ahead) {
  for (auto& Lp : lanes_) {
    TickLane& L = *Lp;
    std::lock_guard<std::mutex> lg(L.mu);
    // a sequence number a coming post will use: door 0's counter (loop ticks: an idle
    // engine's next post goes to its first door) or the lane's own
    uint32_t s = (grid_ ? grid_->door(door_)->posted : L.seq) + (uint32_t)std::max(1, ahead);
    if (s == 0) s = 1;
    for (TickLane::Buf& B : L.bufs)
      for (size_t i = 0; i < B.items_cap; ++i) {
        WorkResult r{};
        r.status = WS_DONE;  // "done, nothing consumed, no output"
        r.seq = s;
        B.h_res[i] = r;
      }
    for (size_t i = 0; i < L.finres_cap; ++i) {
      FinResult r{};
      r.seq = s;
      L.h_finres[i] = r;
    }
  }
}

uint32_t HipEngine::next_seq(TickLane& L) {
  if (++L.seq == 0) ++L.seq;  // 0 never names a tick (fresh result records hold it)
  return L.seq;
}

// The lane's grid is running and will see the next post: launch it when it is not running,
// and replace it when it has been idle long enough that it may be exiting (the host never
// posts to a grid within reach of its idle limit).
void HipEngine::ensure_persistent(TickLane& L) {
  if (L.p_running && steady_s() - L.p_last_post > 0.4e-3 * p_idle_ms_) stop_persistent(L);
  if (L.p_running) return;
  L.h_door->base = L.seq;  // the value posted last before this launch
  hipLaunchKernelGGL(qmx_tick_persistent<2>, dim3(p_grid_), dim3(BS), 0, L.stream, L.h_door, L.d_ctl, p_grid_,
                     ++L.p_gen, (uint32_t)p_idle_ms_ * 100000u, 0);
  HIP_CHECK(hipGetLastError());
  L.p_running = true;
  L.p_last_post = steady_s();
  ++L.p_launches;
}

// Post a stop tick and wait for the grid to leave (it finishes the tick it is on first).
void HipEngine::stop_persistent(TickLane& L) {
  if (!L.p_running) return;
  const uint32_t s = next_seq(L);
  L.h_door->d.stop = 1;
  L.h_door->d.seq = s;
  __atomic_store_n(&L.h_door->posted, s, __ATOMIC_RELEASE);
  L.p_running = false;
  HIP_CHECK(hipStreamSynchronize(L.stream));
}

void HipEngine::ensure_in(TickLane::Buf& B, size_t bytes) {
  if (bytes <= B.in_cap) return;
  if (B.h_in) retire_host(B.h_in);
  B.in_cap = std::max(bytes, B.in_cap * 2);
  B.h_in = (uint8_t*)halloc(B.in_cap + 64);
}
void HipEngine::ensure_out(TickLane& L, size_t bytes) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const size_t k = L.outs.size();
    for (size_t i = 0; i < k; ++i) {  // the last one first: a GPU-warm set of host pages
      const size_t at = (L.out_i + i) % k;
      TickLane::OutArena* a = L.outs[at];
      if (a->refs.load(std::memory_order_acquire) != 0) continue;  // an io loop still reads it
      L.out_i = at;
      if (bytes > a->cap) {
        if (a->p) retire_host(a->p);
        a->cap = std::max(bytes, a->cap * 2);
        a->p = (uint8_t*)halloc(a->cap + 64);
      }
      L.out = a;
      L.h_out = a->p;
      L.out_cap = a->cap;
      return;
    }
    if (k < 16) {  // every arena is still viewed: one more
      L.outs.push_back(new TickLane::OutArena());
      continue;
    }
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10))
      throw std::runtime_error("tick output arenas still viewed by unconsumed results after 10 s");
    sched_yield();
  }
}

void HipEngine::build_params(TickLane& L, int64_t created) {
  KParams& P = L.params;
  put(P.pre1, sizeof(P.pre1), &P.pre1_len, "data: {\"id\": \"chatcmpl-parallel-");
  put(P.pre2, sizeof(P.pre2), &P.pre2_len,
      "\", \"object\": \"chat.completion.chunk\", \"created\": " + std::to_string(created) +
          ", \"model\": \"parallel-proxy\", \"choices\": [{\"index\": 0, \"delta\": {\"content\": \"");
  put(P.suf, sizeof(P.suf), &P.suf_len, kDeltaSuffix);
}

void HipEngine::on_free(int slot) {
  if (slot >= 0 && slot < max_slots_) {
    host_mode_[slot] = 0;
    remote_host_[slot] = 0;
    content_len_[slot] = 0;
  }
}

std::string HipEngine::device_content(int slot, uint32_t len) {
  std::string out(len, '\0');
  if (len) {
    HIP_CHECK(hipSetDevice(device_));  // io loops / exchange threads call this too
    HIP_CHECK(hipMemcpy(&out[0], d_content_ + (size_t)slot * content_cap_, len, hipMemcpyDeviceToHost));
  }
  return out;
}

void* HipEngine::content_device_ptr(int slot, size_t* cap) {
  *cap = 0;
  if (slot < 0 || slot >= max_slots_ || slot >= (int)nslots() || host_mode_[slot]) return nullptr;
  *cap = content_cap_;
  return d_content_ + (size_t)slot * content_cap_;
}

size_t HipEngine::content_size(int slot) {
  if (slot < 0 || slot >= (int)nslots()) return 0;
  if (slot >= max_slots_ || host_mode_[slot] || remote_host_[slot]) return core_[slot].content.size();
  return content_len_[slot];
}

// Spread placement: a remote stream's final text in this (owner) rank's shadow slot, which is
// never fed upstream bytes and is finalized on the GPU like any local stream:
//  * RCCL (bytes == nullptr): the round already wrote it into the slot's HBM content area —
//    its stream was synchronised before the exchange delivered X_BULK, and the finalize that
//    reads it goes out in a later tick, whose items start with a system-scope acquire (the
//    running grid sees it like the host-written tile bytes);
//  * the mesh (bytes): kept with the slot and staged into the finalize item's host-mapped
//    input (prep_finalize), which the item copies into the HBM area first (fin_stage) — no
//    synchronous copy in the io loop;
//  * an RCCL text at world > 1 (host_copied): the exchange's bulk thread copied it out of HBM
//    right after its round (XOptions::host_copy) — staged like a mesh text;
//  * a text longer than the slot's HBM area takes the host path.
void HipEngine::set_remote_content(int slot, const std::string* bytes, size_t len, bool host_copied) {
  if (slot < 0 || slot >= (int)nslots()) return;
  if (slot >= max_slots_ || len > content_cap_) {
    if (slot < max_slots_) host_mode_[slot] = 1;
    core_[slot].content = bytes ? *bytes : std::string();
    return;
  }
  if (bytes) {
    core_[slot].content = *bytes;
    remote_host_[slot] = 1;
    ++(host_copied ? remote_copied_ : remote_staged_);
  } else if (!remote_hbm_direct_) {
    // no host copy came with it (a caller other than the server's exchange path): copy here.
    // (the round's stream was synchronised before the text is applied; this copy is a new
    // dispatch on the device, so it sees the peer's writes)
    core_[slot].content = device_content(slot, len);
    remote_host_[slot] = 1;
    ++remote_copied_;
    ++remote_copied_inline_;
  } else {
    ++remote_dev_;
  }
  content_len_[slot] = (uint32_t)len;
}

void HipEngine::host_open(int slot) {
  // a fresh slot: filter state and content were reset by open(), nothing lives in HBM yet
  if (slot >= 0 && slot < max_slots_) {
    host_mode_[slot] = 1;
    remote_host_[slot] = 0;
    content_len_[slot] = 0;
  }
  ++light_opens_;
}

void HipEngine::escalate(int slot, bool fresh) {
  // migrate the slot to the host path: import filter state + content from HBM
  SlotCore& c = core_[slot];
  if (!fresh) {
    DevSlot ds;
    HIP_CHECK(hipMemcpy(&ds, d_state_ + slot, sizeof(DevSlot), hipMemcpyDeviceToHost));
    c.fs.depth = ds.depth;
    c.fs.tail_len = ds.tail_len;
    std::memcpy(c.fs.tail, ds.tail, kMaxTail);
  } else {
    c.fs = FilterState();
  }
  if (!remote_host_[slot]) c.content = device_content(slot, content_len_[slot]);
  remote_host_[slot] = 0;
  host_mode_[slot] = 1;
  ++escalations_;
}

std::string HipEngine::text(int slot) {
  if (slot < 0 || slot >= (int)nslots()) return std::string();
  const SlotCore& c = core_[slot];
  if (c.aborted) return std::string();
  if (slot >= max_slots_ || host_mode_[slot] || remote_host_[slot]) return c.content;
  return device_content(slot, content_len_[slot]);
}

// One tick of a lane, in phases (HipJob): prepare (arenas filled; may run while the lane's
// previous tick is still on the device), post (doorbell / launch), complete (results).  A
// lane alternates two buffer sets (tiles, items, result records), so the next tick is
// prepared while this one runs and posted the moment it completes (GpuHub, pipelined).
struct HipEngine::HipJob {
  struct Pending {
    int slot;
    size_t carry_len;  // carry bytes that preceded w.data in the tile
    size_t submitted;  // tile bytes
    bool eof_sent;
    Work* w;
  };
  std::vector<Work>* work = nullptr;
  std::vector<FinalizeReq>* fin = nullptr;
  int64_t created = 0;
  int lane = 0, n = 0, m = 0;
  int dk = 0;  // loop ticks: the engine's door the tick went to (its template tables)
  uint32_t seq = 0;
  bool persist = false, new_params = false, posted = false;
  std::vector<Pending> pend;
  std::vector<int> requeue;
  std::vector<Work*> order;
  std::vector<Work*> b[8];
  std::vector<const FinalizeReq*> fin_gpu, fin_host;
  std::vector<SlotResult> host_results;  // escalated streams, processed on the host in prepare
  TickLane::Buf* B = nullptr;
  TickLane::OutArena* arena = nullptr;
  size_t in_off = 0;
  std::chrono::steady_clock::time_point tp0, tp1;
};

void HipEngine::prepare(HipJob& J) {
  TickLane& L = *lanes_[(size_t)J.lane % lanes_.size()];
  std::lock_guard<std::mutex> lg(L.mu);  // kernel_stats() reads the counters under it
  using HC = std::chrono::steady_clock;
  J.tp0 = HC::now();
  J.pend.clear();
  J.requeue.clear();
  J.order.clear();
  J.host_results.clear();
  J.fin_gpu.clear();
  J.fin_host.clear();
  J.posted = false;
  std::vector<Work>& work = *J.work;
  // a buffer set no prepared / in-flight tick holds (two: pipelined lanes, two doors)
  TickLane::Buf* bp = nullptr;
  for (TickLane::Buf& b : L.bufs)
    if (!b.busy) {
      bp = &b;
      break;
    }
  if (!bp) throw std::logic_error("tick prepared with both buffer sets in use");
  TickLane::Buf& B = *bp;
  B.busy = true;
  J.B = &B;
  size_t out_need = 0;
  for (auto& w : work) {
    size_t tot = core_[w.slot].carry.size() + w.data.size();
    size_t sub = std::min(tot, (size_t)tile_);
    out_need += ((12 * sub + 1024) + 15) & ~(size_t)15;
  }
  // tiles at a fixed stride: item n's tile at n x TILE_MAX (the kernel requests its first
  // kSpecTile bytes before it has read the work item)
  ensure_in(B, work.size() * (size_t)TILE_MAX + kSpecTile + 64);
  ensure_out(L, out_need + 64);
  J.arena = L.out;
  // the job holds its arena until complete(): a tick prepared meanwhile (pipelined lanes)
  // must not pick it while this kernel writes it and before any result views it
  J.arena->refs.fetch_add(1, std::memory_order_relaxed);
  if (work.size() > B.items_cap) {
    retire_host(B.h_items);
    retire_host(B.h_res);
    B.items_cap = work.size() * 2;
    B.h_items = (WorkItem*)halloc(sizeof(WorkItem) * B.items_cap);
    B.h_res = (WorkResult*)halloc(sizeof(WorkResult) * B.items_cap);
    std::memset((void*)B.h_res, 0, sizeof(WorkResult) * B.items_cap);  // (pages may be recycled)
  }
  size_t in_off = 0, in_bytes = 0, out_off = 0;
  uint32_t pub_mask = 0;  // backend indices with a publishing item in this tick
  int n = 0;
  // XCD-aware item order: the dispatcher hands workgroup i to XCD i % 8, so item i gets a
  // stream with slot % 8 == i % 8 where possible — a stream's DevSlot state, template and
  // content-arena tail stay in one XCD's L2 from tick to tick.  Host-path streams first.
  {
    for (auto& q : J.b) q.clear();
    for (auto& w : work) {
      if (w.slot >= max_slots_ || host_mode_[w.slot]) J.order.push_back(&w);
      else J.b[w.slot & 7].push_back(&w);
    }
    size_t left = 0;
    for (auto& q : J.b) left += q.size();
    for (int i = 0; left; ++i) {
      int bi = i & 7;
      if (J.b[bi].empty())
        for (int j = 0; j < 8; ++j)
          if (J.b[j].size() > J.b[bi].size()) bi = j;  // affinity bucket empty: the fullest one
      J.order.push_back(J.b[bi].back());
      J.b[bi].pop_back();
      --left;
    }
  }
  for (Work* wp : J.order) {
    Work& w = *wp;
    int slot = w.slot;
    SlotCore& c = core_[slot];
    if (slot >= max_slots_ || host_mode_[slot]) {
      bool was_closed = c.done || c.aborted;
      std::string o;
      process_slot(ts_, c, (const uint8_t*)w.data.data(), w.data.size(), w.eof, J.created, o);
      int flags = (c.done ? RF_DONE : 0) | (c.aborted ? RF_ABORTED : 0) | RF_ESCALATED;
      if (!o.empty() || ((flags & (RF_DONE | RF_ABORTED)) && !was_closed))
        J.host_results.push_back({slot, std::move(o), flags});
      continue;
    }
    if (c.done || c.aborted) continue;
    size_t cl = c.carry.size(), tot = cl + w.data.size();
    size_t sub = std::min(tot, (size_t)tile_);
    bool eof_sent = w.eof && sub == tot;
    // copy carry + data prefix into the arena
    in_off = (size_t)n * TILE_MAX;
    size_t a = std::min(cl, sub);
    std::memcpy(B.h_in + in_off, c.carry.data(), a);
    if (sub > a) std::memcpy(B.h_in + in_off + a, w.data.data(), sub - a);
    WorkItem& it = B.h_items[n];
    it.slot = (uint32_t)slot;
    it.in_off = (uint32_t)in_off;
    it.in_len = (uint32_t)sub;
    it.out_off = (uint32_t)out_off;
    it.out_cap = (uint32_t)(12 * sub + 1024);
    it.flags = (eof_sent ? WF_EOF : 0) | (c.filter ? WF_FILTER : 0) | (c.emit ? WF_EMIT : 0) |
               (c.started ? WF_STARTED : 0) | (w.fresh ? WF_FRESH : 0);
    it.index = (uint32_t)c.index;
    if (c.index >= 0 && c.index < kBackendTpl && !(pub_mask & (1u << c.index))) {
      pub_mask |= 1u << c.index;  // this launch's publisher of its backend's templates
      it.flags |= WF_PUBLISH;
    }
    it.content_len = content_len_[slot];
    in_bytes += sub;
    out_off += ((size_t)it.out_cap + 15) & ~(size_t)15;
    J.pend.push_back({slot, cl, sub, eof_sent, &w});
    ++n;
  }
  J.n = n;
  J.in_off = in_bytes;  // (bytes staged: h2d accounting)
  // finalize requests ride the same launch: workgroups [n, n + m)
  J.fin_gpu = prep_finalize(L, *J.fin, J.fin_host);
  J.m = (int)J.fin_gpu.size();
  // Completion is "record i holds this tick's sequence number", so no record may hold it
  // before this tick's kernel writes it.  Sequence numbers restart with every engine, and
  // pinned host pages freed by an earlier engine in the same process come back from
  // hipHostMalloc with its records in them: a record left at seq v completed tick v of the
  // new engine the moment it was posted (stale consumed / out_len / status, output bytes the
  // kernel was still writing).  That is how backend 1's delta came out labelled
  // chatcmpl-parallel-0 once (profiles/r4/q).  Every record this tick will publish is cleared
  // first; the buffer set and the finalize arenas are this job's alone until complete().
  // (QMX_DEBUG_STALE_RECORDS=1 skips it: the negative control of the stale-record tests)
  if (!keep_stale_records_) {
    for (int i = 0; i < n; ++i) __atomic_store_n(&B.h_res[i].seq, 0u, __ATOMIC_RELAXED);
    for (int i = 0; i < J.m; ++i) __atomic_store_n(&L.h_finres[i].seq, 0u, __ATOMIC_RELAXED);
  }
  if (n + J.m > 0) {
    if (J.created != L.params_created) {  // envelopes carry the second: rebuilt + uploaded once a second
      build_params(L, J.created);
      L.params_created = J.created;
      ++L.params_ver;
    }
    unsigned long long* const dbg0 = L.params.dbg;
    L.params.dbg = nullptr;
    if (stage_timing_) {
      if (B.dbg_cap < (size_t)n) {
        if (B.h_dbg) retire_host(B.h_dbg);
        B.dbg_cap = std::max((size_t)n, B.items_cap);
        HIP_CHECK(hipHostMalloc((void**)&B.h_dbg, sizeof(unsigned long long) * kDbg * B.dbg_cap, hipHostMallocMapped));
      }
      std::memset(B.h_dbg, 0, sizeof(unsigned long long) * kDbg * n);
      L.params.dbg = B.h_dbg;
    }
    if (L.params.dbg != dbg0) ++L.params_ver;
  }
  J.tp1 = HC::now();
  L.host_prep_us += std::chrono::duration<double, std::micro>(J.tp1 - J.tp0).count();
}

void HipEngine::post(HipJob& J) {
  if (J.n + J.m == 0) return;
  TickLane& L = *lanes_[(size_t)J.lane % lanes_.size()];
  std::lock_guard<std::mutex> lg(L.mu);
  TickLane::Buf& B = *J.B;
  // persistent grid (needs polled completion) or a one-shot launch for this tick
  J.persist = grid_ || (persistent_ && poll_);
  if (!J.persist && L.p_running) stop_persistent(L);  // mode switched: the grid must not hold the stream
  J.new_params = B.params_ver != L.params_ver;
  if (J.new_params) {  // the buffer's pinned copy is not touched again until its tick completed
    std::memcpy(B.h_params, &L.params, sizeof(KParams));
    // one-shot launches: a stream-ordered upload; persistent: the grid copies it itself
    if (!J.persist) HIP_CHECK(hipMemcpyAsync(B.d_params, B.h_params, sizeof(KParams), hipMemcpyHostToDevice, L.stream));
    B.params_ver = L.params_ver;
  }
  J.tp1 = std::chrono::steady_clock::now();
  roctxRangePushA("qmx_tick");  // rocprofv3 --marker-trace: one range per tick launch + wait
  L.h2d_bytes += J.in_off;
  // backend template tables of the tick's door set: read its last tick's half, write the other
  J.dk = 0;
  if (grid_) {
    while (J.dk < ndoors_ && door_busy_[J.dk]) ++J.dk;
    if (J.dk == ndoors_) throw std::logic_error("tick posted with every door of the engine busy");
  }
  const uint32_t par = L.tpl_launches[J.dk] & 1;
  BackendTpl* const tpl = L.d_btpl + (size_t)J.dk * 2 * kBackendTpl;
  FinArgs fa{L.h_fin, L.h_fint, L.h_fin_in, L.d_join, L.d_fout, L.h_fout, L.h_finres, L.h_tl, (int2*)L.d_segs};
  if (grid_) {
    // loop-tick mode: this engine's door of the shared grid.  The door's sequence numbers
    // continue from its last post (a grid stop posts stop ticks on every door, under the
    // exclusive side of the guard this post holds the shared side of).
    auto guard = grid_->post_guard();
    PDoor* door = grid_->door(door_ + J.dk);
    door_busy_[J.dk] = 1;
    uint32_t s = door->posted + 1;
    if (s == 0) s = 1;  // (0 never names a tick)
    J.seq = s;
    TickDesc& d = door->d;
    d.items = B.h_items;
    d.in = B.h_in;
    d.out = J.arena->p;
    d.res = B.h_res;
    d.params = B.d_params;
    d.params_src = J.new_params ? B.h_params : nullptr;
    d.btpl_rd = tpl + (size_t)(par ^ 1) * kBackendTpl;
    d.btpl_wr = tpl + (size_t)par * kBackendTpl;
    d.fa = fa;
    d.state = d_state_;
    d.content = d_content_;
    d.seq = s;
    d.n_tick = (uint32_t)J.n;
    d.n_fin = (uint32_t)J.m;
    d.stop = 0;
    __atomic_store_n(&door->posted, s, __ATOMIC_RELEASE);
    grid_->note_post();
    ++L.p_ticks;
    J.posted = true;
    return;
  }
  if (J.persist) ensure_persistent(L);  // before the tick's sequence number: a relaunch starts from L.seq
  J.seq = next_seq(L);
  if (!poll_) HIP_CHECK(hipEventRecord(L.ev0, L.stream));
  if (J.persist) {
    TickDesc& d = L.h_door->d;  // host-mapped: plain stores, then the release store of `posted`
    d.items = B.h_items;
    d.in = B.h_in;
    d.out = J.arena->p;
    d.res = B.h_res;
    d.params = B.d_params;
    d.params_src = J.new_params ? B.h_params : nullptr;
    d.btpl_rd = tpl + (size_t)(par ^ 1) * kBackendTpl;
    d.btpl_wr = tpl + (size_t)par * kBackendTpl;
    d.fa = fa;
    d.state = d_state_;
    d.content = d_content_;
    d.seq = J.seq;
    d.n_tick = (uint32_t)J.n;
    d.n_fin = (uint32_t)J.m;
    d.stop = 0;
    __atomic_store_n(&L.h_door->posted, J.seq, __ATOMIC_RELEASE);
    L.p_last_post = steady_s();
    ++L.p_ticks;
  } else {
    hipLaunchKernelGGL(qmx_tick_kernel, dim3(J.n + J.m), dim3(BS), 0, L.stream, B.h_items, B.h_in, J.arena->p,
                       B.h_res, d_state_, d_content_, B.d_params, J.seq, (uint32_t)J.n, fa,
                       tpl + (size_t)(par ^ 1) * kBackendTpl, tpl + (size_t)par * kBackendTpl);
    HIP_CHECK(hipGetLastError());
  }
  J.posted = true;
}

// Until the posted tick is about to complete (the expected time less the next tick's
// preparation): the lane then prepares the next tick, so it can post it at once.
void HipEngine::wait_near(HipJob& J) {
  if (!J.posted) return;
  TickLane& L = *lanes_[(size_t)J.lane % lanes_.size()];
  const double el = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - J.tp1).count();
  // the device's own clock (kernel span per tick) sets the target: an estimate from host
  // wake-ups would include this very nap and drift upward tick after tick
  const double prep = L.launches ? L.host_prep_us / (double)L.launches : 5.0;
  const double target = L.span_ema_us + 6.0 - prep;
  if (target - el >= 2.0) {
    timespec ts{0, (long)((target - el) * 1000)};
    nanosleep(&ts, nullptr);
  }
}

void HipEngine::complete(HipJob& J, std::vector<SlotResult>& results, std::vector<FinalizeRes>& fres) {
  TickLane& L = *lanes_[(size_t)J.lane % lanes_.size()];
  std::lock_guard<std::mutex> lg(L.mu);
  using HC = std::chrono::steady_clock;
  for (auto& r : J.host_results) results.push_back(std::move(r));
  J.host_results.clear();
  const int n = J.n, m = J.m;
  TickLane::Buf& B = *J.B;
  // one stream's result → slot state + SSE; run as each result record is published (the
  // host's share of a tick overlaps the kernel's stragglers), the rest after the wait
  int n_done = 0;
  auto process_item = [&](int i) {
    HipJob::Pending& p = J.pend[i];
    SlotCore& c = core_[p.slot];
    const WorkResult r = B.h_res[i];
    Work& w = *p.w;
    // the unconsumed remainder (carry + data)[consumed:] becomes the carry, in place
    auto keep_remainder = [&](size_t consumed) {
      const size_t cl = p.carry_len;
      if (consumed < cl) {
        c.carry.erase(0, consumed);
        c.carry += w.data;
      } else {
        c.carry.assign(w.data, consumed - cl, std::string::npos);
      }
    };
    bool no_progress = (r.status & WS_ESCALATE) ||
                       (p.submitted == (size_t)tile_ && r.consumed == 0 && !(r.status & (WS_DONE | WS_ABORTED)));
    if (no_progress) {
      escalate(p.slot, w.fresh);
      keep_remainder(0);
      std::string all;
      all.swap(c.carry);
      bool was_closed = c.done || c.aborted;
      std::string o;
      process_slot(ts_, c, (const uint8_t*)all.data(), all.size(), w.eof, J.created, o);
      int flags = (c.done ? RF_DONE : 0) | (c.aborted ? RF_ABORTED : 0) | RF_ESCALATED;
      if (!o.empty() || ((flags & (RF_DONE | RF_ABORTED)) && !was_closed)) results.push_back({p.slot, std::move(o), flags});
      return;
    }
    if (r.status & WS_STARTED) c.started = true;
    content_len_[p.slot] = r.content_len;
    int flags = 0;
    if (r.status & WS_ABORTED) {
      c.aborted = true;
      c.carry.clear();
      flags |= RF_ABORTED;
    } else {
      keep_remainder(r.consumed);
      if (r.status & WS_DONE) {
        c.done = true;
        c.carry.clear();
        flags |= RF_DONE;
      } else if ((r.status & WS_MORE) || p.submitted < p.carry_len + w.data.size()) {
        J.requeue.push_back(p.slot);  // unprocessed bytes (or a pending EOF) remain
      }
    }
    L.d2h_bytes += r.out_len;
    const char* bytes = (const char*)J.arena->p + B.h_items[i].out_off;
    if (r.out_len && !views_) {
      results.push_back({p.slot, std::string(bytes, r.out_len), flags});
    } else if (r.out_len) {  // a view into this tick's output arena: the io loop copies the bytes once
      SlotResult x{p.slot, std::string(), flags};
      x.view = bytes;
      x.view_len = r.out_len;
      x.hold = ViewRef(&J.arena->refs);
      results.push_back(std::move(x));
    } else if (flags) {
      results.push_back({p.slot, std::string(), flags});
    }
  };
  if (J.posted) {
    // sessions the GPU does not finalize (escalated streams) are finalized here meanwhile
    for (const FinalizeReq* r : J.fin_host) finalize_host(*r, fres);
    if (poll_) {
      // one HIP call per tick, or none: completion and kernel span come from the result records
      wait_results(L, n, m, J.seq, B.h_res, J.tp1, [&](int i) {
        const auto ti = HC::now();
        if (n_done == 0) L.first_result_us += std::chrono::duration<double, std::micro>(ti - J.tp1).count();
        if (i == n_done) process_item(n_done++);
        L.items_host_us += std::chrono::duration<double, std::micro>(HC::now() - ti).count();
      });
      uint64_t a = ~0ull, b = 0, t0max = 0;
      double item_ticks = 0;
      for (int i = 0; i < n; ++i) {
        a = std::min(a, B.h_res[i].t0);
        b = std::max(b, B.h_res[i].t1);
        t0max = std::max(t0max, B.h_res[i].t0);
        item_ticks += (double)(B.h_res[i].t1 - B.h_res[i].t0);
      }
      if (n > 0) {  // do a tick's items run side by side? (one item's run vs the spread of starts)
        L.item_us += item_ticks * 1e-2 / n;
        L.start_spread_us += (double)(t0max - a) * 1e-2;
      }
      if (J.persist && n > 0) {  // the grid's side of the tick (its own clock): doorbell seen ->
        // relayed -> first item started -> last item done
        const PDoor* dr = grid_ ? grid_->door(door_ + J.dk) : L.h_door;
        const uint64_t ts = __atomic_load_n(&dr->t_seen, __ATOMIC_ACQUIRE);
        const uint64_t tr = __atomic_load_n(&dr->t_relayed, __ATOMIC_ACQUIRE);
        if (ts && tr >= ts && a >= tr && b >= a) {
          L.lead_ema_us = 0.85 * L.lead_ema_us + 0.15 * std::min((double)(a - ts) * 1e-2, 500.0);
          if (grid_) {
            // the hops between the two clocks.  Every tick bounds the clock offset (host time −
            // device time): the relay saw the doorbell after the host posted it (off >= post −
            // seen) and the host took the results after the last item finished (off <= now −
            // done).  The offset used is the largest lower bound of the current 100 ms window
            // (and the previous one: drift between the host clock and the 100 MHz device
            // clock stays far below a microsecond there), which includes this tick's: no hop
            // can come out negative.  The window's upper − lower bound is the uncertainty left
            // (clock_window_us); the symmetric round-trip calibration (HipGrid::calibrate) it
            // replaces read post -> seen 1.1 us too short (r4: negative).
            const double post_h = std::chrono::duration<double, std::micro>(J.tp1.time_since_epoch()).count();
            const double now_h = std::chrono::duration<double, std::micro>(HC::now().time_since_epoch()).count();
            const double lo = post_h - (double)ts * 1e-2, hi = now_h - (double)b * 1e-2;
            if (now_h - L.cwin_t0 > 1e5) {  // a new window
              L.clo_prev = L.clo;
              if (L.clo > -1e299 && L.chi < 1e299 && L.chi >= L.clo) {
                L.cwin_sum += L.chi - L.clo;
                ++L.cwin_n;
              }
              L.clo = -1e300;
              L.chi = 1e300;
              L.cwin_t0 = now_h;
            }
            L.clo = std::max(L.clo, lo);
            L.chi = std::min(L.chi, hi);
            const double off = std::max(L.clo, L.clo_prev);
            const double seen_h = (double)ts * 1e-2 + off, done_h = (double)b * 1e-2 + off;
            if (seen_h >= post_h - 5.0 && now_h >= done_h - 5.0) {
              L.post_seen_us += seen_h - post_h;
              L.done_host_us += now_h - done_h;
              ++L.hop_ticks;
            }
          }
          L.relay_us += (double)(tr - ts) * 1e-2;
          L.pickup_us += (double)(a - tr) * 1e-2;
          L.grid_span_us += (double)(b - ts) * 1e-2;
          ++L.grid_ticks;
        }
      }
      for (int i = 0; i < m; ++i) {
        a = std::min(a, L.h_finres[i].t0);
        b = std::max(b, L.h_finres[i].t1);
      }
      if (b > a) {
        L.kernel_ms += (double)(b - a) * 1e-5;  // 100 MHz ticks -> ms
        L.span_ema_us = 0.85 * L.span_ema_us + 0.15 * std::min((double)(b - a) * 1e-2, 2000.0);
      }
    } else {
      HIP_CHECK(hipEventRecord(L.ev1, L.stream));
      wait_stream(L);
      L.timing_pending = true;
      collect_timing(L);
    }
    roctxRangePop();
    L.gpu_wait_us += std::chrono::duration<double, std::micro>(HC::now() - J.tp1).count();
    ++L.launches;
    ++L.tpl_launches[J.dk];
    if (grid_) door_busy_[J.dk] = 0;
    L.items += n;
    if (m > 0) {
      ++L.fin_launches;
      L.fin_items += m;
    }
    if (L.params.dbg && L.params.dbg == B.h_dbg) {
      for (int i = 0; i < n; ++i) {
        const unsigned long long* d = B.h_dbg + kDbg * i;
        if (d[12] > d[11] && d[10] > d[0]) {
          L.clk_cycles += (double)(d[12] - d[11]);
          L.clk_us += (double)(d[10] - d[0]) * 0.01;
        }
        int prev = 0;
        for (int k = 1; k < 11; ++k) {
          if (!d[k]) continue;
          L.stage_us[k] += (double)(d[k] - d[prev]) * 0.01;  // 100 MHz ticks -> us
          prev = k;
        }
        // sub-stages: S3a prepass / S3 event loop / template persist; s4_wave match / cuts / compaction
        auto sub = [&](int slot, int a, int b) {
          if (d[a] && d[b] && d[b] >= d[a]) L.stage_us[slot] += (double)(d[b] - d[a]) * 0.01;
        };
        sub(11, 3, 21);
        sub(12, 21, 22);
        sub(13, 22, 4);
        sub(14, 5, 23);
        sub(15, 23, 24);
        sub(16, 23, 25);  // s4_wave cuts: token list + depth scan / the holdback cuts
        sub(17, 25, 24);
        sub(18, 9, 26);   // S6 write: output window fill / host-memory stores
        sub(19, 26, 10);
        sub(21, 5, 28);   // s4_wave: call entry / candidate scan / MFMA match
        sub(22, 28, 29);
        sub(23, 29, 23);
        sub(24, 25, 30);  // s4 holdback: candidate walk / prefix tests / cut stores
        sub(25, 30, 31);
        sub(26, 31, 24);
        sub(27, 24, 32);  // s4 compaction / s6 sizing on wave 0 / the stage's barrier
        sub(28, 32, 33);
        sub(29, 33, 7);
        sub(30, 3, 34);   // S3a: wave 0's own events / the wait for the slowest wave
        sub(31, 34, 21);
        sub(32, 3, 35);   // S3a on wave 0: before its rounds / round 1 / the rest
        sub(33, 35, 36);
        sub(34, 36, 34);
        sub(35, 35, 38);  // S3a round 1 on wave 0: content-template compare / other shapes (b) / the rest
        sub(36, 38, 39);
        sub(37, 39, 36);
        if (d[27] && d[27] >= B.h_res[i].t1 && B.h_res[i].t1) L.stage_us[20] += (double)(d[27] - B.h_res[i].t1) * 0.01;
      }
      L.stage_n += n;
      for (int i = 0; i < n; ++i) {
        L.s3_full += B.h_dbg[kDbg * i + 13];
        L.s3_tpl += B.h_dbg[kDbg * i + 14];
        L.s3_events += B.h_dbg[kDbg * i + 15];
        L.s3_cyc_full += B.h_dbg[kDbg * i + 16];
        L.s3_cyc_tpl += B.h_dbg[kDbg * i + 17];
        L.s3_cyc_lex += B.h_dbg[kDbg * i + 18];
        L.s3_hole += B.h_dbg[kDbg * i + 19];
        L.s3_cyc_hole += B.h_dbg[kDbg * i + 20];
        L.s3a_unres += B.h_dbg[kDbg * i + 37];
      }
    }
  }
  for (; n_done < n; ++n_done) process_item(n_done);  // the rest (event wait, stage timing)
  if (m > 0) collect_finalize(L, J.fin_gpu, fres);
  if (!J.posted)
    for (const FinalizeReq* r : J.fin_host) finalize_host(*r, fres);
  if (!J.requeue.empty()) {
    std::lock_guard<std::mutex> g(mu_);
    for (int s : J.requeue) {
      Meta& mt = meta_[s];
      if (!mt.live || mt.dirty) continue;
      mt.dirty = true;
      dirty_.push_back(s);
    }
  }
  J.arena->refs.fetch_sub(1, std::memory_order_release);  // results hold their own references
  J.B->busy = false;
  L.process_us += std::chrono::duration<double, std::micro>(HC::now() - J.tp0).count();
}

void HipEngine::run_tick(std::vector<Work>& work, std::vector<FinalizeReq>& fin, int64_t created,
                         std::vector<SlotResult>& results, std::vector<FinalizeRes>& fres, int lane) {
  thread_local HipJob J;
  J.work = &work;
  J.fin = &fin;
  J.created = created;
  J.lane = lane;
  prepare(J);
  post(J);
  complete(J, results, fres);
}

// ---- pipelined ticks (GpuHub lanes) ---------------------------------------------------
HipEngine::HipJob& HipEngine::hjob(Job& j) {
  if (!j.impl) j.impl = std::make_shared<HipJob>();
  HipJob& J = *std::static_pointer_cast<HipJob>(j.impl);
  J.work = &j.work;
  J.fin = &j.fin;
  J.created = j.created;
  J.lane = j.lane;
  return J;
}
int HipEngine::free_doors() const {
  int k = 0;
  for (char b : door_busy_) k += !b;
  return k;
}

bool HipEngine::job_ready(Job& j, double* expect_us) {
  HipJob& J = hjob(j);
  if (expect_us) *expect_us = 0;
  if (!J.posted) return true;
  TickLane& L = *lanes_[(size_t)J.lane % lanes_.size()];
  const WorkResult* res = J.B->h_res;
  for (int i = 0; i < J.n; ++i)
    if (__atomic_load_n(&res[i].seq, __ATOMIC_ACQUIRE) != J.seq) goto pending;
  for (int i = 0; i < J.m; ++i)
    if (__atomic_load_n(&L.h_finres[i].seq, __ATOMIC_ACQUIRE) != J.seq) goto pending;
  return true;
pending:
  // from the device's own clocks (doorbell seen -> first item, kernel span), not from host
  // wake-ups: a poller that sleeps until an estimate built from its own wake-ups never
  // wakes earlier than that estimate, and the estimate only drifts up
  if (expect_us)
    *expect_us = L.lead_ema_us + L.span_ema_us + 3.0 -
                 std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - J.tp1).count();
  return false;
}

void HipEngine::job_prepare(Job& j) { prepare(hjob(j)); }
void HipEngine::job_post(Job& j) { post(hjob(j)); }
void HipEngine::job_wait_near(Job& j) { wait_near(hjob(j)); }
void HipEngine::job_complete(Job& j, std::vector<SlotResult>& results, std::vector<FinalizeRes>& fres) {
  complete(hjob(j), results, fres);
}

void HipEngine::finalize_host(const FinalizeReq& r, std::vector<FinalizeRes>& out) {
  std::vector<std::string> texts;
  for (int s : r.slots) texts.push_back(text(s));
  FinalizeRes fr;
  finalize_texts(ts_, texts, r, fr);
  out.push_back(std::move(fr));
  ++fin_host_;
}

template <class T>
static void grow_mapped(HipEngine* e, T** p, size_t* cap, size_t need, void (HipEngine::*retire)(void*)) {
  if (need <= *cap) return;
  if (*p) (e->*retire)(*p);
  *cap = std::max(need, *cap * 2);
  *p = (T*)e->halloc(sizeof(T) * *cap + 64);
  std::memset((void*)*p, 0, sizeof(T) * *cap + 64);  // (pinned pages may come back recycled)
}
static void grow_device(HipEngine* e, uint8_t** p, size_t* cap, size_t need, void (HipEngine::*retire)(void*)) {
  if (need <= *cap) return;
  if (*p) (e->*retire)(*p);
  *cap = std::max(need, *cap * 2);
  *p = (uint8_t*)e->dalloc(*cap + 64);
}

// Finalize items of a tick, staged in the lane's arenas for the fused launch.  Sessions whose
// texts are all HBM-resident run on the GPU (K3+K4+K5 workgroups); a session with an
// escalated (host-path) stream is finalized on the host.
std::vector<const FinalizeReq*> HipEngine::prep_finalize(TickLane& L, std::vector<FinalizeReq>& reqs,
                                                         std::vector<const FinalizeReq*>& host) {
  std::vector<const FinalizeReq*> gpu;
  if (reqs.empty()) return gpu;
  const int nsl = (int)nslots();
  size_t ntext = 0, in_bytes = 0;
  for (auto& r : reqs) {
    bool dev = true;
    for (int s : r.slots) dev = dev && s >= 0 && s < max_slots_ && s < nsl && !host_mode_[s];
    if (!dev) {
      host.push_back(&r);
      continue;
    }
    gpu.push_back(&r);
    ntext += r.slots.size();
    in_bytes += ((r.joiner.size() + 15) & ~(size_t)15) + 256 + 64;
    for (int s : r.slots)
      if (remote_host_[s] && !core_[s].aborted) in_bytes += (content_len_[s] + 15) & ~(size_t)15;
  }
  if (gpu.empty()) return gpu;
  const int n = (int)gpu.size();
  grow_mapped(this, &L.h_fin, &L.fin_cap, (size_t)n, &HipEngine::retire_host);
  grow_mapped(this, &L.h_finres, &L.finres_cap, (size_t)n, &HipEngine::retire_host);
  grow_mapped(this, &L.h_fint, &L.fint_cap, ntext, &HipEngine::retire_host);
  grow_mapped(this, &L.h_tl, &L.tl_cap, ntext, &HipEngine::retire_host);
  grow_mapped(this, &L.h_fin_in, &L.fin_in_cap, in_bytes, &HipEngine::retire_host);
  size_t join_off = 0, out_off = 0, in_off = 0, t_off = 0, seg_off = 0;
  const std::string suf = kFinalSuffix;
  for (int i = 0; i < n; ++i) {
    const FinalizeReq& r = *gpu[i];
    FinItem& it = L.h_fin[i];
    size_t total = 0, longest = 0;
    it.first_text = (uint32_t)t_off;
    it.n_texts = (uint32_t)r.slots.size();
    it.tl_off = (uint32_t)t_off;
    for (int s : r.slots) {
      const uint32_t len = core_[s].aborted ? 0u : content_len_[s];
      uint32_t stage = kNoStage;
      if (remote_host_[s] && len) {  // a mesh-delivered final: the item copies it to HBM first
        stage = (uint32_t)in_off;
        std::memcpy(L.h_fin_in + in_off, core_[s].content.data(), len);
        in_off += (len + 15) & ~(size_t)15;
        ++L.fin_staged;
      }
      L.h_fint[t_off++] = FinText{(uint32_t)s, len, stage, 0};
      total += len;
      longest = std::max(longest, (size_t)len);
    }
    if (r.slots.size() > 1) total += (r.slots.size() - 1) * r.joiner.size();
    const std::string pre = r.texts ? std::string() : final_prefix(r.created);
    it.flags = (r.strip ? 1u : 0u) | (r.texts ? 2u : 0u);
    it.joiner_off = (uint32_t)in_off;
    it.joiner_len = (uint32_t)r.joiner.size();
    std::memcpy(L.h_fin_in + in_off, r.joiner.data(), r.joiner.size());
    in_off += (r.joiner.size() + 15) & ~(size_t)15;
    it.pre_off = (uint32_t)in_off;
    it.pre_len = (uint32_t)pre.size();
    std::memcpy(L.h_fin_in + in_off, pre.data(), pre.size());
    in_off += (pre.size() + 15) & ~(size_t)15;
    it.suf_off = (uint32_t)in_off;
    it.suf_len = (uint32_t)suf.size();
    std::memcpy(L.h_fin_in + in_off, suf.data(), suf.size());
    in_off += (suf.size() + 15) & ~(size_t)15;
    it.join_off = (uint32_t)join_off;
    join_off += (total + 15) & ~(size_t)15;
    // kept segments of one text: an interval spans >= 7 bytes ("<t></t>"), so <= len/7 + 2
    it.seg_off = (uint32_t)seg_off;
    it.seg_cap = r.strip ? (uint32_t)(longest / 4 + 4) : 1u;
    seg_off += it.seg_cap;
    const size_t cap = r.texts ? total : 6 * total + pre.size() + suf.size();
    it.out_off = (uint32_t)out_off;
    it.out_cap = (uint32_t)cap;
    out_off += (cap + 15) & ~(size_t)15;
  }
  grow_device(this, &L.d_join, &L.join_cap, join_off + 16, &HipEngine::retire_dev);
  grow_device(this, &L.d_fout, &L.dfout_cap, out_off + 16, &HipEngine::retire_dev);
  grow_device(this, &L.d_segs, &L.segs_cap, seg_off * sizeof(int2) + 16, &HipEngine::retire_dev);
  grow_mapped(this, &L.h_fout, &L.fout_cap, out_off + 16, &HipEngine::retire_host);
  return gpu;
}

void HipEngine::collect_finalize(TickLane& L, const std::vector<const FinalizeReq*>& gpu,
                                 std::vector<FinalizeRes>& out) {
  for (size_t i = 0; i < gpu.size(); ++i) {
    const FinalizeReq& r = *gpu[i];
    const FinResult fr = L.h_finres[i];
    if (fr.status) {
      finalize_host(r, out);
      continue;
    }
    FinalizeRes res;
    res.id = r.id;
    const char* base = (const char*)L.h_fout + L.h_fin[i].out_off;
    if (r.texts) {
      res.kind = 2;
      size_t o = 0;
      for (uint32_t k = 0; k < fr.n_kept; ++k) {
        const uint32_t tl = L.h_tl[L.h_fin[i].tl_off + k];
        res.texts.emplace_back(base + o, tl);
        o += tl;
      }
    } else if (fr.n_kept == 0) {
      res.kind = 0;
    } else {
      res.kind = 1;
      res.event.assign(base, fr.out_len);
    }
    out.push_back(std::move(res));
  }
}

std::unordered_map<std::string, double> HipEngine::kernel_stats() {
  std::unordered_map<std::string, double> m;
  double stage[38] = {0}, cyc = 0, cus = 0;
  for (auto& Lp : lanes_) {
    TickLane& L = *Lp;
    std::lock_guard<std::mutex> lg(L.mu);
    m["launches"] += (double)L.launches;
    m["persistent_revivals"] += (double)L.p_revivals;
    m["persistent_grids"] += (double)L.p_launches;  // persistent mode: grid launches (ticks ride doorbells)
    m["persistent_ticks"] += (double)L.p_ticks;
    m["items"] += (double)L.items;
    m["kernel_ms"] += L.kernel_ms;
    m["stage_items"] += (double)L.stage_n;
    m["h2d_bytes"] += (double)L.h2d_bytes;
    m["d2h_bytes"] += (double)L.d2h_bytes;
    m["s3_full_parses"] += (double)L.s3_full;
    m["s3_template_hits"] += (double)L.s3_tpl;
    m["s3_events"] += (double)L.s3_events;
    m["s3_cycles_full"] += (double)L.s3_cyc_full;
    m["s3_cycles_template"] += (double)L.s3_cyc_tpl;
    m["s3_cycles_lex"] += (double)L.s3_cyc_lex;
    m["s3_hole_hits"] += (double)L.s3_hole;
    m["s3_cycles_hole"] += (double)L.s3_cyc_hole;
    m["s3a_unresolved"] += (double)L.s3a_unres;  // events S3a left to its loop (stage timing)
    m["host_prep_us"] += L.host_prep_us;
    m["gpu_wait_us"] += L.gpu_wait_us;
    m["first_result_us"] += L.first_result_us;
    m["item_us"] += L.item_us;
    m["items_host_us"] += L.items_host_us;
    m["relay_us"] += L.relay_us;
    m["pickup_us"] += L.pickup_us;
    m["grid_span_us"] += L.grid_span_us;
    m["grid_ticks"] += L.grid_ticks;
    m["post_seen_us"] += L.post_seen_us;  // loop ticks: host post -> relay saw it (calibrated clocks)
    m["done_host_us"] += L.done_host_us;  // last item done -> the io loop took the results
    m["hop_ticks"] += L.hop_ticks;
    m["clock_window_us"] += L.cwin_sum;  // summed over 100 ms windows (mean: / clock_windows)
    m["clock_windows"] += L.cwin_n;
    m["start_spread_us"] += L.start_spread_us;
    m["process_us"] += L.process_us;
    m["poll_fallbacks"] += (double)L.poll_fallbacks;
    m["fin_launches"] += (double)L.fin_launches;  // tick launches that also carried finalize work
    m["fin_items"] += (double)L.fin_items;
    m["fin_staged_texts"] += (double)L.fin_staged;  // mesh-delivered remote finals staged into items
    for (int k = 1; k < 38; ++k) stage[k] += L.stage_us[k];
    cyc += L.clk_cycles;
    cus += L.clk_us;
  }
  for (int k = 1; k < 11; ++k) m["stage" + std::to_string(k) + "_us"] = stage[k];
  m["stage_s3a_us"] = stage[11];
  m["stage_s3loop_us"] = stage[12];
  m["stage_s3persist_us"] = stage[13];
  m["stage_s4match_us"] = stage[14];
  m["stage_s4cuts_us"] = stage[15];
  m["stage_s4tok_us"] = stage[16];
  m["stage_s4hold_us"] = stage[17];
  m["stage_s6fill_us"] = stage[18];
  m["stage_s6store_us"] = stage[19];
  m["stage_s4entry_us"] = stage[21];
  m["stage_s4scan_us"] = stage[22];
  m["stage_s4mfma_us"] = stage[23];
  m["stage_s4holdwalk_us"] = stage[24];
  m["stage_s4holdpref_us"] = stage[25];
  m["stage_s4holdstore_us"] = stage[26];
  m["stage_s4compact_us"] = stage[27];
  m["stage_s6size_us"] = stage[28];
  m["stage_s4barrier_us"] = stage[29];
  m["stage_s3awave0_us"] = stage[30];
  m["stage_s3await_us"] = stage[31];
  m["stage_s3apre_us"] = stage[32];
  m["stage_s3around1_us"] = stage[33];
  m["stage_s3arest_us"] = stage[34];
  m["stage_s3ar1tpl_us"] = stage[35];
  m["stage_s3ar1b_us"] = stage[36];
  m["stage_s3ar1end_us"] = stage[37];
  m["stage_fence_us"] = stage[20];  // the item's system-scope release fence (L2 write-back)
  m["shader_mhz"] = cus > 0 ? cyc / cus : 0.0;
  m["clk_cycles"] = cyc;  // summable across engines (/metrics sums the io loops' engines)
  m["clk_us"] = cus;
  m["escalations"] = (double)escalations_.load();
  m["light_host_opens"] = (double)light_opens_.load();  // streams opened on the host path (latency mode)
  m["fin_host"] = (double)fin_host_.load();
  m["remote_texts_hbm"] = (double)remote_dev_.load();        // spread owner: finals an RCCL round put in HBM
  m["remote_texts_staged"] = (double)remote_staged_.load();  // ... that came over the mesh
  m["remote_texts_copied"] = (double)remote_copied_.load();  // ... an RCCL round wrote, copied to the host (world > 1)
  m["remote_texts_copied_inline"] = (double)remote_copied_inline_.load();
  m["runtime_allocs"] = (double)allocs_.load();  // arena growths while serving
  m["runtime_alloc_MB"] = 1e-6 * (double)alloc_bytes_.load();
  m["runtime_alloc_us"] = alloc_us_.load();
  m["runtime_alloc_max_us"] = alloc_max_us_.load();  // ... of them by the engine's caller (not the exchange)
  m["lanes"] = (double)lanes_.size();
  m["fin_separate_launches"] = 0.0;  // finalize no longer has a launch (or a wait) of its own
  if (grid_ && door_ == 0)  // the shared grid's counters, once per process
    for (auto& kv : grid_->stats()) m[kv.first] += kv.second;
  if (!grid_ || door_ == 0)  // the process's HIP streams and queue limit, once per process
    for (auto& kv : stream_stats()) m[kv.first] = kv.second;
  return m;
}

// ---- the multi-door grid (loop ticks) ----------------------------------------------------
HipGrid::HipGrid(int device, int doors, int wg_per_door, int idle_ms)
    : device_(device), n_(std::max(1, doors)), wpd_(std::max(1, wg_per_door)), idle_ms_(std::max(5, idle_ms)) {
  // every workgroup of a persistent grid must be resident at once (a relay that is not never
  // relays its door's ticks), and the tick kernels run one workgroup per CU (LDS, VGPRs):
  // keep the grid within half the device's CUs — room for a second process's grid during a
  // rolling reload, and for a partitioned GPU (CPX: 32 CUs per logical device)
  {
    hipDeviceProp_t pr{};
    HIP_CHECK(hipGetDeviceProperties(&pr, device_));
    // processes sharing the GPU (rank rehearsals) split that half between their grids
    const char* sh = env_get("QMX_GPU_SHARERS");
    const int sharers = sh ? std::max(1, atoi(sh)) : 1;
    // QMX_GRID_OCC=2: the register-capped kernel, two workgroups per CU — the budget is half
    // the device's workgroup slots, not half its CUs
    if (const char* oc = env_get("QMX_GRID_OCC")) occ_ = atoi(oc) == 2 ? 2 : 1;
    const int cus = std::max(1, pr.multiProcessorCount), budget = cus * occ_ / 2 / sharers;
    if (n_ * wpd_ > budget) wpd_ = std::max(1, budget / n_);
    if (n_ * wpd_ > budget) throw std::runtime_error("grid: " + std::to_string(n_) + " doors do not fit " +
                                                     std::to_string(cus) + " CUs shared by " +
                                                     std::to_string(sharers) + " processes");
  }
  // XCD-local sub-grids (QMX_GRID_XCD=0: contiguous blocks per door, every door on all XCDs)
  const char* x = env_get("QMX_GRID_XCD");
  interleave_ = (x ? atoi(x) != 0 : true) && n_ % 8 == 0;
  HIP_CHECK(hipSetDevice(device_));
  stream_ = stream_create(StreamKind::Exclusive);  // the grid holds its queue: nothing may queue behind it
  HIP_CHECK(hipHostMalloc((void**)&h_doors_, sizeof(PDoor) * (size_t)n_, hipHostMallocMapped));
  std::memset((void*)h_doors_, 0, sizeof(PDoor) * (size_t)n_);
  HIP_CHECK(hipMalloc((void**)&d_ctls_, sizeof(PCtl) * (size_t)n_));
  HIP_CHECK(hipMemset(d_ctls_, 0, sizeof(PCtl) * (size_t)n_));
  HIP_CHECK(hipDeviceSynchronize());  // the zeroed control blocks before any launch reads them
}

HipGrid::~HipGrid() {
  try {
    stop();
  } catch (const std::exception& e) {
    fprintf(stderr, "qmx: grid stop failed: %s\n", e.what());
  }
  if (stream_) hipStreamSynchronize(stream_);
  if (h_doors_) hipHostFree(h_doors_);
  if (d_ctls_) hipFree(d_ctls_);
  stream_destroy(stream_, StreamKind::Exclusive);
}

PDoor* HipGrid::door(int d) const { return h_doors_ + d; }

std::shared_lock<std::shared_mutex> HipGrid::post_guard() {
  for (;;) {
    std::shared_lock<std::shared_mutex> lk(mu_);
    if (running_.load(std::memory_order_acquire)) return lk;
    lk.unlock();
    std::unique_lock<std::shared_mutex> ex(mu_);
    if (!running_.load(std::memory_order_relaxed)) launch_locked();
  }
}

void HipGrid::note_post() { last_post_.store(steady_s(), std::memory_order_relaxed); }

// Each sub-grid starts from the last tick its door's relay saw: a tick posted to a grid that
// left without relaying it (the host's heartbeat stopped) is picked up by the new launch.
void HipGrid::launch_locked() {
  const double t0 = steady_s();
  HIP_CHECK(hipSetDevice(device_));
  for (int d = 0; d < n_; ++d) h_doors_[d].base = __atomic_load_n(&h_doors_[d].relayed, __ATOMIC_ACQUIRE);
  const uint32_t idle_ticks = 2000u * 100000u;  // 2 s at 100 MHz: only a host that stopped beating
  if (occ_ == 2)
    hipLaunchKernelGGL(qmx_tick_persistent<4>, dim3(n_ * wpd_), dim3(BS), 0, stream_, h_doors_, d_ctls_, wpd_, ++gen_,
                       idle_ticks, interleave_ ? 1 : 0);
  else
    hipLaunchKernelGGL(qmx_tick_persistent<2>, dim3(n_ * wpd_), dim3(BS), 0, stream_, h_doors_, d_ctls_, wpd_, ++gen_,
                       idle_ticks, interleave_ ? 1 : 0);
  HIP_CHECK(hipGetLastError());
  last_post_.store(steady_s(), std::memory_order_relaxed);
  running_.store(true, std::memory_order_release);
  ++launches_;
  const double t1 = steady_s();
  // calibration reuses door 0's descriptor: never while a tick posted there is still unrelayed
  // (a revived grid or a relaunch after an idle exit picks that tick up from `base`; writing
  // the calibration tick over its descriptor would run an empty tick in its place)
  if (__atomic_load_n(&h_doors_[0].relayed, __ATOMIC_ACQUIRE) == h_doors_[0].posted) calibrate_locked();
  // (every door's poster waits for this under the grid lock: its cost is io-loop stall time)
  const double t2 = steady_s();
  launch_us_max_ = std::max(launch_us_max_, 1e6 * (t1 - t0));
  launch_cal_us_max_ = std::max(launch_cal_us_max_, 1e6 * (t2 - t1));
  launch_us_sum_ += 1e6 * (t2 - t0);
}

// Clock calibration (timing only): empty ticks on door 0, each timed on the host from the
// post to the relay's `relayed` store; the relay stamped s_memrealtime when it saw the post.
// The quickest round trip bounds the offset best (error <= its half).  Under the exclusive
// lock: no door is posting.
void HipGrid::calibrate_locked() {
  PDoor& D = h_doors_[0];
  double best = 1e9, off = 0;
  for (int i = 0; i < 12; ++i) {
    uint32_t s = D.posted + 1;
    if (s == 0) s = 1;
    D.d.n_tick = 0;
    D.d.n_fin = 0;
    D.d.stop = 0;
    D.d.params_src = nullptr;
    D.d.seq = s;
    const uint64_t seen0 = __atomic_load_n(&D.t_seen, __ATOMIC_ACQUIRE);
    const double h0 = steady_s();
    __atomic_store_n(&D.posted, s, __ATOMIC_RELEASE);
    // (the relay's wave 0 stores t_seen and its wave 1 `relayed`: the stamp is waited for too)
    while (__atomic_load_n(&D.relayed, __ATOMIC_ACQUIRE) != s || __atomic_load_n(&D.t_seen, __ATOMIC_ACQUIRE) == seen0)
      if (steady_s() - h0 > 0.05) return;  // the grid is not answering: no calibration now
    const double h1 = steady_s();
    const double g = (double)__atomic_load_n(&D.t_seen, __ATOMIC_ACQUIRE) * 1e-2;  // 100 MHz -> us
    if ((h1 - h0) * 1e6 < best) {
      best = (h1 - h0) * 1e6;
      off = 0.5 * (h0 + h1) * 1e6 - g;
    }
  }
  clk_off_us_.store(off, std::memory_order_relaxed);
  clk_rtt_us_.store(best, std::memory_order_relaxed);
  last_cal_.store(steady_s(), std::memory_order_relaxed);
}

// Under the exclusive lock (no door is posting): every posted tick relayed, then a stop tick
// on every door; the grid finishes the ticks it holds and leaves.
void HipGrid::stop_locked() {
  if (!running_.load(std::memory_order_relaxed)) return;
  const double t0 = steady_s();
  const uint32_t left = (1u << 16) | (gen_ & 0xffffu);
  auto exited = [&](int d) { return __atomic_load_n(&h_doors_[d].exits, __ATOMIC_ACQUIRE) == left; };
  for (int d = 0; d < n_; ++d)
    while (__atomic_load_n(&h_doors_[d].relayed, __ATOMIC_ACQUIRE) != h_doors_[d].posted && !exited(d)) {
      if (steady_s() - t0 > 5.0) throw std::runtime_error("grid: door " + std::to_string(d) + " never relayed its tick");
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  for (int d = 0; d < n_; ++d) {
    if (exited(d)) continue;
    PDoor& D = h_doors_[d];
    uint32_t s = D.posted + 1;
    if (s == 0) s = 1;
    D.d.stop = 1;
    D.d.seq = s;
    __atomic_store_n(&D.posted, s, __ATOMIC_RELEASE);
  }
  for (;;) {
    const hipError_t e = hipStreamQuery(stream_);
    if (e == hipSuccess) break;
    if (e != hipErrorNotReady) HIP_CHECK(e);
    if (steady_s() - t0 > 10.0) throw std::runtime_error("grid: did not leave after its stop ticks");
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
  running_.store(false, std::memory_order_release);
  ++stops_;
  stop_us_max_ = std::max(stop_us_max_, 1e6 * (steady_s() - t0));
}

void HipGrid::stop() {
  std::unique_lock<std::shared_mutex> ex(mu_);
  stop_locked();
}

void HipGrid::housekeep() {
  if (!running_.load(std::memory_order_acquire)) return;
  if (steady_s() - last_post_.load(std::memory_order_relaxed) > 1e-3 * idle_ms_) {
    std::unique_lock<std::shared_mutex> ex(mu_, std::try_to_lock);
    if (ex.owns_lock() && steady_s() - last_post_.load(std::memory_order_relaxed) > 1e-3 * idle_ms_) {
      stop_locked();
      return;
    }
  }
  const uint32_t b = beat_.fetch_add(1, std::memory_order_relaxed) + 1;
  for (int d = 0; d < n_; ++d) __atomic_store_n(&h_doors_[d].beat, b, __ATOMIC_RELAXED);
  if (steady_s() - last_cal_.load(std::memory_order_relaxed) > 1.0) {  // the two clocks drift apart by ~us per second
    std::unique_lock<std::shared_mutex> ex(mu_, std::try_to_lock);
    if (ex.owns_lock() && running_.load(std::memory_order_relaxed)) {
      // door 0's tick in flight (if any) must have been relayed: calibration reuses the door
      if (__atomic_load_n(&h_doors_[0].relayed, __ATOMIC_ACQUIRE) == h_doors_[0].posted) calibrate_locked();
    }
  }
}

bool HipGrid::revive_if_exited() {
  std::unique_lock<std::shared_mutex> ex(mu_);
  if (!running_.load(std::memory_order_relaxed)) return false;
  const uint32_t left = (1u << 16) | (gen_ & 0xffffu);
  bool any = false;
  for (int d = 0; d < n_; ++d) any = any || __atomic_load_n(&h_doors_[d].exits, __ATOMIC_ACQUIRE) == left;
  if (!any) return false;
  stop_locked();  // the sub-grids still running take their stop ticks
  launch_locked();
  ++revivals_;
  return true;
}

std::unordered_map<std::string, double> HipGrid::stats() {
  return {{"grid_launches", (double)launches_.load()}, {"grid_stops", (double)stops_.load()},
          {"grid_revivals", (double)revivals_.load()}, {"grid_doors", (double)n_},
          {"grid_clock_rtt_us", clk_rtt_us_.load(std::memory_order_relaxed)}, {"grid_xcd_local", interleave_ ? 1.0 : 0.0},
          {"grid_wg_per_door", (double)wpd_}, {"grid_wg_per_cu", (double)occ_},
          // (written under the exclusive lock; a torn read of a double is harmless here)
          {"grid_launch_us_max", launch_us_max_}, {"grid_launch_calibrate_us_max", launch_cal_us_max_},
          {"grid_launch_us_sum", launch_us_sum_}, {"grid_stop_us_max", stop_us_max_}};
}

}  // namespace qmx
