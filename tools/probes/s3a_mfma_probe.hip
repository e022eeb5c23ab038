// Probe: the tick kernel's S3a event-template equality test on VALU (64-bit SWAR) vs MFMA.
//
// S3a compares every event of a stream tile with the stream's event template (the bytes
// before the content string: ~128 B for the mock's events) and, for a new stream, with its
// backend's hole templates.  The production kernel does it with 64-bit XOR/OR on VALU.  The
// alternative the round-5 review asked to settle with data: v_mfma_i32_16x16x64_i8 with the
// tag matcher's exact squared-distance trick (mfma_match_group) — per byte its base-8 digits
// d0, d1, d2 and d0²+d1²+d2² against -2·template digits and 1, so an output equals -E exactly
// when event and template agree byte for byte.  One MFMA covers 16 events × 16 bytes × 16
// templates; 128 bytes take 8 of them.
//
// Per wave, on LDS-resident data (events[16][L], templates[16][L]), timed with s_memrealtime over
// many repetitions; every variant's 16×T equality matrix is checked against a host oracle:
//   swar1   VALU, each event vs its stream template (what S3a does)
//   swar16  VALU, each event vs 16 templates
//   mfma16  MFMA, each event vs 16 templates at once (building the A operand included)
// Output: one JSON line per variant (ns per 16-event block, and per event x template).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
      exit(1);                                                                              \
    }                                                                                       \
  } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));
constexpr int L = 128;  // compared bytes per event (the mock's event prefix is ~130 B)
constexpr int NE = 16, NT = 16;
constexpr int REPS = 2000;

struct Lds {
  alignas(16) uint8_t ev[NE][L];
  alignas(16) uint8_t tp[NT][L];
};

// SWAR: lane l handles event l / 4, bytes [(l % 4) * 32, +32) as four 64-bit words
__device__ inline uint32_t swar_eq(const Lds& s, int t_of_event_lane, int l) {
  const int e = l >> 2, part = l & 3;
  const uint64_t* a = (const uint64_t*)&s.ev[e][part * 32];
  const uint64_t* b = (const uint64_t*)&s.tp[t_of_event_lane][part * 32];
  const uint64_t d = (a[0] ^ b[0]) | (a[1] ^ b[1]) | (a[2] ^ b[2]) | (a[3] ^ b[3]);
  // an event equals its template iff all 4 of its lanes saw no difference
  const uint64_t diff = __ballot(d != 0);
  uint32_t eqmask = 0;
#pragma unroll
  for (int ee = 0; ee < 16; ++ee) eqmask |= (((diff >> (4 * ee)) & 0xF) == 0 ? 1u : 0u) << ee;
  return eqmask;
}

__global__ void k_swar(const uint8_t* ev, const uint8_t* tp, int ntemplates, uint32_t* out, unsigned long long* ns) {
  __shared__ Lds s;
  const int l = threadIdx.x;
  for (int i = l; i < NE * L; i += 64) (&s.ev[0][0])[i] = ev[i];
  for (int i = l; i < NT * L; i += 64) (&s.tp[0][0])[i] = tp[i];
  __syncthreads();
  uint32_t acc = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int r = 0; r < REPS; ++r) {
    for (int t = 0; t < ntemplates; ++t) {
      const int tt = (t + r) % ntemplates;  // (the template varies: nothing hoisted)
      acc += swar_eq(s, tt, l) * (uint32_t)(tt + 1);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  for (int t = 0; t < ntemplates; ++t) {  // untimed: the result matrix for the oracle
    const uint32_t m = swar_eq(s, t, l);
    if (l == 0) out[t] = m;
  }
  if (l == 0) {
    out[NT] = acc;
    *ns = 10 * (t1 - t0);
  }
}

// MFMA: lane l = row (event) l & 15 of the A operand, feature group l >> 4 (d0, d1, d2, sum of
// squares) of a 16-byte chunk; B: column (template) l & 15, the same group: -2·digit or 1
__global__ void k_mfma(const uint8_t* ev, const uint8_t* tp, const int32_t* negE, uint32_t* out,
                       unsigned long long* ns) {
  __shared__ Lds s;
  const int l = threadIdx.x, r = l & 15, kg = l >> 4;
  for (int i = l; i < NE * L; i += 64) (&s.ev[0][0])[i] = ev[i];
  for (int i = l; i < NT * L; i += 64) (&s.tp[0][0])[i] = tp[i];
  __syncthreads();
  // B fragments of the 8 chunks (template-invariant across event blocks: built once)
  v4i bf[L / 16];
#pragma unroll
  for (int c = 0; c < L / 16; ++c) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t w = *(const uint32_t*)&s.tp[r][16 * c + 4 * q], v = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int x = (w >> (8 * b)) & 255;
        const int f = kg == 0 ? -2 * (x & 7) : kg == 1 ? -2 * ((x >> 3) & 7) : kg == 2 ? -2 * (x >> 6) : 1;
        v |= (uint32_t)(uint8_t)(int8_t)f << (8 * b);
      }
      bf[c][q] = (int)v;
    }
  }
  const int ne = negE[r];
  auto run = [&](int rep) -> uint32_t {  // lane t (< 16) gets template t's 16-event equality mask
    v4i acc = {0, 0, 0, 0};
    const int er = (r + rep) & 15;  // (the row's event varies: the A operand is not hoisted)
#pragma unroll
    for (int c = 0; c < L / 16; ++c) {
      const uint32_t sq_lo = 0x09040100u, sq_hi = 0x31241910u;
      v4i a;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t h = *(const uint32_t*)&s.ev[er][16 * c + 4 * q];
        const uint32_t d0 = h & 0x07070707u, d1 = (h >> 3) & 0x07070707u, d2 = (h >> 6) & 0x03030303u;
        const uint32_t sq = __builtin_amdgcn_perm(sq_hi, sq_lo, d0) + __builtin_amdgcn_perm(sq_hi, sq_lo, d1) +
                            __builtin_amdgcn_perm(sq_hi, sq_lo, d2);
        a[q] = (int)(kg == 0 ? d0 : kg == 1 ? d1 : kg == 2 ? d2 : sq);
      }
      acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, bf[c], acc, 0, 0, 0);
    }
    // output (row 4·(l >> 4) + i, column l & 15): equality bits, gathered per template — the
    // 4 lanes t, t+16, t+32, t+48 hold template t's rows 0-3, 4-7, 8-11, 12-15
    uint32_t bits = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) bits |= (acc[i] == ne ? 1u : 0u) << i;
    uint32_t m = 0;
#pragma unroll
    for (int g = 0; g < 4; ++g) m |= (uint32_t)__shfl(bits, (l & 15) + 16 * g) << (4 * g);
    const int k = rep & 15;  // row ρ held event (ρ + rep) & 15: back to event order
    return ((m << k) | (k ? m >> (16 - k) : 0u)) & 0xFFFFu;
  };
  uint32_t acc_all = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int rep = 0; rep < REPS; ++rep) acc_all += run(rep);
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  const uint32_t res = run(0);  // untimed: the result matrix for the oracle
  if (l < NT) out[l] = res;
  if (l == 0) {
    out[NT] = acc_all;
    *ns = 10 * (t1 - t0);
  }
}

int main() {
  std::mt19937 rng(7);
  // templates: the mock's event prefix shape with per-template variations; events: copies of
  // templates (some modified in one byte, some in the last byte)
  const char* base =
      "data: {\"id\": \"chatcmpl-abcdef0123456789\", \"object\": \"chat.completion.chunk\", \"created\": 1760000000, "
      "\"model\": \"mock-model\", \"choices\": [{\"index\": 0, \"delta\": {\"content\": \"";
  std::vector<uint8_t> tp(NT * L), ev(NE * L);
  for (int t = 0; t < NT; ++t) {
    for (int j = 0; j < L; ++j) tp[t * L + j] = (uint8_t)base[j % strlen(base)];
    if (t) tp[t * L + (t * 7) % L] ^= (uint8_t)(1 + t);  // 15 near-copies
  }
  std::vector<int> ev_t(NE);
  for (int e = 0; e < NE; ++e) {
    ev_t[e] = e % 3 == 0 ? 0 : (int)(rng() % NT);
    for (int j = 0; j < L; ++j) ev[e * L + j] = tp[ev_t[e] * L + j];
    if (e % 5 == 4) ev[e * L + (rng() % L)] ^= 0x20;  // a one-byte difference
    if (e % 7 == 6) ev[e * L + L - 1] ^= 0x01;        // in the last byte
  }
  // host oracle: eq[t] bit e
  std::vector<uint32_t> oracle(NT, 0);
  for (int t = 0; t < NT; ++t)
    for (int e = 0; e < NE; ++e)
      if (!memcmp(&ev[e * L], &tp[t * L], L)) oracle[t] |= 1u << e;
  std::vector<int32_t> negE(NT);
  for (int t = 0; t < NT; ++t) {
    int E = 0;
    for (int j = 0; j < L; ++j) {
      const int x = tp[t * L + j];
      E += (x & 7) * (x & 7) + ((x >> 3) & 7) * ((x >> 3) & 7) + (x >> 6) * (x >> 6);
    }
    negE[t] = -E;
  }
  uint8_t *d_ev, *d_tp;
  int32_t* d_negE;
  uint32_t* d_out;
  unsigned long long* d_cyc;
  CK(hipMalloc(&d_ev, ev.size()));
  CK(hipMalloc(&d_tp, tp.size()));
  CK(hipMalloc(&d_negE, 4 * NT));
  CK(hipMalloc(&d_out, 4 * (NT + 1)));
  CK(hipMalloc(&d_cyc, 8));
  CK(hipMemcpy(d_ev, ev.data(), ev.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_tp, tp.data(), tp.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_negE, negE.data(), 4 * NT, hipMemcpyHostToDevice));
  auto report = [&](const char* name, int ntemp) {
    std::vector<uint32_t> out(NT + 1);
    unsigned long long ns = 0;
    CK(hipMemcpy(out.data(), d_out, 4 * (NT + 1), hipMemcpyDeviceToHost));
    CK(hipMemcpy(&ns, d_cyc, 8, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int t = 0; t < ntemp; ++t) bad += out[t] != oracle[t];
    const double per_rep = (double)ns / REPS;
    printf("{\"variant\": \"%s\", \"templates\": %d, \"bytes\": %d, \"events\": %d, \"ns_per_16_events\": %.1f, "
           "\"ns_per_event_template\": %.3f, \"mismatches_vs_oracle\": %d}\n",
           name, ntemp, L, NE, per_rep, per_rep / (NE * ntemp), bad);
    fflush(stdout);
  };
  // warm-up + timed runs (one wave: the per-wave cost of the test itself)
  for (int w = 0; w < 2; ++w) {
    hipLaunchKernelGGL(k_swar, dim3(1), dim3(64), 0, 0, d_ev, d_tp, 1, d_out, d_cyc);
    CK(hipDeviceSynchronize());
  }
  report("swar1", 1);
  hipLaunchKernelGGL(k_swar, dim3(1), dim3(64), 0, 0, d_ev, d_tp, NT, d_out, d_cyc);
  CK(hipDeviceSynchronize());
  report("swar16", NT);
  for (int w = 0; w < 2; ++w) {
    hipLaunchKernelGGL(k_mfma, dim3(1), dim3(64), 0, 0, d_ev, d_tp, d_negE, d_out, d_cyc);
    CK(hipDeviceSynchronize());
  }
  report("mfma16", NT);
  return 0;
}
