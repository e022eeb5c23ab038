// Probe: cycles per event of the wave lexer (qmx_lex.h) phases on the benchmark's event shape.
//   phase 0: (empty)   1: wave_lex   2: token_grammar (per lane)   3: classify_event (per lane)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../quorum_amd/csrc/qmx_lex.h"

using namespace qmx;

// ablation copy of wave_lex: bit0 no key window, bit1 no scalar check, bit2 no utf8/escape, bit3 no bs flag
namespace qmx {
template <int V>
__device__ inline int wave_lex_v(const uint8_t* x, int a, int b, uint16_t* tpos, uint8_t* ttype, int n0, int cap) {
  constexpr uint64_t W_CHOICES = pack_lit("choices\""), W_CONTENT = pack_lit("content\"");
  constexpr uint64_t W_DELTA = pack_lit("delta\""), M6 = (1ull << 48) - 1;
  constexpr uint64_t W_TRUE = pack_lit("true"), W_NULL = pack_lit("null"), W_FALSE = pack_lit("false");
  const int lane = threadIdx.x & 63;
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  const uint64_t above = lane == 63 ? 0ull : (~0ull << (lane + 1));
  int carry_run = 0, in_str = 0, n = n0;
  bool prev_scal = false, carry_bs = false;
  for (int blk = a; blk < b; blk += 64) {
    const int pos = blk + lane;
    const bool v = pos < b;
    const uint32_t c = v ? x[pos] : (uint32_t)' ';
    const uint64_t BSm = __ballot(v && c == '\\');
    const uint64_t nb = ~BSm & below;
    const int run = nb ? (lane - 1 - (63 - __clzll(nb))) : (lane + carry_run);
    const bool esc = run & 1;
    const bool q = v && c == '"' && !esc;
    const uint64_t Qm = __ballot(q);
    const bool inside = ((__popcll(Qm & below) & 1) ^ in_str) != 0;
    const int stc = inside ? 0 : lex_struct(c);
    const bool sc = v && !inside && !q && !lex_ws(c) && !stc;
    const uint64_t SCm = __ballot(sc);
    const uint64_t Dm = __ballot(sc && c - '0' < 10u);
    const uint64_t BIm = BSm & __ballot(inside);
    const bool sstart = sc && !(lane ? ((SCm >> (lane - 1)) & 1) : prev_scal);
    bool e = false;
    if (!(V & 4) && __ballot(v && c >= 0x80)) {
      if (v && c >= 0x80) e = utf8_lane_bad(x, pos, a, b, c);
    }
    if (!(V & 4) && v && inside && !q) {
      if (c < 0x20) {
        e = true;
      } else if (esc) {  // the escaped character
        if (c == 'u') {
          for (int k = 1; k <= 4; ++k) e = e || pos + k >= b || hexv(x[pos + k]) < 0;
        } else {
          e = !(c == '"' || c == '\\' || c == '/' || c == 'b' || c == 'f' || c == 'n' || c == 'r' || c == 't');
        }
      }
    }
    if (!(V & 2) && sstart) {  // validate the scalar run starting here
      bool fast = false;
      const uint64_t stop = ~SCm & above;
      if (stop) {  // run ends inside this block: digit / literal fast paths from the ballots
        const int le = __ffsll((unsigned long long)stop) - 1;
        const int len = le - lane;
        const uint64_t rm = ((1ull << le) - 1) & ~below;
        if ((rm & ~Dm) == 0) {
          fast = true;
          e = e || (len > 1 && c == '0');
        } else if (c == '-' && len >= 2 && ((rm & ~(1ull << lane)) & ~Dm) == 0) {
          fast = true;
          e = e || (len > 2 && x[pos + 1] == '0');
        } else if (len == 4 || len == 5) {
          const uint64_t w = lds_window8(x, pos, pos + len);
          fast = w == W_TRUE || w == W_NULL || w == W_FALSE;
        }
      }
      if (!fast) {
        int end = pos;
        while (end < b && lex_scalar_byte(x[end])) ++end;
        e = e || !lex_scalar_ok(x, pos, end);
      }
    }
    if (__ballot(e) != 0) return -LEX_INVALID;
    int ty = stc ? stc : q ? (inside ? TK_SCLOSE : TK_SOPEN) : sstart ? TK_SCALAR : 0;
    if (!(V & 1) && q && !inside) {  // string open: is the raw string exactly a target key?
      const uint64_t w = lds_window8(x, pos + 1, b);
      ty |= (w == W_CHOICES ? KID_CHOICES : w == W_CONTENT ? KID_CONTENT : (w & M6) == W_DELTA ? KID_DELTA : 0)
            << KID_SHIFT;
    } else if (!(V & 8) && q) {  // string close: any backslash since its opening quote?
      const uint64_t pq = Qm & below;
      const bool bs = pq ? (BIm & below & (~0ull << (64 - __clzll(pq)))) != 0 : (carry_bs || (BIm & below) != 0);
      if (bs) ty |= TKF_BS;
    }
    const uint64_t Tm = __ballot(ty != 0);
    const int nt = __popcll(Tm);
    if (n + nt > cap) return -LEX_COMPLEX;
    if (ty) {
      const int r = n + __popcll(Tm & below);
      tpos[r] = (uint16_t)pos;
      ttype[r] = (uint8_t)ty;
    }
    n += nt;
    const int in_str_next = in_str ^ (__popcll(Qm) & 1);
    if (!in_str_next) {
      carry_bs = false;
    } else if (Qm) {
      const int lq = 63 - __clzll(Qm);
      carry_bs = lq < 63 && (BIm >> (lq + 1)) != 0;
    } else {
      carry_bs = carry_bs || BIm != 0;
    }
    in_str = in_str_next;
    carry_run = (BSm == ~0ull) ? carry_run + 64 : __clzll(~BSm);
    prev_scal = (SCm >> 63) & 1;
  }
  if (in_str) return -LEX_INVALID;  // unterminated string
  return n - n0;
}

}  // namespace qmx

__global__ __launch_bounds__(256) void k(const uint8_t* ev, int elen, int stride, unsigned long long* out, int* sink) {
  __shared__ alignas(16) uint8_t A[16384];
  __shared__ uint16_t TKP[4][1024];
  __shared__ alignas(8) uint8_t TKT[4][1024];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  for (int i = tid; i < 16384; i += 256) A[i] = ev[i % stride];
  __syncthreads();
  const int nev = 16384 / stride;  // 64 events
  int acc = 0, ntok = 0, my_t0 = 0, my_t1 = 0;
  unsigned long long c0 = __builtin_amdgcn_s_memtime();
  for (int l = 0; l < 16; ++l) {  // 16 events per wave
    int e = 4 * l + w;
    if (e >= nev) break;
    acc += (int)lds_window8(A, e * stride, e * stride + elen);
  }
  unsigned long long c1 = __builtin_amdgcn_s_memtime();
  unsigned long long abl[5];
#define ABL(I, VV)                                                                           \
  {                                                                                          \
    unsigned long long t0 = __builtin_amdgcn_s_memtime();                                    \
    for (int l = 0; l < 16; ++l) {                                                           \
      int e = 4 * l + w;                                                                     \
      acc += wave_lex_v<VV>(A, e * stride + 6, e * stride + elen, TKP[w], TKT[w], 0, 1024); \
    }                                                                                        \
    abl[I] = __builtin_amdgcn_s_memtime() - t0;                                              \
  }
  ABL(0, 0) ABL(1, 1) ABL(2, 2) ABL(3, 4) ABL(4, 15)
  for (int l = 0; l < 16; ++l) {
    int e = 4 * l + w;
    if (e >= nev) break;
    int nt = wave_lex(A, e * stride + 6, e * stride + elen, TKP[w], TKT[w], ntok, 1024);
    if (lane == l) {
      my_t0 = ntok;
      my_t1 = ntok + (nt > 0 ? nt : 0);
    }
    if (nt > 0) ntok += nt;
    acc += nt;
  }
  unsigned long long c2 = __builtin_amdgcn_s_memtime();
  EvResult r;
  int g = -1;
  if (lane < 16) g = token_grammar(TKP[w], TKT[w], my_t0, my_t1, r);
  acc += g * 7 + r.kind + r.str_a;
  unsigned long long c3 = __builtin_amdgcn_s_memtime();
  if (lane < 16) {
    int e = 4 * lane + w;
    EvResult r2 = classify_event_at(A, e * stride, elen);
    acc += r2.kind + r2.str_a;
  }
  unsigned long long c4 = __builtin_amdgcn_s_memtime();
  // wave grammar: re-lex + wave_grammar per event (what the kernel's S3 does per fresh event)
  int wg = 0;
  for (int l = 0; l < 16; ++l) {
    int e = 4 * l + w;
    int nt = wave_lex(A, e * stride + 6, e * stride + elen, TKP[w], TKT[w], 0, 1024);
    EvResult r3;
    bool esc;
    wg += wave_grammar(TKP[w], TKT[w], 0, nt, r3, &esc) * 3 + r3.kind + (nt > 64);
  }
  unsigned long long c5 = __builtin_amdgcn_s_memtime();
  // template compare + string-body check per event
  for (int l = 0; l < 16; ++l) {
    int e = 4 * l + w;
    wg += wave_tpl_match_tile(A, e * stride, e * stride + elen, 0, 150, 160, 26) +
          wave_str_body(A, e * stride + 150, e * stride + 160);
  }
  unsigned long long c6 = __builtin_amdgcn_s_memtime();
  acc += wg;
  if (tid == 0) {
    out[0] = c1 - c0;
    out[1] = c2 - c1;
    out[2] = c3 - c2;
    out[3] = c4 - c3;
    out[4] = (unsigned long long)ntok;
    out[5] = (unsigned long long)g;
    out[6] = (unsigned long long)r.kind;
    for (int i = 0; i < 5; ++i) out[7 + i] = abl[i];
    out[12] = c5 - c4;
    out[13] = c6 - c5;
    out[14] = (unsigned long long)wg;
  }
  sink[tid] = acc;
}

int main() {
  std::string ev =
      "data: {\"id\": \"chatcmpl-mock\", \"object\": \"chat.completion.chunk\", \"created\": 1700000000, \"model\": "
      "\"mock\", \"choices\": [{\"index\": 0, \"delta\": {\"content\": \" quick\"}, \"finish_reason\": null}]}";
  int elen = (int)ev.size(), stride = 256;
  std::vector<uint8_t> buf(stride, ' ');
  memcpy(buf.data(), ev.data(), elen);
  uint8_t* dev;
  unsigned long long* dout;
  int* sink;
  hipMalloc(&dev, stride);
  hipMalloc(&dout, 128);
  hipMalloc(&sink, 1024);
  hipMemcpy(dev, buf.data(), stride, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 3; ++rep) {
    unsigned long long c[15];
    hipLaunchKernelGGL(k, dim3(1), dim3(256), 0, 0, dev, elen, stride, dout, sink);
    hipMemcpy(c, dout, sizeof(c), hipMemcpyDeviceToHost);
    // s_memtime counts shader clocks (~2.4 GHz, see kbench shader_mhz)
    printf("event %dB x16/wave: utf8 %llu  lex %llu  grammar(16 lanes) %llu  classify_event(16 lanes) %llu ticks;"
           " tokens/wave %llu grammar=%lld kind=%llu\n",
           elen, c[0], c[1], c[2], c[3], c[4], (long long)c[5], c[6]);
    printf("  ablation: full %llu  -keywin %llu  -scalar %llu  -utf8/esc %llu  minimal %llu\n", c[7], c[8], c[9], c[10],
           c[11]);
    printf("  lex+wave_grammar x16: %llu ticks; template+body x16: %llu ticks (check %llu)\n", c[12], c[13], c[14]);
  }
  return 0;
}
