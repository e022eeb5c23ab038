// qmx_lex.h — wave-cooperative JSON lexer + per-lane token grammar (CDNA4 device code).
//
// Replaces a byte-serial per-lane scan (latency-bound: one dependent LDS round trip per
// byte, lanes diverging across inlined loops) by two phases:
//
//  1. wave_lex: ONE wave64 tokenises one event, 64 bytes per step. Per block:
//       BS  = ballot(c == '\\')            escapes: lane's preceding backslash run length via
//                                           clz over ~BS below the lane (+ run carried across blocks)
//       Q   = ballot(unescaped '"')         in-string = parity(popc(Q below lane)) ^ carry
//       SC  = ballot(scalar byte)           scalar-run starts; run validated by its first lane
//     errors are ballot-reduced; tokens (structural, string open/close, scalar) are written
//     in order at n + popc(T below lane).  Strict UTF-8 is validated wave-parallel too.
//  2. token_grammar: each lane walks ITS event's ~30 tokens (not ~190 bytes) through the
//     JSON grammar with quorum's choices[0].delta.content role tracking.
//
// Rare shapes (non-object root, non-array `choices`, array/string `delta`, escapes inside a
// target key, nesting > 64, token-buffer overflow) report LEX_COMPLEX and the caller falls
// back to classify_event (qmx_text.h), so the result is always exact.
#pragma once
#include <hip/hip_runtime.h>

#include "qmx_text.h"

namespace qmx {

enum LexTok : uint8_t {
  TK_NONE = 0, TK_LBRACE, TK_RBRACE, TK_LBRACK, TK_RBRACK, TK_COLON, TK_COMMA, TK_SOPEN, TK_SCLOSE, TK_SCALAR
};
// token byte = type | key id << 4 (on TK_SOPEN) | TKF_BS (on TK_SCLOSE: string holds a backslash)
enum : int { TK_TYPE = 15, KID_SHIFT = 4, KID_CHOICES = 1, KID_DELTA = 2, KID_CONTENT = 3, TKF_BS = 64 };
enum : int { LEX_OK = 0, LEX_INVALID = 1, LEX_COMPLEX = 2 };

// Branch-free byte classes (a ?: chain over a divergent byte lowers to a branch tree).
__device__ inline bool lex_ws(uint32_t c) { return c <= 32 && ((0x100002600ull >> c) & 1); }
__device__ inline int lex_struct(uint32_t c) {
  return (c == '{') * TK_LBRACE + (c == '}') * TK_RBRACE + (c == '[') * TK_LBRACK + (c == ']') * TK_RBRACK +
         (c == ':') * TK_COLON + (c == ',') * TK_COMMA;
}
__device__ inline bool lex_scalar_byte(uint32_t c) { return !lex_ws(c) && !lex_struct(c) && c != '"'; }

// Bytes x[p:p+8) (zero past b) from two aligned LDS words; x must be 8-byte aligned with
// >= 16 readable bytes past every b it is used with.
__device__ inline uint64_t lds_window8(const uint8_t* x, int p, int b) {
  const uint64_t* w = (const uint64_t*)x + (p >> 3);
  const int sh = (p & 7) * 8;
  uint64_t v = sh ? (w[0] >> sh) | (w[1] << (64 - sh)) : w[0];
  const int n = b - p;
  if (n < 8) v &= n <= 0 ? 0 : ((1ull << (8 * n)) - 1);
  return v;
}

// Exact check of one scalar run x[p:e): a Python json number or literal.
__device__ inline bool lex_scalar_ok(const uint8_t* x, int p, int e) {
  int n = e - p;
  if (n == 4 && lit_at(x, p, e, QMX_LIT("true"))) return true;
  if (n == 5 && lit_at(x, p, e, QMX_LIT("false"))) return true;
  if (n == 4 && lit_at(x, p, e, QMX_LIT("null"))) return true;
  if (n == 3 && lit_at(x, p, e, QMX_LIT("NaN"))) return true;
  if (n == 8 && lit_at(x, p, e, QMX_LIT("Infinity"))) return true;
  if (n == 9 && x[p] == '-' && lit_at(x, p + 1, e, QMX_LIT("Infinity"))) return true;
  NumScan ns = scan_number(x, p, e);
  return ns.ok && ns.end == e;
}

// Strict UTF-8 (Python bytes.decode) check of the non-ASCII byte c = x[pos] in [a, b).
__device__ inline bool utf8_lane_bad(const uint8_t* x, int pos, int a, int b, uint32_t c) {
  if (c < 0xC0) {  // continuation: must be claimed by a lead 1..3 bytes back
    for (int k = 1; k <= 3; ++k) {
      if (pos - k < a) return true;
      const uint32_t l = x[pos - k];
      if (l < 0x80) return true;
      if (l >= 0xC0) {
        const int need = (l >= 0xC2 && l <= 0xDF) ? 1 : (l >= 0xE0 && l <= 0xEF) ? 2 : (l >= 0xF0 && l <= 0xF4) ? 3 : 0;
        return need < k;
      }
    }
    return true;
  }
  const int need = (c >= 0xC2 && c <= 0xDF) ? 1 : (c >= 0xE0 && c <= 0xEF) ? 2 : (c >= 0xF0 && c <= 0xF4) ? 3 : 0;
  if (need == 0 || pos + need >= b) return true;
  const uint32_t c1 = x[pos + 1];
  const uint32_t lo = c == 0xE0 ? 0xA0 : c == 0xF0 ? 0x90 : 0x80;
  const uint32_t hi = c == 0xED ? 0x9F : c == 0xF4 ? 0x8F : 0xBF;
  bool bad = c1 < lo || c1 > hi;
  for (int k = 2; k <= need; ++k) bad = bad || (x[pos + k] & 0xC0) != 0x80;
  return bad;
}

// Tokenise the JSON text x[a:b) with the whole wave (strict UTF-8 included).  Returns the
// token count, or -LEX_INVALID (malformed: the event is skipped) / -LEX_COMPLEX (token
// buffer overflow).  Wave-uniform.  [a, b) must start and end on code-point boundaries.
__device__ inline int wave_lex(const uint8_t* x, int a, int b, uint16_t* tpos, uint8_t* ttype, int n0, int cap) {
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
    if (__ballot(v && c >= 0x80)) {
      if (v && c >= 0x80) e = utf8_lane_bad(x, pos, a, b, c);
    }
    if (v && inside && !q) {
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
    if (sstart) {  // validate the scalar run starting here
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
    if (q && !inside) {  // string open: is the raw string exactly a target key?
      const uint64_t w = lds_window8(x, pos + 1, b);
      ty |= (w == W_CHOICES ? KID_CHOICES : w == W_CONTENT ? KID_CONTENT : (w & M6) == W_DELTA ? KID_DELTA : 0)
            << KID_SHIFT;
    } else if (q) {  // string close: any backslash since its opening quote?
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

// ---- per-stream shape template -----------------------------------------------------
// One upstream's chunks differ only in the delta text: a stream's last fully-parsed CONTENT
// event is cached as (prefix up to and including the content string's opening quote,
// suffix from its closing quote).  A later event that is byte-identical outside the string
// and whose middle is a valid JSON string body has the same parse, so its content is the
// middle -- one 64-lane compare instead of a lex + grammar.  Exact by construction.
constexpr int TPL_PRE_MAX = 256, TPL_SUF_MAX = 64, TPL_BYTES = TPL_PRE_MAX + TPL_SUF_MAX;

// x[e0:e0+tp) == tpl[0:tp) and x[e1-ts:e1) == tpl[256:256+ts); tpl 8-byte aligned.
__device__ inline bool wave_tpl_match(const uint8_t* x, int e0, int e1, const uint8_t* tpl, int tp, int ts) {
  const int lane = threadIdx.x & 63;
  bool bad = false;
  if (lane < 32) {
    const int o = lane * 8;
    if (o < tp) {
      const int n = min(8, tp - o);
      const uint64_t m = n == 8 ? ~0ull : ((1ull << (8 * n)) - 1);
      bad = lds_window8(x, e0 + o, e0 + tp) != (((const uint64_t*)tpl)[lane] & m);
    }
  } else if (lane < 40) {
    const int o = (lane - 32) * 8;
    if (o < ts) {
      const int n = min(8, ts - o);
      const uint64_t m = n == 8 ? ~0ull : ((1ull << (8 * n)) - 1);
      bad = lds_window8(x, e1 - ts + o, e1) != (((const uint64_t*)(tpl + TPL_PRE_MAX))[lane - 32] & m);
    }
  }
  return __ballot(bad) == 0;
}

// Is x[a:b) a complete JSON string body (no unescaped quote, valid escapes, no control
// characters, strict UTF-8, not ending inside an escape)?  Wave-uniform.
// Returns -1 (no), 0 (yes, no backslash: decoded length = b - a), 1 (yes, has escapes).
__device__ inline int wave_str_body(const uint8_t* x, int a, int b) {
  const int lane = threadIdx.x & 63;
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  int carry_run = 0;
  bool any_bs = false;
  for (int blk = a; blk < b; blk += 64) {
    const int pos = blk + lane;
    const bool v = pos < b;
    const uint32_t c = v ? x[pos] : (uint32_t)'a';
    const uint64_t BSm = __ballot(v && c == '\\');
    any_bs = any_bs || BSm != 0;
    const uint64_t nb = ~BSm & below;
    const int run = nb ? (lane - 1 - (63 - __clzll(nb))) : (lane + carry_run);
    const bool esc = run & 1;
    bool e = v && (c < 0x20 || (c == '"' && !esc));
    if (v && esc) {
      if (c == 'u') {
        for (int k = 1; k <= 4; ++k) e = e || pos + k >= b || hexv(x[pos + k]) < 0;
      } else {
        e = e || !(c == '"' || c == '\\' || c == '/' || c == 'b' || c == 'f' || c == 'n' || c == 'r' || c == 't');
      }
    }
    if (__ballot(v && c >= 0x80)) {
      if (v && c >= 0x80) e = e || utf8_lane_bad(x, pos, a, b, c);
    }
    if (__ballot(e) != 0) return -1;
    const int nv = min(64, b - blk);  // trailing backslash run of this block's valid bytes
    const uint64_t vm = nv == 64 ? ~0ull : ((1ull << nv) - 1);
    const uint64_t bsv = BSm & vm;
    const uint64_t nbs = ~bsv & vm;
    carry_run = nbs ? (nv - 1 - (63 - __clzll(nbs))) : carry_run + nv;
  }
  if (carry_run & 1) return -1;  // an odd run would escape the closing quote
  return any_bs ? 1 : 0;
}

// Wave-parallel grammar + quorum target path for ONE event whose nt <= 64 tokens start at
// t0 (lane j owns token j).  Replaces a per-lane walk (~250 instructions per token) by
// ~O(depth) ballots per event:
//   depth before each token = popc(openers below) - popc(closers below);
//   container of a token    = the last opener below at depth-1 (one ballot per level);
//   JSON validity           = local adjacency rules given the container kind (keys vs values
//                             by the previous token), closers matching their container, a
//                             single root object closing at the last token;
//   path                    = last "choices" key of the root → its "[" → first element →
//                             last "delta" key → its "{" → last "content" key → its value.
// Returns LEX_OK / LEX_INVALID / LEX_COMPLEX exactly like token_grammar (wave-uniform; res
// is valid in every lane).
__device__ inline int wave_grammar(const uint16_t* tpos, const uint8_t* ttype, int t0, int nt, EvResult& res,
                                   bool* content_esc, uint64_t* val_open = nullptr) {
  const int lane = threadIdx.x & 63;
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  res.kind = EV_SKIP;
  res.str_a = res.str_b = 0;
  const bool v = lane < nt;
  const int tb = v ? ttype[t0 + lane] : 0;
  const int ty = tb & TK_TYPE;
  if (__builtin_amdgcn_readlane(ty, 0) != TK_LBRACE) return LEX_COMPLEX;  // non-object root
  const bool isO = ty == TK_LBRACE || ty == TK_LBRACK, isC = ty == TK_RBRACE || ty == TK_RBRACK;
  const uint64_t Om = __ballot(isO), Cm = __ballot(isC);
  const int db = __popcll(Om & below) - __popcll(Cm & below);
  const int da = db + (isO ? 1 : 0) - (isC ? 1 : 0);
  // depth: never negative, root closes exactly at the last token
  if (__ballot(v && (da < 0 || (lane < nt - 1 && da < 1) || (lane == nt - 1 && da != 0))) != 0) return LEX_INVALID;
  // container of each token: last opener below at depth db-1
  // openers occupy every level 0..maxdepth-1 (a token at depth L+1 sits inside an opener
  // at depth L): walk levels until one has no opener — one ballot per level, no reduction
  int cont = -1;
  for (int L = 0; L < 64; ++L) {
    const uint64_t OLall = __ballot(isO && db == L);
    if (OLall == 0) break;
    const uint64_t OL = OLall & below;
    if (db == L + 1 && OL) cont = 63 - __clzll(OL);
  }
  const int ctype = __shfl(ty, cont < 0 ? 0 : cont, 64);
  const bool inObj = cont >= 0 && ctype == TK_LBRACE;
  const int p = __shfl_up(ty, 1, 64);  // previous token type (lane 0: none)
  const bool keyopen = v && lane > 0 && ty == TK_SOPEN && inObj && (p == TK_LBRACE || p == TK_COMMA);
  const uint64_t KOm = __ballot(keyopen);
  if (val_open) *val_open = __ballot(v && ty == TK_SOPEN && !keyopen);  // string values (hole templates)
  const bool keyclose = v && ty == TK_SCLOSE && lane > 0 && ((KOm >> (lane - 1)) & 1);
  const bool valend = v && (ty == TK_SCALAR || isC || (ty == TK_SCLOSE && !keyclose));
  const uint64_t VEm = __ballot(valend), KCm = __ballot(keyclose);
  const bool prevVE = lane > 0 && ((VEm >> (lane - 1)) & 1), prevKC = lane > 0 && ((KCm >> (lane - 1)) & 1);
  bool ok = true;
  if (v && lane > 0) {
    if (ty == TK_SOPEN) ok = inObj ? (p == TK_LBRACE || p == TK_COMMA || p == TK_COLON) : (p == TK_LBRACK || p == TK_COMMA);
    else if (ty == TK_SCLOSE) ok = true;
    else if (ty == TK_COLON) ok = inObj && prevKC;
    else if (ty == TK_COMMA) ok = prevVE;
    else if (ty == TK_RBRACE) ok = inObj && (p == TK_LBRACE || prevVE);
    else if (ty == TK_RBRACK) ok = !inObj && (p == TK_LBRACK || prevVE);
    else ok = inObj ? p == TK_COLON : (p == TK_LBRACK || p == TK_COMMA);  // { [ scalar
  }
  if (__ballot(!ok) != 0) return LEX_INVALID;
  // quorum path: choices[0].delta.content (duplicate keys: the last one wins)
  const int kid = (tb >> KID_SHIFT) & 3;
  const bool bs_next = (__shfl_down(tb, 1, 64) & TKF_BS) != 0;  // key string holds a backslash
  auto last_key = [&](int c, int want, int* k) -> bool {        // false: COMPLEX (escaped key)
    const uint64_t mine = __ballot(keyopen && cont == c && kid == want);
    if (__ballot(keyopen && cont == c && kid != want && bs_next) != 0) return false;
    *k = mine ? 63 - __clzll(mine) : -1;
    return true;
  };
  auto ty_at = [&](int j) { return __builtin_amdgcn_readlane(ty, j); };
  int kc, kd, kk;
  if (!last_key(0, KID_CHOICES, &kc)) return LEX_COMPLEX;
  if (kc < 0) return LEX_OK;
  const int vc = kc + 3;  // "choices" SCLOSE COLON value
  if (ty_at(vc) != TK_LBRACK) return LEX_COMPLEX;
  const int c0 = vc + 1;
  if (ty_at(c0) == TK_RBRACK) return LEX_OK;  // empty choices
  if (ty_at(c0) != TK_LBRACE) {
    res.kind = EV_ABORT;
    return LEX_OK;
  }
  if (!last_key(c0, KID_DELTA, &kd)) return LEX_COMPLEX;
  if (kd < 0) return LEX_OK;
  const int vd = kd + 3, tvd = ty_at(vd);
  if (tvd == TK_LBRACK || tvd == TK_SOPEN) return LEX_COMPLEX;
  if (tvd != TK_LBRACE) {
    res.kind = EV_ABORT;
    return LEX_OK;
  }
  if (!last_key(vd, KID_CONTENT, &kk)) return LEX_COMPLEX;
  if (kk < 0) return LEX_OK;
  const int vk = kk + 3;
  if (ty_at(vk) != TK_SOPEN) {
    res.kind = EV_ABORT;
    return LEX_OK;
  }
  res.kind = EV_CONTENT;
  res.str_a = tpos[t0 + vk] + 1;
  res.str_b = tpos[t0 + vk + 1];
  *content_esc = (__builtin_amdgcn_readlane(tb, vk + 1) & TKF_BS) != 0;
  return LEX_OK;
}

// Template check against an earlier event of the same tile: x[e0:e0+tp) == x[p0:p0+tp) and
// x[e1-ts:e1) == x[s0:s0+ts) (tp <= 256, ts <= 64).
__device__ inline bool wave_tpl_match_tile(const uint8_t* x, int e0, int e1, int p0, int tp, int s0, int ts) {
  const int lane = threadIdx.x & 63;
  bool bad = false;
  if (lane < 32) {
    const int o = lane * 8;
    if (o < tp) bad = lds_window8(x, e0 + o, e0 + tp) != lds_window8(x, p0 + o, p0 + tp);
  } else if (lane < 40) {
    const int o = (lane - 32) * 8;
    if (o < ts) bad = lds_window8(x, e1 - ts + o, e1) != lds_window8(x, s0 + o, s0 + ts);
  }
  return __ballot(bad) == 0;
}

// Per-lane grammar + quorum target-path tracking over tokens [t0, t1).
// Returns LEX_OK (res filled), LEX_INVALID (skip) or LEX_COMPLEX (use classify_event).
// Branch-free per token (predicated selects): lanes walk different events, and a branchy
// state machine costs a wave every arm of every divergent branch on every token.
__device__ inline int token_grammar(const uint16_t* tpos, const uint8_t* ttype, int t0, int t1, EvResult& res) {
  enum { G_VAL0, G_VAL, G_VAL_OR_RB, G_KEY_OR_RC, G_KEY, G_KSTR, G_VSTR, G_COLON, G_AFTER, G_END, G_ERR };
  enum { P_NONE = 0, P_ROOT = 1, P_CHOICES = 2, P_C0 = 3, P_DELTA = 4, P_CONTENT = 5 };
  enum : uint32_t { F_ROOT = 1, F_HCH = 2, F_CHN = 4, F_C0 = 8, F_DP = 16, F_DO = 32, F_HC = 64, F_CS = 128 };
  int st = G_VAL0, d = 0, on = 0, pend = P_NONE, kid = 0, vrole = P_NONE, tca = -1, tcb = -1;
  uint64_t stk = 0;
  uint32_t fl = 0;
  bool cx = false;
  uint64_t tw = 0;
  for (int t = t0; t < t1; ++t) {
    if (t == t0 || (t & 7) == 0) tw = *(const uint64_t*)(ttype + (t & ~7));  // 8 tokens per LDS read
    const int tb = (int)(tw >> ((t & 7) * 8)) & 0xFF;
    const int ty = tb & TK_TYPE;
    const bool top_arr = d > 0 && ((stk >> ((d - 1) & 63)) & 1);
    const bool inV = st <= G_VAL_OR_RB;
    const bool openO = inV && ty == TK_LBRACE, openA = inV && ty == TK_LBRACK, push = openO || openA;
    const bool scal = inV && ty == TK_SCALAR, vso = inV && ty == TK_SOPEN, vstart = push || scal || vso;
    const bool pop = (st == G_VAL_OR_RB && ty == TK_RBRACK) || (st == G_KEY_OR_RC && ty == TK_RBRACE) ||
                     (st == G_AFTER && ((ty == TK_RBRACE && !top_arr) || (ty == TK_RBRACK && top_arr)));
    const bool kso = (st == G_KEY_OR_RC || st == G_KEY) && ty == TK_SOPEN;
    const bool ksc = st == G_KSTR, vsc = st == G_VSTR;  // the lexer pairs quotes: ty is TK_SCLOSE
    const bool colon = st == G_COLON && ty == TK_COLON, comma = st == G_AFTER && ty == TK_COMMA;
    // role of a value starting here, and the quorum-path flags it sets
    const int role = vstart ? (d == 0 ? (int)P_ROOT : pend) : (int)P_NONE;
    cx = cx || (role == P_ROOT && !openO) || (role == P_CHOICES && !openA) || (role == P_DELTA && (openA || vso)) ||
         (push && d >= 64);
    const uint32_t clr = role == P_CHOICES ? (F_CHN | F_C0 | F_DP | F_DO | F_HC | F_CS)
                         : role == P_DELTA ? (F_DO | F_HC | F_CS) : role == P_CONTENT ? F_CS : 0u;
    const uint32_t set = role == P_ROOT ? F_ROOT : role == P_CHOICES ? F_HCH
                         : role == P_C0 ? (F_CHN | (openO ? F_C0 : 0u)) : role == P_DELTA ? (F_DP | (openO ? F_DO : 0u))
                         : role == P_CONTENT ? (F_HC | (vso ? F_CS : 0u)) : 0u;
    fl = (fl & ~clr) | set;
    tca = (role == P_CONTENT && vso) ? t : tca;
    tcb = (vsc && vrole == P_CONTENT) ? t : tcb;
    vrole = vso ? role : vsc ? (int)P_NONE : vrole;
    // key names in the target containers
    const bool tgt = ksc && d == on && (on == 1 || on == 3 || on == 4);
    const int want = on == 1 ? KID_CHOICES : on == 3 ? KID_DELTA : KID_CONTENT;
    const bool kmatch = tgt && kid == want;
    cx = cx || (tgt && !kmatch && (tb & TKF_BS));  // an escaped key might decode to the target name
    const int krole = kmatch ? (on == 1 ? (int)P_CHOICES : on == 3 ? (int)P_DELTA : (int)P_CONTENT) : (int)P_NONE;
    kid = kso ? (tb >> KID_SHIFT) & 3 : kid;
    // depth, target-container tracking, pending role
    const int d2 = d + (push ? 1 : 0) - (pop ? 1 : 0);
    const bool enter = push && ((role == P_ROOT && d2 == 1) || (role == P_CHOICES && d2 == 2) ||
                                (role == P_C0 && d2 == 3 && openO) || (role == P_DELTA && d2 == 4 && openO));
    on = enter ? d2 : (pop && d <= on) ? d - 1 : on;
    pend = push ? (role == P_CHOICES ? (int)P_C0 : (int)P_NONE) : (vstart || pop) ? (int)P_NONE : ksc ? krole : pend;
    // grammar state
    const int endst = d2 == 0 ? G_END : G_AFTER;
    int ns = G_ERR;
    ns = openO ? G_KEY_OR_RC : ns;
    ns = openA ? G_VAL_OR_RB : ns;
    ns = (pop || scal || vsc) ? endst : ns;
    ns = vso ? G_VSTR : ns;
    ns = kso ? G_KSTR : ns;
    ns = ksc ? G_COLON : ns;
    ns = colon ? G_VAL : ns;
    ns = comma ? (top_arr ? G_VAL : G_KEY) : ns;
    st = ns;
    const uint64_t bit = 1ull << (d & 63);
    stk = push ? (openA ? (stk | bit) : (stk & ~bit)) : stk;
    d = d2;
  }
  res.kind = EV_SKIP;
  res.str_a = res.str_b = 0;
  if (cx) return LEX_COMPLEX;
  if (st != G_END) return LEX_INVALID;
  if (!(fl & F_ROOT)) return LEX_COMPLEX;
  if (!(fl & F_HCH) || !(fl & F_CHN)) return LEX_OK;  // no choices[0]
  // choices[0] / delta not an object, content not a string: quorum's handler raises
  if (!(fl & F_C0)) { res.kind = EV_ABORT; return LEX_OK; }
  if (!(fl & F_DP)) return LEX_OK;
  if (!(fl & F_DO)) { res.kind = EV_ABORT; return LEX_OK; }
  if (!(fl & F_HC)) return LEX_OK;
  if (!(fl & F_CS)) { res.kind = EV_ABORT; return LEX_OK; }
  res.kind = EV_CONTENT;
  res.str_a = tpos[tca] + 1;
  res.str_b = tpos[tcb];
  return LEX_OK;
}

// ---- hole templates (qmx_hip.h HoleTpl) --------------------------------------------
// x[a, a+L) == t[q, q+L) with one 8-byte window per lane (L <= 512; t 8-byte aligned with
// >= 16 readable bytes past q+L).  Wave-uniform.
__device__ inline bool wave_lit_eq(const uint8_t* x, int a, const uint8_t* t, int q, int L) {
  const int o = (threadIdx.x & 63) * 8;
  const bool bad = o < L && lds_window8(x, a + o, a + L) != lds_window8(t, q + o, q + L);
  return __ballot(bad) == 0;
}

// The JSON string body that starts at x[a]: the position of its closing (unescaped) quote
// before b, or -1 (no closing quote, a control character, a bad escape, invalid UTF-8).
// *bs: the body holds a backslash.  Wave-uniform; 64 bytes per step.
__device__ inline int wave_str_end(const uint8_t* x, int a, int b, bool* bs) {
  const int lane = threadIdx.x & 63;
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  int carry_run = 0;
  bool any_bs = false;
  for (int blk = a; blk < b; blk += 64) {
    const int pos = blk + lane;
    const bool v = pos < b;
    const uint32_t c = v ? x[pos] : (uint32_t)'a';
    const uint64_t BSm = __ballot(v && c == '\\');
    const uint64_t nb = ~BSm & below;
    const int run = nb ? (lane - 1 - (63 - __clzll(nb))) : (lane + carry_run);
    const bool esc = run & 1;
    const uint64_t Qm = __ballot(v && c == '"' && !esc);
    const int qe = Qm ? __ffsll((unsigned long long)Qm) - 1 : 64;  // the closing quote, if in this block
    const int bb = Qm ? blk + qe : b;
    const bool in = v && lane < qe;  // body bytes of this block
    bool e = in && c < 0x20;
    if (in && esc) {
      if (c == 'u') {
        for (int k = 1; k <= 4; ++k) e = e || pos + k >= bb || hexv(x[pos + k]) < 0;
      } else {
        e = e || !(c == '"' || c == '\\' || c == '/' || c == 'b' || c == 'f' || c == 'n' || c == 'r' || c == 't');
      }
    }
    if (__ballot(in && c >= 0x80)) {
      if (in && c >= 0x80) e = e || utf8_lane_bad(x, pos, a, bb, c);
    }
    if (__ballot(e) != 0) return -1;
    const uint64_t inm = qe >= 64 ? ~0ull : ((1ull << qe) - 1);
    any_bs = any_bs || (BSm & inm) != 0;
    if (Qm) {
      *bs = any_bs;
      return blk + qe;
    }
    const int nv = min(64, b - blk);  // trailing backslash run of this block's valid bytes
    const uint64_t vm = nv == 64 ? ~0ull : ((1ull << nv) - 1);
    const uint64_t nbs = ~(BSm & vm) & vm;
    carry_run = nbs ? (nv - 1 - (63 - __clzll(nbs))) : carry_run + nv;
  }
  return -1;
}

// A number hole at x[p]: the maximal scalar run (<= 32 bytes) must be a JSON number; its
// end, or -1.  One lane.
__device__ inline int num_hole_end(const uint8_t* x, int p, int b) {
  int e = p;
  while (e < b && e - p <= 32 && lex_scalar_byte(x[e])) ++e;
  if (e == p || e - p > 32) return -1;
  const NumScan ns = scan_number(x, p, e);
  return ns.ok && ns.end == e ? e : -1;
}

}  // namespace qmx
