// qmx_text.h — byte-level text primitives shared by the CPU engine and the CDNA4 kernels.
//
// Everything here is `__host__ __device__`: the host engine (qmx_cpu.cpp) and the fused
// tick/finalize kernels (qmx_hip.hip) call the SAME code for the per-event pieces
// (UTF-8 validation, Unicode whitespace, the validating JSON delta extractor, JSON
// string decode, ensure_ascii escape), so the two engines can only differ in the
// data-parallel parts (framing scan, MFMA tag match, depth scan, compaction), which
// the differential tests pin against each other and against the python oracle.
//
// Semantics = SURVEY §2.7 (reference src/quorum/oai_proxy.py:120-139, 262-371, 578-673).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define QMX_HD __host__ __device__ inline

namespace qmx {

// Tag sets the native engines run exactly ("<= ~16 tags"): up to 16 distinct
// (lowercased) tags of up to 61 printable-ASCII bytes with no regex metacharacter and no
// '<', '>' or '/'.  The MFMA matcher compares a 16-byte window per candidate '<' (a pattern
// longer than that — "</" + tag + ">" beyond 16 bytes — is a window prefix match plus a
// compare of its tail bytes), 16 patterns per MFMA column block (open + close of 16 tags:
// two blocks).  The holdback of a partial tag is at most the longest pattern - 1 bytes.
constexpr int kMaxTags = 16;
constexpr int kMaxTagLen = 61;   // "</" + 61 + ">" = 64 bytes
constexpr int kWindow = 16;
constexpr int kMaxTail = 64;
constexpr int kJsonMaxDepth = 256;  // deeper == RecursionError (stream abort)

// ---------------------------------------------------------------------------
// tag patterns
// ---------------------------------------------------------------------------
struct TagSet {
  int n;                                   // distinct lowercase tags
  int len[kMaxTags];
  uint8_t name[kMaxTags][kMaxTagLen + 1];  // lowercase ASCII
};

QMX_HD uint8_t lower_ascii(uint8_t c) { return (c >= 'A' && c <= 'Z') ? (uint8_t)(c + 32) : c; }

// Pattern byte i of pattern `pat` (pat < n: open "<t>", pat >= n: close "</t>").
QMX_HD int pattern_len(const TagSet& ts, int pat) {
  return pat < ts.n ? ts.len[pat] + 2 : ts.len[pat - ts.n] + 3;
}
QMX_HD uint8_t pattern_byte(const TagSet& ts, int pat, int i) {
  bool close = pat >= ts.n;
  int t = close ? pat - ts.n : pat;
  if (i == 0) return '<';
  if (close) {
    if (i == 1) return '/';
    --i;
  }
  return i <= ts.len[t] ? ts.name[t][i - 1] : (uint8_t)'>';
}

// Token at position p of x[0:n): +(t+1) open tag t, -(t+1) close tag t, 0 none.
template <class R>
QMX_HD int match_at(const R& x, int n, int p, const TagSet& ts, int* tok_len) {
  if (x[p] != '<') return 0;
  bool close = (p + 1 < n && x[p + 1] == '/');
  int s = p + 1 + (close ? 1 : 0);
  for (int t = 0; t < ts.n; ++t) {
    int L = ts.len[t];
    if (s + L >= n) continue;  // need x[s+L] == '>'
    bool ok = x[s + L] == '>';
    for (int i = 0; ok && i < L; ++i) ok = lower_ascii(x[s + i]) == ts.name[t][i];
    if (ok) {
      *tok_len = s + L + 1 - p;
      return close ? -(t + 1) : (t + 1);
    }
  }
  return 0;
}

// Is x[q:n) (lowercased) a prefix of some pattern?  opens_only: open patterns only.
template <class R>
QMX_HD bool pattern_prefix(const R& x, int q, int n, const TagSet& ts, bool opens_only) {
  int m = n - q;
  int npat = opens_only ? ts.n : 2 * ts.n;
  for (int pat = 0; pat < npat; ++pat) {
    int P = pattern_len(ts, pat);
    if (m > P) continue;
    bool ok = true;
    for (int i = 0; ok && i < m; ++i) ok = lower_ascii(x[q + i]) == pattern_byte(ts, pat, i);
    if (ok) return true;
  }
  return false;
}

// ---------------------------------------------------------------------------
// Unicode (Python str.isspace) whitespace on UTF-8 bytes
// ---------------------------------------------------------------------------
// Byte length of the whitespace char starting at x[p] (0: not whitespace, -1: incomplete).
template <class R>
QMX_HD int ws_at(const R& x, int p, int n) {
  uint8_t c = x[p];
  if (c < 0x80) return (c == ' ' || (c >= 0x09 && c <= 0x0d) || (c >= 0x1c && c <= 0x1f)) ? 1 : 0;
  if (c == 0xC2) {
    if (p + 1 >= n) return -1;
    return (x[p + 1] == 0x85 || x[p + 1] == 0xA0) ? 2 : 0;
  }
  if (c == 0xE1 || c == 0xE2 || c == 0xE3) {
    if (p + 2 >= n) return -1;
    uint8_t b1 = x[p + 1], b2 = x[p + 2];
    if (c == 0xE1) return (b1 == 0x9A && b2 == 0x80) ? 3 : 0;
    if (c == 0xE3) return (b1 == 0x80 && b2 == 0x80) ? 3 : 0;
    if (b1 == 0x80) return ((b2 >= 0x80 && b2 <= 0x8A) || b2 == 0xA8 || b2 == 0xA9 || b2 == 0xAF) ? 3 : 0;
    if (b1 == 0x81) return b2 == 0x9F ? 3 : 0;
    return 0;
  }
  return 0;
}
// Byte length of a whitespace char ENDING at x[e-1] (lo = lower bound), 0 if none.
template <class R>
QMX_HD int ws_before(const R& x, int lo, int e) {
  if (e - 1 >= lo && x[e - 1] < 0x80) return ws_at(x, e - 1, e) == 1 ? 1 : 0;
  if (e - 2 >= lo && ws_at(x, e - 2, e) == 2) return 2;
  if (e - 3 >= lo && ws_at(x, e - 3, e) == 3) return 3;
  return 0;
}
// Python str.strip() on a UTF-8 range.
template <class R>
QMX_HD void ustrip(const R& x, int* a, int* b) {
  while (*a < *b) {
    int w = ws_at(x, *a, *b);
    if (w <= 0) break;
    *a += w;
  }
  while (*b > *a) {
    int w = ws_before(x, *a, *b);
    if (w <= 0) break;
    *b -= w;
  }
}

// Strict UTF-8 validation (Python bytes.decode('utf-8')): no overlongs, no surrogates.
template <class R>
QMX_HD bool utf8_valid(const R& x, int a, int b) {
  int i = a;
  while (i < b) {
    uint8_t c = x[i];
    if (c < 0x80) { ++i; continue; }
    int need;
    uint32_t cp;
    if (c >= 0xC2 && c <= 0xDF) { need = 1; cp = c & 0x1F; }
    else if (c >= 0xE0 && c <= 0xEF) { need = 2; cp = c & 0x0F; }
    else if (c >= 0xF0 && c <= 0xF4) { need = 3; cp = c & 0x07; }
    else return false;
    if (i + need >= b) return false;
    for (int k = 1; k <= need; ++k) {
      uint8_t d = x[i + k];
      if ((d & 0xC0) != 0x80) return false;
      cp = (cp << 6) | (d & 0x3F);
    }
    if (need == 2 && (cp < 0x800 || (cp >= 0xD800 && cp <= 0xDFFF))) return false;
    if (need == 3 && (cp < 0x10000 || cp > 0x10FFFF)) return false;
    i += need + 1;
  }
  return true;
}

// Decode one (W)UTF-8 code point at y[p] (input known well-formed WTF-8); returns length.
template <class R>
QMX_HD int wtf8_decode(const R& y, int p, int n, uint32_t* cp) {
  uint8_t c = y[p];
  if (c < 0x80) { *cp = c; return 1; }
  if (c < 0xE0 && p + 1 < n) { *cp = ((c & 0x1F) << 6) | (y[p + 1] & 0x3F); return 2; }
  if (c < 0xF0 && p + 2 < n) {
    *cp = ((c & 0x0F) << 12) | ((y[p + 1] & 0x3F) << 6) | (y[p + 2] & 0x3F);
    return 3;
  }
  if (p + 3 < n) {
    *cp = ((c & 0x07) << 18) | ((y[p + 1] & 0x3F) << 12) | ((y[p + 2] & 0x3F) << 6) | (y[p + 3] & 0x3F);
    return 4;
  }
  *cp = 0xFFFD;
  return 1;
}

QMX_HD bool is_cont(uint8_t c) { return (c & 0xC0) == 0x80; }

// ---------------------------------------------------------------------------
// JSON string escaping, json.dumps(ensure_ascii=True) byte-exact
// ---------------------------------------------------------------------------
QMX_HD int escaped_len_cp(uint32_t cp) {
  if (cp >= 0x20 && cp < 0x7F && cp != '"' && cp != '\\') return 1;  // common case first
  if (cp == '"' || cp == '\\' || cp == '\n' || cp == '\r' || cp == '\t' || cp == 0x08 || cp == 0x0C) return 2;
  if (cp >= 0x20 && cp <= 0x7E) return 1;
  if (cp < 0x10000) return 6;
  return 12;
}
QMX_HD uint8_t hexd(uint32_t v) { return (uint8_t)(v < 10 ? '0' + v : 'a' + v - 10); }
QMX_HD int write_u4(uint8_t* o, uint32_t u) {
  o[0] = '\\'; o[1] = 'u';
  o[2] = hexd((u >> 12) & 15); o[3] = hexd((u >> 8) & 15); o[4] = hexd((u >> 4) & 15); o[5] = hexd(u & 15);
  return 6;
}
QMX_HD int escape_cp(uint32_t cp, uint8_t* o) {
  if (cp >= 0x20 && cp < 0x7F && cp != '"' && cp != '\\') {  // common case first (no switch tree)
    o[0] = (uint8_t)cp;
    return 1;
  }
  switch (cp) {
    case '"': o[0] = '\\'; o[1] = '"'; return 2;
    case '\\': o[0] = '\\'; o[1] = '\\'; return 2;
    case '\n': o[0] = '\\'; o[1] = 'n'; return 2;
    case '\r': o[0] = '\\'; o[1] = 'r'; return 2;
    case '\t': o[0] = '\\'; o[1] = 't'; return 2;
    case 0x08: o[0] = '\\'; o[1] = 'b'; return 2;
    case 0x0C: o[0] = '\\'; o[1] = 'f'; return 2;
    default: break;
  }
  if (cp >= 0x20 && cp <= 0x7E) { o[0] = (uint8_t)cp; return 1; }
  if (cp < 0x10000) return write_u4(o, cp);
  uint32_t v = cp - 0x10000;
  write_u4(o, 0xD800 | (v >> 10));
  write_u4(o + 6, 0xDC00 | (v & 0x3FF));
  return 12;
}

// ---------------------------------------------------------------------------
// JSON string decode (into WTF-8) — the body between the quotes, already validated
// ---------------------------------------------------------------------------
QMX_HD int hexv(uint8_t c) {
  if (c >= '0' && c <= '9') return c - '0';
  c = lower_ascii(c);
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  return -1;
}
template <class R>
QMX_HD uint32_t hex4(const R& x, int i) {
  return (uint32_t)((hexv(x[i]) << 12) | (hexv(x[i + 1]) << 8) | (hexv(x[i + 2]) << 4) | hexv(x[i + 3]));
}
QMX_HD int put_wtf8(uint32_t cp, uint8_t* o) {
  if (cp < 0x80) { if (o) o[0] = (uint8_t)cp; return 1; }
  if (cp < 0x800) { if (o) { o[0] = 0xC0 | (cp >> 6); o[1] = 0x80 | (cp & 0x3F); } return 2; }
  if (cp < 0x10000) {
    if (o) { o[0] = 0xE0 | (cp >> 12); o[1] = 0x80 | ((cp >> 6) & 0x3F); o[2] = 0x80 | (cp & 0x3F); }
    return 3;
  }
  if (o) {
    o[0] = 0xF0 | (cp >> 18); o[1] = 0x80 | ((cp >> 12) & 0x3F);
    o[2] = 0x80 | ((cp >> 6) & 0x3F); o[3] = 0x80 | (cp & 0x3F);
  }
  return 4;
}
// Decode JSON string body x[a:b) → out (may be null: length only). Python json semantics:
// \uD8xx\uDCxx pairs combine, lone surrogates are kept (as 3-byte WTF-8).
template <class R>
QMX_HD int json_unescape(const R& x, int a, int b, uint8_t* out) {
  int o = 0, i = a;
  while (i < b) {
    uint8_t c = x[i];
    if (c != '\\') {
      if (out) out[o] = c;
      ++o; ++i;
      continue;
    }
    uint8_t e = x[i + 1];
    uint32_t cp;
    if (e == 'u') {
      cp = hex4(x, i + 2);
      i += 6;
      if (cp >= 0xD800 && cp <= 0xDBFF && i + 6 <= b && x[i] == '\\' && x[i + 1] == 'u') {
        uint32_t lo = hex4(x, i + 2);
        if (lo >= 0xDC00 && lo <= 0xDFFF) {
          cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          i += 6;
        }
      }
    } else {
      i += 2;
      switch (e) {
        case 'n': cp = '\n'; break;
        case 't': cp = '\t'; break;
        case 'r': cp = '\r'; break;
        case 'b': cp = 0x08; break;
        case 'f': cp = 0x0C; break;
        default: cp = e; break;  // " \ /
      }
    }
    o += put_wtf8(cp, out ? out + o : nullptr);
  }
  return o;
}

// ---------------------------------------------------------------------------
// Validating JSON delta extractor (Python json.loads + quorum's exception semantics)
// ---------------------------------------------------------------------------
// Literals are packed into 64-bit immediates (byte k = char k): device code must never
// index string literals in per-byte loops (that is a global-memory load per byte).
constexpr uint64_t pack_lit(const char* s) {
  uint64_t v = 0;
  for (int k = 0; s[k] && k < 8; ++k) v |= (uint64_t)(uint8_t)s[k] << (8 * k);
  return v;
}
constexpr int lit_len(const char* s) {
  int k = 0;
  while (s[k]) ++k;
  return k;
}
// packed with the LAST char in the lowest byte (for a left-shifting rolling window)
constexpr uint64_t pack_rev(const char* s) {
  uint64_t v = 0;
  int n = lit_len(s);
  for (int k = 0; k < n; ++k) v = (v << 8) | (uint8_t)s[k];
  return v;
}
QMX_HD uint8_t lit_ch(uint64_t v, int k) { return (uint8_t)(v >> (8 * k)); }

enum EvKind : int { EV_SKIP = 0, EV_CONTENT = 1, EV_ABORT = 2 };
struct EvResult {
  int kind;
  int str_a, str_b;  // content string body (between quotes) when kind == EV_CONTENT
};

enum : int { K_NONE = 0, K_OBJ, K_ARR, K_STR, K_NUM, K_TRUE, K_FALSE, K_NULL };
enum : int { R_NONE = 0, R_ROOT, R_CHOICES, R_C0, R_DELTA, R_CONTENT, R_ROOTELEM, R_DELTAELEM };

// small KMP-free matcher for the two substring targets (no self-overlap issues handled
// generically: we restart at each code unit with a tiny window compare)
struct StrScan {
  bool ok;
  bool eq_choices, eq_delta, eq_content;
  bool has_choices, has_content;
  bool nonempty;
  int end;  // position after closing quote
};

// Scan a JSON string starting at x[p] == '"'.  Validates (control chars, escapes) and
// computes equality / containment against the fixed ASCII targets on DECODED chars.
template <class R>
QMX_HD StrScan scan_string(const R& x, int p, int b, bool want_contains) {
  StrScan r;
  r.ok = false; r.eq_choices = r.eq_delta = r.eq_content = false;
  r.has_choices = r.has_content = false; r.nonempty = false; r.end = p;
  constexpr uint64_t T0 = pack_lit("choices"), T1 = pack_lit("delta"), T2 = pack_lit("content");
  constexpr uint64_t R0 = pack_rev("choices"), R2 = pack_rev("content");
  constexpr uint64_t M56 = (1ull << 56) - 1;
  int k = 0;               // decoded unit index
  bool e0 = true, e1 = true, e2 = true;
  // rolling window of the last 7 decoded units (ASCII, 0 for non-ASCII), newest in byte 0
  uint64_t win = 0;
  int i = p + 1;
  while (true) {
    if (i >= b) return r;
    uint8_t c = x[i];
    uint32_t u;  // decoded unit: ASCII char or 0x100 for "other"
    if (c == '"') { ++i; break; }
    if (c < 0x20) return r;
    if (c == '\\') {
      if (i + 1 >= b) return r;
      uint8_t e = x[i + 1];
      if (e == 'u') {
        if (i + 5 >= b) return r;
        for (int q = 2; q < 6; ++q) if (hexv(x[i + q]) < 0) return r;
        uint32_t cp = hex4(x, i + 2);
        u = cp < 0x80 ? cp : 0x100;
        i += 6;
      } else {
        switch (e) {
          case '"': u = '"'; break;
          case '\\': u = '\\'; break;
          case '/': u = '/'; break;
          case 'b': u = 0x08; break;
          case 'f': u = 0x0C; break;
          case 'n': u = '\n'; break;
          case 'r': u = '\r'; break;
          case 't': u = '\t'; break;
          default: return r;
        }
        i += 2;
      }
    } else if (c >= 0x80) {
      // one code point = one "other" unit; skip its continuation bytes
      int ln = c >= 0xF0 ? 4 : c >= 0xE0 ? 3 : 2;
      u = 0x100;
      i += ln;
    } else {
      u = c;
      ++i;
    }
    e0 = e0 && k < 7 && u == lit_ch(T0, k);
    e1 = e1 && k < 5 && u == lit_ch(T1, k);
    e2 = e2 && k < 7 && u == lit_ch(T2, k);
    ++k;
    if (want_contains) {
      win = ((win << 8) | (u < 0x80 ? u : 0u)) & M56;
      r.has_choices = r.has_choices || (k >= 7 && win == R0);
      r.has_content = r.has_content || (k >= 7 && win == R2);
    }
  }
  r.ok = true;
  r.eq_choices = e0 && k == 7;
  r.eq_delta = e1 && k == 5;
  r.eq_content = e2 && k == 7;
  r.nonempty = k > 0;
  r.end = i;
  return r;
}

struct NumScan {
  bool ok;
  bool zero;
  int end;
};
// Python NUMBER_RE: -?(0|[1-9]\d*)(\.\d+)?([eE][-+]?\d+)?  (+ float underflow to 0.0)
template <class R>
QMX_HD NumScan scan_number(const R& x, int p, int b) {
  NumScan r{false, true, p};
  int i = p;
  if (i < b && x[i] == '-') ++i;
  if (i >= b) return r;
  int first_nz_exp = 0;  // decimal exponent of first nonzero digit (before applying e)
  bool seen_nz = false;
  int int_start = i;
  if (x[i] == '0') {
    ++i;
  } else if (x[i] >= '1' && x[i] <= '9') {
    while (i < b && x[i] >= '0' && x[i] <= '9') ++i;
  } else {
    return r;
  }
  int int_len = i - int_start;
  for (int q = int_start; q < i; ++q)
    if (x[q] != '0') { seen_nz = true; first_nz_exp = int_len - 1 - (q - int_start); break; }
  bool is_float = false;
  if (i + 1 < b && x[i] == '.' && x[i + 1] >= '0' && x[i + 1] <= '9') {
    is_float = true;
    ++i;
    int f0 = i;
    while (i < b && x[i] >= '0' && x[i] <= '9') {
      if (!seen_nz && x[i] != '0') { seen_nz = true; first_nz_exp = -(i - f0 + 1); }
      ++i;
    }
  }
  if (i < b && (x[i] == 'e' || x[i] == 'E')) {
    int j = i + 1;
    bool neg = false;
    if (j < b && (x[j] == '+' || x[j] == '-')) { neg = x[j] == '-'; ++j; }
    if (j < b && x[j] >= '0' && x[j] <= '9') {
      is_float = true;
      long ev = 0;
      while (j < b && x[j] >= '0' && x[j] <= '9') {
        if (ev < 100000) ev = ev * 10 + (x[j] - '0');
        ++j;
      }
      i = j;
      if (seen_nz && is_float) {
        long e10 = first_nz_exp + (neg ? -ev : ev);
        if (e10 < -324) seen_nz = false;  // underflows to 0.0
      }
    }
  }
  r.ok = true;
  r.zero = !seen_nz;
  r.end = i;
  return r;
}

template <class R>
QMX_HD bool lit_at(const R& x, int p, int b, uint64_t lit, int len) {
  if (p + len > b) return false;
  for (int i = 0; i < len; ++i)
    if (x[p + i] != lit_ch(lit, i)) return false;
  return true;
}
#define QMX_LIT(s) pack_lit(s), lit_len(s)

QMX_HD bool json_ws(uint8_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

// Classify one framed SSE event e[0:m) (see reference.classify_event for the contract).
template <class R>
QMX_HD EvResult classify_event(const R& e, int m) {
  EvResult res{EV_SKIP, 0, 0};
  if (!lit_at(e, 0, m, QMX_LIT("data: "))) return res;
  if (!utf8_valid(e, 0, m)) return res;
  int a = 6, b = m;
  ustrip(e, &a, &b);
  if (b - a == 6 && lit_at(e, a, b, QMX_LIT("[DONE]"))) return res;

  // --- parse ---------------------------------------------------------------------
  uint64_t stk[kJsonMaxDepth / 64] = {0, 0, 0, 0};  // bit = container is array
  int depth = 0;
  int crole[5] = {0, 0, 0, 0, 0};   // role of the container at depth 1..4
  int ccount[5] = {0, 0, 0, 0, 0};  // members/elements seen
  int keyrole = R_NONE;             // role for the next object member value
  // decision state
  int root_kind = K_NONE;
  bool root_has = false;  // root array elem == "choices" / root str contains "choices"
  bool has_choices = false;
  int ch_kind = K_NONE;
  bool ch_truthy = false;
  int c0_kind = K_NONE;
  bool d_present = false;
  int d_kind = K_NONE;
  bool d_has = false;  // delta array elem == "content" / delta str contains "content"
  bool has_content = false;
  int content_kind = K_NONE;
  int ca = 0, cb = 0;

  int pos = a;
  int role = R_ROOT;
  // state: 0 = expect value, 1 = expect key, 2 = after value
  int state = 0;
  int vkind = K_NONE;
  bool vtruthy = false;
  while (true) {
    if (state == 0 || state == 1) {
      while (pos < b && json_ws(e[pos])) ++pos;
      if (pos >= b) return res;  // JSONDecodeError -> skip
    }
    if (state == 1) {
      if (e[pos] != '"') return res;
      StrScan s = scan_string(e, pos, b, false);
      if (!s.ok) return res;
      int cr = depth <= 4 ? crole[depth] : R_NONE;
      keyrole = R_NONE;
      if (cr == R_ROOT && s.eq_choices) {
        keyrole = R_CHOICES;
        has_choices = true; ch_kind = K_NONE; ch_truthy = false; c0_kind = K_NONE;
        d_present = false; d_kind = K_NONE; d_has = false; has_content = false; content_kind = K_NONE;
      } else if (cr == R_C0 && s.eq_delta) {
        keyrole = R_DELTA;
        d_present = true; d_kind = K_NONE; d_has = false; has_content = false; content_kind = K_NONE;
      } else if (cr == R_DELTA && s.eq_content) {
        keyrole = R_CONTENT;
        has_content = true; content_kind = K_NONE;
      }
      pos = s.end;
      while (pos < b && json_ws(e[pos])) ++pos;
      if (pos >= b || e[pos] != ':') return res;
      ++pos;
      role = keyrole;
      state = 0;
      continue;
    }
    if (state == 0) {
      uint8_t c = e[pos];
      if (c == '{' || c == '[') {
        if (depth >= kJsonMaxDepth) { res.kind = EV_ABORT; return res; }
        bool arr = c == '[';
        if (arr) stk[depth >> 6] |= (1ull << (depth & 63));
        else stk[depth >> 6] &= ~(1ull << (depth & 63));
        ++depth;
        if (depth <= 4) { crole[depth] = role; ccount[depth] = 0; }
        if (role == R_ROOT) root_kind = arr ? K_ARR : K_OBJ;
        else if (role == R_CHOICES) ch_kind = arr ? K_ARR : K_OBJ;
        else if (role == R_C0) c0_kind = arr ? K_ARR : K_OBJ;
        else if (role == R_DELTA) d_kind = arr ? K_ARR : K_OBJ;
        else if (role == R_CONTENT) content_kind = arr ? K_ARR : K_OBJ;
        ++pos;
        while (pos < b && json_ws(e[pos])) ++pos;
        if (pos >= b) return res;
        if (e[pos] == (arr ? ']' : '}')) {
          ++pos;
          --depth;
          vkind = arr ? K_ARR : K_OBJ;
          vtruthy = false;
          // role of the just-closed container was `role`
          state = 2;
          goto after_value_container;
        }
        if (arr) {
          // element 0
          int cr = depth <= 4 ? crole[depth] : R_NONE;
          role = cr == R_CHOICES ? R_C0 : cr == R_ROOT ? R_ROOTELEM : cr == R_DELTA ? R_DELTAELEM : R_NONE;
          if (depth <= 4) ccount[depth] = 1;
          state = 0;
        } else {
          if (depth <= 4) ccount[depth] = 1;
          state = 1;
        }
        continue;
      }
      // scalar value
      if (c == '"') {
        bool want = role == R_ROOT || role == R_DELTA;
        StrScan s = scan_string(e, pos, b, want);
        if (!s.ok) return res;
        vkind = K_STR;
        vtruthy = s.nonempty;
        if (role == R_ROOT) root_has = s.has_choices;
        else if (role == R_DELTA) d_has = s.has_content;
        else if (role == R_ROOTELEM) root_has = root_has || s.eq_choices;
        else if (role == R_DELTAELEM) d_has = d_has || s.eq_content;
        else if (role == R_CONTENT) { ca = pos + 1; cb = s.end - 1; }
        pos = s.end;
      } else if (c == '-' || (c >= '0' && c <= '9')) {
        if (c == '-' && lit_at(e, pos, b, pack_lit("-Infinit"), 8) && lit_at(e, pos + 8, b, QMX_LIT("y"))) {
          pos += 9; vkind = K_NUM; vtruthy = true;
        } else {
          NumScan ns = scan_number(e, pos, b);
          if (!ns.ok) return res;
          pos = ns.end; vkind = K_NUM; vtruthy = !ns.zero;
        }
      } else if (lit_at(e, pos, b, QMX_LIT("true"))) { pos += 4; vkind = K_TRUE; vtruthy = true; }
      else if (lit_at(e, pos, b, QMX_LIT("false"))) { pos += 5; vkind = K_FALSE; vtruthy = false; }
      else if (lit_at(e, pos, b, QMX_LIT("null"))) { pos += 4; vkind = K_NULL; vtruthy = false; }
      else if (lit_at(e, pos, b, QMX_LIT("NaN"))) { pos += 3; vkind = K_NUM; vtruthy = true; }
      else if (lit_at(e, pos, b, QMX_LIT("Infinity"))) { pos += 8; vkind = K_NUM; vtruthy = true; }
      else return res;
      if (role == R_ROOT) root_kind = vkind;
      else if (role == R_CHOICES) { ch_kind = vkind; ch_truthy = vtruthy; }
      else if (role == R_C0) c0_kind = vkind;
      else if (role == R_DELTA) d_kind = vkind;
      else if (role == R_CONTENT) content_kind = vkind;
      state = 2;
    }
  after_value_container:
    // state 2: after a complete value at the current depth
    if (state == 2) {
      if (depth == 0) {
        while (pos < b && json_ws(e[pos])) ++pos;
        if (pos != b) return res;  // extra data
        break;
      }
      while (pos < b && json_ws(e[pos])) ++pos;
      if (pos >= b) return res;
      bool arr = (stk[(depth - 1) >> 6] >> ((depth - 1) & 63)) & 1;
      uint8_t c = e[pos];
      if (c == ',') {
        ++pos;
        if (depth <= 4) ++ccount[depth];
        if (arr) {
          role = R_NONE;
          int cr = depth <= 4 ? crole[depth] : R_NONE;
          if (cr == R_ROOT) role = R_ROOTELEM;
          else if (cr == R_DELTA) role = R_DELTAELEM;
          state = 0;
        } else {
          state = 1;
        }
        continue;
      }
      if (c == (arr ? ']' : '}')) {
        ++pos;
        int closed_role = depth <= 4 ? crole[depth] : R_NONE;
        int cnt = depth <= 4 ? ccount[depth] : 1;
        --depth;
        if (closed_role == R_CHOICES) ch_truthy = cnt > 0;
        role = closed_role;
        state = 2;
        goto after_value_container;
      }
      return res;
    }
  }

  // --- quorum decision (oai_proxy.py:608-616 under Python semantics) ---------------
  switch (root_kind) {
    case K_OBJ: break;
    case K_ARR:
    case K_STR: res.kind = root_has ? EV_ABORT : EV_SKIP; return res;
    default: res.kind = EV_ABORT; return res;  // `in` on number/bool/None -> TypeError
  }
  if (!has_choices || !ch_truthy) return res;
  if (ch_kind != K_ARR) { res.kind = EV_ABORT; return res; }
  if (c0_kind != K_OBJ) { res.kind = EV_ABORT; return res; }
  if (!d_present) return res;  // .get("delta", {}) -> {} -> no content
  switch (d_kind) {
    case K_OBJ: break;
    case K_ARR:
    case K_STR: res.kind = d_has ? EV_ABORT : EV_SKIP; return res;
    default: res.kind = EV_ABORT; return res;
  }
  if (!has_content) return res;
  if (content_kind != K_STR) { res.kind = EV_ABORT; return res; }
  res.kind = EV_CONTENT;
  res.str_a = ca;
  res.str_b = cb;
  return res;
}

// Reader adaptors: R is a raw pointer on the host; on the device an LDS word reader.
template <class R>
struct OffsetReader {
  const R& r;
  int off;
  QMX_HD uint8_t operator[](int i) const { return r[off + i]; }
};
// Event at x[e0 : e0+m); string offsets in the result are relative to e0.
template <class R>
QMX_HD EvResult classify_event_at(const R& x, int e0, int m) {
  OffsetReader<R> o{x, e0};
  return classify_event(o, m);
}

}  // namespace qmx
