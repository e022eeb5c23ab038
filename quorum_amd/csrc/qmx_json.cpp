// qmx_json.cpp — Python-compatible JSON DOM (see qmx_json.h).
#include "qmx_json.h"

#include <charconv>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "qmx_text.h"

namespace qmx {

const JVal* JVal::get(const std::string& k) const {
  if (t != OBJ) return nullptr;
  for (auto& kv : o)
    if (kv.first == k) return &kv.second;
  return nullptr;
}
JVal* JVal::get(const std::string& k) {
  if (t != OBJ) return nullptr;
  for (auto& kv : o)
    if (kv.first == k) return &kv.second;
  return nullptr;
}
void JVal::set(const std::string& k, JVal v) {
  for (auto& kv : o)
    if (kv.first == k) {
      kv.second = std::move(v);
      return;
    }
  o.emplace_back(k, std::move(v));
}
bool JVal::truthy() const {
  switch (t) {
    case NUL:
    case FALSE_: return false;
    case TRUE_: return true;
    case INT: return !(s == "0" || s == "-0");
    case FLOAT: return d != 0.0;
    case STR: return !s.empty();
    case ARR: return !a.empty();
    case OBJ: return !o.empty();
  }
  return false;
}

// ------------------------------------------------------------------------------------
// parser
// ------------------------------------------------------------------------------------
namespace {
struct Parser {
  const uint8_t* p;
  size_t n, i = 0;
  std::string err;
  int depth = 0;

  void ws() {
    while (i < n && (p[i] == ' ' || p[i] == '\t' || p[i] == '\n' || p[i] == '\r')) ++i;
  }
  bool fail(const char* what) {
    if (err.empty()) {
      size_t line = 1, col = 1;
      for (size_t k = 0; k < i && k < n; ++k) {
        if (p[k] == '\n') {
          ++line;
          col = 1;
        } else {
          ++col;
        }
      }
      err = std::string(what) + ": line " + std::to_string(line) + " column " + std::to_string(col) + " (char " +
            std::to_string(i) + ")";
    }
    return false;
  }
  bool lit(const char* s) {
    size_t L = strlen(s);
    if (i + L <= n && memcmp(p + i, s, L) == 0) {
      i += L;
      return true;
    }
    return false;
  }
  bool string(std::string& out) {
    // p[i] == '"'
    size_t start = i;
    StrScan sc = scan_string(p, (int)i, (int)n, false);
    if (!sc.ok) return fail("Unterminated string starting at");
    int dl = json_unescape(p, (int)start + 1, sc.end - 1, nullptr);
    out.resize(dl);
    json_unescape(p, (int)start + 1, sc.end - 1, (uint8_t*)&out[0]);
    i = sc.end;
    return true;
  }
  bool value(JVal& v) {
    ws();
    if (i >= n) return fail("Expecting value");
    uint8_t c = p[i];
    if (c == '{') {
      if (++depth > 900) return fail("maximum recursion depth exceeded");
      ++i;
      v.t = JVal::OBJ;
      ws();
      if (i < n && p[i] == '}') {
        ++i;
        --depth;
        return true;
      }
      while (true) {
        ws();
        if (i >= n || p[i] != '"') return fail("Expecting property name enclosed in double quotes");
        std::string k;
        if (!string(k)) return false;
        ws();
        if (i >= n || p[i] != ':') return fail("Expecting ':' delimiter");
        ++i;
        JVal child;
        if (!value(child)) return false;
        v.set(k, std::move(child));
        ws();
        if (i < n && p[i] == ',') {
          ++i;
          continue;
        }
        if (i < n && p[i] == '}') {
          ++i;
          break;
        }
        return fail("Expecting ',' delimiter");
      }
      --depth;
      return true;
    }
    if (c == '[') {
      if (++depth > 900) return fail("maximum recursion depth exceeded");
      ++i;
      v.t = JVal::ARR;
      ws();
      if (i < n && p[i] == ']') {
        ++i;
        --depth;
        return true;
      }
      while (true) {
        JVal child;
        if (!value(child)) return false;
        v.a.push_back(std::move(child));
        ws();
        if (i < n && p[i] == ',') {
          ++i;
          continue;
        }
        if (i < n && p[i] == ']') {
          ++i;
          break;
        }
        return fail("Expecting ',' delimiter");
      }
      --depth;
      return true;
    }
    if (c == '"') {
      v.t = JVal::STR;
      return string(v.s);
    }
    if (lit("true")) { v.t = JVal::TRUE_; return true; }
    if (lit("false")) { v.t = JVal::FALSE_; return true; }
    if (lit("null")) { v.t = JVal::NUL; return true; }
    if (lit("NaN")) { v.t = JVal::FLOAT; v.d = std::nan(""); return true; }
    if (lit("Infinity")) { v.t = JVal::FLOAT; v.d = INFINITY; return true; }
    if (lit("-Infinity")) { v.t = JVal::FLOAT; v.d = -INFINITY; return true; }
    if (c == '-' || (c >= '0' && c <= '9')) {
      NumScan ns = scan_number(p, (int)i, (int)n);
      if (!ns.ok) return fail("Expecting value");
      std::string tok((const char*)p + i, ns.end - i);
      i = ns.end;
      bool isf = tok.find_first_of(".eE") != std::string::npos;
      if (isf) {
        v.t = JVal::FLOAT;
        v.d = strtod(tok.c_str(), nullptr);
      } else {
        v.t = JVal::INT;
        v.s = (tok == "-0") ? "0" : tok;
      }
      return true;
    }
    return fail("Expecting value");
  }
};
}  // namespace

bool json_parse(const char* p, size_t n, JVal& out, std::string* err) {
  Parser ps{(const uint8_t*)p, n};
  out = JVal();
  if (!utf8_valid((const uint8_t*)p, 0, (int)n)) {
    if (err) *err = "invalid utf-8 in request body";
    return false;
  }
  if (!ps.value(out)) {
    if (err) *err = ps.err;
    return false;
  }
  ps.ws();
  if (ps.i != n) {
    ps.fail("Extra data");
    if (err) *err = ps.err;
    return false;
  }
  return true;
}

// ------------------------------------------------------------------------------------
// dump
// ------------------------------------------------------------------------------------
std::string py_float_repr(double d) {
  if (std::isnan(d)) return "NaN";
  if (std::isinf(d)) return d > 0 ? "Infinity" : "-Infinity";
  char buf[64];
  auto r = std::to_chars(buf, buf + sizeof(buf), d, std::chars_format::scientific);
  std::string s(buf, r.ptr);
  bool neg = s[0] == '-';
  if (neg) s.erase(0, 1);
  size_t e = s.find('e');
  std::string mant = s.substr(0, e);
  int exp = atoi(s.c_str() + e + 1);
  std::string digits;
  for (char c : mant)
    if (c != '.') digits.push_back(c);
  while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
  std::string out = neg ? "-" : "";
  if (exp >= -4 && exp < 16) {
    if (exp >= 0) {
      std::string ip = digits.substr(0, std::min<size_t>(digits.size(), exp + 1));
      while ((int)ip.size() < exp + 1) ip.push_back('0');
      std::string fp = (int)digits.size() > exp + 1 ? digits.substr(exp + 1) : "";
      out += ip + "." + (fp.empty() ? "0" : fp);
    } else {
      out += "0." + std::string(-exp - 1, '0') + digits;
    }
  } else {
    out += digits.substr(0, 1);
    if (digits.size() > 1) out += "." + digits.substr(1);
    char eb[16];
    snprintf(eb, sizeof(eb), "e%c%02d", exp < 0 ? '-' : '+', exp < 0 ? -exp : exp);
    out += eb;
  }
  return out;
}

void json_dump_str(const std::string& w, std::string& out) {
  out.push_back('"');
  const uint8_t* y = (const uint8_t*)w.data();
  uint8_t buf[12];
  for (size_t q = 0; q < w.size();) {
    uint32_t cp;
    q += wtf8_decode(y, (int)q, (int)w.size(), &cp);
    out.append((const char*)buf, escape_cp(cp, buf));
  }
  out.push_back('"');
}

void json_dump(const JVal& v, std::string& out) {
  switch (v.t) {
    case JVal::NUL: out += "null"; break;
    case JVal::FALSE_: out += "false"; break;
    case JVal::TRUE_: out += "true"; break;
    case JVal::INT: out += v.s; break;
    case JVal::FLOAT: out += py_float_repr(v.d); break;
    case JVal::STR: json_dump_str(v.s, out); break;
    case JVal::ARR:
      out.push_back('[');
      for (size_t k = 0; k < v.a.size(); ++k) {
        if (k) out += ", ";
        json_dump(v.a[k], out);
      }
      out.push_back(']');
      break;
    case JVal::OBJ:
      out.push_back('{');
      for (size_t k = 0; k < v.o.size(); ++k) {
        if (k) out += ", ";
        json_dump_str(v.o[k].first, out);
        out += ": ";
        json_dump(v.o[k].second, out);
      }
      out.push_back('}');
      break;
  }
}

std::string json_dumps(const JVal& v) {
  std::string s;
  json_dump(v, s);
  return s;
}

// ------------------------------------------------------------------------------------
// Python str()/repr() (for str.format of non-string values)
// ------------------------------------------------------------------------------------
static std::string py_str_repr(const std::string& w) {
  bool has_sq = w.find('\'') != std::string::npos, has_dq = w.find('"') != std::string::npos;
  char q = (has_sq && !has_dq) ? '"' : '\'';
  std::string out(1, q);
  const uint8_t* y = (const uint8_t*)w.data();
  for (size_t i = 0; i < w.size();) {
    uint32_t cp;
    int L = wtf8_decode(y, (int)i, (int)w.size(), &cp);
    char b[16];
    if (cp == (uint32_t)q || cp == '\\') { out.push_back('\\'); out.push_back((char)cp); }
    else if (cp == '\n') out += "\\n";
    else if (cp == '\r') out += "\\r";
    else if (cp == '\t') out += "\\t";
    else if (cp < 0x20 || cp == 0x7f) { snprintf(b, sizeof(b), "\\x%02x", cp); out += b; }
    else if (cp >= 0x80 && cp < 0xa0) { snprintf(b, sizeof(b), "\\x%02x", cp); out += b; }
    else if (cp >= 0xD800 && cp <= 0xDFFF) { snprintf(b, sizeof(b), "\\u%04x", cp); out += b; }
    else out.append(w, i, L);
    i += L;
  }
  out.push_back(q);
  return out;
}

std::string py_repr(const JVal& v) {
  switch (v.t) {
    case JVal::NUL: return "None";
    case JVal::FALSE_: return "False";
    case JVal::TRUE_: return "True";
    case JVal::INT: return v.s;
    case JVal::FLOAT:
      if (std::isnan(v.d)) return "nan";
      if (std::isinf(v.d)) return v.d > 0 ? "inf" : "-inf";
      return py_float_repr(v.d);
    case JVal::STR: return py_str_repr(v.s);
    case JVal::ARR: {
      std::string o = "[";
      for (size_t k = 0; k < v.a.size(); ++k) {
        if (k) o += ", ";
        o += py_repr(v.a[k]);
      }
      return o + "]";
    }
    case JVal::OBJ: {
      std::string o = "{";
      for (size_t k = 0; k < v.o.size(); ++k) {
        if (k) o += ", ";
        o += py_str_repr(v.o[k].first) + ": " + py_repr(v.o[k].second);
      }
      return o + "}";
    }
  }
  return "";
}

std::string py_str(const JVal& v) { return v.t == JVal::STR ? v.s : py_repr(v); }

bool py_format(const std::string& t, const std::string& name, const std::string& value, std::string& out) {
  out.clear();
  for (size_t i = 0; i < t.size(); ++i) {
    char c = t[i];
    if (c == '{') {
      if (i + 1 < t.size() && t[i + 1] == '{') {
        out.push_back('{');
        ++i;
        continue;
      }
      size_t j = t.find('}', i);
      if (j == std::string::npos) return false;
      if (t.compare(i + 1, j - i - 1, name) != 0 || j - i - 1 != name.size()) return false;
      out += value;
      i = j;
    } else if (c == '}') {
      if (i + 1 < t.size() && t[i + 1] == '}') {
        out.push_back('}');
        ++i;
        continue;
      }
      return false;
    } else {
      out.push_back(c);
    }
  }
  return true;
}

}  // namespace qmx
