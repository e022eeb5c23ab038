// qmx_json.h — JSON DOM with Python json.loads / json.dumps semantics (native data plane).
//
// * parse: strict JSON + NaN/Infinity/-Infinity, duplicate keys keep the FIRST position with
//   the LAST value (Python dict assignment), strings decoded to WTF-8 (lone surrogates kept).
// * dump: json.dumps defaults — ", " / ": " separators, ensure_ascii escaping, Python float
//   repr (shortest round-trip, exponent outside [-4, 16)), big ints preserved verbatim.
// * py_str: Python str() of a value (for str.format of non-string message content).
#pragma once
#include <stdint.h>

#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace qmx {

struct JVal {
  enum Type : uint8_t { NUL, FALSE_, TRUE_, INT, FLOAT, STR, ARR, OBJ };
  Type t = NUL;
  std::string s;  // STR (WTF-8) / INT (canonical decimal text)
  double d = 0;   // FLOAT
  std::vector<JVal> a;
  std::vector<std::pair<std::string, JVal>> o;

  static JVal str(std::string v) {
    JVal j;
    j.t = STR;
    j.s = std::move(v);
    return j;
  }
  static JVal integer(long long v) {
    JVal j;
    j.t = INT;
    j.s = std::to_string(v);
    return j;
  }
  static JVal boolean(bool b) {
    JVal j;
    j.t = b ? TRUE_ : FALSE_;
    return j;
  }
  const JVal* get(const std::string& k) const;
  JVal* get(const std::string& k);
  void set(const std::string& k, JVal v);  // Python dict assignment (keeps position)
  bool truthy() const;
  bool is_str() const { return t == STR; }
};

// Returns false with a Python-style message on malformed input.
bool json_parse(const char* p, size_t n, JVal& out, std::string* err = nullptr);
void json_dump(const JVal& v, std::string& out);
std::string json_dumps(const JVal& v);
void json_dump_str(const std::string& wtf8, std::string& out);  // quoted + ensure_ascii
std::string py_float_repr(double d);
std::string py_str(const JVal& v);   // str(value)
std::string py_repr(const JVal& v);  // repr(value)

// Minimal str.format for templates whose only fields are `{name}` (plus {{ }} escapes).
// Returns false (KeyError/ValueError in Python) if any other field/format spec appears.
bool py_format(const std::string& tmpl, const std::string& name, const std::string& value, std::string& out);

}  // namespace qmx
