// ke_json.h — the wire formats koord-scheduler reads from the apiserver, decoded on the host:
// a small JSON DOM with Go encoding/json's lookup rules, and the apimachinery / Go scalar syntaxes the
// Kubernetes objects use (resource.Quantity, metav1.Duration, metav1.Time).  Used by ke_decode.cpp.
#pragma once
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace ke {
namespace json {

struct Value {
  enum Type { NUL, BOOL, NUM, STR, ARR, OBJ } t = NUL;
  bool b = false;
  std::string s;  // string contents (unescaped) or the number's literal text
  std::vector<Value> a;
  std::vector<std::pair<std::string, Value>> o;  // members in document order (duplicates kept)

  bool is_obj() const { return t == OBJ; }
  bool is_null() const { return t == NUL; }
  // a map key (exact match; Go keeps the last duplicate)
  const Value* key(const char* k) const;
  // a struct field: Go's decoder prefers an exact match of the json tag, else a case-insensitive one
  // (encoding/json: "preferring an exact match but also accepting a case-insensitive match"); the last
  // matching member wins
  const Value* field(const char* k) const;
};

// RFC 8259 parse of the whole input (trailing whitespace only).  false + err on malformed input.
bool parse(const char* p, size_t n, Value& out, std::string& err);

// Go encoding/json into int64: an integer literal (no fraction / exponent) within range
bool as_int64(const Value& v, int64_t* out);
// Go encoding/json into float64 (strconv.ParseFloat of the literal)
bool as_float64(const Value& v, double* out);

}  // namespace json

// k8s.io/apimachinery resource.ParseQuantity + Value() / MilliValue() (both round up); false on a malformed
// quantity, UNSUPPORTED-range values (beyond int64 after rounding) set *overflow.
bool parse_quantity(const std::string& s, int64_t* value, int64_t* milli, bool* overflow);
// Quantity.UnmarshalJSON: a JSON string or a bare number
bool quantity_json(const json::Value& v, int64_t* value, int64_t* milli, bool* overflow);
// the same quantities exactly, in units of 1e-9 (sums of quantities round once, like Quantity.Add + Value())
bool quantity_nanos(const std::string& s, __int128* nanos, bool* overflow);
bool quantity_json_nanos(const json::Value& v, __int128* nanos, bool* overflow);
bool nanos_value(__int128 nanos, int64_t* value, int64_t* milli);
// Go time.ParseDuration -> nanoseconds
bool parse_duration(const std::string& s, int64_t* ns);
// metav1.Time (time.RFC3339, optional fractional seconds) -> unix nanoseconds
bool parse_rfc3339(const std::string& s, int64_t* ns);
// Go strconv.ParseInt(s, 10, 64)
bool parse_int64(const std::string& s, int64_t* out);

}  // namespace ke
