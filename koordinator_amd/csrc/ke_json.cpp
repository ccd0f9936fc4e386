// ke_json.cpp — JSON DOM + the Kubernetes scalar syntaxes (ke_json.h).
#include "ke_json.h"

#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstring>

namespace ke {
namespace json {

namespace {

struct Parser {
  const char* p;
  const char* e;
  std::string err;
  int depth = 0;

  void ws() {
    while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++;
  }
  bool fail(const char* m) {
    if (err.empty()) err = m;
    return false;
  }
  static void utf8(std::string& out, uint32_t c) {
    if (c < 0x80) {
      out += (char)c;
    } else if (c < 0x800) {
      out += (char)(0xC0 | (c >> 6));
      out += (char)(0x80 | (c & 0x3F));
    } else if (c < 0x10000) {
      out += (char)(0xE0 | (c >> 12));
      out += (char)(0x80 | ((c >> 6) & 0x3F));
      out += (char)(0x80 | (c & 0x3F));
    } else {
      out += (char)(0xF0 | (c >> 18));
      out += (char)(0x80 | ((c >> 12) & 0x3F));
      out += (char)(0x80 | ((c >> 6) & 0x3F));
      out += (char)(0x80 | (c & 0x3F));
    }
  }
  bool hex4(uint32_t* v) {
    if (e - p < 4) return fail("truncated \\u escape");
    uint32_t x = 0;
    for (int i = 0; i < 4; i++) {
      const char c = p[i];
      x <<= 4;
      if (c >= '0' && c <= '9') x |= (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f') x |= (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') x |= (uint32_t)(c - 'A' + 10);
      else return fail("bad \\u escape");
    }
    p += 4;
    *v = x;
    return true;
  }
  bool str(std::string& out) {
    p++;  // opening quote
    while (true) {
      if (p >= e) return fail("unterminated string");
      const unsigned char c = (unsigned char)*p;
      if (c == '"') {
        p++;
        return true;
      }
      if (c < 0x20) return fail("control character in string");
      if (c != '\\') {
        out += (char)c;
        p++;
        continue;
      }
      if (++p >= e) return fail("unterminated escape");
      const char x = *p++;
      switch (x) {
        case '"': out += '"'; break;
        case '\\': out += '\\'; break;
        case '/': out += '/'; break;
        case 'b': out += '\b'; break;
        case 'f': out += '\f'; break;
        case 'n': out += '\n'; break;
        case 'r': out += '\r'; break;
        case 't': out += '\t'; break;
        case 'u': {
          uint32_t u;
          if (!hex4(&u)) return false;
          if (u >= 0xD800 && u < 0xDC00) {  // a high surrogate: a low one must follow, else U+FFFD (Go)
            uint32_t lo = 0;
            if (e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
              const char* save = p;
              p += 2;
              if (!hex4(&lo)) return false;
              if (lo >= 0xDC00 && lo < 0xE000) {
                u = 0x10000 + ((u - 0xD800) << 10) + (lo - 0xDC00);
              } else {
                p = save;
                u = 0xFFFD;
              }
            } else {
              u = 0xFFFD;
            }
          } else if (u >= 0xDC00 && u < 0xE000) {
            u = 0xFFFD;
          }
          utf8(out, u);
          break;
        }
        default:
          return fail("bad escape");
      }
    }
  }
  bool num(Value& v) {
    const char* s = p;
    if (p < e && *p == '-') p++;
    if (p >= e) return fail("bad number");
    if (*p == '0') {
      p++;
    } else if (*p >= '1' && *p <= '9') {
      while (p < e && *p >= '0' && *p <= '9') p++;
    } else {
      return fail("bad number");
    }
    if (p < e && *p == '.') {
      p++;
      if (p >= e || !(*p >= '0' && *p <= '9')) return fail("bad number fraction");
      while (p < e && *p >= '0' && *p <= '9') p++;
    }
    if (p < e && (*p == 'e' || *p == 'E')) {
      p++;
      if (p < e && (*p == '+' || *p == '-')) p++;
      if (p >= e || !(*p >= '0' && *p <= '9')) return fail("bad number exponent");
      while (p < e && *p >= '0' && *p <= '9') p++;
    }
    v.t = Value::NUM;
    v.s.assign(s, (size_t)(p - s));
    return true;
  }
  bool lit(const char* w, size_t n) {
    if ((size_t)(e - p) < n || std::memcmp(p, w, n) != 0) return fail("bad literal");
    p += n;
    return true;
  }
  bool value(Value& v) {
    ws();
    if (p >= e) return fail("unexpected end of input");
    if (++depth > 512) return fail("nesting too deep");
    bool ok;
    switch (*p) {
      case '{': {
        v.t = Value::OBJ;
        p++;
        ws();
        if (p < e && *p == '}') {
          p++;
          ok = true;
          break;
        }
        ok = true;
        while (ok) {
          ws();
          if (p >= e || *p != '"') {
            ok = fail("expected object key");
            break;
          }
          std::string k;
          if (!str(k)) {
            ok = false;
            break;
          }
          ws();
          if (p >= e || *p != ':') {
            ok = fail("expected ':'");
            break;
          }
          p++;
          v.o.emplace_back(std::move(k), Value());
          if (!value(v.o.back().second)) {
            ok = false;
            break;
          }
          ws();
          if (p < e && *p == ',') {
            p++;
            continue;
          }
          if (p < e && *p == '}') {
            p++;
            break;
          }
          ok = fail("expected ',' or '}'");
        }
        break;
      }
      case '[': {
        v.t = Value::ARR;
        p++;
        ws();
        if (p < e && *p == ']') {
          p++;
          ok = true;
          break;
        }
        ok = true;
        while (ok) {
          v.a.emplace_back();
          if (!value(v.a.back())) {
            ok = false;
            break;
          }
          ws();
          if (p < e && *p == ',') {
            p++;
            continue;
          }
          if (p < e && *p == ']') {
            p++;
            break;
          }
          ok = fail("expected ',' or ']'");
        }
        break;
      }
      case '"':
        v.t = Value::STR;
        ok = str(v.s);
        break;
      case 't':
        v.t = Value::BOOL;
        v.b = true;
        ok = lit("true", 4);
        break;
      case 'f':
        v.t = Value::BOOL;
        v.b = false;
        ok = lit("false", 5);
        break;
      case 'n':
        v.t = Value::NUL;
        ok = lit("null", 4);
        break;
      default:
        ok = num(v);
    }
    depth--;
    return ok;
  }
};

bool ieq(const std::string& a, const char* b) {
  const size_t n = std::strlen(b);
  if (a.size() != n) return false;
  for (size_t i = 0; i < n; i++) {
    char x = a[i], y = b[i];
    if (x >= 'A' && x <= 'Z') x = (char)(x - 'A' + 'a');
    if (y >= 'A' && y <= 'Z') y = (char)(y - 'A' + 'a');
    if (x != y) return false;
  }
  return true;
}

}  // namespace

const Value* Value::key(const char* k) const {
  if (t != OBJ) return nullptr;
  const Value* r = nullptr;
  for (const auto& m : o)
    if (m.first == k) r = &m.second;
  return r;
}

const Value* Value::field(const char* k) const {
  if (t != OBJ) return nullptr;
  const Value* r = nullptr;
  for (const auto& m : o)  // encoding/json assigns every member that maps to the field: the last one wins
    if (m.first == k || ieq(m.first, k)) r = &m.second;
  return r;
}

bool parse(const char* p, size_t n, Value& out, std::string& err) {
  Parser ps{p, p + n, {}};
  out = Value();
  if (!ps.value(out)) {
    err = ps.err;
    return false;
  }
  ps.ws();
  if (ps.p != ps.e) {
    err = "trailing data after the JSON value";
    return false;
  }
  return true;
}

bool as_int64(const Value& v, int64_t* out) { return v.t == Value::NUM && parse_int64(v.s, out); }

bool as_float64(const Value& v, double* out) {
  if (v.t != Value::NUM) return false;
  errno = 0;
  char* end = nullptr;
  const double d = std::strtod(v.s.c_str(), &end);
  if (end != v.s.c_str() + v.s.size() || errno == ERANGE) return false;  // ParseFloat: out of range -> error
  *out = d;
  return true;
}

}  // namespace json

bool parse_int64(const std::string& s, int64_t* out) {
  size_t i = 0;
  bool neg = false;
  if (i < s.size() && (s[i] == '+' || s[i] == '-')) neg = s[i++] == '-';
  if (i >= s.size()) return false;
  unsigned __int128 v = 0;
  for (; i < s.size(); i++) {
    if (s[i] < '0' || s[i] > '9') return false;
    v = v * 10 + (unsigned)(s[i] - '0');
    if (v > ((unsigned __int128)1 << 63)) return false;
  }
  if (!neg && v > (unsigned __int128)INT64_MAX) return false;
  *out = neg ? (int64_t)(-(__int128)v) : (int64_t)v;
  return true;
}

// ---- resource.Quantity (k8s.io/apimachinery/pkg/api/resource/quantity.go, v0.28) ---------------------------
namespace {
using i128 = __int128;

bool mul_ok(i128 a, i128 b, i128* r) { return !__builtin_mul_overflow(a, b, r); }

i128 pow10_128(int k) {
  i128 r = 1;
  for (int i = 0; i < k; i++) r *= 10;
  return r;
}

// ceil(n / d) for n >= 0, d > 0
i128 ceil_div(i128 n, i128 d) { return n / d + (n % d != 0 ? 1 : 0); }

// |q| = n * 10^e, n >= 0, after ParseQuantity's rounding up to nano (amount.Round(amount, Nano, RoundUp)), in
// units of 1e-9; false when it does not fit
bool to_nanos(i128 n, int e, i128* out) {
  if (e < -9) {
    n = (-9 - e > 38) ? (n != 0 ? 1 : 0) : ceil_div(n, pow10_128(-9 - e));
    e = -9;
  }
  const int s = e + 9;
  if (s > 38) return n == 0 ? (*out = 0, true) : false;
  return mul_ok(n, pow10_128(s), out);
}
}  // namespace

bool quantity_nanos(const std::string& str, __int128* nanos, bool* overflow) {
  *overflow = false;
  if (str.empty()) return false;
  if (str == "0") {
    *nanos = 0;
    return true;
  }
  size_t pos = 0;
  const size_t end = str.size();
  bool positive = true;
  if (str[0] == '-') positive = false, pos++;
  else if (str[0] == '+') pos++;
  size_t num0 = pos;
  while (pos < end && str[pos] >= '0' && str[pos] <= '9') pos++;
  std::string num = str.substr(num0, pos - num0), denom;
  if (pos < end && str[pos] == '.') {
    pos++;
    const size_t d0 = pos;
    while (pos < end && str[pos] >= '0' && str[pos] <= '9') pos++;
    denom = str.substr(d0, pos - d0);
  }
  if (num.empty() && denom.empty()) return false;
  const size_t suf0 = pos;
  while (pos < end && std::strchr("eEinumkKMGTP", str[pos])) pos++;
  if (pos < end && (str[pos] == '-' || str[pos] == '+')) pos++;
  while (pos < end && str[pos] >= '0' && str[pos] <= '9') pos++;
  if (pos != end) return false;
  const std::string suffix = str.substr(suf0);
  // quantitySuffixer.interpret (suffix.go)
  int e10 = 0, e2 = 0;
  static const struct { const char* s; int e10, e2; } SUF[] = {
      {"", 0, 0},   {"n", -9, 0}, {"u", -6, 0},  {"m", -3, 0},  {"k", 3, 0},   {"M", 6, 0},   {"G", 9, 0},
      {"T", 12, 0}, {"P", 15, 0}, {"E", 18, 0},  {"Ki", 0, 10}, {"Mi", 0, 20}, {"Gi", 0, 30}, {"Ti", 0, 40},
      {"Pi", 0, 50}, {"Ei", 0, 60}};
  bool found = false;
  for (const auto& x : SUF)
    if (suffix == x.s) e10 = x.e10, e2 = x.e2, found = true;
  if (!found) {
    int64_t ex;
    if (suffix.size() > 1 && (suffix[0] == 'e' || suffix[0] == 'E') && parse_int64(suffix.substr(1), &ex) &&
        ex > -1000 && ex < 1000)
      e10 = (int)ex;
    else
      return false;
  }
  std::string digits = num + denom;  // mantissa digits, leading zeros dropped
  size_t z = 0;
  while (z + 1 < digits.size() && digits[z] == '0') z++;
  digits = digits.substr(z);
  if (digits.size() > 36) {
    *overflow = true;
    return false;
  }
  i128 n = 0;
  for (char c : digits) n = n * 10 + (c - '0');
  if (!positive && n != 0) {  // negative quantities are neither requests nor capacities
    *overflow = true;
    return false;
  }
  if ((e2 && !mul_ok(n, (i128)1 << e2, &n)) || !to_nanos(n, e10 - (int)denom.size(), nanos)) {
    *overflow = true;
    return false;
  }
  return true;
}

bool nanos_value(__int128 nanos, int64_t* value, int64_t* milli) {  // Value() / MilliValue(): round up
  const i128 v = ceil_div(nanos, 1000000000), m = ceil_div(nanos, 1000000);
  if (m > (i128)INT64_MAX) return false;
  *value = (int64_t)v;
  *milli = (int64_t)m;
  return true;
}

bool parse_quantity(const std::string& str, int64_t* value, int64_t* milli, bool* overflow) {
  __int128 n;
  if (!quantity_nanos(str, &n, overflow)) return false;
  if (!nanos_value(n, value, milli)) {
    *overflow = true;
    return false;
  }
  return true;
}

bool quantity_json_nanos(const json::Value& v, __int128* nanos, bool* overflow) {
  *overflow = false;
  std::string s;
  if (v.t == json::Value::STR || v.t == json::Value::NUM) s = v.s;
  else return false;
  size_t a = 0, b = s.size();  // Quantity.UnmarshalJSON: strings.TrimSpace
  while (a < b && std::strchr(" \t\n\r\v\f", s[a])) a++;
  while (b > a && std::strchr(" \t\n\r\v\f", s[b - 1])) b--;
  return quantity_nanos(s.substr(a, b - a), nanos, overflow);
}

bool quantity_json(const json::Value& v, int64_t* value, int64_t* milli, bool* overflow) {
  __int128 n;
  if (!quantity_json_nanos(v, &n, overflow)) return false;
  if (!nanos_value(n, value, milli)) {
    *overflow = true;
    return false;
  }
  return true;
}

// ---- time.ParseDuration (Go src/time/format.go) ------------------------------------------------------------
bool parse_duration(const std::string& s0, int64_t* ns) {
  std::string s = s0;
  bool neg = false;
  if (!s.empty() && (s[0] == '-' || s[0] == '+')) {
    neg = s[0] == '-';
    s = s.substr(1);
  }
  if (s == "0") {
    *ns = 0;
    return true;
  }
  if (s.empty()) return false;
  uint64_t d = 0;
  size_t i = 0;
  while (i < s.size()) {
    uint64_t v = 0, f = 0;
    double scale = 1;
    if (!(s[i] == '.' || (s[i] >= '0' && s[i] <= '9'))) return false;
    const size_t i0 = i;
    while (i < s.size() && s[i] >= '0' && s[i] <= '9') {
      if (v > (1ull << 63) / 10) return false;
      v = v * 10 + (uint64_t)(s[i] - '0');
      if (v > (1ull << 63)) return false;
      i++;
    }
    const bool pre = i != i0;
    bool post = false;
    if (i < s.size() && s[i] == '.') {
      i++;
      const size_t f0 = i;
      bool overflow = false;
      while (i < s.size() && s[i] >= '0' && s[i] <= '9') {
        if (!overflow) {
          if (f > (1ull << 63) / 10) {
            overflow = true;
          } else {
            const uint64_t y = f * 10 + (uint64_t)(s[i] - '0');
            if (y > (1ull << 63)) overflow = true;
            else f = y, scale *= 10;
          }
        }
        i++;
      }
      post = i != f0;
    }
    if (!pre && !post) return false;
    const size_t u0 = i;
    while (i < s.size() && s[i] != '.' && !(s[i] >= '0' && s[i] <= '9')) i++;
    const std::string u = s.substr(u0, i - u0);
    uint64_t unit;
    if (u == "ns") unit = 1;
    else if (u == "us" || u == "\xc2\xb5s" || u == "\xce\xbcs") unit = 1000;
    else if (u == "ms") unit = 1000000;
    else if (u == "s") unit = 1000000000ull;
    else if (u == "m") unit = 60ull * 1000000000ull;
    else if (u == "h") unit = 3600ull * 1000000000ull;
    else return false;  // missing or unknown unit
    if (v > (1ull << 63) / unit) return false;
    v *= unit;
    if (f > 0) {
      v += (uint64_t)((double)f * ((double)unit / scale));
      if (v > (1ull << 63)) return false;
    }
    d += v;
    if (d > (1ull << 63)) return false;
  }
  if (neg) {
    *ns = -(int64_t)d;
    return true;
  }
  if (d > (uint64_t)INT64_MAX) return false;
  *ns = (int64_t)d;
  return true;
}

// ---- metav1.Time: time.Parse(time.RFC3339, s) ----------------------------------------------------------
namespace {
int64_t days_from_civil(int64_t y, unsigned m, unsigned d) {  // H. Hinnant's algorithm
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const unsigned yoe = (unsigned)(y - era * 400);
  const unsigned doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + (int64_t)doe - 719468;
}
bool digits(const std::string& s, size_t at, size_t n, int* out) {
  if (at + n > s.size()) return false;
  int v = 0;
  for (size_t i = at; i < at + n; i++) {
    if (s[i] < '0' || s[i] > '9') return false;
    v = v * 10 + (s[i] - '0');
  }
  *out = v;
  return true;
}
}  // namespace

bool parse_rfc3339(const std::string& s, int64_t* ns) {
  int Y, M, D, h, m, sec;
  if (!digits(s, 0, 4, &Y) || s.size() < 20 || s[4] != '-' || !digits(s, 5, 2, &M) || s[7] != '-' ||
      !digits(s, 8, 2, &D) || s[10] != 'T' || !digits(s, 11, 2, &h) || s[13] != ':' || !digits(s, 14, 2, &m) ||
      s[16] != ':' || !digits(s, 17, 2, &sec))
    return false;
  static const int mdays[] = {31, 29, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  const bool leap = (Y % 4 == 0 && Y % 100 != 0) || Y % 400 == 0;
  if (M < 1 || M > 12 || D < 1 || D > mdays[M - 1] || (M == 2 && D == 29 && !leap) || h > 23 || m > 59 || sec > 59)
    return false;
  size_t i = 19;
  int64_t frac = 0;
  if (i < s.size() && (s[i] == '.' || s[i] == ',')) {  // fractional seconds (Go accepts them after "05")
    i++;
    int nd = 0;
    while (i < s.size() && s[i] >= '0' && s[i] <= '9') {
      if (nd < 9) frac = frac * 10 + (s[i] - '0');
      nd++;
      i++;
    }
    if (nd == 0) return false;
    for (int k = nd; k < 9; k++) frac *= 10;
  }
  int64_t off = 0;
  if (i < s.size() && s[i] == 'Z') {
    i++;
  } else if (i < s.size() && (s[i] == '+' || s[i] == '-')) {
    int oh, om;
    if (!digits(s, i + 1, 2, &oh) || i + 3 >= s.size() || s[i + 3] != ':' || !digits(s, i + 4, 2, &om) || oh > 23 ||
        om > 59)
      return false;
    off = (s[i] == '-' ? -1 : 1) * ((int64_t)oh * 3600 + om * 60);
    i += 6;
  } else {
    return false;
  }
  if (i != s.size()) return false;
  const int64_t secs = days_from_civil(Y, (unsigned)M, (unsigned)D) * 86400 + h * 3600 + m * 60 + sec - off;
  // int64 unix nanoseconds cover 1677-09-21 .. 2262-04-11 (Go: UnixNano undefined outside); later times are
  // not representable here
  int64_t t;
  if (__builtin_mul_overflow(secs, (int64_t)1000000000, &t) || __builtin_add_overflow(t, frac, &t)) return false;
  *ns = t;
  return true;
}

}  // namespace ke
