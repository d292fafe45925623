// Compact JSON DOM + parser + serializer used by the native document store and broker.
//
// Objects keep insertion order (two parallel vectors) so stored documents round-trip
// byte-for-byte through the query path.  Numbers are doubles (JSON semantics).
#pragma once

#include <emmintrin.h>

#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

namespace tt {

struct Value {
  enum Type : uint8_t { Null = 0, Bool = 1, Number = 2, String = 3, Array = 4, Object = 5 };
  Type t = Null;
  bool b = false;
  double n = 0.0;
  std::string s;                 // String payload
  std::vector<Value> items;      // Array items / Object values
  std::vector<std::string> keys; // Object keys (parallel to items)

  static Value null() { return Value(); }
  static Value boolean(bool v) { Value x; x.t = Bool; x.b = v; return x; }
  static Value number(double v) { Value x; x.t = Number; x.n = v; return x; }
  static Value string(std::string v) { Value x; x.t = String; x.s = std::move(v); return x; }

  const Value* get(std::string_view key) const {
    if (t != Object) return nullptr;
    for (size_t i = 0; i < keys.size(); ++i)
      if (keys[i] == key) return &items[i];
    return nullptr;
  }
  // case-insensitive fallback (camelCase vs PascalCase producers)
  const Value* get_ci(std::string_view key) const {
    if (t != Object) return nullptr;
    if (auto* v = get(key)) return v;
    for (size_t i = 0; i < keys.size(); ++i) {
      const std::string& k = keys[i];
      if (k.size() != key.size()) continue;
      bool eq = true;
      for (size_t j = 0; j < k.size() && eq; ++j) eq = std::tolower((unsigned char)k[j]) == std::tolower((unsigned char)key[j]);
      if (eq) return &items[i];
    }
    return nullptr;
  }
  // Dotted path lookup ("a.b.c"); array indices allowed as numeric segments.
  const Value* path(std::string_view p) const {
    const Value* cur = this;
    size_t pos = 0;
    while (cur && pos <= p.size()) {
      size_t dot = p.find('.', pos);
      std::string_view seg = p.substr(pos, dot == std::string_view::npos ? std::string_view::npos : dot - pos);
      if (cur->t == Object) {
        cur = cur->get_ci(seg);
      } else if (cur->t == Array) {
        size_t idx = 0;
        bool ok = !seg.empty();
        for (char c : seg) { if (c < '0' || c > '9') { ok = false; break; } idx = idx * 10 + (c - '0'); }
        cur = (ok && idx < cur->items.size()) ? &cur->items[idx] : nullptr;
      } else {
        return nullptr;
      }
      if (dot == std::string_view::npos) break;
      pos = dot + 1;
    }
    return cur;
  }
};

struct ParseError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// Recursive-descent parser that builds each value in place (no temporaries moved into the
// parent's vectors), reserves small containers up front, finds the end of a string run 16 bytes
// at a time (SSE2) and converts plain integers without strtod.  `strict`: raw control characters
// inside strings are an error (Python's json.loads), which the task codecs need.
class Parser {
 public:
  explicit Parser(std::string_view s, bool strict = false) : p_(s.data()), e_(s.data() + s.size()), strict_(strict) {}
  Value parse() {
    Value v;
    value(v, 0);
    ws();
    if (p_ != e_) throw ParseError("trailing characters after JSON value");
    return v;
  }

 private:
  const char* p_;
  const char* e_;
  bool strict_;

  void ws() { while (p_ < e_ && (*p_ == ' ' || *p_ == '\n' || *p_ == '\r' || *p_ == '\t')) ++p_; }
  [[noreturn]] void fail(const char* m) { throw ParseError(m); }

  void value(Value& v, int depth) {
    if (depth > 256) fail("JSON nesting too deep");
    ws();
    if (p_ >= e_) fail("unexpected end of JSON");
    switch (*p_) {
      case '{': object(v, depth); return;
      case '[': array(v, depth); return;
      case '"': v.t = Value::String; str(v.s); return;
      case 't': lit("true", 4); v.t = Value::Bool; v.b = true; return;
      case 'f': lit("false", 5); v.t = Value::Bool; v.b = false; return;
      case 'n': lit("null", 4); return;
      default: num(v);
    }
  }
  void lit(const char* w, size_t n) {
    if ((size_t)(e_ - p_) < n || std::memcmp(p_, w, n) != 0) fail("invalid literal");
    p_ += n;
  }
  // The token is the longest run of [0-9.eE+-] after an optional sign, and must be a complete
  // strtod number; up to 15 plain digits are exact as an integer conversion.
  void num(Value& v) {
    const char* s = p_;
    if (p_ < e_ && (*p_ == '-' || *p_ == '+')) ++p_;
    const char* d0 = p_;
    while (p_ < e_ && *p_ >= '0' && *p_ <= '9') ++p_;
    const char* d1 = p_;
    while (p_ < e_ && ((*p_ >= '0' && *p_ <= '9') || *p_ == '.' || *p_ == 'e' || *p_ == 'E' || *p_ == '-' || *p_ == '+')) ++p_;
    if (p_ == s) fail("invalid JSON token");
    v.t = Value::Number;
    if (p_ == d1 && d1 > d0 && d1 - d0 <= 15) {
      int64_t x = 0;
      for (const char* q = d0; q < d1; ++q) x = x * 10 + (*q - '0');
      v.n = *s == '-' ? -(double)x : (double)x;
      return;
    }
    char buf[64];
    std::string big;
    const size_t n = (size_t)(p_ - s);
    const char* c;
    if (n < sizeof buf) {
      std::memcpy(buf, s, n);
      buf[n] = 0;
      c = buf;
    } else {
      big.assign(s, n);
      c = big.c_str();
    }
    char* end = nullptr;
    v.n = std::strtod(c, &end);
    if (end != c + n) fail("invalid number");
  }
  static void utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) out += (char)cp;
    else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) { out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F)); }
    else { out += (char)(0xF0 | (cp >> 18)); out += (char)(0x80 | ((cp >> 12) & 0x3F)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F)); }
  }
  uint32_t hex4() {
    if (e_ - p_ < 4) fail("bad \\u escape");
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
      char c = *p_++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad hex digit");
    }
    return v;
  }
  // First '"' or '\\' (strict: or control character) at or after p, else e.
  const char* stop(const char* p) const {
    const __m128i q = _mm_set1_epi8('"'), bs = _mm_set1_epi8('\\'), ctl = _mm_set1_epi8(0x1F);
    while (e_ - p >= 16) {
      __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p));
      __m128i hit = _mm_or_si128(_mm_cmpeq_epi8(x, q), _mm_cmpeq_epi8(x, bs));
      if (strict_) hit = _mm_or_si128(hit, _mm_cmpeq_epi8(_mm_max_epu8(x, ctl), ctl));
      int m = _mm_movemask_epi8(hit);
      if (m) return p + __builtin_ctz((unsigned)m);
      p += 16;
    }
    while (p < e_ && *p != '"' && *p != '\\' && !(strict_ && (unsigned char)*p < 0x20)) ++p;
    return p;
  }
  void str(std::string& out) {
    ++p_;  // opening quote
    const char* run = p_;
    while (true) {
      p_ = stop(p_);
      if (p_ >= e_) fail("unterminated string");
      char c = *p_;
      if (c == '"') { out.append(run, p_); ++p_; return; }
      if (c != '\\') fail("control character in string");
      out.append(run, p_);
      ++p_;
      if (p_ >= e_) fail("bad escape");
      char x = *p_++;
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
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00 && e_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') {
            p_ += 2;
            uint32_t lo = hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          utf8(out, cp);
          break;
        }
        default: fail("bad escape");
      }
      run = p_;
    }
  }
  void array(Value& v, int depth) {
    ++p_;
    v.t = Value::Array;
    ws();
    if (p_ < e_ && *p_ == ']') { ++p_; return; }
    v.items.reserve(4);
    while (true) {
      v.items.emplace_back();
      value(v.items.back(), depth + 1);
      ws();
      if (p_ >= e_) fail("unterminated array");
      if (*p_ == ',') { ++p_; continue; }
      if (*p_ == ']') { ++p_; return; }
      fail("expected , or ]");
    }
  }
  void object(Value& v, int depth) {
    ++p_;
    v.t = Value::Object;
    ws();
    if (p_ < e_ && *p_ == '}') { ++p_; return; }
    v.keys.reserve(8);
    v.items.reserve(8);
    while (true) {
      ws();
      if (p_ >= e_ || *p_ != '"') fail("expected object key");
      v.keys.emplace_back();
      str(v.keys.back());
      ws();
      if (p_ >= e_ || *p_ != ':') fail("expected :");
      ++p_;
      v.items.emplace_back();
      value(v.items.back(), depth + 1);
      ws();
      if (p_ >= e_) fail("unterminated object");
      if (*p_ == ',') { ++p_; continue; }
      if (*p_ == '}') { ++p_; return; }
      fail("expected , or }");
    }
  }
};

inline Value parse(std::string_view s) { return Parser(s).parse(); }
// json.loads' strictness: raw control characters inside strings are rejected.
inline Value parse_strict(std::string_view s) { return Parser(s, true).parse(); }

// Allocation-free check that `s` is one JSON value Parser would accept (same grammar: number
// tokens, escapes, nesting limit), for the data plane's "is this body JSON?" questions.
class Validator {
 public:
  explicit Validator(std::string_view s) : p_(s.data()), e_(s.data() + s.size()) {}
  bool ok() {
    if (!value(0)) return false;
    ws();
    return p_ == e_;
  }

 private:
  const char* p_;
  const char* e_;
  void ws() { while (p_ < e_ && (*p_ == ' ' || *p_ == '\n' || *p_ == '\r' || *p_ == '\t')) ++p_; }
  bool value(int depth) {
    if (depth > 256) return false;
    ws();
    if (p_ >= e_) return false;
    switch (*p_) {
      case '{': return object(depth);
      case '[': return array(depth);
      case '"': return str();
      case 't': return lit("true", 4);
      case 'f': return lit("false", 5);
      case 'n': return lit("null", 4);
      default: return num();
    }
  }
  bool lit(const char* w, size_t n) {
    if ((size_t)(e_ - p_) < n || std::memcmp(p_, w, n) != 0) return false;
    p_ += n;
    return true;
  }
  bool num() {
    const char* s = p_;
    if (p_ < e_ && (*p_ == '-' || *p_ == '+')) ++p_;
    const char* d0 = p_;
    while (p_ < e_ && *p_ >= '0' && *p_ <= '9') ++p_;
    const char* d1 = p_;
    while (p_ < e_ && ((*p_ >= '0' && *p_ <= '9') || *p_ == '.' || *p_ == 'e' || *p_ == 'E' || *p_ == '-' || *p_ == '+')) ++p_;
    if (p_ == s) return false;
    if (p_ == d1 && d1 > d0) return true;  // sign + digits: always a complete strtod number
    char buf[64];
    std::string big;
    const size_t n = (size_t)(p_ - s);
    const char* c;
    if (n < sizeof buf) {
      std::memcpy(buf, s, n);
      buf[n] = 0;
      c = buf;
    } else {
      big.assign(s, n);
      c = big.c_str();
    }
    char* end = nullptr;
    std::strtod(c, &end);
    return end == c + n;
  }
  bool str() {
    ++p_;
    const __m128i q = _mm_set1_epi8('"'), bs = _mm_set1_epi8('\\');
    while (true) {
      while (e_ - p_ >= 16) {
        __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p_));
        int m = _mm_movemask_epi8(_mm_or_si128(_mm_cmpeq_epi8(x, q), _mm_cmpeq_epi8(x, bs)));
        if (m) {
          p_ += __builtin_ctz((unsigned)m);
          break;
        }
        p_ += 16;
      }
      while (p_ < e_ && *p_ != '"' && *p_ != '\\') ++p_;
      if (p_ >= e_) return false;
      if (*p_ == '"') {
        ++p_;
        return true;
      }
      ++p_;  // backslash
      if (p_ >= e_) return false;
      char x = *p_++;
      switch (x) {
        case '"': case '\\': case '/': case 'b': case 'f': case 'n': case 'r': case 't': break;
        case 'u': {
          if (!hex4()) return false;
          break;
        }
        default: return false;
      }
    }
  }
  bool hex4() {
    if (e_ - p_ < 4) return false;
    uint32_t cp = 0;
    for (int i = 0; i < 4; ++i) {
      char c = *p_++;
      cp <<= 4;
      if (c >= '0' && c <= '9') cp |= c - '0';
      else if (c >= 'a' && c <= 'f') cp |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') cp |= c - 'A' + 10;
      else return false;
    }
    // Parser: a high surrogate followed by "\u" consumes the second escape as its low half
    if (cp >= 0xD800 && cp < 0xDC00 && e_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') {
      p_ += 2;
      for (int i = 0; i < 4; ++i) {
        char c = *p_++;
        if (!((c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'))) return false;
      }
    }
    return true;
  }
  bool array(int depth) {
    ++p_;
    ws();
    if (p_ < e_ && *p_ == ']') { ++p_; return true; }
    while (true) {
      if (!value(depth + 1)) return false;
      ws();
      if (p_ >= e_) return false;
      if (*p_ == ',') { ++p_; continue; }
      if (*p_ == ']') { ++p_; return true; }
      return false;
    }
  }
  bool object(int depth) {
    ++p_;
    ws();
    if (p_ < e_ && *p_ == '}') { ++p_; return true; }
    while (true) {
      ws();
      if (p_ >= e_ || *p_ != '"' || !str()) return false;
      ws();
      if (p_ >= e_ || *p_ != ':') return false;
      ++p_;
      if (!value(depth + 1)) return false;
      ws();
      if (p_ >= e_) return false;
      if (*p_ == ',') { ++p_; continue; }
      if (*p_ == '}') { ++p_; return true; }
      return false;
    }
  }
};

inline bool valid(std::string_view s) { return Validator(s).ok(); }

// Scanning a validated JSON text without building values: end of the whitespace at p, and end
// of the value starting at p (raw slices of a request body, e.g. the state items' values).
inline const char* ws_end(const char* p, const char* e) {
  while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  return p;
}

inline const char* skip_value(const char* p, const char* e) {
  p = ws_end(p, e);
  if (p >= e) return p;
  if (*p == '"') {
    ++p;
    while (p < e && *p != '"') p += (*p == '\\') ? 2 : 1;
    return p + 1;
  }
  if (*p == '{' || *p == '[') {
    int depth = 0;
    while (p < e) {
      char c = *p;
      if (c == '"') {
        p = skip_value(p, e);
        continue;
      }
      if (c == '{' || c == '[') ++depth;
      if (c == '}' || c == ']') {
        if (--depth == 0) return p + 1;
      }
      ++p;
    }
    return p;
  }
  while (p < e && *p != ',' && *p != '}' && *p != ']' && *p != ' ' && *p != '\n' && *p != '\r' && *p != '\t') ++p;
  return p;
}

// Copy of a valid JSON text without insignificant whitespace; runs without quotes, backslashes
// or whitespace are copied 16 bytes at a time.
inline std::string compact(std::string_view s) {
  std::string o;
  o.reserve(s.size());
  const char* p = s.data();
  const char* e = p + s.size();
  bool in_str = false;
  const __m128i q = _mm_set1_epi8('"'), bs = _mm_set1_epi8('\\'), sp = _mm_set1_epi8(' '), nl = _mm_set1_epi8('\n'),
                cr = _mm_set1_epi8('\r'), tb = _mm_set1_epi8('\t');
  while (p < e) {
    if (e - p >= 16) {
      __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p));
      __m128i hit = _mm_or_si128(_mm_cmpeq_epi8(x, q), _mm_cmpeq_epi8(x, bs));
      if (!in_str)
        hit = _mm_or_si128(hit, _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(x, sp), _mm_cmpeq_epi8(x, nl)),
                                             _mm_or_si128(_mm_cmpeq_epi8(x, cr), _mm_cmpeq_epi8(x, tb))));
      int m = _mm_movemask_epi8(hit);
      if (m == 0) {
        o.append(p, 16);
        p += 16;
        continue;
      }
      int k = __builtin_ctz((unsigned)m);
      o.append(p, (size_t)k);
      p += k;
    }
    char c = *p++;
    if (in_str) {
      o += c;
      if (c == '\\' && p < e) o += *p++;
      else if (c == '"') in_str = false;
    } else if (c == '"') {
      in_str = true;
      o += c;
    } else if (c != ' ' && c != '\n' && c != '\r' && c != '\t') {
      o += c;
    }
  }
  return o;
}

inline void escape_to(std::string& out, std::string_view s) {
  out += '"';
  const char* run = s.data();  // plain characters go out in runs, not one push_back each
  const char* e = s.data() + s.size();
  for (const char* p = run; p < e; ++p) {
    const unsigned char c = (unsigned char)*p;
    if (c >= 0x20 && c != '"' && c != '\\') continue;
    out.append(run, (size_t)(p - run));
    run = p + 1;
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      default:
        char buf[8];
        std::snprintf(buf, sizeof buf, "\\u%04x", c);
        out += buf;
    }
  }
  out.append(run, (size_t)(e - run));
  out += '"';
}

inline void number_to(std::string& out, double d) {
  if (std::isfinite(d) && d == std::floor(d) && std::fabs(d) < 9.007199254740992e15) {
    char buf[32];
    std::snprintf(buf, sizeof buf, "%lld", (long long)d);
    out += buf;
  } else if (!std::isfinite(d)) {
    out += "null";
  } else {
    char buf[32];
    std::snprintf(buf, sizeof buf, "%.17g", d);
    out += buf;
  }
}

inline void dump_to(std::string& out, const Value& v) {
  switch (v.t) {
    case Value::Null: out += "null"; break;
    case Value::Bool: out += v.b ? "true" : "false"; break;
    case Value::Number: number_to(out, v.n); break;
    case Value::String: escape_to(out, v.s); break;
    case Value::Array:
      out += '[';
      for (size_t i = 0; i < v.items.size(); ++i) { if (i) out += ','; dump_to(out, v.items[i]); }
      out += ']';
      break;
    case Value::Object:
      out += '{';
      for (size_t i = 0; i < v.items.size(); ++i) {
        if (i) out += ',';
        escape_to(out, v.keys[i]);
        out += ':';
        dump_to(out, v.items[i]);
      }
      out += '}';
      break;
  }
}

inline std::string dump(const Value& v) { std::string o; dump_to(o, v); return o; }

// Total order across JSON values: null < bool < number < string < array < object.
inline int compare(const Value& a, const Value& b) {
  if (a.t != b.t) return a.t < b.t ? -1 : 1;
  switch (a.t) {
    case Value::Null: return 0;
    case Value::Bool: return (int)a.b - (int)b.b;
    case Value::Number: return a.n < b.n ? -1 : (a.n > b.n ? 1 : 0);
    case Value::String: { int c = a.s.compare(b.s); return c < 0 ? -1 : (c > 0 ? 1 : 0); }
    case Value::Array: {
      size_t n = std::min(a.items.size(), b.items.size());
      for (size_t i = 0; i < n; ++i) { int c = compare(a.items[i], b.items[i]); if (c) return c; }
      return a.items.size() < b.items.size() ? -1 : (a.items.size() > b.items.size() ? 1 : 0);
    }
    case Value::Object: { std::string x = dump(a), y = dump(b); int c = x.compare(y); return c < 0 ? -1 : (c > 0 ? 1 : 0); }
  }
  return 0;
}

inline bool equals(const Value& a, const Value& b) { return compare(a, b) == 0; }

// Canonical hash-index key for a scalar value.
inline std::string index_key(const Value& v) {
  std::string k;
  k += (char)('0' + v.t);
  switch (v.t) {
    case Value::Bool: k += v.b ? '1' : '0'; break;
    case Value::Number: number_to(k, v.n); break;
    case Value::String: k += v.s; break;
    case Value::Null: break;
    default: dump_to(k, v); break;
  }
  return k;
}

}  // namespace tt
