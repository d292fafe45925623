// Small text helpers shared by the native HTTP components (sidecar data plane, backing front,
// load generator): URL percent-coding, JSON string quoting, UTF-8 validation, base64.
#pragma once

#include <cctype>
#include <cstdint>
#include <string>
#include <string_view>

#include "json.hpp"

namespace tt::text {

inline int hexv(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

// urllib.parse.unquote (plus_space: unquote_plus for query strings)
inline std::string unquote(std::string_view s, bool plus_space = false) {
  std::string o;
  o.reserve(s.size());
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '%' && i + 2 < s.size() && hexv(s[i + 1]) >= 0 && hexv(s[i + 2]) >= 0) {
      o += (char)(hexv(s[i + 1]) * 16 + hexv(s[i + 2]));
      i += 2;
    } else if (plus_space && s[i] == '+') {
      o += ' ';
    } else {
      o += s[i];
    }
  }
  return o;
}

// urllib.parse.quote(s, safe="")
inline std::string quote_all(std::string_view s) {
  static const char* d = "0123456789ABCDEF";
  std::string o;
  for (unsigned char c : s) {
    if (std::isalnum(c) || c == '_' || c == '.' || c == '-' || c == '~') {
      o += (char)c;
    } else {
      o += '%';
      o += d[c >> 4];
      o += d[c & 15];
    }
  }
  return o;
}

inline std::string lower(std::string_view s) {
  std::string o(s);
  for (auto& c : o) c = (char)std::tolower((unsigned char)c);
  return o;
}

// JSON string literal (quotes + escapes)
inline std::string json_str(std::string_view s) {
  std::string o;
  escape_to(o, s);
  return o;
}

inline bool valid_utf8(std::string_view s) {
  for (size_t i = 0; i < s.size();) {
    unsigned char c = (unsigned char)s[i];
    size_t n = c < 0x80 ? 0 : (c >> 5) == 6 ? 1 : (c >> 4) == 14 ? 2 : (c >> 3) == 30 ? 3 : 99;
    if (n == 99 || i + n >= s.size() + (n == 0)) return n == 0;
    for (size_t k = 1; k <= n; ++k)
      if (((unsigned char)s[i + k] >> 6) != 2) return false;
    i += n + 1;
  }
  return true;
}

inline std::string base64(std::string_view in) {
  static const char* t = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  std::string o;
  size_t i = 0;
  for (; i + 2 < in.size(); i += 3) {
    uint32_t v = ((uint8_t)in[i] << 16) | ((uint8_t)in[i + 1] << 8) | (uint8_t)in[i + 2];
    o += t[v >> 18];
    o += t[(v >> 12) & 63];
    o += t[(v >> 6) & 63];
    o += t[v & 63];
  }
  if (i + 1 == in.size()) {
    uint32_t v = (uint8_t)in[i] << 16;
    o += t[v >> 18];
    o += t[(v >> 12) & 63];
    o += "==";
  } else if (i + 2 == in.size()) {
    uint32_t v = ((uint8_t)in[i] << 16) | ((uint8_t)in[i + 1] << 8);
    o += t[v >> 18];
    o += t[(v >> 12) & 63];
    o += t[(v >> 6) & 63];
    o += '=';
  }
  return o;
}

inline std::string unbase64(std::string_view in) {
  std::string o;
  uint32_t acc = 0;
  int bits = 0;
  for (char c : in) {
    int v = c >= 'A' && c <= 'Z' ? c - 'A' : c >= 'a' && c <= 'z' ? c - 'a' + 26 : c >= '0' && c <= '9' ? c - '0' + 52
            : c == '+' ? 62 : c == '/' ? 63 : -1;
    if (v < 0) continue;
    acc = (acc << 6) | (uint32_t)v;
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      o += (char)((acc >> bits) & 0xFF);
    }
  }
  return o;
}

}  // namespace tt::text
