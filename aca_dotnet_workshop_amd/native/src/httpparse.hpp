// HTTP/1.1 message-head parsing for the Python web layer (server requests and client
// responses).  The head (request/status line + header lines, without the blank line) is
// parsed in one pass; header names are lower-cased, values trimmed, repeated headers
// joined with ", " (``set-cookie`` keeps a list, exposed separately).
#pragma once

#include <cctype>
#include <stdexcept>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace tt {

struct HttpHead {
  std::string a, b, c;  // request: method, target, version; response: version, status, reason
  std::vector<std::pair<std::string, std::string>> headers;
};

inline std::string_view trim(std::string_view s) {
  size_t i = 0, j = s.size();
  while (i < j && (s[i] == ' ' || s[i] == '\t')) ++i;
  while (j > i && (s[j - 1] == ' ' || s[j - 1] == '\t' || s[j - 1] == '\r')) --j;
  return s.substr(i, j - i);
}

// ASCII lower case (header names are tokens): no locale lookup per character
inline char ascii_lower(char c) { return c >= 'A' && c <= 'Z' ? (char)(c + ('a' - 'A')) : c; }

inline HttpHead parse_head(std::string_view head) {
  HttpHead h;
  size_t eol = head.find("\r\n");
  std::string_view first = head.substr(0, eol);
  size_t s1 = first.find(' ');
  if (s1 == std::string_view::npos) throw std::invalid_argument("malformed start line");
  size_t s2 = first.find(' ', s1 + 1);
  h.a = std::string(first.substr(0, s1));
  if (s2 == std::string_view::npos) {
    h.b = std::string(first.substr(s1 + 1));
  } else {
    h.b = std::string(first.substr(s1 + 1, s2 - s1 - 1));
    h.c = std::string(first.substr(s2 + 1));
  }
  size_t pos = eol == std::string_view::npos ? head.size() : eol + 2;
  h.headers.reserve(16);  // one allocation for a typical head instead of growing 1, 2, 4, 8
  while (pos < head.size()) {
    size_t e = head.find("\r\n", pos);
    if (e == std::string_view::npos) e = head.size();
    std::string_view line = head.substr(pos, e - pos);
    pos = e + 2;
    if (line.empty()) continue;
    size_t colon = line.find(':');
    if (colon == std::string_view::npos) throw std::invalid_argument("malformed header line");
    std::string name(trim(line.substr(0, colon)));
    for (auto& ch : name) ch = ascii_lower(ch);
    h.headers.emplace_back(std::move(name), std::string(trim(line.substr(colon + 1))));
  }
  return h;
}

}  // namespace tt
