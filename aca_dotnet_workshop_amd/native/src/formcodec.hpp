// The frontend's Create page post (reference Pages/Tasks/Create.cshtml.cs:30-51) in one native
// pass: the urlencoded form, the cookies, the antiforgery check and the [Required] binding of
// TaskAddModel, producing the JSON body the page sends to `api/tasks` through the sidecar.
//
// Exactly the decisions of services/frontend/app.py (Request.form / Request.cookies /
// Antiforgery.validate / _bind) for the posts a browser sends; anything outside that envelope
// -- a missing or blank field (the page re-renders with errors), an unusual date, whitespace the
// binder would strip, malformed escapes, non-UTF-8 bytes, a token in a header instead of the
// form -- is declined and the Python page handles it.
#pragma once

#include <openssl/crypto.h>
#include <openssl/evp.h>
#include <openssl/hmac.h>

#include <string>
#include <string_view>
#include <vector>

#include "json.hpp"
#include "taskcodec.hpp"

namespace formcodec {

enum class Verdict { kDecline, kOk, kBadToken };

inline int hexval(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

// urllib's unquote (plus_to_space: unquote_plus) restricted to well-formed input: false on a '%'
// without two hex digits or a result that is not UTF-8 (Python would keep / replace those).
inline bool unquote(std::string_view s, bool plus, std::string& out) {
  out.clear();
  out.reserve(s.size());
  for (size_t i = 0; i < s.size(); ++i) {
    char c = s[i];
    if (c == '%') {
      if (i + 2 >= s.size()) return false;
      int h = hexval(s[i + 1]), l = hexval(s[i + 2]);
      if (h < 0 || l < 0) return false;
      out += (char)(h * 16 + l);
      i += 2;
    } else if (plus && c == '+') {
      out += ' ';
    } else {
      out += c;
    }
  }
  return taskcodec::valid_utf8(out);
}

// A bound [Required] value: str.strip() would change it (or it is blank) -> the Python binder.
inline bool plain_value(const std::string& v) {
  if (v.empty()) return false;
  auto edge = [](unsigned char c) { return c <= 0x20 || c >= 0x7f; };  // ASCII space/control or non-ASCII
  return !edge((unsigned char)v.front()) && !edge((unsigned char)v.back());
}

inline bool digits(std::string_view s, size_t at, size_t n, int& out) {
  if (at + n > s.size()) return false;
  out = 0;
  for (size_t i = at; i < at + n; ++i) {
    if (s[i] < '0' || s[i] > '9') return false;
    out = out * 10 + (s[i] - '0');
  }
  return true;
}

// parse_datetime(v).strftime("%Y-%m-%dT%H:%M:%S") for "YYYY-MM-DD[THH:MM[:SS[.f{1,9}]]]"
// (the date input's value, or a datetime-local one); offsets and other forms are declined.
inline bool due_date(std::string_view v, std::string& out) {
  int y, mo, d, h = 0, mi = 0, s = 0;
  if (v.size() < 10 || !digits(v, 0, 4, y) || v[4] != '-' || !digits(v, 5, 2, mo) || v[7] != '-' ||
      !digits(v, 8, 2, d))
    return false;
  size_t i = 10;
  if (i < v.size()) {
    if (v[i] != 'T' || !digits(v, i + 1, 2, h) || i + 3 >= v.size() || v[i + 3] != ':' || !digits(v, i + 4, 2, mi))
      return false;
    i += 6;
    if (i < v.size()) {
      if (v[i] != ':' || !digits(v, i + 1, 2, s)) return false;
      i += 3;
      if (i < v.size()) {
        if (v[i] != '.') return false;
        size_t j = i + 1;
        while (j < v.size() && v[j] >= '0' && v[j] <= '9') ++j;
        if (j == i + 1 || j - i - 1 > 9 || j != v.size()) return false;
        i = j;
      }
    }
  }
  static const int mdays[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  if (y < 1000 || mo < 1 || mo > 12 || d < 1 || d > mdays[mo - 1] + (mo == 2 && taskcodec::leap(y)) || h > 23 ||
      mi > 59 || s > 59)
    return false;
  out.clear();
  taskcodec::put4(out, y); out += '-'; taskcodec::put2(out, mo); out += '-'; taskcodec::put2(out, d);
  out += 'T';
  taskcodec::put2(out, h); out += ':'; taskcodec::put2(out, mi); out += ':'; taskcodec::put2(out, s);
  return true;
}

inline std::string hmac_sha256_hex(std::string_view key, std::string_view msg) {
  unsigned char mac[EVP_MAX_MD_SIZE];
  unsigned int len = 0;
  HMAC(EVP_sha256(), key.data(), (int)key.size(), reinterpret_cast<const unsigned char*>(msg.data()), msg.size(), mac,
       &len);
  static const char* hx = "0123456789abcdef";
  std::string out(2 * len, '0');
  for (unsigned int i = 0; i < len; ++i) {
    out[2 * i] = hx[mac[i] >> 4];
    out[2 * i + 1] = hx[mac[i] & 15];
  }
  return out;
}

// `body`: the form; `cookie`: the Cookie header; `key`: the antiforgery key.  kOk: `json` holds
// {"taskName","taskCreatedBy","taskDueDate","taskAssignedTo"}; kBadToken: the page answers 400.
inline Verdict create_task(std::string_view body, std::string_view cookie, std::string_view key,
                           std::string_view af_cookie_name, std::string_view identity_cookie_name, std::string& json) {
  if (!taskcodec::valid_utf8(body) || !taskcodec::valid_utf8(cookie)) return Verdict::kDecline;
  // cookies: `;`-separated, stripped, name=value, value percent-decoded, the last one wins
  std::string af, who, tmp;
  bool have_af = false, have_who = false;
  for (size_t i = 0; i <= cookie.size();) {
    size_t j = cookie.find(';', i);
    if (j == std::string_view::npos) j = cookie.size();
    std::string_view part = cookie.substr(i, j - i);
    while (!part.empty() && (part.front() == ' ' || part.front() == '\t')) part.remove_prefix(1);
    while (!part.empty() && (part.back() == ' ' || part.back() == '\t')) part.remove_suffix(1);
    size_t eq = part.find('=');
    if (eq != std::string_view::npos) {
      std::string_view name = part.substr(0, eq);
      if (name == af_cookie_name || name == identity_cookie_name) {
        if (!unquote(part.substr(eq + 1), false, tmp)) return Verdict::kDecline;
        if (name == af_cookie_name) af = tmp, have_af = true;
        else who = tmp, have_who = true;
      }
    }
    i = j + 1;
  }
  // form: `&`-separated name=value pairs, unquote_plus, the first one wins
  static const char* names[4] = {"__RequestVerificationToken", "TaskAdd.TaskName", "TaskAdd.TaskDueDate",
                                 "TaskAdd.TaskAssignedTo"};
  std::string vals[4];
  bool seen[4] = {false, false, false, false};
  std::string name;
  for (size_t i = 0; i < body.size();) {
    size_t j = body.find('&', i);
    if (j == std::string_view::npos) j = body.size();
    std::string_view field = body.substr(i, j - i);
    i = j + 1;
    if (field.empty()) continue;
    size_t eq = field.find('=');
    if (eq == std::string_view::npos) return Verdict::kDecline;
    if (!unquote(field.substr(0, eq), true, name)) return Verdict::kDecline;
    for (int k = 0; k < 4; ++k)
      if (name == names[k] && !seen[k]) {
        if (!unquote(field.substr(eq + 1), true, vals[k])) return Verdict::kDecline;
        seen[k] = true;
      }
  }
  if (!seen[0] || vals[0].empty()) return Verdict::kDecline;  // a header token, or none: the page decides
  if (!have_af || af.empty()) return Verdict::kBadToken;
  const std::string want = hmac_sha256_hex(key, af);
  if (want.size() != vals[0].size() || CRYPTO_memcmp(want.data(), vals[0].data(), want.size()) != 0)
    return Verdict::kBadToken;
  for (int k = 1; k < 4; ++k)
    if (!seen[k] || !plain_value(vals[k])) return Verdict::kDecline;
  if (!have_who || who.empty()) return Verdict::kDecline;
  std::string due;
  if (!due_date(vals[2], due)) return Verdict::kDecline;
  json.clear();
  json += "{\"taskName\":";
  tt::escape_to(json, vals[1]);
  json += ",\"taskCreatedBy\":";
  tt::escape_to(json, who);
  json += ",\"taskDueDate\":\"";
  json += due;
  json += "\",\"taskAssignedTo\":";
  tt::escape_to(json, vals[3]);
  json += '}';
  return Verdict::kOk;
}

// -- the other posts of the UI: Edit (Pages/Tasks/Edit.cshtml.cs:57-71) and Index's Complete /
// Delete handlers (Pages/Tasks/Index.cshtml.cs:57-71), with the same envelope rules.

// The antiforgery and identity cookies (Request.cookies: `;`-separated, stripped, percent-
// decoded, the last one wins); false on an undecodable value.
inline bool read_cookies(std::string_view cookie, std::string_view af_name, std::string_view id_name, std::string& af,
                         bool& have_af, std::string& who, bool& have_who) {
  std::string tmp;
  have_af = have_who = false;
  for (size_t i = 0; i <= cookie.size();) {
    size_t j = cookie.find(';', i);
    if (j == std::string_view::npos) j = cookie.size();
    std::string_view part = cookie.substr(i, j - i);
    while (!part.empty() && (part.front() == ' ' || part.front() == '\t')) part.remove_prefix(1);
    while (!part.empty() && (part.back() == ' ' || part.back() == '\t')) part.remove_suffix(1);
    size_t eq = part.find('=');
    if (eq != std::string_view::npos) {
      std::string_view name = part.substr(0, eq);
      if (name == af_name || (!id_name.empty() && name == id_name)) {
        if (!unquote(part.substr(eq + 1), false, tmp)) return false;
        if (name == af_name) af = tmp, have_af = true;
        else who = tmp, have_who = true;
      }
    }
    i = j + 1;
  }
  return true;
}

// The form's fields `names[0..n)` (Request.form: `&`-separated, unquote_plus, the first wins);
// false on a malformed pair.
inline bool read_form(std::string_view body, const char* const* names, int n, std::string* vals, bool* seen) {
  std::string name;
  for (int k = 0; k < n; ++k) seen[k] = false;
  for (size_t i = 0; i < body.size();) {
    size_t j = body.find('&', i);
    if (j == std::string_view::npos) j = body.size();
    std::string_view field = body.substr(i, j - i);
    i = j + 1;
    if (field.empty()) continue;
    size_t eq = field.find('=');
    if (eq == std::string_view::npos) return false;
    if (!unquote(field.substr(0, eq), true, name)) return false;
    for (int k = 0; k < n; ++k)
      if (name == names[k] && !seen[k]) {
        if (!unquote(field.substr(eq + 1), true, vals[k])) return false;
        seen[k] = true;
      }
  }
  return true;
}

// Antiforgery.validate for a token in the form (a header token: the page decides).
inline Verdict check_token(bool seen_token, const std::string& token, bool have_af, const std::string& af,
                           std::string_view key) {
  if (!seen_token || token.empty()) return Verdict::kDecline;
  if (!have_af || af.empty()) return Verdict::kBadToken;
  const std::string want = hmac_sha256_hex(key, af);
  if (want.size() != token.size() || CRYPTO_memcmp(want.data(), token.data(), want.size()) != 0)
    return Verdict::kBadToken;
  return Verdict::kOk;
}

// POST Tasks/Edit/{id}: antiforgery, TaskUpdateModel's [Required] binding, the PUT body
// {"taskId","taskName","taskDueDate","taskAssignedTo"} and the id it goes to (the form's TaskId,
// else the route's `path_id`; a GUID in the 36-character form, else the page decides).
inline Verdict edit_task(std::string_view body, std::string_view cookie, std::string_view key,
                         std::string_view af_cookie_name, std::string_view path_id, std::string& json,
                         std::string& task_id) {
  if (!taskcodec::valid_utf8(body) || !taskcodec::valid_utf8(cookie)) return Verdict::kDecline;
  std::string af, who;
  bool have_af, have_who;
  if (!read_cookies(cookie, af_cookie_name, {}, af, have_af, who, have_who)) return Verdict::kDecline;
  static const char* names[5] = {"__RequestVerificationToken", "TaskUpdate.TaskId", "TaskUpdate.TaskName",
                                 "TaskUpdate.TaskDueDate", "TaskUpdate.TaskAssignedTo"};
  std::string vals[5];
  bool seen[5];
  if (!read_form(body, names, 5, vals, seen)) return Verdict::kDecline;
  Verdict v = check_token(seen[0], vals[0], have_af, af, key);
  if (v != Verdict::kOk) return v;
  for (int k = 2; k < 5; ++k)
    if (!seen[k] || !plain_value(vals[k])) return Verdict::kDecline;
  std::string due;
  if (!due_date(vals[3], due)) return Verdict::kDecline;
  task_id = seen[1] && !vals[1].empty() ? vals[1] : std::string(path_id);
  if (!taskcodec::is_guid36(task_id)) return Verdict::kDecline;
  json.clear();
  json += "{\"taskId\":";
  tt::escape_to(json, task_id);
  json += ",\"taskName\":";
  tt::escape_to(json, vals[2]);
  json += ",\"taskDueDate\":\"";
  json += due;
  json += "\",\"taskAssignedTo\":";
  tt::escape_to(json, vals[4]);
  json += '}';
  return Verdict::kOk;
}

// POST Tasks/Index?handler=complete|delete&id=: the antiforgery check of the form (the handler and
// the id come from the query string; in the form instead: the page decides).
inline Verdict index_post(std::string_view body, std::string_view cookie, std::string_view key,
                          std::string_view af_cookie_name) {
  if (!taskcodec::valid_utf8(body) || !taskcodec::valid_utf8(cookie)) return Verdict::kDecline;
  std::string af, who;
  bool have_af, have_who;
  if (!read_cookies(cookie, af_cookie_name, {}, af, have_af, who, have_who)) return Verdict::kDecline;
  static const char* names[3] = {"__RequestVerificationToken", "handler", "id"};
  std::string vals[3];
  bool seen[3];
  if (!read_form(body, names, 3, vals, seen)) return Verdict::kDecline;
  if (seen[1] || seen[2]) return Verdict::kDecline;
  return check_token(seen[0], vals[0], have_af, af, key);
}

}  // namespace formcodec
