// TaskModel wire codec for the Backend API's create path (POST /api/tasks).
//
// The reference binds the request body to TaskAddModel, creates a TaskModel with a new Guid and
// DateTime.UtcNow (Backend.Api Services/TasksStoreManager.cs:27-38), serialises it once for
// SaveStateAsync and PublishEventAsync.  The Python service does the same through pydantic
// (models/task.py); this is the same binding and serialisation in one pass over the body:
//
//   * the body is a JSON object; the four TaskAddModel properties are taken by their camelCase
//     names, unrelated properties are ignored (ASP.NET drops extras);
//   * taskDueDate accepts the ISO-8601 forms of models/dotnet.py:parse_datetime without a UTC
//     offset ("YYYY-MM-DD", "...THH:MM[:SS[.fffffff]]", optional "Z") and is written back the way
//     System.Text.Json writes it (trimmed fraction, "Z" only for UTC values);
//   * the id is a random (version 4) Guid, taskCreatedOn the current UTC time in microseconds.
//
// Anything outside that envelope -- a differently cased or snake_case property name, a duplicate,
// a non-string value, an offset, an out-of-range date, invalid UTF-8 -- is NOT decided here:
// create() returns false and the caller runs the general binder, which produces the exact
// validation error (400 ProblemDetails) or the remapped value.  Output is byte-identical to
// TaskModel.model_dump_json(by_alias=True) (tests/test_task_codec.py).
#pragma once

#include <sys/random.h>

#include <cstdint>
#include <cstring>
#include <ctime>
#include <algorithm>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

#include "json.hpp"

namespace taskcodec {

struct Created {
  std::string id;           // lowercase hyphenated Guid
  std::string name;         // decoded taskName (log lines)
  std::string assigned_to;  // decoded taskAssignedTo
  std::string task_json;    // TaskModel JSON (state value and event data)
  std::string state_body;   // [{"key":"<id>","value":<task_json>}]
};

inline bool valid_utf8(std::string_view s) {
  const unsigned char* p = reinterpret_cast<const unsigned char*>(s.data());
  const unsigned char* e = p + s.size();
  while (p < e) {
    unsigned char c = *p;
    if (c < 0x80) {
      ++p;
      while (e - p >= 8) {  // ASCII runs 8 bytes at a time
        uint64_t w;
        std::memcpy(&w, p, 8);
        if (w & 0x8080808080808080ull) break;
        p += 8;
      }
      continue;
    }
    int n;
    uint32_t cp;
    if ((c & 0xE0) == 0xC0) { n = 1; cp = c & 0x1F; if (c < 0xC2) return false; }
    else if ((c & 0xF0) == 0xE0) { n = 2; cp = c & 0x0F; }
    else if ((c & 0xF8) == 0xF0) { n = 3; cp = c & 0x07; if (c > 0xF4) return false; }
    else return false;
    if (e - p <= n) return false;
    for (int i = 1; i <= n; ++i) {
      if ((p[i] & 0xC0) != 0x80) return false;
      cp = (cp << 6) | (p[i] & 0x3F);
    }
    if ((n == 2 && (cp < 0x800 || (cp >= 0xD800 && cp < 0xE000))) || (n == 3 && (cp < 0x10000 || cp > 0x10FFFF)))
      return false;
    p += n + 1;
  }
  return true;
}

// Random bytes from the kernel CSPRNG (what uuid.uuid4 / Guid.NewGuid use), drawn in blocks.
class Entropy {
 public:
  bool take(uint8_t* out, size_t n) {
    if (pos_ + n > sizeof buf_) {
      size_t got = 0;
      while (got < sizeof buf_) {
        ssize_t r = getrandom(buf_ + got, sizeof buf_ - got, 0);
        if (r <= 0) return false;
        got += (size_t)r;
      }
      pos_ = 0;
    }
    std::memcpy(out, buf_ + pos_, n);
    pos_ += n;
    return true;
  }

 private:
  uint8_t buf_[4096];
  size_t pos_ = sizeof buf_;
};

inline bool new_guid(Entropy& rng, std::string& out) {
  uint8_t b[16];
  if (!rng.take(b, 16)) return false;
  b[6] = (uint8_t)((b[6] & 0x0F) | 0x40);  // version 4
  b[8] = (uint8_t)((b[8] & 0x3F) | 0x80);  // RFC 4122 variant
  static const char* hx = "0123456789abcdef";
  out.clear();
  for (int i = 0; i < 16; ++i) {
    if (i == 4 || i == 6 || i == 8 || i == 10) out += '-';
    out += hx[b[i] >> 4];
    out += hx[b[i] & 15];
  }
  return true;
}

inline void put2(std::string& o, int v) { o += (char)('0' + v / 10); o += (char)('0' + v % 10); }
inline void put4(std::string& o, int v) { put2(o, v / 100); put2(o, v % 100); }

// System.Text.Json DateTime: "yyyy-MM-ddTHH:mm:ss[.f{1,6} trimmed][Z]"; `fixed7`: the
// round-trip "O" form instead, always 7 fractional digits -- how the store holds TaskCreatedOn,
// so the string order the store sorts by is the DateTime order (models/dotnet.py
// format_roundtrip; the API's ORDER BY page and the reference's OrderBy then agree).
inline void format_dt(std::string& o, int y, int mo, int d, int h, int mi, int s, int us, bool utc,
                      bool fixed7 = false) {
  put4(o, y); o += '-'; put2(o, mo); o += '-'; put2(o, d); o += 'T';
  put2(o, h); o += ':'; put2(o, mi); o += ':'; put2(o, s);
  if (fixed7) {
    char f[8];
    for (int i = 5; i >= 0; --i) { f[i] = (char)('0' + us % 10); us /= 10; }
    f[6] = '0';  // microsecond precision: the tick digit
    o += '.';
    o.append(f, 7);
  } else if (us) {
    char f[7];
    for (int i = 5; i >= 0; --i) { f[i] = (char)('0' + us % 10); us /= 10; }
    int n = 6;
    while (n > 0 && f[n - 1] == '0') --n;
    o += '.';
    o.append(f, n);
  }
  if (utc) o += 'Z';
}

inline bool leap(int y) { return (y % 4 == 0 && y % 100 != 0) || y % 400 == 0; }

// parse_datetime's grammar minus offsets; false = let the general binder decide.  `fixed7`: the
// store's round-trip form (format_dt).
inline bool parse_due(std::string_view v, std::string& out, bool fixed7 = false) {
  auto dig = [&](size_t i, size_t n, int& r) {
    if (i + n > v.size()) return false;
    r = 0;
    for (size_t k = i; k < i + n; ++k) {
      if (v[k] < '0' || v[k] > '9') return false;
      r = r * 10 + (v[k] - '0');
    }
    return true;
  };
  int y, mo, d, h = 0, mi = 0, s = 0, us = 0;
  bool utc = false;
  if (!dig(0, 4, y) || v.size() < 10 || v[4] != '-' || !dig(5, 2, mo) || v[7] != '-' || !dig(8, 2, d)) return false;
  size_t i = 10;
  if (i < v.size() && (v[i] == 'T' || v[i] == ' ')) {
    if (!dig(i + 1, 2, h) || i + 3 >= v.size() || v[i + 3] != ':' || !dig(i + 4, 2, mi)) return false;
    i += 6;
    if (i < v.size() && v[i] == ':') {
      if (!dig(i + 1, 2, s)) return false;
      i += 3;
      if (i < v.size() && (v[i] == '.' || v[i] == ',')) {
        size_t j = i + 1, n = 0;
        while (j < v.size() && v[j] >= '0' && v[j] <= '9') { if (n < 6) us = us * 10 + (v[j] - '0'); ++j; ++n; }
        if (n == 0 || n > 9) return false;
        for (size_t k = n; k < 6; ++k) us *= 10;
        i = j;
      }
    }
  }
  if (i < v.size() && (v[i] == 'Z' || v[i] == 'z')) { utc = true; ++i; }
  if (i != v.size()) return false;  // offsets, whitespace, junk
  static const int mdays[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  if (y < 1 || mo < 1 || mo > 12 || d < 1 || d > mdays[mo - 1] + (mo == 2 && leap(y)) || h > 23 || mi > 59 || s > 59)
    return false;
  format_dt(out, y, mo, d, h, mi, s, us, utc, fixed7);
  return true;
}

// json.loads (strict) rejects raw control characters inside strings (tt::parse_strict does too).
inline bool no_raw_controls_in_strings(std::string_view s) {
  bool in = false;
  for (size_t i = 0; i < s.size(); ++i) {
    unsigned char c = (unsigned char)s[i];
    if (!in) { if (c == '"') in = true; continue; }
    if (c == '\\') { ++i; continue; }
    if (c == '"') in = false;
    else if (c < 0x20) return false;
  }
  return true;
}

inline bool create(std::string_view body, Entropy& rng, Created& out) {
  if (!valid_utf8(body)) return false;
  tt::Value doc;
  try {
    doc = tt::parse_strict(body);
  } catch (const tt::ParseError&) {
    return false;
  }
  if (doc.t != tt::Value::Object) return false;
  static const char* names[4] = {"taskName", "taskCreatedBy", "taskDueDate", "taskAssignedTo"};
  static const char* other[8] = {"task_name", "task_created_by", "task_due_date", "task_assigned_to",
                                 "taskname", "taskcreatedby", "taskduedate", "taskassignedto"};
  const tt::Value* f[4] = {nullptr, nullptr, nullptr, nullptr};
  for (size_t k = 0; k < doc.keys.size(); ++k) {
    const std::string& key = doc.keys[k];
    int hit = -1;
    for (int j = 0; j < 4; ++j)
      if (key == names[j]) hit = j;
    if (hit >= 0) {
      if (f[hit] != nullptr) return false;  // duplicate: json.loads keeps the last one
      f[hit] = &doc.items[k];
      continue;
    }
    // an unrelated property: only scalars whose grammar both parsers share (numbers and nested
    // values go to the general binder, whose JSON parser is the authority on them)
    const tt::Value& x = doc.items[k];
    if (x.t != tt::Value::String && x.t != tt::Value::Bool && x.t != tt::Value::Null) return false;
    std::string low(key);
    for (char& c : low) c = (char)std::tolower((unsigned char)c);
    for (const char* o : other)
      if (key == o || low == o) return false;  // remapped by the general binder
  }
  for (int j = 0; j < 4; ++j)  // strings only, and no lone surrogates from \\u escapes
    if (f[j] != nullptr && (f[j]->t != tt::Value::String || !valid_utf8(f[j]->s))) return false;
  std::string due;
  if (f[2] == nullptr) due = "0001-01-01T00:00:00";
  else if (!parse_due(f[2]->s, due)) return false;

  if (!new_guid(rng, out.id)) return false;
  struct timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  time_t secs = ts.tv_sec;
  struct tm tmv;
  gmtime_r(&secs, &tmv);
  std::string& j = out.task_json;
  j.clear();
  j.reserve(256 + body.size());
  j += "{\"taskId\":\"";
  j += out.id;
  j += "\",\"taskName\":";
  tt::escape_to(j, f[0] ? std::string_view(f[0]->s) : std::string_view());
  j += ",\"taskCreatedBy\":";
  tt::escape_to(j, f[1] ? std::string_view(f[1]->s) : std::string_view());
  j += ",\"taskCreatedOn\":\"";
  format_dt(j, tmv.tm_year + 1900, tmv.tm_mon + 1, tmv.tm_mday, tmv.tm_hour, tmv.tm_min, tmv.tm_sec,
            (int)(ts.tv_nsec / 1000), true, true);
  j += "\",\"taskDueDate\":\"";
  j += due;
  j += "\",\"taskAssignedTo\":";
  tt::escape_to(j, f[3] ? std::string_view(f[3]->s) : std::string_view());
  j += ",\"isCompleted\":false,\"isOverDue\":false}";
  out.name = f[0] ? f[0]->s : std::string();
  out.assigned_to = f[3] ? f[3]->s : std::string();
  out.state_body.clear();
  out.state_body.reserve(j.size() + 64);
  out.state_body += "[{\"key\":\"";
  out.state_body += out.id;
  out.state_body += "\",\"value\":";
  out.state_body += j;
  out.state_body += "}]";
  return true;
}

// -------------------------------------------------------------------------------------------
// The processor's side: a CloudEvents envelope from the sidecar and the TaskModel inside it.

// CloudEvents 1.0 structured mode (what app.UseCloudEvents() unwraps, Processor/Program.cs:29):
// the envelope's attributes and its JSON `data` re-serialised compactly.  false = the general
// (Python) unwrapper decides: not an object, data_base64, a string payload, or numbers anywhere in
// the data (their text form is the Python parser's business).
struct Unwrapped {
  std::string data;
  std::string content_type = "application/json";
  std::vector<std::pair<std::string, const tt::Value*>> attrs;
  tt::Value doc;
};

inline bool has_number(const tt::Value& v) {
  if (v.t == tt::Value::Number) return true;
  for (const auto& x : v.items)
    if (has_number(x)) return true;
  return false;
}

inline bool unwrap_cloudevent(std::string_view body, Unwrapped& out) {
  if (!valid_utf8(body)) return false;
  try {
    out.doc = tt::parse_strict(body);
  } catch (const tt::ParseError&) {
    return false;
  }
  const tt::Value& ce = out.doc;
  if (ce.t != tt::Value::Object) return false;
  const tt::Value* data = nullptr;
  out.attrs.clear();
  for (size_t i = 0; i < ce.keys.size(); ++i) {
    const std::string& k = ce.keys[i];
    for (size_t j = 0; j < i; ++j)
      if (ce.keys[j] == k) return false;  // duplicate attribute
    if (k == "data_base64") return false;
    if (k == "data") { data = &ce.items[i]; continue; }
    if (k == "datacontenttype") {
      if (ce.items[i].t != tt::Value::String) return false;
      out.content_type = ce.items[i].s;
    }
    out.attrs.emplace_back(k, &ce.items[i]);
  }
  if (data == nullptr || data->t == tt::Value::String || has_number(*data)) return false;
  for (const auto& kv : out.attrs)
    if (has_number(*kv.second) || (kv.second->t == tt::Value::String && !valid_utf8(kv.second->s))) return false;
  out.data.clear();
  tt::dump_to(out.data, *data);
  return valid_utf8(out.data);
}

inline bool is_guid36(const std::string& s) {
  if (s.size() != 36) return false;
  for (size_t i = 0; i < 36; ++i) {
    char c = s[i];
    if (i == 8 || i == 13 || i == 18 || i == 23) { if (c != '-') return false; continue; }
    if (!((c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'))) return false;
  }
  return true;
}

// TaskModel binding check (TaskModel.model_validate of the event data, Processor
// TasksNotifierController.cs:26): the taskName when the object binds within the envelope of
// create(); false = the general binder decides (and produces any 400).
inline bool task_model_name(std::string_view body, std::string& name) {
  if (!valid_utf8(body)) return false;
  tt::Value doc;
  try {
    doc = tt::parse_strict(body);
  } catch (const tt::ParseError&) {
    return false;
  }
  if (doc.t != tt::Value::Object) return false;
  static const char* names[8] = {"taskId", "taskName", "taskCreatedBy", "taskCreatedOn",
                                 "taskDueDate", "taskAssignedTo", "isCompleted", "isOverDue"};
  static const char* snake[8] = {"task_id", "task_name", "task_created_by", "task_created_on",
                                 "task_due_date", "task_assigned_to", "is_completed", "is_over_due"};
  const tt::Value* f[8] = {nullptr};
  for (size_t k = 0; k < doc.keys.size(); ++k) {
    const std::string& key = doc.keys[k];
    int hit = -1;
    for (int j = 0; j < 8; ++j)
      if (key == names[j]) hit = j;
    if (hit >= 0) {
      if (f[hit] != nullptr) return false;
      f[hit] = &doc.items[k];
      continue;
    }
    const tt::Value& x = doc.items[k];
    if (x.t != tt::Value::String && x.t != tt::Value::Bool && x.t != tt::Value::Null) return false;
    std::string low(key);
    for (char& c : low) c = (char)std::tolower((unsigned char)c);
    for (int j = 0; j < 8; ++j) {
      std::string ln(names[j]);
      for (char& c : ln) c = (char)std::tolower((unsigned char)c);
      if (key == snake[j] || low == ln) return false;
    }
  }
  std::string scratch;
  for (int j = 0; j < 8; ++j) {
    const tt::Value* v = f[j];
    if (v == nullptr) continue;
    if (j == 6 || j == 7) { if (v->t != tt::Value::Bool) return false; continue; }
    if (v->t != tt::Value::String || !valid_utf8(v->s)) return false;
    if (j == 0 && !is_guid36(v->s)) return false;
    if ((j == 3 || j == 4) && !parse_due(v->s, scratch)) return false;
  }
  name = f[1] ? f[1]->s : std::string();
  return true;
}

// -------------------------------------------------------------------------------------------
// Lists of TaskModels: the overdue sweep (Processor ScheduledTasksManagerController.cs:19-46 ->
// API OverdueTasksController.cs:26-32 -> TasksStoreManager.MarkOverdueTasks).  A TaskModel object
// that binds within the envelope of task_model_name() is written back canonically -- model
// property order, Guid lower-case, DateTimes as System.Text.Json writes them, defaults for
// missing properties -- the JSON of TaskModel.to_wire().

// Index of `key` among TaskModel's wire names, or -1: a length test first, then one memcmp (the
// sweep binds ~1000 tasks per page through here; a strcmp against every name was ~40 % of it).
inline int task_field_index(const std::string& key) {
  static const std::string_view names[8] = {"taskId", "taskName", "taskCreatedBy", "taskCreatedOn",
                                            "taskDueDate", "taskAssignedTo", "isCompleted", "isOverDue"};
  for (int j = 0; j < 8; ++j)
    if (key.size() == names[j].size() && std::memcmp(key.data(), names[j].data(), key.size()) == 0) return j;
  return -1;
}

inline bool task_fields(const tt::Value& doc, const tt::Value* (&f)[8]) {
  if (doc.t != tt::Value::Object) return false;
  static const char* names[8] = {"taskId", "taskName", "taskCreatedBy", "taskCreatedOn",
                                 "taskDueDate", "taskAssignedTo", "isCompleted", "isOverDue"};
  static const char* snake[8] = {"task_id", "task_name", "task_created_by", "task_created_on",
                                 "task_due_date", "task_assigned_to", "is_completed", "is_over_due"};
  for (auto& x : f) x = nullptr;
  for (size_t k = 0; k < doc.keys.size(); ++k) {
    const std::string& key = doc.keys[k];
    const int hit = task_field_index(key);
    if (hit >= 0) {
      if (f[hit] != nullptr) return false;
      f[hit] = &doc.items[k];
      continue;
    }
    const tt::Value& x = doc.items[k];
    if (x.t != tt::Value::String && x.t != tt::Value::Bool && x.t != tt::Value::Null) return false;
    std::string low(key);
    for (char& c : low) c = (char)std::tolower((unsigned char)c);
    for (int j = 0; j < 8; ++j) {
      std::string ln(names[j]);
      for (char& c : ln) c = (char)std::tolower((unsigned char)c);
      if (key == snake[j] || low == ln) return false;
    }
  }
  return true;
}

// PUT api/tasks/{id}'s body bound as TaskUpdateModel (TasksController.cs:48-59; its taskId is
// not used -- the route's id is): the new name, assignee and due date (canonical text).
struct Update {
  std::string name, assigned_to, due = "0001-01-01T00:00:00";
};

// Canonical TaskModel JSON of `doc` (isOverDue forced true when `overdue`); `due_day` receives
// the due date's "YYYY-MM-DD".  `store_form`: TaskCreatedOn in the store's round-trip form
// (format_dt fixed7) -- for a document written back to the store.  `upd`: the task as
// UpdateTask leaves it (name, assignee, due date replaced: TasksStoreManager.cs:85-99);
// `complete`: as MarkTaskCompleted leaves it (:71-81).  false = outside the envelope.
inline bool write_task(const tt::Value& doc, bool overdue, std::string& out, std::string& id, std::string& due_day,
                       bool store_form = false, const Update* upd = nullptr, bool complete = false) {
  const tt::Value* f[8];
  if (!task_fields(doc, f)) return false;
  for (int j = 0; j < 6; ++j)
    if (f[j] != nullptr && (f[j]->t != tt::Value::String || !valid_utf8(f[j]->s))) return false;
  for (int j = 6; j < 8; ++j)
    if (f[j] != nullptr && f[j]->t != tt::Value::Bool) return false;
  if (f[0]) id.assign(f[0]->s);
  else id.assign("00000000-0000-0000-0000-000000000000");
  if (!is_guid36(id)) return false;
  for (char& c : id) c = (char)std::tolower((unsigned char)c);
  // per-thread scratch: a 19+ character date does not fit the small-string buffer, and this
  // runs once per task of a sweep page
  static thread_local std::string created, due;
  created.assign(store_form ? "0001-01-01T00:00:00.0000000" : "0001-01-01T00:00:00");  // format_roundtrip(MinValue)
  due.assign("0001-01-01T00:00:00");
  if (f[3] && (created.clear(), !parse_due(f[3]->s, created, store_form))) return false;
  if (f[4] && (due.clear(), !parse_due(f[4]->s, due))) return false;  // the stored task must bind
  if (upd) {
    due.clear();
    if (!parse_due(upd->due, due)) return false;
  }
  due_day.assign(due, 0, 10);
  static const std::string empty;
  out += "{\"taskId\":\"";
  out += id;
  out += "\",\"taskName\":";
  tt::escape_to(out, upd ? std::string_view(upd->name) : f[1] ? std::string_view(f[1]->s) : std::string_view(empty));
  out += ",\"taskCreatedBy\":";
  tt::escape_to(out, f[2] ? std::string_view(f[2]->s) : std::string_view(empty));
  out += ",\"taskCreatedOn\":\"";
  out += created;
  out += "\",\"taskDueDate\":\"";
  out += due;
  out += "\",\"taskAssignedTo\":";
  tt::escape_to(out, upd ? std::string_view(upd->assigned_to) : f[5] ? std::string_view(f[5]->s) : std::string_view(empty));
  out += ",\"isCompleted\":";
  out += (complete || (f[6] && f[6]->b)) ? "true" : "false";
  out += ",\"isOverDue\":";
  out += (overdue || (f[7] && f[7]->b)) ? "true" : "false";
  out += '}';
  return true;
}

// TaskUpdateModel's binder for the bodies it shares with the general one (create's envelope
// rules: the camelCase names once each, other properties only as strings / booleans / null, no
// name the general binder would remap); false = let it decide.
inline bool bind_update(std::string_view body, Update& u) {
  if (!valid_utf8(body)) return false;
  tt::Value doc;
  try {
    doc = tt::parse_strict(body);
  } catch (const tt::ParseError&) {
    return false;
  }
  if (doc.t != tt::Value::Object) return false;
  static const char* names[4] = {"taskId", "taskName", "taskDueDate", "taskAssignedTo"};
  static const char* other[8] = {"task_id", "task_name", "task_due_date", "task_assigned_to",
                                 "taskid", "taskname", "taskduedate", "taskassignedto"};
  const tt::Value* f[4] = {nullptr, nullptr, nullptr, nullptr};
  for (size_t k = 0; k < doc.keys.size(); ++k) {
    const std::string& key = doc.keys[k];
    int hit = -1;
    for (int j = 0; j < 4; ++j)
      if (key == names[j]) hit = j;
    if (hit >= 0) {
      if (f[hit] != nullptr) return false;
      f[hit] = &doc.items[k];
      continue;
    }
    const tt::Value& x = doc.items[k];
    if (x.t != tt::Value::String && x.t != tt::Value::Bool && x.t != tt::Value::Null) return false;
    std::string low(key);
    for (char& c : low) c = (char)std::tolower((unsigned char)c);
    for (const char* o : other)
      if (key == o || low == o) return false;
  }
  for (int j = 0; j < 4; ++j)
    if (f[j] != nullptr && (f[j]->t != tt::Value::String || !valid_utf8(f[j]->s))) return false;
  if (f[0] != nullptr && !is_guid36(f[0]->s)) return false;  // the Guid binder's text forms are its own
  u.name = f[1] ? f[1]->s : std::string();
  u.assigned_to = f[3] ? f[3]->s : std::string();
  u.due.clear();
  if (f[2] == nullptr) u.due = "0001-01-01T00:00:00";
  else if (!parse_due(f[2]->s, u.due)) return false;
  return true;
}

// A stored task through one of the API's read-modify-writes (TasksStoreManager.cs:71-99):
// the document written back (store form) with `upd` / `complete` applied, its id and the stored
// assignee (for the assignee-change publish).  false = outside the envelope (Python decides).
inline bool edit_task(std::string_view stored, const Update* upd, bool complete, std::string& out, std::string& id,
                      std::string& old_assignee) {
  if (!valid_utf8(stored)) return false;
  tt::Value doc;
  try {
    doc = tt::parse_strict(stored);
  } catch (const tt::ParseError&) {
    return false;
  }
  const tt::Value* f[8];
  if (!task_fields(doc, f)) return false;
  old_assignee = f[5] && f[5]->t == tt::Value::String ? f[5]->s : std::string();
  std::string day;
  out.clear();
  return write_task(doc, false, out, id, day, true, upd, complete);
}

// GET api/tasks/{id}'s answer from the stored document: the TaskModel JSON (to_json).
inline bool task_json(std::string_view stored, std::string& out) {
  if (!valid_utf8(stored)) return false;
  tt::Value doc;
  try {
    doc = tt::parse_strict(stored);
  } catch (const tt::ParseError&) {
    return false;
  }
  std::string id, day;
  out.clear();
  return write_task(doc, false, out, id, day);
}

// ASCII-only case-insensitive equality (str.lower() agrees on ASCII); -1 when either side has
// other characters (Python compares them).
inline int ascii_ieq(std::string_view a, std::string_view b) {
  for (unsigned char c : a)
    if (c >= 0x80) return -1;
  for (unsigned char c : b)
    if (c >= 0x80) return -1;
  if (a.size() != b.size()) return 0;
  for (size_t i = 0; i < a.size(); ++i)
    if (std::tolower((unsigned char)a[i]) != std::tolower((unsigned char)b[i])) return 0;
  return 1;
}

inline bool parse_array(std::string_view body, tt::Value& doc) {
  if (!valid_utf8(body)) return false;
  try {
    doc = tt::parse_strict(body);
  } catch (const tt::ParseError&) {
    return false;
  }
  return doc.t == tt::Value::Array;
}

// The same order as a number: "yyyy-MM-ddTHH:mm:ss[.f{1,7}]" (canonical, as write_task writes it)
// -> (seconds of the calendar fields, mixed radix) * 10^6 + microseconds.  Monotone in the
// DateTime; the fraction's 7th digit (100 ns) is below the TaskModel's microsecond precision.
inline uint64_t created_key(std::string_view c) {
  auto d = [&](size_t i, size_t n) {
    uint64_t r = 0;
    for (size_t k = i; k < i + n && k < c.size(); ++k) r = r * 10 + (uint64_t)(c[k] - '0');
    return r;
  };
  uint64_t secs = ((((d(0, 4) * 13 + d(5, 2)) * 32 + d(8, 2)) * 24 + d(11, 2)) * 60 + d(14, 2)) * 60 + d(17, 2);
  uint64_t us = 0;
  size_t i = 19, n = 0;
  if (i < c.size() && c[i] == '.')
    for (++i; i < c.size() && c[i] >= '0' && c[i] <= '9' && n < 6; ++i, ++n) us = us * 10 + (uint64_t)(c[i] - '0');
  for (; n < 6; ++n) us *= 10;
  return secs * 1000000 + us;
}

// The closing quote of a JSON string literal whose opening quote is at p[-1], when the literal
// has no escapes and no raw control characters (16 bytes a step); nullptr otherwise.
inline const char* plain_string_end(const char* p, const char* e) {
  const __m128i q = _mm_set1_epi8('"'), bs = _mm_set1_epi8('\\'), ctl = _mm_set1_epi8(0x1f);
  while (e - p >= 16) {
    const __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p));
    const __m128i hit = _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(x, q), _mm_cmpeq_epi8(x, bs)),
                                     _mm_cmpeq_epi8(_mm_max_epu8(x, ctl), ctl));  // byte <= 0x1f
    const int m = _mm_movemask_epi8(hit);
    if (m) {
      p += __builtin_ctz((unsigned)m);
      return *p == '"' ? p : nullptr;
    }
    p += 16;
  }
  for (; p < e; ++p) {
    if (*p == '"') return p;
    if (*p == '\\' || (unsigned char)*p < 0x20) return nullptr;
  }
  return nullptr;
}

// A task in the layout the API stores it (write_task, store form: the fields in order, compact,
// strings without escapes) at t[i..], -> write_task's output for it appended to `out`, `i` past
// it, `key` its created_key; no value tree.  False = another layout (the caller binds it through
// the tree; the output would be the same).
// `overdue`: written with isOverDue set (markoverdue's save); `store_form`: the created date in
// the store's round-trip form (write_task's); `flags` (optional): the task's own isCompleted and
// isOverDue as read; `id_out` (optional): the id as written (lower case).
inline bool fast_task_at(std::string_view t, size_t& i, std::string& out, uint64_t& key,
                         std::string* due_day = nullptr, bool overdue = false, bool store_form = false,
                         std::pair<bool, bool>* flags = nullptr, std::string* id_out = nullptr) {
  const char* const e = t.data() + t.size();
  auto lit = [&](std::string_view w) {
    if (t.compare(i, w.size(), w) != 0) return false;
    i += w.size();
    return true;
  };
  auto str = [&](std::string_view& v) {
    if (i >= t.size() || t[i] != '"') return false;
    const char* q = plain_string_end(t.data() + i + 1, e);
    if (!q) return false;
    const size_t j = (size_t)(q - t.data());
    v = t.substr(i, j + 1 - i);
    i = j + 1;
    return true;
  };
  auto boolean = [&](bool& b) { return lit("true") ? (b = true) : lit("false") ? !(b = false) : false; };
  std::string_view id, name, by, created, due, to;
  bool done = false, over = false;
  if (!lit("{\"taskId\":") || !str(id) || !lit(",\"taskName\":") || !str(name) || !lit(",\"taskCreatedBy\":") ||
      !str(by) || !lit(",\"taskCreatedOn\":") || !str(created) || !lit(",\"taskDueDate\":") || !str(due) ||
      !lit(",\"taskAssignedTo\":") || !str(to) || !lit(",\"isCompleted\":") || !boolean(done) ||
      !lit(",\"isOverDue\":") || !boolean(over) || !lit("}"))
    return false;
  id = id.substr(1, id.size() - 2);
  if (id.size() != 36) return false;
  for (size_t k = 0; k < 36; ++k) {
    const char c = id[k];
    if (k == 8 || k == 13 || k == 18 || k == 23) {
      if (c != '-') return false;
    } else if (!((c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'))) {
      return false;
    }
  }
  // a 28-byte date does not fit the small-string buffer: per-thread scratch, no allocation a task
  static thread_local std::string c, d;
  c.clear();
  d.clear();
  if (!parse_due(created.substr(1, created.size() - 2), c, store_form) || !parse_due(due.substr(1, due.size() - 2), d))
    return false;
  out += "{\"taskId\":\"";
  const size_t at = out.size();
  out.append(id);
  for (size_t k = at; k < out.size(); ++k) out[k] = (char)std::tolower((unsigned char)out[k]);
  if (id_out) id_out->assign(out, at, 36);
  if (flags) *flags = {done, over};
  out += "\",\"taskName\":";
  out.append(name);
  out += ",\"taskCreatedBy\":";
  out.append(by);
  out += ",\"taskCreatedOn\":\"";
  out += c;
  out += "\",\"taskDueDate\":\"";
  out += d;
  out += "\",\"taskAssignedTo\":";
  out.append(to);
  out += done ? ",\"isCompleted\":true" : ",\"isCompleted\":false";
  out += (over || overdue) ? ",\"isOverDue\":true}" : ",\"isOverDue\":false}";
  key = created_key(c);
  if (due_day) due_day->assign(d, 0, 10);
  return true;
}

struct TaskRow {
  uint64_t key;
  size_t at, len;
};

// The state-query response as the backing's page assembly writes it (DocStore::mirror_results,
// `{"results":[{"key":..,"data":..,"etag":".."},..],"token":".."}`, compact) with every task in
// the stored layout: the rows written into `buf` in one pass over the text, which the layout
// itself validates.  False = any other text (the value tree reads it).
inline bool fast_query_tasks(std::string_view b, std::string& buf, std::vector<TaskRow>& rows, bool& token) {
  size_t i = 0;
  const char* const e = b.data() + b.size();
  auto lit = [&](std::string_view w) {
    if (b.compare(i, w.size(), w) != 0) return false;
    i += w.size();
    return true;
  };
  auto str = [&](size_t& len) {
    if (i >= b.size() || b[i] != '"') return false;
    const char* q = plain_string_end(b.data() + i + 1, e);
    if (!q) return false;
    const size_t j = (size_t)(q - b.data());
    len = j - i - 1;
    i = j + 1;
    return true;
  };
  if (!lit("{\"results\":[")) return false;
  if (!lit("]")) {
    while (true) {
      size_t klen = 0, elen = 0;
      if (!lit("{\"key\":") || !str(klen) || !lit(",\"data\":")) return false;
      const size_t at = buf.size();
      uint64_t key = 0;
      if (!fast_task_at(b, i, buf, key)) return false;
      rows.push_back({key, at, buf.size() - at});
      if (!lit(",\"etag\":") || !str(elen) || !lit("}")) return false;
      if (lit(",")) continue;
      if (lit("]")) break;
      return false;
    }
  }
  token = false;
  if (lit(",\"token\":")) {
    size_t tlen = 0;
    if (!str(tlen)) return false;
    token = tlen > 0;
  }
  return lit("}") && i == b.size();
}

// POST api/overduetasks/markoverdue: the ids (for the per-task log lines) and the state API's
// bulk-save body [{"key": id, "value": TaskModel with isOverDue = true}, ...].
inline bool mark_overdue(std::string_view body, std::vector<std::string>& ids, std::string& bulk) {
  tt::Value doc;
  if (!parse_array(body, doc)) return false;
  ids.clear();
  bulk.assign("[");
  std::string id, day;
  for (size_t i = 0; i < doc.items.size(); ++i) {
    if (i) bulk += ',';
    bulk += "{\"key\":\"";
    const size_t key_at = bulk.size();
    bulk += "\",\"value\":";
    if (!write_task(doc.items[i], true, bulk, id, day)) return false;
    bulk += '}';
    bulk.insert(key_at, id);
    ids.push_back(id);
  }
  bulk += ']';
  return true;
}

// The conditional half of markoverdue: the state API's bulk-get answer for the page's ids
// ([{"key", "data", "etag"} | {"key"}]) -> a bulk save that sets isOverDue on the STORED task
// (not the caller's copy) only where it is still open and not yet overdue, each item guarded by
// the ETag it was read with (first-write): a completion that lands between the sweep's query
// and this save makes the save fail for that item (409) instead of reverting it.  `ids`: the
// tasks written; `skipped`: completed / already overdue / deleted ones.
// conditional_mark over the sidecar's bulk-get answer as the data plane lays it out
// (`[{"key":..,"data":<stored task>,"etag":".."}|{"key":..}]`, compact) with every task in the
// stored layout, in one pass; false = any other text.
inline bool fast_conditional_mark(std::string_view b, std::string& bulk, std::vector<std::string>& ids,
                                  size_t& skipped) {
  if (!valid_utf8(b)) return false;
  const char* const e = b.data() + b.size();
  size_t i = 0;
  auto lit = [&](std::string_view w) {
    if (b.compare(i, w.size(), w) != 0) return false;
    i += w.size();
    return true;
  };
  auto str = [&](std::string_view& v) {
    if (i >= b.size() || b[i] != '"') return false;
    const char* q = plain_string_end(b.data() + i + 1, e);
    if (!q) return false;
    const size_t j = (size_t)(q - b.data());
    v = b.substr(i, j + 1 - i);
    i = j + 1;
    return true;
  };
  ids.clear();
  skipped = 0;
  bulk.assign("[");
  bulk.reserve(b.size() + 64 * 128);
  if (!lit("[")) return false;
  if (lit("]")) {
    bulk += ']';
    return i == b.size();
  }
  std::string id;
  while (true) {
    std::string_view key, etag;
    if (!lit("{\"key\":") || !str(key)) return false;
    if (lit("}")) {
      ++skipped;  // deleted since the sweep's query
    } else {
      if (!lit(",\"data\":")) return false;
      const size_t mark = bulk.size();
      if (ids.size()) bulk += ',';
      bulk += "{\"key\":";
      bulk.append(key);
      bulk += ",\"value\":";
      uint64_t k = 0;
      std::pair<bool, bool> flags;
      if (!fast_task_at(b, i, bulk, k, nullptr, true, true, &flags, &id)) return false;
      if (!lit(",\"etag\":") || !str(etag) || !lit("}")) return false;
      if (flags.first || flags.second) {  // completed or already overdue: not written
        bulk.resize(mark);
        ++skipped;
      } else {
        if (etag.size() > 2) {
          bulk += ",\"etag\":";
          bulk.append(etag);
        }
        bulk += ",\"options\":{\"concurrency\":\"first-write\"}}";
        ids.push_back(id);
      }
    }
    if (lit(",")) continue;
    if (lit("]")) break;
    return false;
  }
  bulk += ']';
  return i == b.size();
}

inline bool conditional_mark(std::string_view got, std::string& bulk, std::vector<std::string>& ids,
                             size_t& skipped) {
  // the data plane's own answer around the stored tasks: one pass; anything else below
  if (fast_conditional_mark(got, bulk, ids, skipped)) return true;
  tt::Value doc;
  if (!parse_array(got, doc)) return false;
  ids.clear();
  skipped = 0;
  bulk.assign("[");
  std::string id, day;
  for (const auto& it : doc.items) {
    if (it.t != tt::Value::Object) return false;
    const tt::Value* key = it.get("key");
    const tt::Value* data = it.get("data");
    const tt::Value* etag = it.get("etag");
    if (key == nullptr || key->t != tt::Value::String) return false;
    if (data == nullptr || data->t == tt::Value::Null) {  // deleted since the sweep's query
      ++skipped;
      continue;
    }
    const tt::Value* f[8];
    if (!task_fields(*data, f)) return false;
    if ((f[6] && f[6]->t == tt::Value::Bool && f[6]->b) || (f[7] && f[7]->t == tt::Value::Bool && f[7]->b)) {
      ++skipped;
      continue;
    }
    if (ids.size()) bulk += ',';
    bulk += "{\"key\":";
    tt::escape_to(bulk, key->s);
    bulk += ",\"value\":";
    if (!write_task(*data, true, bulk, id, day, true)) return false;
    if (etag != nullptr && etag->t == tt::Value::String && !etag->s.empty()) {
      bulk += ",\"etag\":";
      tt::escape_to(bulk, etag->s);
    }
    bulk += ",\"options\":{\"concurrency\":\"first-write\"}}";
    ids.push_back(id);
  }
  bulk += ']';
  return true;
}

// The cron job's filter (ScheduledTasksManagerController.cs:31-36): of the API's overdue page,
// the tasks whose due date is before the run's date (UTC), as a TaskModel JSON array; also the
// page's size.  `starts` (optional): the offset in `out` of each kept task's object, so the
// caller can cut the array into chunks without scanning it again.
// overdue_filter over a page in the layout the API answers it (query_tasks's output: compact,
// the fields in order, strings without escapes), in one pass; false = any other text.
inline bool fast_overdue_filter(std::string_view b, std::string_view run_day, size_t& retrieved, size_t& kept,
                                std::string& out, std::vector<size_t>* starts) {
  if (run_day.size() != 10 || !valid_utf8(b) || b.empty() || b[0] != '[') return false;
  size_t i = 1;
  retrieved = kept = 0;
  out.assign("[");
  out.reserve(b.size() + 2);
  std::string day;
  if (b.size() == 2 && b[1] == ']') {
    out += ']';
    return true;
  }
  while (true) {
    const size_t mark = out.size();
    if (kept) out += ',';
    uint64_t key = 0;
    if (!fast_task_at(b, i, out, key, &day)) return false;
    ++retrieved;
    if (std::string_view(day) < run_day) {
      if (starts) starts->push_back(mark + (kept ? 1 : 0));
      ++kept;
    } else {
      out.resize(mark);
    }
    if (i < b.size() && b[i] == ',') {
      ++i;
      continue;
    }
    if (i + 1 == b.size() && b[i] == ']') break;
    return false;
  }
  out += ']';
  return true;
}

inline bool overdue_filter(std::string_view body, std::string_view run_day, size_t& retrieved, size_t& kept,
                           std::string& out, std::vector<size_t>* starts = nullptr) {
  // the API's own page: one pass, no value tree (1,000 tasks a sweep); anything else below
  const size_t nstarts = starts ? starts->size() : 0;
  if (fast_overdue_filter(body, run_day, retrieved, kept, out, starts)) return true;
  if (starts) starts->resize(nstarts);
  tt::Value doc;
  if (!parse_array(body, doc) || run_day.size() != 10) return false;
  retrieved = doc.items.size();
  kept = 0;
  out.assign("[");
  out.reserve(body.size() + 2);
  std::string id, day;
  for (const auto& item : doc.items) {
    // written in place, and cut back off when the task is not due before the run's date
    const size_t mark = out.size();
    if (kept) out += ',';
    if (!write_task(item, false, out, id, day)) return false;
    if (std::string_view(day) < run_day) {
      if (starts) starts->push_back(mark + (kept ? 1 : 0));  // where this task's object begins
      ++kept;
    } else {
      out.resize(mark);
    }
  }
  out += ']';
  return true;
}


// State-query response of the task collection (Dapr `{"results": [{"key", "data", "etag"}],
// "token", "metadata"}`) -> the TaskModel JSON array of the results that carry data: the API's
// GET api/overduetasks page (TasksStoreManager.GetYesterdaysDueTasks, range sweep).  With
// `by_created` the tasks come out ordered by TaskCreatedOn as a DateTime, ascending (or with
// `descending`, newest first: the GET api/tasks list) and stable
// (the reference's `.OrderBy(o => o.TaskCreatedOn)`, TasksStoreManager.cs:136): System.Text.Json
// trims the fraction, so the strings do not sort chronologically within one second ("...:42Z"
// is earlier than "...:42.1Z").  `more`: the response carries a continuation token.
inline bool query_tasks_tree(std::string_view body, std::string& out, size_t& count, bool by_created, bool* more,
                             bool descending);

inline bool query_tasks(std::string_view body, std::string& out, size_t& count, bool by_created = false,
                        bool* more = nullptr, bool descending = false) {
  if (!valid_utf8(body)) return false;
  // the page as the backing assembles it from the API's own writes: one pass over the text,
  // every task copied with its dates re-formatted -- no value tree for a 1,000-task sweep page;
  // any other text goes through the tree
  std::vector<TaskRow> rows;
  std::string buf;
  buf.reserve(body.size());
  bool token = false;
  if (!fast_query_tasks(body, buf, rows, token)) return query_tasks_tree(body, out, count, by_created, more, descending);
  if (more) *more = token;
  if (by_created) {
    if (descending)
      std::stable_sort(rows.begin(), rows.end(), [](const TaskRow& a, const TaskRow& b) { return a.key > b.key; });
    else
      std::stable_sort(rows.begin(), rows.end(), [](const TaskRow& a, const TaskRow& b) { return a.key < b.key; });
  }
  count = 0;
  out.assign("[");
  out.reserve(buf.size() + rows.size() + 2);
  for (const TaskRow& r : rows) {
    if (count++) out += ',';
    out.append(buf, r.at, r.len);
  }
  out += ']';
  return true;
}

// query_tasks through the value tree (any text the one-pass reader declines)
inline bool query_tasks_tree(std::string_view body, std::string& out, size_t& count, bool by_created, bool* more,
                             bool descending) {
  tt::Value doc;
  try {
    doc = tt::parse_strict(body);
  } catch (const tt::ParseError&) {
    return false;
  }
  if (doc.t != tt::Value::Object) return false;
  if (more) {
    const tt::Value* tok = doc.get("token");
    *more = tok != nullptr && tok->t == tt::Value::String && !tok->s.empty();
  }
  const tt::Value* results = doc.get("results");
  if (results == nullptr || results->t == tt::Value::Null) {
    out = "[]";
    count = 0;
    return true;
  }
  if (results->t != tt::Value::Array) return false;
  count = 0;
  std::string id, day;
  if (!by_created) {
    out.assign("[");
    for (const auto& r : results->items) {
      if (r.t != tt::Value::Object) return false;
      const tt::Value* data = r.get("data");
      if (data == nullptr || data->t == tt::Value::Null) continue;
      if (count++) out += ',';
      if (!write_task(*data, false, out, id, day)) return false;
    }
    out += ']';
    return true;
  }
  // every task written once into `buf`; ordered by a numeric DateTime key (the canonical
  // created-on text sits right after `"taskCreatedOn":"` in write_task's fixed field order)
  struct Row {
    uint64_t key;
    size_t at, len;
  };
  std::vector<Row> rows;
  rows.reserve(results->items.size());
  std::string buf;
  buf.reserve(body.size());
  static const std::string_view tag = "\"taskCreatedOn\":\"";
  for (const auto& r : results->items) {
    if (r.t != tt::Value::Object) return false;
    const tt::Value* data = r.get("data");
    if (data == nullptr || data->t == tt::Value::Null) continue;
    const size_t at = buf.size();
    if (!write_task(*data, false, buf, id, day)) return false;
    const size_t c = buf.find(tag, at);
    if (c == std::string::npos) return false;
    rows.push_back({created_key(std::string_view(buf).substr(c + tag.size())), at, buf.size() - at});
  }
  // `descending`: newest first, ties in result order -- the reference's list,
  // `.OrderByDescending(o => o.TaskCreatedOn)` (TasksStoreManager.cs:66), is a stable sort too
  if (descending)
    std::stable_sort(rows.begin(), rows.end(), [](const Row& a, const Row& b) { return a.key > b.key; });
  else
    std::stable_sort(rows.begin(), rows.end(), [](const Row& a, const Row& b) { return a.key < b.key; });
  out.assign("[");
  out.reserve(buf.size() + rows.size() + 2);
  for (const Row& r : rows) {
    if (count++) out += ',';
    out.append(buf, r.at, r.len);
  }
  out += ']';
  return true;
}

}  // namespace taskcodec
