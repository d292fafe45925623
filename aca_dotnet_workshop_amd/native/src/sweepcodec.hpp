// The overdue sweep's protobuf hops in one pass each (apphost.hpp api_overdue / mark_pass): the
// sidecar's gRPC answers read straight into the API's output, instead of pb -> the state HTTP
// API's JSON (daprpb.hpp) -> the task codec (taskcodec.hpp) -> pb again.  A 1,000-task page
// crosses the app host twice per sweep (the GET's page, the markoverdue chunks' bulk get and
// save); each function here returns exactly what that chain returns, or false for anything
// outside the layouts it reads (the caller then runs the chain): tasks in the stored layout
// (taskcodec::fast_task_at), keys and etags as plain strings.
//   query_pb_tasks      QueryStateResponse -> the API's overdue / list page
//                       (= query_response_json + query_tasks)
//   conditional_mark_pb GetBulkStateResponse -> the ETag-guarded SaveStateRequest
//                       (= bulk_state_response_json + conditional_mark + save_state_bulk)
//   mark_overdue_ids    markoverdue's body (the API's own page layout) -> its ids
//                       (= mark_overdue's ids, no value tree)
#pragma once

#include <string>
#include <string_view>
#include <utility>
#include <vector>

#include "daprpb.hpp"
#include "pb.hpp"
#include "taskcodec.hpp"

namespace taskcodec {

// A string the state JSON layout carries as is: valid UTF-8, no quote, backslash or control
// character (what fast_task_at's reader and the data plane's writer pass through unchanged).
inline bool plain_text(std::string_view s) {
  for (unsigned char c : s)
    if (c < 0x20 || c == '"' || c == '\\') return false;
  return valid_utf8(s);
}

struct PbItem {
  std::string_view key, data, etag, error;
};

// one QueryStateItem / BulkStateItem {key = 1, data = 2, etag = 3, error = 4}
inline bool pb_item(std::string_view v, PbItem& it) {
  tt::pb::Reader ir(v);
  uint32_t g, gwt;
  std::string_view x;
  it = {};
  while (ir.next(g, gwt)) {
    if (g == 1 && gwt == tt::pb::LEN && ir.bytes(x)) it.key = x;
    else if (g == 2 && gwt == tt::pb::LEN && ir.bytes(x)) it.data = x;
    else if (g == 3 && gwt == tt::pb::LEN && ir.bytes(x)) it.etag = x;
    else if (g == 4 && gwt == tt::pb::LEN && ir.bytes(x)) it.error = x;
    else if (!ir.skip(gwt)) break;
  }
  return ir.ok;
}

inline bool query_pb_tasks(std::string_view msg, std::string& out, size_t& count, bool by_created, bool* more,
                           bool descending) {
  tt::pb::Reader rd(msg);
  uint32_t f, wt;
  std::string_view v, token;
  std::vector<TaskRow> rows;
  std::string buf;
  buf.reserve(msg.size());
  while (rd.next(f, wt)) {
    if (f == 1 && wt == tt::pb::LEN && rd.bytes(v)) {
      PbItem it;
      if (!pb_item(v, it) || it.data.empty() || !plain_text(it.key) || !plain_text(it.etag) ||
          !valid_utf8(it.data))
        return false;
      size_t i = 0;
      const size_t at = buf.size();
      uint64_t key = 0;
      if (!fast_task_at(it.data, i, buf, key) || i != it.data.size()) return false;
      rows.push_back({key, at, buf.size() - at});
    } else if (f == 2 && wt == tt::pb::LEN && rd.bytes(v)) {
      token = v;
    } else if (!rd.skip(wt)) {
      break;
    }
  }
  if (!rd.ok) return false;
  if (more) *more = !token.empty();
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

inline bool conditional_mark_pb(std::string_view msg, std::string_view store, std::string& save,
                                std::vector<std::string>& ids, size_t& skipped) {
  tt::pb::Reader rd(msg);
  uint32_t f, wt;
  std::string_view v;
  tt::pb::Writer w;
  w.s.reserve(msg.size() + 64);
  w.str(1, store);
  ids.clear();
  skipped = 0;
  static thread_local std::string task;
  std::string id;
  static constexpr char kFirstWrite[] = {0x08, 0x01};  // StateOptions {concurrency = FIRST_WRITE}
  while (rd.next(f, wt)) {
    if (f == 1 && wt == tt::pb::LEN && rd.bytes(v)) {
      PbItem it;
      if (!pb_item(v, it) || !it.error.empty() || !plain_text(it.key)) return false;
      if (it.data == "null") it.data = {};  // a missing key, as some servers write it
      if (it.data.empty()) {  // deleted since the sweep's query
        ++skipped;
        continue;
      }
      if (!plain_text(it.etag) || !valid_utf8(it.data)) return false;
      task.clear();
      size_t i = 0;
      uint64_t k = 0;
      std::pair<bool, bool> flags;
      if (!fast_task_at(it.data, i, task, k, nullptr, true, true, &flags, &id) || i != it.data.size()) return false;
      if (flags.first || flags.second) {  // completed or already overdue: not written
        ++skipped;
        continue;
      }
      // StateItem {key = 1, value = 2, etag = 3: Etag {value = 1}, options = 5}
      const size_t etag_msg = tt::pb::str_size(1, it.etag.size());
      w.len_header(2, tt::pb::len_field_size(1, it.key.size()) + tt::pb::len_field_size(2, task.size()) +
                          (it.etag.empty() ? 0 : tt::pb::len_field_size(3, etag_msg)) +
                          tt::pb::len_field_size(5, sizeof kFirstWrite));
      w.len_field(1, it.key);
      w.len_field(2, task);
      if (!it.etag.empty()) {
        w.len_header(3, etag_msg);
        w.str(1, it.etag);
      }
      w.len_field(5, std::string_view(kFirstWrite, sizeof kFirstWrite));
      ids.push_back(id);
    } else if (!rd.skip(wt)) {
      break;
    }
  }
  if (!rd.ok) return false;
  save = std::move(w.s);
  return true;
}

inline bool mark_overdue_ids(std::string_view body, std::vector<std::string>& ids) {
  if (body.size() < 2 || body[0] != '[' || !valid_utf8(body)) return false;
  ids.clear();
  if (body == "[]") return true;
  static thread_local std::string scratch;
  std::string id;
  size_t i = 1;
  while (true) {
    scratch.clear();
    uint64_t k = 0;
    if (!fast_task_at(body, i, scratch, k, nullptr, true, false, nullptr, &id)) return false;
    ids.push_back(id);
    if (i < body.size() && body[i] == ',') {
      ++i;
      continue;
    }
    return i + 1 == body.size() && body[i] == ']';
  }
}

}  // namespace taskcodec
