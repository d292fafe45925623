// The dapr.proto.runtime.v1 messages of the reference SDK's hot calls, written and read without
// message objects -- what the .NET DaprClient sends for SaveStateAsync / GetBulkStateAsync /
// QueryStateAsync / PublishEventAsync (TasksStoreManager.cs:35,61,147,155) -- shared by the app
// host's native routes (apphost.hpp) and the Python SDK's gRPC client (sdk/grpc_client.py via
// module.cpp), so both write the same bytes.  Field numbers: sdk/proto.py (the public Dapr 1.14
// protos).  The answers are turned into the state HTTP API's JSON layout, the text the task codec
// (taskcodec.hpp) reads in one pass.
#pragma once

#include <string>
#include <string_view>
#include <vector>

#include "json.hpp"
#include "pb.hpp"

namespace tt::daprpb {

// SaveStateRequest {store_name = 1, states = 2: StateItem {key = 1, value = 2}} -- the common save
// (no ETag, metadata or options), every field written (sdk/grpc_client.py encode_save_state)
inline std::string save_state(std::string_view store, std::string_view key, std::string_view value) {
  pb::Writer item, w;
  item.len_field(1, key);
  item.len_field(2, value);
  w.len_field(1, store);
  w.len_field(2, item.s);
  return w.s;
}

// PublishEventRequest {pubsub_name = 1, topic = 2, data = 3, data_content_type = 4}
inline std::string publish_event(std::string_view pubsub, std::string_view topic, std::string_view data,
                                 std::string_view ctype) {
  pb::Writer w;
  w.len_field(1, pubsub);
  w.len_field(2, topic);
  w.len_field(3, data);
  w.len_field(4, ctype);
  return w.s;
}

// QueryStateRequest {store_name = 1, query = 2}, as message.SerializeToString writes it
inline std::string query_state(std::string_view store, std::string_view query) {
  pb::Writer w;
  w.str(1, store);
  w.str(2, query);
  return w.s;
}

// GetBulkStateRequest {store_name = 1, keys = 2 (repeated), parallelism = 3}
inline std::string get_bulk_state(std::string_view store, const std::vector<std::string>& keys, int parallelism) {
  pb::Writer w;
  w.str(1, store);
  for (auto& k : keys) w.len_field(2, k);
  w.u64(3, (uint64_t)parallelism);
  return w.s;
}

// The state HTTP API's save body ([{"key", "value", "etag", "options": {"concurrency",
// "consistency"}, "metadata": {..}}]) as a SaveStateRequest: StateItem {key = 1, value = 2 (the
// value's compact JSON text), etag = 3 (Etag {value = 1}), metadata = 4 (map), options = 5
// (StateOptions {concurrency = 1: first-write 1 / last-write 2, consistency = 2: eventual 1 /
// strong 2})}, fields in number order, the way protobuf serializes the SDK's message.  False: not
// such a body (a value that is not JSON, a key that is not a string, ...).
inline bool save_state_bulk(std::string_view store, std::string_view body, std::string& out) {
  if (!tt::valid(body)) return false;
  const char* p = body.data();
  const char* const e = p + body.size();
  auto lit = [&](char ch) {
    p = tt::ws_end(p, e);
    if (p < e && *p == ch) {
      ++p;
      return true;
    }
    return false;
  };
  auto string_at = [&](std::string& s) {  // a JSON string value, unescaped
    p = tt::ws_end(p, e);
    if (p >= e || *p != '"') return false;
    const char* s0 = p;
    p = tt::skip_value(p, e);
    std::string_view raw(s0, (size_t)(p - s0));
    if (raw.find('\\') == std::string_view::npos) {
      s.assign(raw.substr(1, raw.size() - 2));
      return true;
    }
    tt::Value v = tt::parse(raw);
    if (v.t != tt::Value::String) return false;
    s = std::move(v.s);
    return true;
  };
  pb::Writer w;
  w.str(1, store);
  if (!lit('[')) return false;
  if (lit(']')) {
    out = std::move(w.s);
    return tt::ws_end(p, e) == e;
  }
  while (true) {
    if (!lit('{')) return false;
    std::string key, etag, value = "null";
    bool have_key = false, have_etag = false;
    uint64_t concurrency = 0, consistency = 0;
    std::vector<std::pair<std::string, std::string>> meta;
    if (!lit('}')) {
      while (true) {
        std::string f;
        if (!string_at(f) || !lit(':')) return false;
        p = tt::ws_end(p, e);
        const char* v0 = p;
        if (f == "key") {
          if (!string_at(key)) return false;
          have_key = true;
        } else if (f == "value") {
          p = tt::skip_value(p, e);
          value = tt::compact(std::string_view(v0, (size_t)(p - v0)));
        } else if (f == "etag") {
          p = tt::skip_value(p, e);
          tt::Value v = tt::parse(std::string_view(v0, (size_t)(p - v0)));
          if (v.t == tt::Value::String) etag = v.s, have_etag = true;
          else if (auto* x = v.get("value"); x && x->t == tt::Value::String) etag = x->s, have_etag = true;
        } else if (f == "options" || f == "metadata") {
          p = tt::skip_value(p, e);
          tt::Value v = tt::parse(std::string_view(v0, (size_t)(p - v0)));
          if (v.t != tt::Value::Object) return false;
          for (size_t i = 0; i < v.keys.size(); ++i) {
            const tt::Value& x = v.items[i];
            std::string text = x.t == tt::Value::String ? x.s : tt::dump(x);
            if (f == "metadata") {
              meta.emplace_back(v.keys[i], std::move(text));
            } else if (v.keys[i] == "concurrency") {
              concurrency = text == "first-write" ? 1 : text == "last-write" ? 2 : 0;
            } else if (v.keys[i] == "consistency") {
              consistency = text == "eventual" ? 1 : text == "strong" ? 2 : 0;
            }
          }
        } else {
          p = tt::skip_value(p, e);
        }
        if (p > e) return false;
        if (lit(',')) continue;
        if (lit('}')) break;
        return false;
      }
    }
    if (!have_key) return false;
    pb::Writer item;
    item.len_field(1, key);
    item.len_field(2, value);
    if (have_etag) {
      pb::Writer et;
      et.str(1, etag);
      item.len_field(3, et.s);
    }
    for (auto& kv : meta) item.map_entry(4, kv.first, kv.second);
    if (concurrency || consistency) {
      pb::Writer opt;
      opt.u64(1, concurrency);
      opt.u64(2, consistency);
      item.len_field(5, opt.s);
    }
    w.len_field(2, item.s);
    if (lit(',')) continue;
    if (lit(']')) break;
    return false;
  }
  if (tt::ws_end(p, e) != e) return false;
  out = std::move(w.s);
  return true;
}

namespace detail {
// The end of the JSON string whose opening quote is at p[-1] (past its closing quote), 16 bytes
// a step; the same end tt::skip_value finds (an escape skips the byte after the backslash).
inline const char* string_end(const char* p, const char* e) {
  const __m128i q = _mm_set1_epi8('"'), bs = _mm_set1_epi8('\\');
  while (true) {
    while (e - p >= 16) {
      const __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p));
      const int m = _mm_movemask_epi8(_mm_or_si128(_mm_cmpeq_epi8(x, q), _mm_cmpeq_epi8(x, bs)));
      if (m) {
        p += __builtin_ctz((unsigned)m);
        break;
      }
      p += 16;
    }
    while (p < e && *p != '"' && *p != '\\') ++p;
    if (p >= e) return p + 1;
    if (*p == '"') return p + 1;
    p += 2;  // an escape: the next byte is part of it
    if (p >= e) return p + 1;
  }
}

// tt::skip_value's end of the value at p (no leading whitespace), with strings skipped 16 bytes
// a step; `ws`: whether the value holds whitespace outside its strings (tt::compact would
// change it).
inline const char* value_end(const char* p, const char* e, bool& ws) {
  ws = false;
  if (p >= e) return p;
  if (*p == '"') return string_end(p + 1, e);
  if (*p == '{' || *p == '[') {
    int depth = 0;
    while (p < e) {
      const char c = *p;
      if (c == '"') {
        p = string_end(p + 1, e);
        continue;
      }
      if (c == '{' || c == '[') ++depth;
      else if (c == '}' || c == ']') {
        if (--depth == 0) return p + 1;
      } else if (c == ' ' || c == '\n' || c == '\r' || c == '\t') {
        ws = true;
      }
      ++p;
    }
    return p;
  }
  while (p < e && *p != ',' && *p != '}' && *p != ']' && *p != ' ' && *p != '\n' && *p != '\r' && *p != '\t') ++p;
  return p;
}
}  // namespace detail

// The state query API's answer ({"results":[{"key","data","etag"[,"error"]}],"token"}) as a
// QueryStateResponse in one pass, without a value tree: a sweep page of thousands of tasks
// costs a scan, not a parse and a dump per task.  Keys, etags and the token must be plain
// strings (no escapes), each data value goes over compacted (as it is when it has no whitespace
// to drop); any other shape (metadata, escapes) returns false and the tree path encodes it.
inline bool query_response_pb(std::string_view b, std::string& out) {
  const char* p = b.data();
  const char* const e = p + b.size();
  auto lit = [&](char ch) {
    p = tt::ws_end(p, e);
    if (p < e && *p == ch) {
      ++p;
      return true;
    }
    return false;
  };
  auto null = [&] {
    p = tt::ws_end(p, e);
    if (e - p >= 4 && std::string_view(p, 4) == "null") {
      p += 4;
      return true;
    }
    return false;
  };
  auto plain = [&](std::string_view& s) {
    p = tt::ws_end(p, e);
    if (p >= e || *p != '"') return false;
    const char* q = detail::string_end(p + 1, e) - 1;  // the closing quote, or a backslash's run
    if (q >= e || *q != '"') return false;
    for (const char* x = p + 1; x < q; ++x)
      if (*x == '\\') return false;
    s = std::string_view(p + 1, (size_t)(q - p - 1));
    p = q + 1;
    return true;
  };
  pb::Writer w;
  w.s.reserve(b.size());
  std::string squeezed;
  if (!lit('{')) return false;
  if (!lit('}')) {
    while (true) {
      std::string_view k;
      if (!plain(k) || !lit(':')) return false;
      if (k == "results") {
        if (!null()) {
          if (!lit('[')) return false;
          if (!lit(']')) {
            while (true) {
              if (!lit('{')) return false;
              std::string_view key, etag, err, data;
              if (!lit('}')) {
                while (true) {
                  std::string_view f;
                  if (!plain(f) || !lit(':')) return false;
                  if (f == "data") {
                    if (!null()) {
                      const char* s0 = tt::ws_end(p, e);
                      bool ws = false;
                      p = detail::value_end(s0, e, ws);
                      if (p > e || p == s0) return false;
                      data = std::string_view(s0, (size_t)(p - s0));
                      if (ws) {
                        squeezed = tt::compact(data);
                        data = squeezed;
                      }
                    }
                  } else if (f == "key" || f == "etag" || f == "error") {
                    std::string_view v;
                    if (!null() && !plain(v)) return false;
                    (f == "key" ? key : f == "etag" ? etag : err) = v;
                  } else {
                    return false;
                  }
                  if (lit(',')) continue;
                  if (lit('}')) break;
                  return false;
                }
              }
              // QueryStateItem {key = 1, data = 2, etag = 3, error = 4}, its length first
              w.len_header(1, pb::str_size(1, key.size()) + pb::str_size(2, data.size()) +
                                  pb::str_size(3, etag.size()) + pb::str_size(4, err.size()));
              w.str(1, key);
              w.str(2, data);
              w.str(3, etag);
              w.str(4, err);
              if (lit(',')) continue;
              if (lit(']')) break;
              return false;
            }
          }
        }
      } else if (k == "token") {
        std::string_view t;
        if (!null() && !plain(t)) return false;
        w.str(2, t);
      } else {
        return false;
      }
      if (lit(',')) continue;
      if (lit('}')) break;
      return false;
    }
  }
  if (tt::ws_end(p, e) != e) return false;
  out = std::move(w.s);
  return true;
}

namespace detail {
inline void item_json(std::string& out, std::string_view key, std::string_view data, std::string_view etag,
                      bool etag_always) {
  out += "{\"key\":";
  tt::escape_to(out, key);
  if (!data.empty() || etag_always) {
    out += ",\"data\":";
    if (data.empty()) out += "null";
    else out.append(data);
    out += ",\"etag\":";
    tt::escape_to(out, etag);
  }
  out += '}';
}
}  // namespace detail

// QueryStateResponse {results = 1 {key, data, etag, error}, token = 2} as the state query API's
// JSON answer ({"results":[{"key","data","etag"}],"token"}); false when an item's data is not
// JSON text.
inline bool query_response_json(std::string_view msg, std::string& out) {
  pb::Reader rd(msg);
  uint32_t f, wt;
  std::string_view v, token;
  out.assign("{\"results\":[");
  bool first = true;
  while (rd.next(f, wt)) {
    if (f == 1 && wt == pb::LEN && rd.bytes(v)) {
      pb::Reader ir(v);
      uint32_t g, gwt;
      std::string_view x, key, data, etag;
      while (ir.next(g, gwt)) {
        if (g == 1 && gwt == pb::LEN && ir.bytes(x)) key = x;
        else if (g == 2 && gwt == pb::LEN && ir.bytes(x)) data = x;
        else if (g == 3 && gwt == pb::LEN && ir.bytes(x)) etag = x;
        else if (!ir.skip(gwt)) break;
      }
      if (!ir.ok || (!data.empty() && !tt::valid(data))) return false;
      if (!first) out += ',';
      first = false;
      detail::item_json(out, key, data, etag, true);
    } else if (f == 2 && wt == pb::LEN && rd.bytes(v)) {
      token = v;
    } else if (!rd.skip(wt)) {
      break;
    }
  }
  if (!rd.ok) return false;
  out += ']';
  if (!token.empty()) {
    out += ",\"token\":";
    tt::escape_to(out, token);
  }
  out += '}';
  return true;
}

// GetBulkStateResponse {items = 1: BulkStateItem {key = 1, data = 2, etag = 3, error = 4}} as
// the state bulk-get API's answer ([{"key","data","etag"} | {"key"}] -- a key without data is
// missing); false when data is not JSON text or an item carries an error.
inline bool bulk_state_response_json(std::string_view msg, std::string& out) {
  pb::Reader rd(msg);
  uint32_t f, wt;
  std::string_view v;
  out.assign("[");
  bool first = true;
  while (rd.next(f, wt)) {
    if (f == 1 && wt == pb::LEN && rd.bytes(v)) {
      pb::Reader ir(v);
      uint32_t g, gwt;
      std::string_view x, key, data, etag, error;
      while (ir.next(g, gwt)) {
        if (g == 1 && gwt == pb::LEN && ir.bytes(x)) key = x;
        else if (g == 2 && gwt == pb::LEN && ir.bytes(x)) data = x;
        else if (g == 3 && gwt == pb::LEN && ir.bytes(x)) etag = x;
        else if (g == 4 && gwt == pb::LEN && ir.bytes(x)) error = x;
        else if (!ir.skip(gwt)) break;
      }
      if (!ir.ok || !error.empty() || (!data.empty() && !tt::valid(data))) return false;
      if (data == "null") data = {};  // a missing key, as some servers write it
      if (!first) out += ',';
      first = false;
      detail::item_json(out, key, data, etag, false);
    } else if (!rd.skip(wt)) {
      break;
    }
  }
  if (!rd.ok) return false;
  out += ']';
  return true;
}

}  // namespace tt::daprpb
