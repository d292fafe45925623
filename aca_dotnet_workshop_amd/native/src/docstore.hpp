// Native document store: the state-store engine behind `state.azure.cosmosdb`,
// `state.redis` and `state.in-memory` components.
//
// Capabilities mirrored from what the reference relies on:
//   * key -> JSON document with a monotonically increasing ETag per write;
//   * first-write / last-write optimistic concurrency (ETag mismatch -> EtagMismatch);
//   * TTL (Dapr `ttlInSeconds` metadata);
//   * multi-key atomic transactions;
//   * the state query API: filter EQ/NEQ/GT/GTE/LT/LTE/IN/AND/OR over JSON paths, multi-key
//     sort, limit + continuation token (reference Services/TasksStoreManager.cs:54-69, 104-139);
//   * automatic secondary hash indexes on equality paths (Cosmos indexes every path by
//     default) so `EQ taskCreatedBy` / `EQ taskDueDate` are O(matches), not O(collection);
//   * durability through an append-only log with online compaction.
#pragma once

#include <sys/random.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "applog.hpp"
#include "json.hpp"
#include "shardedmap.hpp"

namespace tt {

struct EtagMismatch : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct QueryError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

inline int64_t now_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::system_clock::now().time_since_epoch()).count();
}

struct Filter {
  enum Op { ALL, EQ, NEQ, GT, GTE, LT, LTE, IN, AND, OR } op = ALL;
  std::string path;
  Value val;
  std::vector<Value> vals;
  std::vector<Filter> kids;
};

inline bool ieq(std::string_view a, const char* b) {
  size_t n = std::strlen(b);
  if (a.size() != n) return false;
  for (size_t i = 0; i < n; ++i)
    if (std::toupper((unsigned char)a[i]) != b[i]) return false;
  return true;
}

inline Filter compile_filter(const Value& f) {
  Filter out;
  if (f.t == Value::Null) return out;
  if (f.t != Value::Object) throw QueryError("filter must be an object");
  if (f.keys.empty()) return out;
  if (f.keys.size() != 1) throw QueryError("filter object must have exactly one operator");
  const std::string& op = f.keys[0];
  const Value& arg = f.items[0];
  if (ieq(op, "AND") || ieq(op, "OR")) {
    out.op = ieq(op, "AND") ? Filter::AND : Filter::OR;
    if (arg.t != Value::Array || arg.items.empty()) throw QueryError(op + " expects a non-empty array");
    for (auto& k : arg.items) out.kids.push_back(compile_filter(k));
    return out;
  }
  static const std::pair<const char*, Filter::Op> table[] = {
      {"EQ", Filter::EQ}, {"NEQ", Filter::NEQ}, {"GT", Filter::GT}, {"GTE", Filter::GTE},
      {"LT", Filter::LT}, {"LTE", Filter::LTE}, {"IN", Filter::IN}};
  bool found = false;
  for (auto& [name, code] : table)
    if (ieq(op, name)) { out.op = code; found = true; }
  if (!found) throw QueryError("unsupported filter operator " + op);
  if (arg.t != Value::Object || arg.keys.size() != 1) throw QueryError(op + " expects {\"path\": value}");
  out.path = arg.keys[0];
  if (out.op == Filter::IN) {
    if (arg.items[0].t != Value::Array) throw QueryError("IN expects an array of values");
    out.vals = arg.items[0].items;
  } else {
    out.val = arg.items[0];
  }
  return out;
}

inline bool eval_filter(const Filter& f, const Value& doc) {
  switch (f.op) {
    case Filter::ALL: return true;
    case Filter::AND:
      for (auto& k : f.kids) if (!eval_filter(k, doc)) return false;
      return true;
    case Filter::OR:
      for (auto& k : f.kids) if (eval_filter(k, doc)) return true;
      return false;
    case Filter::IN: {
      const Value* v = doc.path(f.path);
      if (!v) return false;
      for (auto& x : f.vals) if (equals(*v, x)) return true;
      return false;
    }
    default: {
      const Value* v = doc.path(f.path);
      if (!v) return f.op == Filter::NEQ;
      if (f.op == Filter::EQ) return equals(*v, f.val);
      if (f.op == Filter::NEQ) return !equals(*v, f.val);
      if (v->t != f.val.t) return false;  // ranges only compare like types
      int c = compare(*v, f.val);
      switch (f.op) {
        case Filter::GT: return c > 0;
        case Filter::GTE: return c >= 0;
        case Filter::LT: return c < 0;
        case Filter::LTE: return c <= 0;
        default: return false;
      }
    }
  }
}

struct SortKey {
  std::string path;
  bool desc = false;
};

struct Doc {
  std::string value;
  Value parsed;
  uint64_t etag = 0;
  uint64_t seq = 0;
  int64_t expire_ms = 0;
  uint32_t mrow = UINT32_MAX;  // row in the column mirror (UINT32_MAX = none)
};

// Canonical dictionary key of a JSON scalar with the query engine's equality: numbers by
// value (-0.0 == 0.0), strings / booleans / null by value, arrays / objects by canonical JSON.
inline void mirror_key(const Value& v, std::string& k) {
  k.clear();
  switch (v.t) {
    case Value::Null: k = "n"; break;
    case Value::Bool: k = v.b ? "b1" : "b0"; break;
    case Value::Number: {
      double d = v.n + 0.0;  // folds -0.0
      uint64_t bits;
      std::memcpy(&bits, &d, sizeof bits);
      k.assign("d");
      k.append(reinterpret_cast<const char*>(&bits), sizeof bits);
      break;
    }
    case Value::String: k = "s"; k += v.s; break;
    default: k = "j"; dump_to(k, v);
  }
}

// Columnar mirror of a collection, maintained on every write under the store lock -- the
// source of the GPU query accelerator (ops/columnar.py ColumnarIndex.from_native).  One row
// per document version: an update kills the document's row and appends a new one (same seq,
// so orderings keep the native engine's insertion-order semantics); deletes kill the row.
// Readers pull deltas (rows appended since a cursor, new dictionary values, killed rows)
// instead of re-encoding, and the native write path never leaves C++.  Compaction drops dead
// rows and bumps the generation (readers then reload).
struct MirrorColumn {
  std::string path;
  ShardedMap<int32_t> dict;                       // canonical key -> id
  std::vector<std::string> values;                // JSON text per id, in order of first use
  std::vector<int32_t> ids;                       // per row (-1 = path missing)
};

struct ColumnMirror {
  bool on = false;
  bool disabled = false;  // TTL writes: expiry is evaluated by the native engine only
  uint64_t gen = 1;
  std::vector<MirrorColumn> cols;
  // per row: the owning map node -- key and document, no lookup by key (valid while live)
  std::vector<std::pair<const std::string, Doc>*> nodes;
  std::vector<int64_t> seqs;
  std::vector<uint8_t> live;
  std::vector<uint32_t> kills;  // rows killed since this generation began
  size_t live_rows = 0;
  uint64_t compactions = 0;
};

struct MirrorDelta {
  uint64_t gen = 0;
  bool on = false, disabled = false, full = false;
  size_t n = 0, from = 0, kill_cursor = 0;
  std::vector<std::string> paths;
  std::vector<size_t> dict_from;
  std::vector<std::vector<std::string>> new_values;
  std::vector<std::vector<int32_t>> ids;
  std::vector<int64_t> seqs;
  std::vector<uint8_t> live;     // rows [from, n)  (from == 0 when full)
  std::vector<uint32_t> kills;   // rows < from killed since the reader's kill cursor
};

struct TxOp {
  bool is_delete = false;
  std::string key;
  std::string value;
  std::optional<std::string> etag;
  bool first_write = false;
  int64_t ttl_ms = 0;
};

class DocStore {
 public:
  explicit DocStore(const std::string& path = "", int fsync_mode = 0, size_t index_threshold = 256)
      : index_threshold_(index_threshold) {
    if (!path.empty()) {
      log_.open(path, fsync_mode);
      log_.replay([this](char kind, std::vector<std::string_view>& f) { apply_log(kind, f); });
    }
  }

  // ---------------------------------------------------------------- writes
  std::string set(const std::string& key, const std::string& value, const std::optional<std::string>& etag,
                  bool first_write, int64_t ttl_ms) {
    Value parsed = parse(value);  // validate before taking the lock
    std::string text(value);
    std::vector<Doc> graveyard;  // declared before the lock: the replaced version is freed after it
    std::lock_guard<std::mutex> g(mu_);
    int64_t now = now_ms();
    auto it = docs_.find(key);
    check_etag_at(it, etag, first_write, now);
    it = put_at(it, key, std::move(text), std::move(parsed), ttl_ms > 0 ? now + ttl_ms : 0, &graveyard);
    log_put(key, it->second.value, it->second.etag, it->second.expire_ms);
    maybe_compact();
    return std::to_string(it->second.etag);
  }

  // Bulk write (Dapr BulkSet: not atomic -- every item succeeds or fails on its own): values
  // parsed before the lock, then ONE lock hold and ONE log write(2) for the whole batch, instead
  // of one of each per item.  Per item: the new etag, or err 1 (etag precondition) / 2 (invalid
  // JSON) with its detail.
  // Per item, one lookup of the key (etag check, write and log record share it); a caller that
  // already holds the value's parse tree (the native front parsed the request body) passes it
  // in `parsed` with `have_parsed`, and `value` is then its canonical text.  The replaced
  // documents are freed after the lock is released.
  struct BulkItem {
    std::string key, value;
    std::optional<std::string> etag;
    bool first_write = false;
    bool have_parsed = false;
    Value parsed;
  };
  struct BulkResult {
    std::string etag;
    int err = 0;
    std::string detail;
  };
  std::vector<BulkResult> set_many(std::vector<BulkItem>& items) {
    std::vector<BulkResult> out(items.size());
    for (size_t i = 0; i < items.size(); ++i) {
      if (items[i].have_parsed) continue;
      try {
        items[i].parsed = parse(items[i].value);
      } catch (const ParseError& e) {
        out[i].err = 2;
        out[i].detail = std::string("invalid JSON: ") + e.what();
      }
    }
    std::vector<Doc> graveyard;
    graveyard.reserve(items.size());
    {
      std::lock_guard<std::mutex> g(mu_);
      {
        AppLog::BatchScope batch(log_);
        const int64_t now = now_ms();
        for (size_t i = 0; i < items.size(); ++i) {
          if (out[i].err) continue;
          BulkItem& it = items[i];
          auto dit = docs_.find(it.key);
          const bool exists = dit != docs_.end() && !expired(dit->second, now);
          if (it.etag && !it.etag->empty()) {
            if (!exists || *it.etag != std::to_string(dit->second.etag)) {
              out[i].err = 1;
              out[i].detail = "possible etag mismatch";
              continue;
            }
          } else if (it.first_write && exists) {
            out[i].err = 1;
            out[i].detail = "possible etag mismatch: first-write on existing key without etag";
            continue;
          }
          dit = put_at(dit, it.key, std::move(it.value), std::move(it.parsed), 0, &graveyard);
          log_put(it.key, dit->second.value, dit->second.etag, dit->second.expire_ms);
          out[i].etag = std::to_string(dit->second.etag);
        }
      }
      maybe_compact();
    }
    return out;
  }

  std::optional<std::pair<std::string, std::string>> get(const std::string& key) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = docs_.find(key);
    if (it == docs_.end()) return std::nullopt;
    if (expired(it->second, now_ms())) { erase_locked(key, true); return std::nullopt; }
    return std::make_pair(it->second.value, std::to_string(it->second.etag));
  }

  bool del(const std::string& key, const std::optional<std::string>& etag) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = docs_.find(key);
    int64_t now = now_ms();
    if (it == docs_.end() || expired(it->second, now)) {
      if (etag && !etag->empty()) throw EtagMismatch("possible etag mismatch: key not found");
      return false;
    }
    if (etag && !etag->empty() && *etag != std::to_string(it->second.etag)) throw EtagMismatch("possible etag mismatch");
    erase_locked(key, true);
    maybe_compact();
    return true;
  }

  // All-or-nothing: every precondition is checked before any mutation is applied.
  void transact(const std::vector<TxOp>& ops) {
    std::vector<Value> parsed(ops.size());
    for (size_t i = 0; i < ops.size(); ++i)
      if (!ops[i].is_delete) parsed[i] = parse(ops[i].value);
    std::lock_guard<std::mutex> g(mu_);
    int64_t now = now_ms();
    for (auto& op : ops) {
      if (op.is_delete) {
        if (op.etag && !op.etag->empty()) {
          auto it = docs_.find(op.key);
          if (it == docs_.end() || *op.etag != std::to_string(it->second.etag)) throw EtagMismatch("possible etag mismatch in transaction");
        }
      } else {
        check_etag(op.key, op.etag, op.first_write, now);
      }
    }
    log_.append('T', {std::string_view("begin")});
    for (size_t i = 0; i < ops.size(); ++i) {
      auto& op = ops[i];
      if (op.is_delete) {
        if (docs_.count(op.key)) erase_locked(op.key, true);
      } else {
        uint64_t e = put(op.key, op.value, std::move(parsed[i]), op.ttl_ms > 0 ? now + op.ttl_ms : 0);
        log_put(op.key, op.value, e, docs_[op.key].expire_ms);
      }
    }
    log_.append('T', {std::string_view("commit")});
    maybe_compact();
  }

  // ---------------------------------------------------------------- query
  // One result of a sort-keys projection: {"key", "etag", "sort": [the document's value at each
  // sort path, null when missing]} -- the first phase of a cross-partition page (the sidecar
  // merges the shards' sort keys and fetches only the page's documents, dataplane.cpp).
  static void sort_keys_to(std::string& out, std::string_view key, const Doc& d, const std::vector<std::string>& paths) {
    out += "{\"key\":";
    escape_to(out, key);
    out += ",\"etag\":\"";
    out += std::to_string(d.etag);
    out += "\",\"sort\":[";
    for (size_t j = 0; j < paths.size(); ++j) {
      if (j) out += ',';
      const Value* v = d.parsed.path(paths[j]);
      if (v) dump_to(out, *v);
      else out += "null";
    }
    out += "]}";
  }

  // Returns {"results":[{"key","data","etag"}...],"token":"..."} as JSON text; `sort_keys`: the
  // results as sort-keys projections instead (sort_keys_to).
  std::string query(const std::string& query_json, const std::string& prefix, bool sort_keys = false) {
    Value q = parse(query_json.empty() ? std::string("{}") : query_json);
    if (q.t != Value::Object) throw QueryError("query must be a JSON object");
    Filter f;
    if (auto* fv = q.get_ci("filter")) f = compile_filter(*fv);
    std::vector<SortKey> sort;
    if (auto* sv = q.get_ci("sort")) {
      if (sv->t != Value::Array) throw QueryError("sort must be an array");
      for (auto& s : sv->items) {
        const Value* k = s.get_ci("key");
        if (!k || k->t != Value::String) throw QueryError("sort entry needs a string key");
        SortKey sk{k->s, false};
        if (auto* o = s.get_ci("order")) sk.desc = o->t == Value::String && ieq(o->s, "DESC");
        sort.push_back(sk);
      }
    }
    size_t limit = 0, offset = 0;
    if (auto* pv = q.get_ci("page")) {
      if (auto* l = pv->get_ci("limit")) limit = l->t == Value::Number && l->n > 0 ? (size_t)l->n : 0;
      if (auto* t = pv->get_ci("token")) {
        if (t->t == Value::String && !t->s.empty()) offset = (size_t)std::strtoull(t->s.c_str(), nullptr, 10);
      }
    }

    std::lock_guard<std::mutex> g(mu_);
    int64_t now = now_ms();
    ensure_indexes(f);
    std::vector<std::pair<const std::string*, const Doc*>> hits;
    auto consider = [&](const std::string& key, const Doc& d) {
      if (!prefix.empty() && key.compare(0, prefix.size(), prefix) != 0) return;
      if (expired(d, now)) return;
      if (!eval_filter(f, d.parsed)) return;
      hits.emplace_back(&key, &d);
    };
    std::unordered_set<std::string> cand;
    if (candidates(f, cand)) {
      ++stats_indexed_queries_;
      for (auto& k : cand) {
        auto it = docs_.find(k);
        if (it != docs_.end()) consider(it->first, it->second);
      }
    } else {
      ++stats_scan_queries_;
      for (auto& [k, d] : docs_) consider(k, d);
    }
    if (sort.empty()) {
      std::sort(hits.begin(), hits.end(), [](auto& a, auto& b) { return a.second->seq < b.second->seq; });
    } else {
      static const Value kNull;
      std::stable_sort(hits.begin(), hits.end(), [&](auto& a, auto& b) {
        for (auto& sk : sort) {
          const Value* x = a.second->parsed.path(sk.path);
          const Value* y = b.second->parsed.path(sk.path);
          int c = compare(x ? *x : kNull, y ? *y : kNull);
          if (c) return sk.desc ? c > 0 : c < 0;
        }
        return a.second->seq < b.second->seq;
      });
    }
    size_t begin = std::min(offset, hits.size());
    size_t end = limit ? std::min(hits.size(), begin + limit) : hits.size();
    std::string out = "{\"results\":[";
    std::vector<std::string> sort_paths;
    if (sort_keys)
      for (auto& sk : sort) sort_paths.push_back(sk.path);
    for (size_t i = begin; i < end; ++i) {
      if (i > begin) out += ',';
      if (sort_keys) {
        sort_keys_to(out, std::string_view(*hits[i].first).substr(prefix.size()), *hits[i].second, sort_paths);
        continue;
      }
      out += "{\"key\":";
      escape_to(out, std::string_view(*hits[i].first).substr(prefix.size()));
      out += ",\"data\":";
      out += hits[i].second->value;
      out += ",\"etag\":\"";
      out += std::to_string(hits[i].second->etag);
      out += "\"}";
    }
    out += "]";
    if (limit && end < hits.size()) {
      out += ",\"token\":\"" + std::to_string(end) + "\"";
    }
    out += "}";
    return out;
  }

  std::vector<std::string> keys(const std::string& prefix, size_t limit) {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<std::pair<uint64_t, std::string>> ks;
    int64_t now = now_ms();
    for (auto& [k, d] : docs_)
      if ((prefix.empty() || k.compare(0, prefix.size(), prefix) == 0) && !expired(d, now)) ks.emplace_back(d.seq, k);
    std::sort(ks.begin(), ks.end());
    std::vector<std::string> out;
    for (auto& p : ks) { if (limit && out.size() >= limit) break; out.push_back(p.second); }
    return out;
  }

  // Column export for the GPU scan path: one (seq-ordered) row per live document whose key
  // starts with `prefix`; returns keys and, per path, the raw JSON scalar values.
  // Dictionary-encoded columns of the documents under `prefix`, in insertion (seq) order: the
  // bulk load of the columnar query accelerator (ops/columnar.py ColumnarIndex.from_encoded).
  // Per path: the distinct values (JSON text, in order of first appearance) and one int32 id
  // per document (-1 = path missing).  Equality follows the query engine: numbers by value
  // (-0.0 == 0.0), strings/booleans/null by value, arrays/objects by canonical JSON.  Two
  // pseudo-paths: "\x00keyprefix" = the key's "<app-id>||" prefix, "\x00value" = the document.
  struct EncodedColumn {
    std::vector<std::string> values;
    std::vector<int32_t> ids;
  };
  struct Encoded {
    std::string key_blob;          // all keys concatenated (seq order)
    std::vector<int64_t> key_off;  // n + 1 offsets into key_blob
    std::vector<int64_t> seqs;
    std::vector<EncodedColumn> cols;
  };
  Encoded encode_columns(const std::string& prefix, const std::vector<std::string>& paths) {
    std::lock_guard<std::mutex> g(mu_);
    int64_t now = now_ms();
    std::vector<std::pair<uint64_t, const std::pair<const std::string, Doc>*>> rows;
    rows.reserve(docs_.size());
    for (auto& kv : docs_)
      if ((prefix.empty() || kv.first.compare(0, prefix.size(), prefix) == 0) && !expired(kv.second, now))
        rows.emplace_back(kv.second.seq, &kv);
    std::sort(rows.begin(), rows.end(), [](auto& a, auto& b) { return a.first < b.first; });
    Encoded out;
    out.key_off.reserve(rows.size() + 1);
    out.seqs.reserve(rows.size());
    out.key_off.push_back(0);
    for (auto& r : rows) {
      out.key_blob += r.second->first;
      out.key_off.push_back((int64_t)out.key_blob.size());
      out.seqs.push_back((int64_t)r.first);
    }
    out.cols.resize(paths.size());
    // one worker thread per column (read-only over the locked store)
    auto encode_one = [&](size_t c) {
      const std::string& path = paths[c];
      EncodedColumn& col = out.cols[c];
      col.ids.resize(rows.size());
      std::unordered_map<std::string, int32_t> dict;
      std::string k;
      for (size_t i = 0; i < rows.size(); ++i) {
        const std::string& key = rows[i].second->first;
        const Value& doc = rows[i].second->second.parsed;
        Value tmp;
        const Value* v;
        if (path == std::string("\x00keyprefix", 10)) {
          size_t p = key.find("||");
          tmp = Value::string(p == std::string::npos ? std::string() : key.substr(0, p + 2));
          v = &tmp;
        } else if (path == std::string("\x00value", 6)) {
          v = doc.t == Value::Object ? nullptr : &doc;
        } else {
          v = doc.path(path);
        }
        if (!v) {
          col.ids[i] = -1;
          continue;
        }
        mirror_key(*v, k);
        auto it = dict.find(k);
        if (it == dict.end()) {
          it = dict.emplace(k, (int32_t)col.values.size()).first;
          col.values.push_back(dump(*v));
        }
        col.ids[i] = it->second;
      }
        };
    if (paths.size() <= 1 || rows.size() < 100000) {
      for (size_t c = 0; c < paths.size(); ++c) encode_one(c);
    } else {
      std::vector<std::thread> ts;
      for (size_t c = 0; c < paths.size(); ++c) ts.emplace_back(encode_one, c);
      for (auto& t : ts) t.join();
    }
    return out;
  }

  // ------------------------------------------------------ provisioned throughput (RU/s)
  // Cosmos request-unit budget of the container (bicep/modules/cosmos-db.bicep:68-72,
  // autoscale max 4000 RU/s): a token bucket refilled at `ru_per_s` holding at most one second
  // of budget.  `charge` admits an operation (returns 0) or says how many milliseconds until
  // it would be admitted -- the caller answers 429 + x-ms-retry-after-ms and nothing is spent.
  // 0 RU/s = not provisioned (unlimited).  Costs follow Cosmos' published shape: a point read
  // is 1 RU per KiB, a write / delete 5 RU per KiB, a query 2.5 RU + 1 RU per KiB returned.
  static double read_ru(size_t bytes) { return std::max<double>(1.0, std::ceil(bytes / 1024.0)); }
  static double write_ru(size_t bytes) { return 5.0 * std::max<double>(1.0, std::ceil(bytes / 1024.0)); }
  static double query_ru(size_t result_bytes) { return 2.5 + std::ceil(result_bytes / 1024.0); }

  void set_throughput(double ru_per_s, double ticket_ttl_s = kTicketTtlS) {
    std::lock_guard<std::mutex> g(ru_mu_);
    ru_ticket_ttl_s_ = ticket_ttl_s;
    ru_rate_ = std::max(0.0, ru_per_s);
    ru_on_.store(ru_rate_ > 0, std::memory_order_relaxed);
    // the bucket starts empty and refills at the provisioned rate: over any window from the
    // start, what is admitted stays within rate x window (+ the call in flight) -- no free
    // first second of budget on top
    ru_tokens_ = 0;
    ru_last_ = mono_s();
    ru_tickets_.clear();
    ru_by_slot_.clear();
    ru_by_bind_.clear();
  }

  // Admission with reservations.  A caller the bucket cannot serve now is not just told its own
  // deficit (every waiter would wake at once and collide again): its RU are RESERVED -- the
  // bucket goes negative by the demand admitted for later -- and the 429's hint
  // (x-ms-retry-after-ms) is the moment the refill has paid for it, i.e. that caller's slot behind
  // every earlier waiter.  The reservation is bound to the request (`bind`: a hash of its method
  // and target, or of a query's text) and the 429 also carries an unguessable ticket
  // (`x-tt-ru-ticket`).  The retry is admitted at or after its slot without a second charge when
  //   * it presents the ticket (and is the same request), or
  //   * it follows only the Cosmos contract -- retries after the hint, no ticket -- and is the
  //     same request: it claims its own due reservation by `bind`;
  // an unticketed retry BEFORE its slot just gets the time left (no second reservation).  A
  // reservation more than kMaxReserveS ahead is refused outright (the SDK's 30 s wait budget
  // could not reach it).  One not claimed within kTicketTtlS of its slot lapses -- its caller
  // gave up -- and its RU go back to the bucket.
  static constexpr double kMaxReserveS = 25.0;
  static constexpr double kTicketTtlS = 10.0;
  // what a charge is for: the throttled-call breakdown of throughput_stats
  enum Kind : int { kRead = 0, kWrite = 1, kQuery = 2, kDelete = 3 };

  int64_t charge(double ru) {
    uint64_t unused = 0;
    return charge(ru, 0, unused);
  }
  // a provisioned budget (RU/s > 0): only then does admission need the request's `bind`
  bool provisioned() const { return ru_on_.load(std::memory_order_relaxed); }

  // FNV-1a of a request's identity (method + target, or a query's text): the `bind` of charge.
  static uint64_t bind_of(std::string_view a, std::string_view b = {}) {
    uint64_t h = 1469598103934665603ull;
    for (unsigned char c : a) h = (h ^ c) * 1099511628211ull;
    h = (h ^ 0xff) * 1099511628211ull;
    for (unsigned char c : b) h = (h ^ c) * 1099511628211ull;
    return h ? h : 1;
  }

  int64_t charge(double ru, uint64_t ticket, uint64_t& ticket_out, uint64_t bind = 0, int kind = kWrite) {
    std::lock_guard<std::mutex> g(ru_mu_);
    ticket_out = 0;
    if (ru_rate_ <= 0) {  // not provisioned: admitted, still metered (what the workload would need)
      ru_consumed_ += ru;
      return 0;
    }
    double now = mono_s();
    ru_tokens_ = std::min(ru_rate_, ru_tokens_ + (now - ru_last_) * ru_rate_);
    ru_last_ = now;
    lapse(now);
    // the request's own reservation: by its ticket, else (a Cosmos-contract retry) by `bind`
    auto own = ru_tickets_.end();
    if (ticket) {
      own = ru_tickets_.find(ticket);
      if (own != ru_tickets_.end() && bind && own->second.bind != bind) own = ru_tickets_.end();  // another's ticket
    }
    if (own == ru_tickets_.end() && bind) {
      auto range = ru_by_bind_.equal_range(bind);
      for (auto it = range.first; it != range.second; ++it) {
        auto t = ru_tickets_.find(it->second);
        if (t != ru_tickets_.end() && (own == ru_tickets_.end() || t->second.slot < own->second.slot)) own = t;
      }
    }
    if (own != ru_tickets_.end()) {
      if (now + 5e-4 >= own->second.slot) {  // its slot came: paid for by the reservation
        ru_consumed_ += own->second.ru;
        ++ru_reserved_admits_;
        drop(own);
        return 0;
      }
      ticket_out = own->first;  // early: keep the slot
      ++ru_throttled_;
      ++ru_early_retries_;
      return std::max<int64_t>(1, (int64_t)std::ceil((own->second.slot - now) * 1000.0));
    }
    ru = std::min(ru, ru_rate_);  // a request bigger than a second's budget waits for a full bucket
    ++ru_calls_;
    if (ru_tokens_ >= ru) {
      ru_tokens_ -= ru;
      ru_consumed_ += ru;
      return 0;
    }
    ++ru_throttled_;
    ++ru_throttled_kind_[kind & 3];
    double wait = (ru - ru_tokens_) / ru_rate_;  // until the refill has paid every earlier reservation and this one
    if (wait > kMaxReserveS) return std::max<int64_t>(1, (int64_t)std::ceil(wait * 1000.0));
    ru_tokens_ -= ru;
    do ticket_out = next_ticket();
    while (ru_tickets_.count(ticket_out));
    Reservation res{now + wait, ru, bind};
    ru_tickets_.emplace(ticket_out, res);
    ru_by_slot_.emplace(res.slot, ticket_out);
    if (bind) ru_by_bind_.emplace(bind, ticket_out);
    return std::max<int64_t>(1, (int64_t)std::ceil(wait * 1000.0));
  }

  // RU owed after the fact (a query's result-size part): spent whatever the balance, so later
  // callers wait for it.
  void debit(double ru) {
    std::lock_guard<std::mutex> g(ru_mu_);
    ru_consumed_ += ru;
    if (ru_rate_ <= 0) return;
    double now = mono_s();
    ru_tokens_ = std::min(ru_rate_, ru_tokens_ + (now - ru_last_) * ru_rate_) - ru;
    ru_last_ = now;
  }

  std::unordered_map<std::string, double> throughput_stats() {
    std::lock_guard<std::mutex> g(ru_mu_);
    return {{"ru_per_s", ru_rate_}, {"ru_consumed", ru_consumed_}, {"throttled", (double)ru_throttled_},
            {"reserved_admits", (double)ru_reserved_admits_}, {"open_reservations", (double)ru_tickets_.size()},
            {"calls", (double)ru_calls_}, {"early_retries", (double)ru_early_retries_},
            {"lapsed_reservations", (double)ru_lapsed_}, {"refunded_ru", ru_refunded_},
            {"throttled_read", (double)ru_throttled_kind_[kRead]}, {"throttled_write", (double)ru_throttled_kind_[kWrite]},
            {"throttled_query", (double)ru_throttled_kind_[kQuery]},
            {"throttled_delete", (double)ru_throttled_kind_[kDelete]},
            {"mono", mono_s()}};  // the store's clock: windows measured on the side that meters them
  }

  // ------------------------------------------------------------ column mirror
  // Mirror `paths` (added to the mirrored set; existing rows are encoded for new paths).  The
  // first call builds the mirror from the live documents in insertion order.  Returns false
  // when the collection cannot be mirrored (a TTL write was seen).
  bool mirror_enable(const std::vector<std::string>& paths) {
    std::lock_guard<std::mutex> g(mu_);
    if (mirror_.disabled) return false;
    std::vector<std::string> add;
    for (auto& p : paths) {
      bool have = false;
      for (auto& c : mirror_.cols) have = have || c.path == p;
      for (auto& a : add) have = have || a == p;
      if (!have) add.push_back(p);
    }
    if (mirror_.on && add.empty()) return true;
    if (!mirror_.on) {
      for (auto& [k, d] : docs_)
        if (d.expire_ms) { mirror_.disabled = true; return false; }
      mirror_.on = true;
      mirror_.cols.clear();
      for (auto& p : add) { mirror_.cols.emplace_back(); mirror_.cols.back().path = p; }
      mirror_rebuild_rows();
    } else {
      size_t first = mirror_.cols.size();
      for (auto& p : add) { mirror_.cols.emplace_back(); mirror_.cols.back().path = p; }
      auto enc = [&](size_t c) {
        MirrorColumn& col = mirror_.cols[c];
        col.ids.assign(mirror_.nodes.size(), -1);
        std::string k;
        for (size_t r = 0; r < mirror_.nodes.size(); ++r) {
          if (!mirror_.live[r]) continue;
          auto& kv = *mirror_.nodes[r];
          col.ids[r] = mirror_encode(col, kv.first, kv.second.parsed, k);
        }
      };
      parallel_for_columns(first, mirror_.cols.size(), enc);
      ++mirror_.gen;
      mirror_.kills.clear();
    }
    return true;
  }

  // Changes since a reader's cursor (generation, rows seen, kill-log position, dictionary
  // sizes per column); a different generation (or column set) returns everything.
  MirrorDelta mirror_delta(uint64_t gen, size_t from, size_t kill_from, const std::vector<size_t>& dict_sizes) {
    std::lock_guard<std::mutex> g(mu_);
    MirrorDelta d;
    d.gen = mirror_.gen;
    d.on = mirror_.on;
    d.disabled = mirror_.disabled;
    if (!mirror_.on) return d;
    size_t n = mirror_.nodes.size();
    d.full = gen != mirror_.gen || dict_sizes.size() != mirror_.cols.size() || from > n ||
             kill_from > mirror_.kills.size();
    if (d.full) from = 0, kill_from = mirror_.kills.size();
    d.n = n;
    d.from = from;
    d.kill_cursor = mirror_.kills.size();
    for (size_t i = kill_from; i < mirror_.kills.size(); ++i)
      if (mirror_.kills[i] < from) d.kills.push_back(mirror_.kills[i]);
    d.seqs.assign(mirror_.seqs.begin() + from, mirror_.seqs.end());
    d.live.assign(mirror_.live.begin() + from, mirror_.live.end());
    for (size_t c = 0; c < mirror_.cols.size(); ++c) {
      auto& col = mirror_.cols[c];
      size_t df = d.full ? 0 : std::min(dict_sizes[c], col.values.size());
      d.paths.push_back(col.path);
      d.dict_from.push_back(df);
      d.new_values.emplace_back(col.values.begin() + df, col.values.end());
      d.ids.emplace_back(col.ids.begin() + from, col.ids.end());
    }
    return d;
  }

  // Query result JSON for mirror rows (in the given order): {"results":[{"key","data","etag"}]}
  // with `prefix` stripped from the keys.  Rows killed since the reader's sync (the document
  // changed or went away) are skipped; `skipped` reports how many.  `gen` is the mirror
  // generation the reader's row numbers come from: a compaction (or a new column) renumbers the
  // rows, so a different generation returns false (`*stale` = true) without touching `out` --
  // a stale row number could name another live document, which would then be returned for a
  // filter it does not match.
  // `sort_paths` (non-null): sort-keys projections instead of documents (sort_keys_to).
  bool mirror_results(const int32_t* rows, size_t nrows, const std::string& prefix, const std::string& token,
                      uint64_t gen, std::string& out, size_t* skipped = nullptr,
                      const std::vector<std::string>* sort_paths = nullptr) {
    std::lock_guard<std::mutex> g(mu_);
    if (gen != mirror_.gen) return false;
    int64_t now = now_ms();
    out.clear();
    // one allocation for the page (~300 KB for the sweep's 1,024 tasks), not a doubling series
    if (!sort_paths && !docs_.empty()) out.reserve(32 + token.size() + nrows * (live_bytes_ / docs_.size() + 48));
    out += "{\"results\":[";
    size_t skip = 0;
    bool first = true;
    for (size_t i = 0; i < nrows; ++i) {
      uint32_t r = (uint32_t)rows[i];
      if (r >= mirror_.nodes.size() || !mirror_.live[r]) { ++skip; continue; }
      auto* it = mirror_.nodes[r];  // a live row's node: no hash lookup of the key
      const std::string& key = it->first;
      if (it->second.mrow != r || expired(it->second, now)) { ++skip; continue; }
      if (!first) out += ',';
      first = false;
      if (sort_paths) {
        sort_keys_to(out, std::string_view(key).substr(std::min(prefix.size(), key.size())), it->second, *sort_paths);
        continue;
      }
      out += "{\"key\":";
      escape_to(out, std::string_view(key).substr(std::min(prefix.size(), key.size())));
      out += ",\"data\":";
      out += it->second.value;
      out += ",\"etag\":\"";
      out += std::to_string(it->second.etag);
      out += "\"}";
    }
    out += "]";
    if (!token.empty()) out += ",\"token\":\"" + token + "\"";
    out += "}";
    if (skipped) *skipped = skip;
    return true;
  }

  std::unordered_map<std::string, uint64_t> mirror_stats() {
    std::lock_guard<std::mutex> g(mu_);
    return {{"on", mirror_.on}, {"disabled", mirror_.disabled}, {"gen", mirror_.gen},
            {"rows", mirror_.nodes.size()}, {"live_rows", mirror_.live_rows}, {"columns", mirror_.cols.size()},
            {"compactions", mirror_.compactions}};
  }

  size_t size() {
    std::lock_guard<std::mutex> g(mu_);
    return docs_.size();
  }

  void compact() {
    std::lock_guard<std::mutex> g(mu_);
    compact_locked();
  }

  void sync() { std::lock_guard<std::mutex> g(mu_); log_.sync(); }
  // group commit (AppLog fsync_mode 2): a writer's mark after its write, and the wait for the
  // sync that covers it (the backing front answers from the callback; Python callers block)
  bool group_commit() const { return log_.group(); }
  uint64_t log_mark() const { return log_.mark(); }
  void after_durable(uint64_t mark, std::function<void()> cb) { log_.after_durable(mark, std::move(cb)); }
  void wait_durable() { log_.wait_durable(); }
  AppLog::CommitStats commit_stats() { return log_.commit_stats(); }

  std::unordered_map<std::string, uint64_t> stats() {
    std::lock_guard<std::mutex> g(mu_);
    return {{"docs", docs_.size()}, {"live_bytes", live_bytes_}, {"log_bytes", log_.bytes()},
            {"indexes", indexes_.size()}, {"indexed_queries", stats_indexed_queries_},
            {"scan_queries", stats_scan_queries_}, {"etag", etag_}};
  }

  std::vector<std::string> indexed_paths() {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<std::string> out;
    for (auto& [p, _] : indexes_) out.push_back(p);
    std::sort(out.begin(), out.end());
    return out;
  }

 private:
  using Index = std::unordered_map<std::string, std::unordered_set<std::string>>;
  using Docs = ShardedMap<Doc>;  // grows a shard at a time: no whole-collection rehash under mu_

  static bool expired(const Doc& d, int64_t now) { return d.expire_ms && d.expire_ms <= now; }

  void check_etag(const std::string& key, const std::optional<std::string>& etag, bool first_write, int64_t now) {
    check_etag_at(docs_.find(key), etag, first_write, now);
  }

  void check_etag_at(Docs::iterator it, const std::optional<std::string>& etag,
                     bool first_write, int64_t now) {
    bool exists = it != docs_.end() && !expired(it->second, now);
    if (etag && !etag->empty()) {
      if (!exists || *etag != std::to_string(it->second.etag)) throw EtagMismatch("possible etag mismatch");
    } else if (first_write && exists) {
      throw EtagMismatch("possible etag mismatch: first-write on existing key without etag");
    }
  }

  uint64_t put(const std::string& key, const std::string& value, Value parsed, int64_t expire_ms) {
    return put_at(docs_.find(key), key, std::string(value), std::move(parsed), expire_ms, nullptr)->second.etag;
  }

  // Strict equality of two scalars (same type, same bits): equal values have equal index keys
  // and equal mirror dictionary keys, so an update that leaves a path unchanged keeps its index
  // entry and its dictionary id without re-keying.
  static bool same_scalar(const Value* a, const Value* b) {
    if (!a || !b) return a == b;
    if (a->t != b->t) return false;
    switch (a->t) {
      case Value::Null: return true;
      case Value::Bool: return a->b == b->b;
      case Value::Number: return std::memcmp(&a->n, &b->n, sizeof(double)) == 0;
      case Value::String: return a->s == b->s;
      default: return false;
    }
  }

  // The write itself, at `it` = docs_.find(key) done once by the caller.  Bulk writes pass a
  // `graveyard` that takes the replaced document's parsed tree and text, so their frees run
  // after the store lock is released.
  Docs::iterator put_at(Docs::iterator it,
                                                       const std::string& key, std::string&& value, Value parsed,
                                                       int64_t expire_ms, std::vector<Doc>* graveyard) {
    uint64_t e = ++etag_;
    if (expire_ms && mirror_.on) mirror_disable();
    int32_t* reuse = nullptr;
    if (it == docs_.end()) {
      Doc d;
      live_bytes_ += key.size() + value.size();
      d.value = std::move(value);
      d.parsed = std::move(parsed);
      d.etag = e;
      d.seq = ++seq_;
      d.expire_ms = expire_ms;
      index_add(key, d.parsed);
      it = docs_.emplace(key, std::move(d)).first;
    } else {
      Doc& d = it->second;
      index_update(key, d.parsed, parsed);
      if (mirror_.on && d.mrow < mirror_.live.size() && mirror_.live[d.mrow]) {
        reuse_.resize(mirror_.cols.size());
        for (size_t c = 0; c < mirror_.cols.size(); ++c)
          reuse_[c] = same_column_value(mirror_.cols[c], d.parsed, parsed) ? mirror_.cols[c].ids[d.mrow] : kEncode;
        reuse = reuse_.data();
      }
      live_bytes_ += value.size();
      live_bytes_ -= d.value.size();
      if (graveyard) {
        graveyard->emplace_back();
        graveyard->back().value.swap(d.value);
        graveyard->back().parsed = std::move(d.parsed);
      }
      d.value = std::move(value);
      d.parsed = std::move(parsed);
      d.etag = e;
      d.expire_ms = expire_ms;
      mirror_kill(d);
    }
    if (mirror_.on) mirror_append(*it, reuse);
    return it;
  }

  void erase_locked(const std::string& key, bool log) {
    auto it = docs_.find(key);
    if (it == docs_.end()) return;
    index_remove(key, it->second.parsed);
    mirror_kill(it->second);
    live_bytes_ -= key.size() + it->second.value.size();
    docs_.erase(it);
    if (log) log_.append('D', {key});
  }

  void log_put(const std::string& key, const std::string& value, uint64_t etag, int64_t expire) {
    if (!log_.is_open()) return;
    log_.append('P', {key, value, AppLog::pod(etag), AppLog::pod(expire)});
  }

  void apply_log(char kind, std::vector<std::string_view>& f) {
    if (kind == 'P' && f.size() == 4) {
      std::string key(f[0]), value(f[1]);
      uint64_t e;
      int64_t exp;
      std::memcpy(&e, f[2].data(), 8);
      std::memcpy(&exp, f[3].data(), 8);
      Value parsed;
      try { parsed = parse(value); } catch (...) { return; }
      put(key, value, std::move(parsed), exp);
      docs_[key].etag = e;
      etag_ = std::max(etag_, e);
    } else if (kind == 'D' && f.size() == 1) {
      erase_locked(std::string(f[0]), false);
    }
  }

  void maybe_compact() {
    if (!log_.is_open()) return;
    uint64_t live = live_bytes_ + docs_.size() * 40;
    if (log_.bytes() > (1u << 20) && log_.bytes() > 4 * live) compact_locked();
  }

  void compact_locked() {
    if (!log_.is_open()) return;
    std::vector<std::pair<uint64_t, const std::pair<const std::string, Doc>*>> rows;
    for (auto& kv : docs_) rows.emplace_back(kv.second.seq, &kv);
    std::sort(rows.begin(), rows.end(), [](auto& a, auto& b) { return a.first < b.first; });
    log_.rewrite([&](AppLog& out) {
      for (auto& r : rows)
        out.append('P', {r.second->first, r.second->second.value, AppLog::pod(r.second->second.etag),
                         AppLog::pod(r.second->second.expire_ms)});
    });
  }

  // ----------------------------------------------------------- column mirror (locked)
  template <class F>
  void parallel_for_columns(size_t lo, size_t hi, F&& f) {
    if (hi - lo <= 1 || mirror_.nodes.size() < 100000) {
      for (size_t c = lo; c < hi; ++c) f(c);
      return;
    }
    std::vector<std::thread> ts;
    for (size_t c = lo; c < hi; ++c) ts.emplace_back(f, c);
    for (auto& t : ts) t.join();
  }

  // Dictionary id of `path` in document `doc` under `key` (pseudo-paths as encode_columns).
  static int32_t mirror_encode(MirrorColumn& col, const std::string& key, const Value& doc, std::string& k) {
    static const std::string kPrefix("\x00keyprefix", 10), kValue("\x00value", 6);
    Value tmp;
    const Value* v;
    if (col.path == kPrefix) {
      size_t p = key.find("||");
      tmp = Value::string(p == std::string::npos ? std::string() : key.substr(0, p + 2));
      v = &tmp;
    } else if (col.path == kValue) {
      v = doc.t == Value::Object ? nullptr : &doc;
    } else {
      v = doc.path(col.path);
    }
    if (!v) return -1;
    mirror_key(*v, k);
    auto it = col.dict.find(k);
    if (it == col.dict.end()) {
      it = col.dict.emplace(k, (int32_t)col.values.size()).first;
      col.values.push_back(dump(*v));
    }
    return it->second;
  }

  // Whether column `col` of the updated document keeps the previous version's dictionary id.
  static bool same_column_value(const MirrorColumn& col, const Value& before, const Value& after) {
    static const std::string kPrefix("\x00keyprefix", 10), kValue("\x00value", 6);
    if (col.path == kPrefix) return true;  // a function of the key alone
    if (col.path == kValue)
      return before.t != Value::Object && after.t != Value::Object && same_scalar(&before, &after);
    return same_scalar(before.path(col.path), after.path(col.path));
  }

  // `reuse` (optional, one per column): a dictionary id carried over from the replaced row, or
  // kEncode to look the value up.
  void mirror_append(std::pair<const std::string, Doc>& kv, const int32_t* reuse = nullptr) {
    uint32_t r = (uint32_t)mirror_.nodes.size();
    mirror_.nodes.push_back(&kv);
    mirror_.seqs.push_back((int64_t)kv.second.seq);
    mirror_.live.push_back(1);
    std::string k;
    for (size_t c = 0; c < mirror_.cols.size(); ++c) {
      MirrorColumn& col = mirror_.cols[c];
      col.ids.push_back(reuse && reuse[c] != kEncode ? reuse[c] : mirror_encode(col, kv.first, kv.second.parsed, k));
    }
    kv.second.mrow = r;
    ++mirror_.live_rows;
    if (mirror_.nodes.size() > 65536 && mirror_.nodes.size() > 2 * mirror_.live_rows) mirror_compact();
  }

  void mirror_kill(Doc& d) {
    if (d.mrow == UINT32_MAX) return;
    if (mirror_.on && d.mrow < mirror_.live.size() && mirror_.live[d.mrow]) {
      mirror_.live[d.mrow] = 0;
      mirror_.kills.push_back(d.mrow);
      --mirror_.live_rows;
    }
    d.mrow = UINT32_MAX;
  }

  void mirror_disable() {
    for (auto& kv : docs_) kv.second.mrow = UINT32_MAX;
    uint64_t gen = mirror_.gen;
    mirror_ = ColumnMirror{};
    mirror_.gen = gen + 1;
    mirror_.disabled = true;
  }

  // Every live document, in insertion order, re-encoded into fresh rows (new generation).
  void mirror_rebuild_rows() {
    std::vector<std::pair<uint64_t, std::pair<const std::string, Doc>*>> rows;
    rows.reserve(docs_.size());
    for (auto& kv : docs_) rows.emplace_back(kv.second.seq, &kv);
    std::sort(rows.begin(), rows.end(), [](auto& a, auto& b) { return a.first < b.first; });
    mirror_.nodes.clear();
    mirror_.seqs.clear();
    mirror_.kills.clear();
    mirror_.nodes.reserve(rows.size());
    for (auto& r : rows) {
      r.second->second.mrow = (uint32_t)mirror_.nodes.size();
      mirror_.nodes.push_back(r.second);
      mirror_.seqs.push_back((int64_t)r.first);
    }
    mirror_.live.assign(rows.size(), 1);
    mirror_.live_rows = rows.size();
    auto enc = [&](size_t c) {
      MirrorColumn& col = mirror_.cols[c];
      col.ids.resize(rows.size());
      std::string k;
      for (size_t i = 0; i < rows.size(); ++i)
        col.ids[i] = mirror_encode(col, rows[i].second->first, rows[i].second->second.parsed, k);
    };
    parallel_for_columns(0, mirror_.cols.size(), enc);
    ++mirror_.gen;
  }

  // Drop dead rows (renumbering the survivors in row order); dictionaries are kept.
  void mirror_compact() {
    size_t w = 0, n = mirror_.nodes.size();
    for (size_t r = 0; r < n; ++r) {
      if (!mirror_.live[r]) continue;
      if (w != r) {
        mirror_.nodes[w] = mirror_.nodes[r];
        mirror_.seqs[w] = mirror_.seqs[r];
        for (auto& col : mirror_.cols) col.ids[w] = col.ids[r];
        mirror_.nodes[w]->second.mrow = (uint32_t)w;
      }
      ++w;
    }
    mirror_.nodes.resize(w);
    mirror_.seqs.resize(w);
    for (auto& col : mirror_.cols) col.ids.resize(w);
    mirror_.live.assign(w, 1);
    mirror_.live_rows = w;
    mirror_.kills.clear();
    ++mirror_.gen;
    ++mirror_.compactions;
  }

  // ----------------------------------------------------------- secondary indexes
  void collect_eq_paths(const Filter& f, std::vector<std::string>& out) {
    if (f.op == Filter::EQ || f.op == Filter::IN) out.push_back(f.path);
    for (auto& k : f.kids) collect_eq_paths(k, out);
  }

  void ensure_indexes(const Filter& f) {
    if (docs_.size() < index_threshold_) return;
    std::vector<std::string> paths;
    collect_eq_paths(f, paths);
    for (auto& p : paths) {
      if (indexes_.count(p)) continue;
      Index& idx = indexes_[p];
      for (auto& [k, d] : docs_) {
        const Value* v = d.parsed.path(p);
        if (v && v->t != Value::Array && v->t != Value::Object) idx[index_key(*v)].insert(k);
      }
    }
  }

  void index_add(const std::string& key, const Value& doc) {
    for (auto& [p, idx] : indexes_) {
      const Value* v = doc.path(p);
      if (v && v->t != Value::Array && v->t != Value::Object) idx[index_key(*v)].insert(key);
    }
  }

  // Re-index an updated document: paths whose value is unchanged keep their entry.
  void index_update(const std::string& key, const Value& before, const Value& after) {
    for (auto& [p, idx] : indexes_) {
      const Value* a = before.path(p);
      const Value* b = after.path(p);
      if (same_scalar(a, b)) continue;
      if (a && a->t != Value::Array && a->t != Value::Object) {
        auto it = idx.find(index_key(*a));
        if (it != idx.end()) {
          it->second.erase(key);
          if (it->second.empty()) idx.erase(it);
        }
      }
      if (b && b->t != Value::Array && b->t != Value::Object) idx[index_key(*b)].insert(key);
    }
  }

  void index_remove(const std::string& key, const Value& doc) {
    for (auto& [p, idx] : indexes_) {
      const Value* v = doc.path(p);
      if (!v || v->t == Value::Array || v->t == Value::Object) continue;
      auto it = idx.find(index_key(*v));
      if (it != idx.end()) {
        it->second.erase(key);
        if (it->second.empty()) idx.erase(it);
      }
    }
  }

  // Candidate key set from indexes; false = needs a full scan.
  bool candidates(const Filter& f, std::unordered_set<std::string>& out) {
    switch (f.op) {
      case Filter::EQ: {
        auto ix = indexes_.find(f.path);
        if (ix == indexes_.end() || f.val.t == Value::Array || f.val.t == Value::Object) return false;
        auto it = ix->second.find(index_key(f.val));
        if (it != ix->second.end()) out.insert(it->second.begin(), it->second.end());
        return true;
      }
      case Filter::IN: {
        auto ix = indexes_.find(f.path);
        if (ix == indexes_.end()) return false;
        for (auto& v : f.vals) {
          if (v.t == Value::Array || v.t == Value::Object) return false;
          auto it = ix->second.find(index_key(v));
          if (it != ix->second.end()) out.insert(it->second.begin(), it->second.end());
        }
        return true;
      }
      case Filter::AND: {
        bool any = false;
        std::unordered_set<std::string> best;
        for (auto& k : f.kids) {
          std::unordered_set<std::string> c;
          if (candidates(k, c) && (!any || c.size() < best.size())) { best.swap(c); any = true; }
        }
        if (any) out.insert(best.begin(), best.end());
        return any;
      }
      case Filter::OR: {
        std::unordered_set<std::string> acc;
        for (auto& k : f.kids)
          if (!candidates(k, acc)) return false;
        out.insert(acc.begin(), acc.end());
        return true;
      }
      default: return false;
    }
  }

  std::mutex mu_;
  Docs docs_;
  std::unordered_map<std::string, Index> indexes_;
  AppLog log_;
  uint64_t etag_ = 0;
  uint64_t seq_ = 0;
  uint64_t live_bytes_ = 0;
  uint64_t stats_indexed_queries_ = 0;
  uint64_t stats_scan_queries_ = 0;
  size_t index_threshold_;
  ColumnMirror mirror_;
  static constexpr int32_t kEncode = INT32_MIN;  // mirror_append: no id carried over
  std::vector<int32_t> reuse_;                   // put_at's per-column carried ids (under mu_)
  std::mutex ru_mu_;
  std::atomic<bool> ru_on_{false};
  double ru_rate_ = 0, ru_tokens_ = 0, ru_last_ = 0, ru_consumed_ = 0;
  // calls: charged requests (a ticketed retry is not a new one); early_retries: tickets
  // presented before their slot (a second 429 for the same call)
  uint64_t ru_throttled_ = 0, ru_reserved_admits_ = 0, ru_calls_ = 0, ru_early_retries_ = 0, ru_lapsed_ = 0;
  uint64_t ru_throttled_kind_[4] = {0, 0, 0, 0};
  double ru_refunded_ = 0;
  double ru_ticket_ttl_s_ = kTicketTtlS;
  struct Reservation {
    double slot, ru;
    uint64_t bind;
  };
  std::unordered_map<uint64_t, Reservation> ru_tickets_;      // ticket -> reservation
  std::multimap<double, uint64_t> ru_by_slot_;                 // slot -> ticket (lapse order)
  std::unordered_multimap<uint64_t, uint64_t> ru_by_bind_;     // request -> ticket
  uint64_t ru_rng_[2] = {0, 0};
  // tickets are random (xorshift128+ seeded from getrandom): a request cannot claim another's slot
  // by counting
  uint64_t next_ticket() {
    if ((ru_rng_[0] | ru_rng_[1]) == 0) {
      if (getrandom(ru_rng_, sizeof ru_rng_, 0) != (ssize_t)sizeof ru_rng_ || (ru_rng_[0] | ru_rng_[1]) == 0)
        ru_rng_[0] = 0x9e3779b97f4a7c15ull ^ (uint64_t)(mono_s() * 1e9);
    }
    uint64_t a = ru_rng_[0];
    const uint64_t b = ru_rng_[1];
    ru_rng_[0] = b;
    a ^= a << 23;
    ru_rng_[1] = a ^ b ^ (a >> 17) ^ (b >> 26);
    uint64_t v = (ru_rng_[1] + b) >> 1;  // 63 bits: the decimal header text parses as unsigned either way
    return v ? v : 1;
  }
  void drop(std::unordered_map<uint64_t, Reservation>::iterator it) {
    auto range = ru_by_slot_.equal_range(it->second.slot);
    for (auto s = range.first; s != range.second; ++s)
      if (s->second == it->first) {
        ru_by_slot_.erase(s);
        break;
      }
    if (it->second.bind) {
      auto b = ru_by_bind_.equal_range(it->second.bind);
      for (auto x = b.first; x != b.second; ++x)
        if (x->second == it->first) {
          ru_by_bind_.erase(x);
          break;
        }
    }
    ru_tickets_.erase(it);
  }
  // reservations not claimed within kTicketTtlS of their slot: their callers gave up; the RU
  // they held go back to the bucket (capped at a second's budget, like any refill)
  void lapse(double now) {
    while (!ru_by_slot_.empty() && ru_by_slot_.begin()->first + ru_ticket_ttl_s_ < now) {
      auto t = ru_tickets_.find(ru_by_slot_.begin()->second);
      if (t == ru_tickets_.end()) {
        ru_by_slot_.erase(ru_by_slot_.begin());
        continue;
      }
      ru_tokens_ = std::min(ru_rate_, ru_tokens_ + t->second.ru);
      ru_refunded_ += t->second.ru;
      ++ru_lapsed_;
      drop(t);
    }
  }
  static double mono_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }
};

}  // namespace tt
