// Native HTTP front for the backing-services emulator (backing/server.py).
//
// Runs an epoll loop on its own thread inside the backing-services process and serves the
// per-task hot routes directly against the SAME DocStore / Broker engine objects the Python
// handlers use (both are internally synchronised), without touching the GIL:
//
//   PUT|GET|DELETE /cosmos/{account}/{db}/{coll}/docs/{key}
//   POST           /cosmos/{account}/{db}/{coll}/bulkset
//   POST           /servicebus/{ns}/topics/{topic}/messages
//   POST           /servicebus/{ns}/receive?entity&max&lockMs&waitMs   (long poll)
//   POST           /servicebus/{ns}/settle
//   GET            /servicebus/{ns}/counts?entity
//   POST / GET     /storage/{account}/queues/{queue}/messages   (put; receive, long poll)
//   DELETE / PUT   /storage/{account}/queues/{queue}/messages/{receipt}   (delete; visibility)
//   PUT            /storage/{account}/blobs/{container}/{name}   (files under the blob root)
//   GET            /storage/{account}/blobs/{container}?count=true
//
// Everything else (entity management, queries, transactions, blobs, key vault, sendgrid,
// admin) and every request for an engine the Python side has not attached yet is forwarded
// verbatim to the Python server on a private Unix socket.  Responses, status codes and RBAC
// decisions mirror backing/server.py and backing/auth.py (role assignments are pushed down
// as principal -> (scope prefix, actions)).  Collections mirrored by the columnar query
// accelerator keep their writes here: the DocStore maintains its column mirror itself
// (docstore.hpp ColumnMirror) on every write, whichever front made it.
#pragma once

#include <condition_variable>
#include <deque>
#include <filesystem>
#include <unordered_set>

#include <fcntl.h>
#include <unistd.h>

#include <sys/eventfd.h>

#include <array>
#include <atomic>
#include <cassert>
#include <cstring>
#include <map>
#include <mutex>
#include <shared_mutex>
#include <thread>
#include <unordered_map>

#include "broker.hpp"
#include "docstore.hpp"
#include "evhttp.hpp"
#include "json.hpp"
#include "textutil.hpp"

namespace tt {

namespace bf {

using text::unquote;
inline std::string jstr(std::string_view s) { return text::json_str(s); }
inline bool utf8_ok(std::string_view s) { return text::valid_utf8(s); }
inline std::string b64(std::string_view in) { return text::base64(in); }

// RFC 7807 body exactly like web/http.py problem()
inline std::string problem_json(int status, std::string_view detail) {
  return "{\"type\": \"https://tools.ietf.org/html/rfc9110#section-15." + std::to_string(status / 100) +
         "\", \"title\": " + jstr(ev::reason_phrase(status)) + ", \"status\": " + std::to_string(status) +
         ", \"detail\": " + jstr(detail) + "}";
}

struct Grant {
  std::string principal, scope;
  std::vector<std::string> actions;  // "*" = any
};

}  // namespace bf

// The items of a bulkset body, scanned without building its tree: a value sent as a JSON
// value (the data plane's form) is kept as its raw text, whitespace compacted, and parsed once
// by the store; a value sent as a string holds JSON text.  False (left to Python's handler):
// invalid JSON, not an array of objects, a key that is not a string, or a TTL write.
inline bool scan_bulk_items(const std::string& body, std::vector<DocStore::BulkItem>& out) {
  std::string_view text = body.empty() ? std::string_view("[]") : std::string_view(body);
  if (!valid(text)) return false;
  const char* p = ws_end(text.data(), text.data() + text.size());
  const char* e = text.data() + text.size();
  if (*p != '[') return false;
  ++p;
  while (true) {
    p = ws_end(p, e);
    if (*p == ']') return true;
    if (*p != '{') return false;
    ++p;
    DocStore::BulkItem b;
    bool have_key = false, have_value = false;
    while (true) {
      p = ws_end(p, e);
      if (*p == '}') { ++p; break; }
      const char* ks = p;
      p = skip_value(p, e);
      std::string_view ktok(ks, (size_t)(p - ks));
      std::string k = ktok.find('\\') == std::string_view::npos ? std::string(ktok.substr(1, ktok.size() - 2))
                                                               : parse(ktok).s;
      p = ws_end(ws_end(p, e) + 1, e);  // ':'
      const char* vs = p;
      p = skip_value(p, e);
      std::string_view raw(vs, (size_t)(p - vs));
      if (k == "key") {
        if (raw.front() != '"') return false;
        b.key = raw.find('\\') == std::string_view::npos ? std::string(raw.substr(1, raw.size() - 2)) : parse(raw).s;
        have_key = true;
      } else if (k == "value") {
        have_value = true;
        b.value = raw.front() == '"' ? parse(raw).s : compact(raw);
      } else if (k == "etag") {
        b.etag.reset();
        if (raw.front() == '"') {
          std::string s = parse(raw).s;
          if (!s.empty()) b.etag = std::move(s);
        }
      } else if (k == "firstWrite") {
        b.first_write = raw == "true";
      } else if (k == "ttlMs") {
        if (raw.front() != 'n' && raw.front() != '"' && std::strtod(std::string(raw).c_str(), nullptr) != 0) return false;
      }
      p = ws_end(p, e);
      if (*p == ',') ++p;
    }
    if (!have_key) return false;
    if (!have_value) b.value = "null";
    out.push_back(std::move(b));
    p = ws_end(p, e);
    if (*p == ',') ++p;
  }
}

// The stored text of every item's value in a bulkset body, as the native front stores it (a
// JSON string value: the JSON text it holds; anything else: its compact text), for the items
// the front leaves to Python (TTL writes) -- both paths store the same bytes.  false: not a
// valid array of objects (Python answers).
inline bool scan_value_array(const char* p, const char* e, std::vector<std::string>& out);

inline bool scan_bulk_values(const std::string& body, std::vector<std::string>& out) {
  std::string_view text = body.empty() ? std::string_view("[]") : std::string_view(body);
  if (!valid(text)) return false;
  return scan_value_array(ws_end(text.data(), text.data() + text.size()), text.data() + text.size(), out);
}

// The same for a transaction body (`{"ops": [{"op", "key", "value", ...}]}`): every op's value
// as stored -- the request's own bytes, compacted -- so a transaction stores what a save does.
inline bool scan_tx_values(const std::string& body, std::vector<std::string>& out) {
  std::string_view text(body);
  if (text.empty() || !valid(text)) return false;
  const char* e = text.data() + text.size();
  const char* p = ws_end(text.data(), e);
  if (*p != '{') return false;
  ++p;
  bool found = false;
  while (true) {
    p = ws_end(p, e);
    if (*p == '}') return found;
    const char* ks = p;
    p = skip_value(p, e);
    std::string_view ktok(ks, (size_t)(p - ks));
    std::string k = ktok.find('\\') == std::string_view::npos ? std::string(ktok.substr(1, ktok.size() - 2))
                                                             : parse(ktok).s;
    p = ws_end(ws_end(p, e) + 1, e);  // ':'
    if (k == "ops") {
      out.clear();  // a repeated key: the last one wins, as in json.loads
      if (!scan_value_array(p, e, out)) return false;
      found = true;
    }
    p = ws_end(skip_value(p, e), e);
    if (*p == ',') ++p;
  }
}

inline bool scan_value_array(const char* p, const char* e, std::vector<std::string>& out) {
  if (*p != '[') return false;
  ++p;
  while (true) {
    p = ws_end(p, e);
    if (*p == ']') return true;
    if (*p != '{') return false;
    ++p;
    std::string value = "null";
    while (true) {
      p = ws_end(p, e);
      if (*p == '}') { ++p; break; }
      const char* ks = p;
      p = skip_value(p, e);
      std::string_view ktok(ks, (size_t)(p - ks));
      std::string k = ktok.find('\\') == std::string_view::npos ? std::string(ktok.substr(1, ktok.size() - 2))
                                                               : parse(ktok).s;
      p = ws_end(ws_end(p, e) + 1, e);  // ':'
      const char* vs = p;
      p = skip_value(p, e);
      std::string_view raw(vs, (size_t)(p - vs));
      if (k == "value") value = raw.front() == '"' ? parse(raw).s : compact(raw);
      p = ws_end(p, e);
      if (*p == ',') ++p;
    }
    out.push_back(std::move(value));
    p = ws_end(p, e);
    if (*p == ',') ++p;
  }
}

class BackingFront {
 public:
  // `threads` event loops share the port via SO_REUSEPORT (connections are spread by the kernel).
  // `uds`: also serve on this Unix socket -- the environment's processes on this host reach the
  // backing over it (a local stream socket costs about half a loopback TCP exchange's CPU); the
  // shards share the one listening socket (EPOLLEXCLUSIVE: one loop is woken per connection).
  BackingFront(const std::string& host, int port, const std::string& fallback_uds, int threads = 1,
               const std::string& uds = "")
      : fallback_(ev::Endpoint::parse("unix:" + fallback_uds)) {
    ev::reserve_fd_table();  // accept() must not grow the fd table (RCU wait) under load
    threads = std::max(1, std::min(threads, 64));
    for (int i = 0; i < threads; ++i) {
      shards_.push_back(std::make_shared<Shard>(*this));
      shards_.back()->self = shards_.back();
    }
    ev::Endpoint ep;
    ep.unix_socket = false;
    ep.host = host;
    ep.port = port;
    for (auto& sh : shards_) {
      int p = ev::listen_on(sh->loop, ep, sh->handler, threads > 1);
      if (ep.port == 0) ep.port = p;  // the other shards join the port the first one got
    }
    port_ = ep.port;
    if (!uds.empty()) {
      ev::Endpoint u;
      u.path = uds;
      int unused = 0;
      int fd = ev::bind_listen(u, false, unused);
      for (size_t i = 0; i < shards_.size(); ++i) {
        int f = i == 0 ? fd : ::fcntl(fd, F_DUPFD_CLOEXEC, 0);
        if (f < 0) break;
        auto l = std::make_shared<ev::Listener>(shards_[i]->loop, f, shards_[i]->handler);
        // whichever loop wakes for a connection, they are dealt to the loops in turn: the local
        // clients hold few long-lived (pipelined) connections, and an idle loop tends to win
        // every wake-up, which would leave one loop with all of them
        l->hand_off = [this, i](int c) {
          size_t to = next_uds_shard_.fetch_add(1, std::memory_order_relaxed) % shards_.size();
          if (to == i) return false;
          Shard* sh = shards_[to].get();
          sh->post_task([sh, c] { ev::adopt(sh->loop, c, sh->handler); });
          return true;
        };
        shards_[i]->loop.add(l, EPOLLIN | EPOLLEXCLUSIVE);
      }
    }
    for (auto& sh : shards_) sh->start();
  }
  ~BackingFront() { stop(); }

  // A query the indexes do not answer (a scan the columnar / GPU accelerator may take) runs on
  // a small pool of query worker threads (kQueryWorkers, TT_BACKING_QUERY_THREADS; the Python
  // route's query_pool had 4) through `query_fn` -- the Python planner, backing/server.py
  // BackingServices.run_query, called with the GIL -- and its answer goes back from the front's
  // loop: the page of results makes no extra HTTP hop through the Python server's event loop.
  // One slow scan (or a collection's first mirror build) holds one worker, not every other
  // collection's queries; the accelerator's per-collection lock keeps a collection's GPU use
  // serial.
  struct QueryJob {
    std::string account, db, coll, body, prefix, traceparent, sent_mono, front_mono;
    bool sort_keys = false;
  };
  struct QueryResult {
    int status = 0;  // 0: not taken -- the request goes to the Python server
    std::string body;
    ev::HeaderList headers;
  };
  using QueryFn = std::function<QueryResult(const QueryJob&)>;
  void set_query_fn(QueryFn fn) {
    std::lock_guard l(q_mu_);
    query_fn_ = std::move(fn);
    if (q_threads_.empty() && query_fn_) {
      int n = 4;
      if (const char* v = std::getenv("TT_BACKING_QUERY_THREADS"); v && std::atoi(v) > 0) n = std::min(32, std::atoi(v));
      for (int i = 0; i < n; ++i)
        q_threads_.emplace_back([this] {
          pthread_setname_np(pthread_self(), "tt-front-query");
          query_loop();
        });
    }
  }

  int port() const { return port_; }
  int threads() const { return (int)shards_.size(); }

  void stop() {
    if (stopped_) return;
    stopped_ = true;
    {
      std::lock_guard l(q_mu_);
      q_stop_ = true;
    }
    q_cv_.notify_all();
    for (auto& t : q_threads_)
      if (t.joinable()) t.join();
    q_threads_.clear();
    {
      std::lock_guard l(q_mu_);
      query_fn_ = nullptr;  // drop the Python callable before the interpreter may go
    }
    for (auto& sh : shards_) sh->request_stop();
    for (auto& sh : shards_) sh->join();
  }

  // -- configuration pushed from Python (any thread) -----------------------------------
  void attach_store(const std::string& account, const std::string& db, const std::string& coll, DocStore* s) {
    std::unique_lock l(cfg_mu_);
    auto& c = colls_[account + "\x1f" + db + "\x1f" + coll];
    if (!c) c = std::make_unique<Coll>();
    c->store = s;
  }
  void attach_broker(const std::string& ns, Broker* b) {
    std::unique_lock l(cfg_mu_);
    brokers_[ns] = b;
  }
  void set_policy(const std::string& mode, const std::vector<std::pair<std::string, std::string>>& keys,
                  const std::vector<std::tuple<std::string, std::string, std::vector<std::string>>>& grants) {
    std::unique_lock l(cfg_mu_);
    enforce_ = mode == "enforce";
    keys_ = keys;
    grants_.clear();
    for (auto& [p, s, a] : grants) grants_.push_back(bf::Grant{p, s, a});
  }
  // -- blobs --------------------------------------------------------------------------------
  // backing/server.py blob_root: the front writes blobs there as the Python route does.
  void set_blob_root(const std::string& root) {
    std::lock_guard l(blob_mu_);
    blob_root_ = root;
  }
  // A container's blob names: one directory scan on first use, then kept by every put and
  // delete -- the front's own, and Python's through blob_note -- so a count walks nothing.
  // `account` / `container` are the on-disk (sanitised) names.
  void blob_note(const std::string& account, const std::string& container, const std::string& name, bool added) {
    std::lock_guard l(blob_mu_);
    auto& names = blob_names_locked(account, container);
    if (added) names.insert(name);
    else names.erase(name);
  }
  size_t blob_count(const std::string& account, const std::string& container, const std::string& prefix) {
    std::lock_guard l(blob_mu_);
    auto& names = blob_names_locked(account, container);
    if (prefix.empty()) return names.size();
    size_t n = 0;
    for (auto& x : names) n += x.compare(0, prefix.size(), prefix) == 0;
    return n;
  }

  // Python-side broker activity (publish / abandon) for parked native long-polls.
  void notify(const std::string& ns, const std::string& entity) {
    for (auto& sh : shards_) sh->post(ns + "|" + entity);
  }
  std::map<std::string, uint64_t> stats() {
    std::map<std::string, uint64_t> out;
    for (size_t i = 0; i < kCounters.size(); ++i)
      if (uint64_t v = counters_[i].load(std::memory_order_relaxed)) out[kCounters[i]] = v;
    return out;
  }

 private:
  struct Coll {
    DocStore* store = nullptr;
  };
  struct Shard;
  struct QueuedQuery {
    std::shared_ptr<QueryJob> job;
    Shard* sh = nullptr;
    ev::Reply reply;
  };
  std::mutex q_mu_;
  std::condition_variable q_cv_;
  std::deque<QueuedQuery> q_jobs_;
  QueryFn query_fn_;
  std::vector<std::thread> q_threads_;
  bool q_stop_ = false;
  struct Parked {
    std::string ns, entity;
    size_t max;
    int64_t lock_ms;
    double deadline;
    ev::Reply reply;
    bool storage = false;  // a storage-queue receive: its answer has the queue API's shape
  };
  struct Shard;
  struct Wake : ev::IoObj {
    Shard* sh;
    explicit Wake(Shard* x) : sh(x) {}
    void on_event(uint32_t) override;  // defined after Shard
  };
  // One event loop + thread; parked long-polls live on the shard that received them.
  struct Shard {
    BackingFront& f;
    ev::Loop loop;
    ev::Client client;
    ev::Handler handler;
    std::thread thread;
    int wake_fd = -1;
    std::atomic<bool> stop_flag{false};
    std::mutex mu;
    std::vector<std::string> posted;               // cross-thread notifications
    std::vector<std::function<void()>> tasks;      // cross-thread work for this loop (query answers)
    std::multimap<std::string, Parked> parked;     // "ns|entity" -> waiting receives
    std::weak_ptr<Shard> self;                     // for answers posted back after a group commit

    explicit Shard(BackingFront& front) : f(front), client(loop) {
      handler = [this](ev::Message&& m, ev::Reply r) { f.on_request(*this, std::move(m), std::move(r)); };
      wake_fd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
      auto w = std::make_shared<Wake>(this);
      w->fd = dup(wake_fd);
      loop.add(w, EPOLLIN);
    }
    ~Shard() {
      if (wake_fd >= 0) ::close(wake_fd);
    }
    void start() {
      thread = std::thread([this] {
        pthread_setname_np(pthread_self(), "tt-front");  // per-thread CPU reports (bench hot_threads)
        ev::GapTracer gaps("backing-front");
        gaps.attach(loop);
        loop.run([this, &gaps](double t) {
          gaps.tick(t);
          on_tick(t);
        });
      });
    }
    // one eventfd write per loop wake-up, however many posts land before the loop runs (a
    // group commit releases a batch of answers at once); the loop clears the flag before it
    // takes the posted work, so a post after that takes a new write
    std::atomic<bool> wake_pending{false};
    void wake() {
      if (wake_pending.exchange(true, std::memory_order_acq_rel)) return;
      uint64_t one = 1;
      ssize_t r = ::write(wake_fd, &one, sizeof one);
      (void)r;
    }
    void post(std::string key) {
      {
        std::lock_guard l(mu);
        posted.push_back(std::move(key));
      }
      wake();
    }
    void post_task(std::function<void()> fn) {
      {
        std::lock_guard l(mu);
        tasks.push_back(std::move(fn));
      }
      wake();
    }
    void request_stop() {
      stop_flag = true;
      wake();
    }
    void join() {
      if (thread.joinable()) thread.join();
    }
    void on_wake() {
      if (stop_flag) {
        for (auto& kv : parked) kv.second.reply.json(503, bf::problem_json(503, "shutting down"));
        parked.clear();
        loop.stop();
        return;
      }
      std::vector<std::string> keys;
      std::vector<std::function<void()>> todo;
      wake_pending.store(false, std::memory_order_release);
      {
        std::lock_guard l(mu);
        keys.swap(posted);
        todo.swap(tasks);
      }
      for (auto& k : keys) f.retry_parked(*this, k);
      for (auto& fn : todo) fn();
    }
    void on_tick(double now) {
      if (stop_flag) {
        on_wake();
        return;
      }
      // deadlines + periodic re-check (delayed / scheduled messages, expired locks)
      std::vector<std::string> keys;
      for (auto& kv : parked)
        if (keys.empty() || keys.back() != kv.first) keys.push_back(kv.first);
      for (auto& k : keys) f.retry_parked(*this, k, now);
    }
  };

  ev::Endpoint fallback_;
  std::vector<std::shared_ptr<Shard>> shards_;
  std::atomic<size_t> next_uds_shard_{0};  // the Unix listener deals connections in turn
  int port_ = 0;
  bool stopped_ = false;

  std::shared_mutex cfg_mu_;
  std::unordered_map<std::string, std::unique_ptr<Coll>> colls_;
  std::unordered_map<std::string, Broker*> brokers_;
  bool enforce_ = false;
  std::vector<std::pair<std::string, std::string>> keys_;
  std::vector<bf::Grant> grants_;
  std::mutex blob_mu_;
  std::string blob_root_;
  std::unordered_map<std::string, std::unordered_set<std::string>> blob_names_;  // "account/container"

  std::unordered_set<std::string>& blob_names_locked(const std::string& account, const std::string& container) {
    std::string key = account + "/" + container;
    auto it = blob_names_.find(key);
    if (it != blob_names_.end()) return it->second;
    auto& names = blob_names_[key];
    namespace fs = std::filesystem;
    std::error_code ec;
    fs::path root = fs::path(blob_root_) / account / container;
    if (!blob_root_.empty() && fs::is_directory(root, ec))
      for (auto i = fs::recursive_directory_iterator(root, ec); !ec && i != fs::recursive_directory_iterator();
           i.increment(ec)) {
        if (!i->is_regular_file(ec)) continue;
        std::string n = i->path().lexically_relative(root).string();
        if (!ends_with(n, ".meta.json") && !ends_with(n, ".tmp")) names.insert(std::move(n));
      }
    return names;
  }
  static bool ends_with(const std::string& s, const char* suf) {
    size_t n = std::strlen(suf);
    return s.size() >= n && s.compare(s.size() - n, n, suf) == 0;
  }
  // backing/server.py _safe for ASCII names (non-ASCII ones stay with Python's regex)
  static bool safe_name(const std::string& in, std::string& out) {
    out.clear();
    for (unsigned char c : in) {
      if (c >= 0x80) return false;
      bool keep = (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '.' || c == '_' ||
                  c == '-';
      out += keep ? (char)c : '_';
    }
    return true;
  }
  static bool write_file(const std::string& path, std::string_view data) {
    int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    if (fd < 0) return false;
    size_t off = 0;
    while (off < data.size()) {
      ssize_t w = ::write(fd, data.data() + off, data.size() - off);
      if (w < 0 && errno == EINTR) continue;
      if (w <= 0) {
        ::close(fd);
        return false;
      }
      off += (size_t)w;
    }
    return ::close(fd) == 0;
  }

  // PUT /storage/{account}/blobs/{container}/{name}: the Python route's files (the blob, written
  // to a .tmp and renamed; its .meta.json) and answer.  Names Python might resolve differently
  // (dot segments, non-ASCII, its own .tmp / .meta.json suffixes) go to it.
  bool handle_blob(ev::Message& m, ev::Reply& r, const std::vector<std::string>& seg, const std::string& qs) {
    std::string acct, cont, root;
    if (!safe_name(seg[1], acct) || !safe_name(seg[3], cont)) return false;
    {
      std::lock_guard l(blob_mu_);
      root = blob_root_;
    }
    if (root.empty()) return false;
    if (seg.size() == 4 && m.method == "GET") {
      std::string c = query_get(qs, "count");
      for (auto& ch : c) ch = ::tt::ascii_lower(ch);
      if (c != "1" && c != "true") return false;  // the listing stays with Python
      if (!authorize(m, r, "blob.read", "storage/" + seg[1])) return true;
      count("blob.count");
      r.send(200, {{"content-type", "application/json"}},
             "{\"count\": " + std::to_string(blob_count(acct, cont, query_get(qs, "prefix"))) + "}");
      return true;
    }
    if (seg.size() < 5 || m.method != "PUT") return false;
    std::string name;
    for (size_t i = 4; i < seg.size(); ++i) {
      const std::string& p = seg[i];
      if (p.empty() || p == "." || p == ".." || p.find('/') != std::string::npos) return false;
      for (unsigned char c : p)
        if (c < 0x20 || c >= 0x80) return false;
      if (i > 4) name += '/';
      name += p;
    }
    if (ends_with(name, ".tmp") || ends_with(name, ".meta.json")) return false;
    if (!authorize(m, r, "blob.write", "storage/" + seg[1])) return true;
    count("blob.put");
    namespace fs = std::filesystem;
    fs::path f = fs::path(root) / acct / cont / name;
    std::error_code ec;
    fs::create_directories(f.parent_path(), ec);
    const std::string tmp = f.string() + ".tmp";
    auto* ct = m.header("content-type");
    char meta[160];
    std::snprintf(meta, sizeof meta, ", \"lastModified\": %.6f, \"size\": %zu}",
                  std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count(),
                  m.body.size());
    if (ec || !write_file(tmp, m.body) || ::rename(tmp.c_str(), f.c_str()) != 0 ||
        !write_file(f.string() + ".meta.json",
                    "{\"contentType\": " + bf::jstr(ct ? *ct : "application/octet-stream") + meta)) {
      r.send(500, {{"content-type", "application/problem+json; charset=utf-8"}},
             bf::problem_json(500, "blob write failed: " + f.string()));
      return true;
    }
    blob_note(acct, cont, name, true);
    r.send(201, {{"content-type", "application/json"}},
           "{\"blobURL\": " + bf::jstr("/storage/" + seg[1] + "/blobs/" + seg[3] + "/" + name) + "}");
    return true;
  }

  // Request counters, bumped by every loop on every request: one relaxed atomic per name, no
  // lock and no string (the hottest names first).
  static constexpr std::array<const char*, 19> kCounters = {
      "doc.put", "sb.publish", "sb.receive", "sb.settle", "doc.get", "doc.bulkget", "doc.bulkset", "doc.query",
      "doc.throttled", "doc.delete", "doc.query_worker", "doc.query_worker_done", "forwarded",
      "queue.put", "queue.get", "queue.delete", "queue.update", "blob.put", "blob.count"};
  std::array<std::atomic<uint64_t>, kCounters.size()> counters_{};

  void count(const char* k) {
    for (size_t i = 0; i < kCounters.size(); ++i)
      if (std::strcmp(kCounters[i], k) == 0) {
        counters_[i].fetch_add(1, std::memory_order_relaxed);
        return;
      }
    assert(!"unknown backing front counter");
  }
  // A broker event on one shard wakes parked receives on every shard.
  void broadcast(Shard& here, const std::string& key) {
    retry_parked(here, key);
    if (shards_.size() > 1)
      for (auto& sh : shards_)
        if (sh.get() != &here) sh->post(key);
  }

  // -- auth: backing/auth.py AccessPolicy.check ----------------------------------------
  bool allowed(const ev::Message& m, const std::string& action, const std::string& scope) {
    std::shared_lock l(cfg_mu_);
    if (!enforce_) return true;
    auto* key = m.header("x-tt-key");
    if (key && !key->empty())
      for (auto& [ks, k] : keys_)
        if (scope.rfind(ks, 0) == 0 && *key == k) return true;
    auto* ident = m.header("x-tt-identity");
    if (ident && !ident->empty())
      for (auto& g : grants_) {
        if (g.principal != *ident || scope.rfind(g.scope, 0) != 0) continue;
        for (auto& a : g.actions)
          if (a == "*" || a == action) return true;
      }
    return false;
  }
  bool authorize(const ev::Message& m, const ev::Reply& r, const std::string& action, const std::string& scope) {
    if (allowed(m, action, scope)) return true;
    auto* ident = m.header("x-tt-identity");
    std::string who = ident && !ident->empty() ? *ident : "anonymous";
    r.send(403, {{"content-type", "application/problem+json; charset=utf-8"}},
           bf::problem_json(403, who + " is not authorized to perform " + action + " on " + scope));
    return false;
  }

  // -- dispatch ---------------------------------------------------------------------------
  static void split(const std::string& target, std::string& path, std::string& qs) {
    auto q = target.find('?');
    path = target.substr(0, q);
    qs = q == std::string::npos ? "" : target.substr(q + 1);
  }
  static std::string query_get(const std::string& qs, const std::string& name) {
    size_t i = 0;
    while (i <= qs.size() && !qs.empty()) {
      size_t j = qs.find('&', i);
      if (j == std::string::npos) j = qs.size();
      std::string_view kv(qs.data() + i, j - i);
      size_t eq = kv.find('=');
      if (bf::unquote(kv.substr(0, eq), true) == name)
        return eq == std::string_view::npos ? "" : bf::unquote(kv.substr(eq + 1), true);
      i = j + 1;
    }
    return "";
  }

  void on_request(Shard& sh, ev::Message&& m, ev::Reply r) {
    std::string path, qs;
    split(m.target, path, qs);
    std::vector<std::string> seg;
    seg.reserve(8);
    for (size_t i = 1; i <= path.size();) {
      size_t j = path.find('/', i);
      if (j == std::string::npos) j = path.size();
      seg.push_back(bf::unquote(std::string_view(path).substr(i, j - i)));
      i = j + 1;
    }
    if (seg.size() == 6 && seg[0] == "cosmos" && seg[4] == "docs" && handle_doc(sh, m, r, seg)) return;
    if (seg.size() == 5 && seg[0] == "cosmos" && seg[4] == "bulkset" && m.method == "POST" &&
        handle_bulkset(sh, m, r, seg))
      return;
    if (seg.size() == 5 && seg[0] == "cosmos" && seg[4] == "bulkget" && m.method == "POST" && handle_bulkget(m, r, seg))
      return;
    if (seg.size() == 5 && seg[0] == "cosmos" && seg[4] == "query" && m.method == "POST" && handle_query(sh, m, r, seg, qs))
      return;
    if (seg.size() >= 3 && seg[0] == "servicebus" && handle_bus(sh, m, r, seg, qs)) return;
    if (seg.size() >= 5 && seg[0] == "storage" && seg[2] == "queues" && handle_storage_queue(sh, m, r, seg, qs)) return;
    if (seg.size() >= 4 && seg[0] == "storage" && seg[2] == "blobs" && handle_blob(m, r, seg, qs)) return;
    forward(sh, std::move(m), std::move(r));
  }

  void forward(Shard& sh, ev::Message&& m, ev::Reply r) {
    count("forwarded");
    ev::HeaderList h;
    for (auto& kv : m.headers)
      if (!ev::is_hop_header(kv.first)) h.push_back(kv);
    if (m.header("traceparent")) {  // a traced caller: when the front forwarded (CLOCK_MONOTONIC s)
      char t[32];
      std::snprintf(t, sizeof t, "%.6f", ev::now_s());
      h.emplace_back("x-tt-front-mono", t);
    }
    sh.client.request(fallback_, m.method, m.target, h, m.body, 0, [r](ev::ClientResult&& res) {
      if (res.err) {
        r.send(503, {{"content-type", "application/problem+json; charset=utf-8"}},
               bf::problem_json(503, "backing control plane unreachable"));
        return;
      }
      if (res.resp.header("x-tt-handler-end-mono")) {  // a traced query: when the front had the answer
        ev::HeaderList h2 = res.resp.headers;
        char t[32];
        std::snprintf(t, sizeof t, "%.6f", ev::now_s());
        h2.emplace_back("x-tt-front-rx-mono", t);
        r.send(res.resp.status, h2, res.resp.body);
        return;
      }
      r.send(res.resp.status, res.resp.headers, res.resp.body);
    });
  }

  // Provisioned-throughput admission (DocStore::charge): 429 + x-ms-retry-after-ms when the
  // container's RU/s budget is spent, as Cosmos answers; the sidecars retry after the hint.
  // The 429 carries the reservation's ticket (x-tt-ru-ticket); a retry presenting it is admitted
  // at its slot without a second charge (DocStore::charge).
  // `kind`: what the call is for (DocStore::Kind, the throttled-call breakdown); the reservation
  // is bound to the request: method + target, plus the body of a query or a bulk write.
  bool throttled(ev::Message& m, ev::Reply& r, DocStore* s, double ru, int kind) {
    if (!s->provisioned()) {  // unlimited: metered only
      s->charge(ru);
      return false;
    }
    uint64_t ticket = 0, out = 0;
    if (const std::string* t = m.header("x-tt-ru-ticket")) ticket = std::strtoull(t->c_str(), nullptr, 10);
    const uint64_t bind = DocStore::bind_of(m.method + " " + m.target,
                                            kind == DocStore::kQuery || m.method == "POST" ? std::string_view(m.body)
                                                                                           : std::string_view());
    int64_t wait_ms = s->charge(ru, ticket, out, bind, kind);
    if (!wait_ms) return false;
    count("doc.throttled");
    ev::HeaderList h{{"x-ms-retry-after-ms", std::to_string(wait_ms)},
                     {"retry-after", std::to_string((wait_ms + 999) / 1000)},
                     {"content-type", "application/problem+json; charset=utf-8"}};
    if (out) h.emplace_back("x-tt-ru-ticket", std::to_string(out));
    r.send(429, h, bf::problem_json(429, "Request rate is large: the container's provisioned throughput is exhausted"));
    return true;
  }

  // The native collection a cosmos path names (/cosmos/{account}/{db}/{container}/...), or null;
  // the lookup key is built in a per-thread buffer (no allocation per request).
  Coll* coll_of(const std::vector<std::string>& seg) {
    thread_local std::string k;
    k.assign(seg[1]);
    k += '\x1f';
    k += seg[2];
    k += '\x1f';
    k += seg[3];
    std::shared_lock l(cfg_mu_);
    auto it = colls_.find(k);
    return it != colls_.end() && it->second->store ? it->second.get() : nullptr;
  }

  // Answers a write once it is durable: now, or -- group commit (AppLog fsync_mode 2) -- from
  // the engine's log committer once the sync covering this write is done, handed back to the
  // shard's loop.  The loop goes on serving meanwhile; the writes of a sync period share one
  // fdatasync.
  template <class Engine>
  void send_durable(Shard& sh, Engine* eng, ev::Reply& r, int status, ev::HeaderList h, std::string body) {
    if (!eng->group_commit()) {
      r.send(status, h, body);
      return;
    }
    std::weak_ptr<Shard> w = sh.self;
    eng->after_durable(eng->log_mark(), [w, r, status, h = std::move(h), body = std::move(body)] {
      if (auto s = w.lock()) s->post_task([r, status, h, body] { r.send(status, h, body); });
    });
  }

  // -- cosmos documents ----------------------------------------------------------------------
  bool handle_doc(Shard& sh, ev::Message& m, ev::Reply& r, const std::vector<std::string>& seg) {
    Coll* c = coll_of(seg);
    if (!c) return false;
    const std::string& key = seg[5];
    const std::string scope = "cosmos/" + seg[1];
    if (m.method == "GET") {
      if (!authorize(m, r, "cosmos.read", scope)) return true;
      count("doc.get");
      if (throttled(m, r, c->store, DocStore::read_ru(0), DocStore::kRead)) return true;
      auto v = c->store->get(key);
      if (!v) r.empty(404);
      else r.send(200, {{"etag", v->second}, {"content-type", "application/json"}}, v->first);
      return true;
    }
    if (m.method != "PUT" && m.method != "DELETE") return false;
    auto* ttl = m.header("x-tt-ttl-ms");
    if (ttl && !ttl->empty() && *ttl != "0") return false;  // TTL writes disable the accelerator (Python)
    if (!authorize(m, r, "cosmos.write", scope)) return true;
    auto* im = m.header("if-match");
    std::optional<std::string> etag;
    if (im && !im->empty()) etag = *im;
    const char* pj = "application/problem+json; charset=utf-8";
    if (throttled(m, r, c->store, DocStore::write_ru(m.method == "PUT" ? m.body.size() : 0),
                  m.method == "PUT" ? DocStore::kWrite : DocStore::kDelete))
      return true;
    if (m.method == "PUT") {
      count("doc.put");
      auto* fw = m.header("x-tt-first-write");
      try {
        std::string e = c->store->set(key, m.body, etag, fw && *fw == "1", 0);
        send_durable(sh, c->store, r, 200, {{"etag", e}, {"content-type", "application/json"}},
                     "{\"etag\": " + bf::jstr(e) + "}");
      } catch (const EtagMismatch& ex) {
        r.send(412, {{"content-type", pj}}, bf::problem_json(412, ex.what()));
      } catch (const ParseError& ex) {
        r.send(400, {{"content-type", pj}}, bf::problem_json(400, std::string("invalid JSON: ") + ex.what()));
      }
      return true;
    }
    count("doc.delete");
    try {
      bool ok = c->store->del(key, etag);
      if (ok) send_durable(sh, c->store, r, 204, {}, {});
      else r.empty(404);
    } catch (const EtagMismatch& ex) {
      r.send(412, {{"content-type", pj}}, bf::problem_json(412, ex.what()));
    }
    return true;
  }

  // POST .../bulkset: [{"key", "value" (JSON text or value), "etag", "firstWrite", "ttlMs"}]
  bool handle_bulkset(Shard& sh, ev::Message& m, ev::Reply& r, const std::vector<std::string>& seg) {
    Coll* c = coll_of(seg);
    if (!c) return false;
    std::vector<DocStore::BulkItem> batch;
    if (!scan_bulk_items(m.body, batch)) return false;  // Python produces the error response
    if (!authorize(m, r, "cosmos.write", "cosmos/" + seg[1])) return true;
    count("doc.bulkset");
    double ru = 0;
    for (auto& b : batch) ru += DocStore::write_ru(b.value.size());
    if (throttled(m, r, c->store, ru, DocStore::kWrite)) return true;
    const std::vector<DocStore::BulkResult> res = c->store->set_many(batch);
    std::string out = "[";
    bool etag_err = false, other_err = false;
    for (size_t i = 0; i < res.size(); ++i) {
      if (i) out += ", ";
      out += "{\"key\": " + bf::jstr(batch[i].key);
      if (res[i].err == 0) {
        out += ", \"etag\": " + bf::jstr(res[i].etag) + "}";
      } else {
        (res[i].err == 1 ? etag_err : other_err) = true;
        out += std::string(", \"error\": ") + (res[i].err == 1 ? "\"etag\"" : "\"invalid\"") +
               ", \"detail\": " + bf::jstr(res[i].detail) + "}";
      }
    }
    out += "]";
    send_durable(sh, c->store, r, etag_err ? 412 : other_err ? 400 : 200, {{"content-type", "application/json"}}, out);
    return true;
  }

  // POST .../bulkget {"keys": [...]} -> [{"key", "data" (the stored JSON, as is), "etag"} | {"key"}]
  // in key order (a missing document has no data): the read half of a bulk read-modify-write
  bool handle_bulkget(ev::Message& m, ev::Reply& r, const std::vector<std::string>& seg) {
    Coll* c = coll_of(seg);
    if (!c) return false;
    Value body;
    try {
      body = parse(m.body);
    } catch (const ParseError&) {
      return false;  // Python produces the error response
    }
    const Value* keys = body.get("keys");
    if (!keys || keys->t != Value::Array) return false;
    for (auto& k : keys->items)
      if (k.t != Value::String) return false;
    if (!authorize(m, r, "cosmos.read", "cosmos/" + seg[1])) return true;
    count("doc.bulkget");
    if (throttled(m, r, c->store, DocStore::read_ru(0) * (double)std::max<size_t>(1, keys->items.size()), DocStore::kRead))
      return true;
    std::string out = "[";
    for (size_t i = 0; i < keys->items.size(); ++i) {
      const std::string& k = keys->items[i].s;
      if (i) out += ", ";
      out += "{\"key\": " + bf::jstr(k);
      if (auto v = c->store->get(k)) out += ", \"data\": " + v->first + ", \"etag\": " + bf::jstr(v->second);
      out += "}";
    }
    out += "]";
    r.send(200, {{"content-type", "application/json"}}, out);
    return true;
  }

  // POST .../query whose filter the hash indexes answer (backing/accel.py ``indexable``: the
  // planner sends those to the native engine, never to the columnar accelerator) -- the list of
  // a creator's tasks (TasksStoreManager.cs:54-69) -- runs here, on the front's loop, without
  // the Python server's event loop and GIL in the way.  Everything else (scans the accelerator
  // may take, sampled traces that record the store's spans, malformed queries) goes to Python.
  static bool indexable(const Value* f) {
    if (!f || f->t != Value::Object || f->keys.size() != 1) return false;
    std::string op = f->keys[0];
    for (auto& ch : op) ch = (char)std::toupper((unsigned char)ch);
    const Value& arg = f->items[0];
    if (op == "EQ" || op == "IN") {
      // equality on booleans / null is not selective: the planner scans instead
      if (arg.t != Value::Object || arg.items.empty()) return false;
      const Value& v = arg.items[0];
      auto plain = [](const Value& x) { return x.t == Value::Null || x.t == Value::Bool; };
      if (v.t != Value::Array) return !plain(v);
      for (auto& x : v.items)
        if (!plain(x)) return true;
      return false;
    }
    if (op == "AND") {
      if (arg.t != Value::Array) return false;
      for (auto& x : arg.items)
        if (indexable(&x)) return true;
      return false;
    }
    if (op == "OR") {
      if (arg.t != Value::Array || arg.items.empty()) return false;
      for (auto& x : arg.items)
        if (!indexable(&x)) return false;
      return true;
    }
    return false;
  }
  static bool sampled(const ev::Message& m) {
    const std::string* tp = m.header("traceparent");
    if (!tp || tp->size() < 55) return false;
    return (std::strtol(tp->c_str() + tp->size() - 2, nullptr, 16) & 1) != 0;
  }

  bool to_query_worker(Shard& sh, ev::Message& m, ev::Reply& r, Coll* c, const std::vector<std::string>& seg,
                       const std::string& qs) {
    {
      std::lock_guard l(q_mu_);
      if (!query_fn_ || q_stop_) return false;  // no worker: the Python server's route
    }
    if (!authorize(m, r, "cosmos.read", "cosmos/" + seg[1])) return true;
    if (throttled(m, r, c->store, DocStore::query_ru(0), DocStore::kQuery)) return true;
    count("doc.query_worker");
    auto job = std::make_shared<QueryJob>();
    job->account = seg[1];
    job->db = seg[2];
    job->coll = seg[3];
    job->body = std::move(m.body);
    job->prefix = query_get(qs, "prefix");
    std::string project = query_get(qs, "project");
    for (auto& ch : project) ch = (char)std::tolower((unsigned char)ch);
    job->sort_keys = project == "sortkeys";
    if (const std::string* tp = m.header("traceparent")) job->traceparent = *tp;
    if (const std::string* t = m.header("x-tt-sent-mono")) job->sent_mono = *t;
    char t[32];
    std::snprintf(t, sizeof t, "%.6f", ev::now_s());
    job->front_mono = t;
    {
      std::lock_guard l(q_mu_);
      q_jobs_.push_back({job, &sh, r});
    }
    q_cv_.notify_one();
    return true;
  }

  void query_loop() {
    while (true) {
      QueuedQuery qq;
      QueryFn fn;
      {
        std::unique_lock l(q_mu_);
        q_cv_.wait(l, [this] { return q_stop_ || !q_jobs_.empty(); });
        if (q_stop_) {
          for (auto& j : q_jobs_)  // answered from their loops: the front is going down
            j.sh->post_task([r = j.reply] { r.json(503, bf::problem_json(503, "shutting down")); });
          q_jobs_.clear();
          return;
        }
        qq = std::move(q_jobs_.front());
        q_jobs_.pop_front();
        fn = query_fn_;
      }
      QueryResult res;
      try {
        res = fn(*qq.job);
      } catch (const std::exception& ex) {
        res.status = 500;
        res.body = ex.what();
      }
      qq.sh->post_task([this, qq, res = std::move(res)]() mutable {
        count("doc.query_worker_done");
        if (res.status == 200) {
          if (!res.headers.empty()) {  // a traced query: when the front had the answer
            char t[32];
            std::snprintf(t, sizeof t, "%.6f", ev::now_s());
            res.headers.emplace_back("x-tt-front-rx-mono", t);
          }
          res.headers.emplace_back("content-type", "application/json");
          qq.reply.send(200, res.headers, res.body);
        } else {
          qq.reply.send(res.status ? res.status : 500, {{"content-type", "application/problem+json; charset=utf-8"}},
                        bf::problem_json(res.status ? res.status : 500, res.body));
        }
      });
    }
  }

  bool handle_query(Shard& sh, ev::Message& m, ev::Reply& r, const std::vector<std::string>& seg, const std::string& qs) {
    Coll* c = coll_of(seg);
    if (!c) return false;
    bool indexed = false;
    try {
      Value q = parse(m.body.empty() ? std::string("{}") : m.body);
      if (q.t != Value::Object) return false;
      indexed = indexable(q.get("filter"));
    } catch (const ParseError&) {
      return false;
    }
    if (!indexed || sampled(m)) return to_query_worker(sh, m, r, c, seg, qs);
    if (!authorize(m, r, "cosmos.read", "cosmos/" + seg[1])) return true;
    if (throttled(m, r, c->store, DocStore::query_ru(0), DocStore::kQuery)) return true;
    std::string body;
    try {
      std::string project = query_get(qs, "project");
      for (auto& ch : project) ch = (char)std::tolower((unsigned char)ch);
      body = c->store->query(m.body, query_get(qs, "prefix"), project == "sortkeys");
    } catch (const std::exception& ex) {  // the caller's query: 400, as the Python handler answers
      r.send(400, {{"content-type", "application/problem+json; charset=utf-8"}}, bf::problem_json(400, ex.what()));
      return true;
    }
    count("doc.query");
    c->store->debit(DocStore::query_ru(body.size()) - DocStore::query_ru(0));  // the result-size part
    r.send(200, {{"content-type", "application/json"}}, body);
    return true;
  }

  // -- service bus ---------------------------------------------------------------------------
  static std::string entity_scope(const std::string& entity) {
    auto p = entity.find("/subscriptions/");
    if (p != std::string::npos) return "topics/" + entity.substr(0, p);
    return "queues/" + entity;
  }

  bool handle_bus(Shard& sh, ev::Message& m, ev::Reply& r, const std::vector<std::string>& seg,
                  const std::string& qs) {
    Broker* b = nullptr;
    {
      std::shared_lock l(cfg_mu_);
      auto it = brokers_.find(seg[1]);
      if (it != brokers_.end()) b = it->second;
    }
    if (!b) return false;
    const std::string& ns = seg[1];
    if (seg.size() == 5 && seg[2] == "topics" && seg[4] == "messages" && m.method == "POST") {
      if (!authorize(m, r, "sb.send", "servicebus/" + ns + "/topics/" + seg[3])) return true;
      count("sb.publish");
      auto* ct = m.header("content-type");
      auto* props = m.header("x-tt-props");
      auto* mid = m.header("x-tt-message-id");
      auto* ttl = m.header("x-tt-ttl-ms");
      auto* delay = m.header("x-tt-delay-ms");
      uint64_t seq = b->publish(seg[3], m.body, ct ? *ct : "application/json", props ? *props : "{}", mid ? *mid : "",
                                ttl && !ttl->empty() ? std::atoll(ttl->c_str()) : 0,
                                delay && !delay->empty() ? std::atoll(delay->c_str()) : 0);
      send_durable(sh, b, r, 201, {{"content-type", "application/json"}}, "{\"seq\": " + std::to_string(seq) + "}");
      for (auto& sub : b->subscriptions(seg[3])) broadcast(sh, ns + "|" + seg[3] + "/subscriptions/" + sub);
      return true;
    }
    if (seg.size() == 3 && seg[2] == "receive" && m.method == "POST") {
      std::string entity = query_get(qs, "entity");
      if (!authorize(m, r, "sb.receive", "servicebus/" + ns + "/" + entity_scope(entity))) return true;
      count("sb.receive");
      std::string mx = query_get(qs, "max"), lk = query_get(qs, "lockMs"), wt = query_get(qs, "waitMs");
      Parked p{ns, entity, (size_t)std::max(1, mx.empty() ? 1 : std::atoi(mx.c_str())),
               lk.empty() ? 0 : std::atoll(lk.c_str()), ev::now_s() + (wt.empty() ? 0 : std::atoi(wt.c_str())) / 1000.0,
               r};
      if (!try_receive(b, p, false)) sh.parked.emplace(ns + "|" + entity, std::move(p));
      return true;
    }
    if (seg.size() == 3 && seg[2] == "settle" && m.method == "POST") {
      Value body;
      try {
        body = parse(m.body.empty() ? std::string_view("{}") : std::string_view(m.body));
      } catch (const std::exception&) {
        return false;  // let Python produce its error
      }
      std::string entity;
      if (auto* e = body.get("entity"); e && e->t == Value::String) entity = e->s;
      if (!authorize(m, r, "sb.receive", "servicebus/" + ns + "/" + entity_scope(entity))) return true;
      count("sb.settle");
      auto list = [&](const char* k) -> const std::vector<Value>* {
        auto* v = body.get(k);
        return v && v->t == Value::Array ? &v->items : nullptr;
      };
      auto str = [](const Value& o, const char* k) {
        auto* v = o.get(k);
        return v && v->t == Value::String ? v->s : std::string();
      };
      auto num = [](const Value& o, const char* k) {
        auto* v = o.get(k);
        return v && v->t == Value::Number ? (int64_t)v->n : (int64_t)0;
      };
      std::string out = "{\"complete\": [";
      if (auto* l = list("complete"))
        for (size_t i = 0; i < l->size(); ++i) out += std::string(i ? ", " : "") + (b->complete(entity, (*l)[i].s) ? "true" : "false");
      out += "], \"abandon\": [";
      bool abandoned = false;
      if (auto* l = list("abandon"))
        for (size_t i = 0; i < l->size(); ++i) {
          abandoned = true;
          out += std::string(i ? ", " : "") +
                 (b->abandon(entity, str((*l)[i], "token"), num((*l)[i], "delayMs")) ? "true" : "false");
        }
      out += "], \"deadletter\": [";
      if (auto* l = list("deadletter"))
        for (size_t i = 0; i < l->size(); ++i)
          out += std::string(i ? ", " : "") +
                 (b->dead_letter(entity, str((*l)[i], "token"), str((*l)[i], "reason")) ? "true" : "false");
      out += "], \"renew\": [";
      if (auto* l = list("renew"))
        for (size_t i = 0; i < l->size(); ++i)
          out += std::string(i ? ", " : "") +
                 (b->renew(entity, str((*l)[i], "token"), num((*l)[i], "lockMs")) ? "true" : "false");
      out += "]}";
      send_durable(sh, b, r, 200, {{"content-type", "application/json"}}, out);
      if (abandoned) broadcast(sh, ns + "|" + entity);
      return true;
    }
    if (seg.size() == 3 && seg[2] == "counts" && m.method == "GET") {
      auto [a, s, l, d, e, c, rc] = b->counts(query_get(qs, "entity"));
      r.send(200, {{"content-type", "application/json"}},
             "{\"active\": " + std::to_string(a) + ", \"scheduled\": " + std::to_string(s) + ", \"locked\": " +
                 std::to_string(l) + ", \"dead_letter\": " + std::to_string(d) + ", \"enqueued\": " + std::to_string(e) +
                 ", \"completed\": " + std::to_string(c) + ", \"received\": " + std::to_string(rc) + "}");
      return true;
    }
    return false;
  }

  // -- storage queues (backing/server.py _storage_routes, the same broker "storage-<account>") --
  // A query value the Python route would parse differently (not a plain non-negative integer)
  // leaves the request to it.
  static bool plain_uint(const std::string& v, int64_t& out) {
    if (v.empty() || v.size() > 15) return false;
    int64_t x = 0;
    for (char c : v) {
      if (c < '0' || c > '9') return false;
      x = x * 10 + (c - '0');
    }
    out = x;
    return true;
  }
  static bool uint_param(const std::string& qs, const char* name, int64_t dflt, int64_t& out) {
    std::string v = query_get(qs, name);
    if (v.empty()) {
      out = dflt;
      return true;
    }
    return plain_uint(v, out);
  }

  bool handle_storage_queue(Shard& sh, ev::Message& m, ev::Reply& r, const std::vector<std::string>& seg,
                            const std::string& qs) {
    const std::string ns = "storage-" + seg[1];
    Broker* b = nullptr;
    {
      std::shared_lock l(cfg_mu_);
      auto it = brokers_.find(ns);
      if (it != brokers_.end()) b = it->second;
    }
    if (!b) return false;  // the Python route creates the account's broker on first use
    const std::string& account = seg[1];
    const std::string& queue = seg[3];
    if (seg.size() == 5 && seg[4] == "messages" && m.method == "POST") {
      int64_t ttl_s, delay_s;
      if (!uint_param(qs, "messagettl", 0, ttl_s) || !uint_param(qs, "visibilitytimeout", 0, delay_s)) return false;
      if (!authorize(m, r, "queue.send", "storage/" + account)) return true;
      count("queue.put");
      uint64_t seq = b->send(queue, m.body, "text/plain", "{}", "", ttl_s * 1000, delay_s * 1000);
      send_durable(sh, b, r, 201, {{"content-type", "application/json"}},
                   "{\"messageId\": \"" + std::to_string(seq) + "\"}");
      broadcast(sh, ns + "|" + queue);
      return true;
    }
    if (seg.size() == 5 && seg[4] == "messages" && m.method == "GET") {
      int64_t mx, vis, wait_ms;
      if (!uint_param(qs, "numofmessages", 1, mx) || mx < 1 || !uint_param(qs, "visibilityMs", 30000, vis) ||
          !uint_param(qs, "waitMs", 0, wait_ms))
        return false;
      if (!authorize(m, r, "queue.receive", "storage/" + account)) return true;
      count("queue.get");
      Parked p{ns, queue, (size_t)mx, vis, ev::now_s() + (double)wait_ms / 1000.0, r, true};
      if (!try_receive(b, p, false)) sh.parked.emplace(ns + "|" + queue, std::move(p));
      return true;
    }
    if (seg.size() == 6 && seg[4] == "messages" && (m.method == "DELETE" || m.method == "PUT")) {
      int64_t vis = 0;
      if (m.method == "PUT" && !uint_param(qs, "visibilityMs", 0, vis)) return false;
      if (!authorize(m, r, "queue.receive", "storage/" + account)) return true;
      count(m.method == "DELETE" ? "queue.delete" : "queue.update");
      bool ok = m.method == "DELETE" ? b->complete(queue, seg[5]) : b->abandon(queue, seg[5], vis);
      send_durable(sh, b, r, ok ? 204 : 404, {}, "");
      if (m.method == "PUT") broadcast(sh, ns + "|" + queue);
      return true;
    }
    return false;
  }

  // Returns true when the request was answered (messages, or deadline reached).
  bool try_receive(Broker* b, Parked& p, bool expired) {
    // a receiver that went away (its process died mid long poll) must not lock messages it can
    // never settle -- they would sit out the whole lock duration before redelivery
    if (p.reply.abandoned()) {
      p.reply.send(204, {}, {});  // nobody reads it: lets the half-closed connection finish and close
      return true;
    }
    std::vector<Received> msgs;
    try {
      msgs = b->receive(p.entity, p.max, p.lock_ms);
    } catch (const std::exception& e) {
      p.reply.send(404, {{"content-type", "application/problem+json; charset=utf-8"}}, bf::problem_json(404, e.what()));
      return true;
    }
    if (msgs.empty() && !expired && ev::now_s() < p.deadline) return false;
    std::string out = "[";
    if (p.storage) {  // backing/server.py get_messages: messageId, popReceipt, dequeueCount, insertionMs, body
      for (size_t i = 0; i < msgs.size(); ++i) {
        auto& x = msgs[i];
        if (i) out += ", ";
        out += "{\"messageId\": \"" + std::to_string(x.seq) + "\", \"popReceipt\": " + bf::jstr(x.lock_token) +
               ", \"dequeueCount\": " + std::to_string(x.delivery_count) +
               ", \"insertionMs\": " + std::to_string(x.enqueued_wall);
        if (bf::utf8_ok(x.body)) out += ", \"body\": " + bf::jstr(x.body) + "}";
        else out += ", \"bodyB64\": \"" + bf::b64(x.body) + "\"}";
      }
      out += "]";
      p.reply.send(200, {{"content-type", "application/json"}}, out);
      return true;
    }
    for (size_t i = 0; i < msgs.size(); ++i) {
      auto& x = msgs[i];
      if (i) out += ", ";
      std::string props = x.props.empty() ? "{}" : x.props;
      out += "{\"lockToken\": " + bf::jstr(x.lock_token) + ", \"seq\": " + std::to_string(x.seq) + ", \"id\": " +
             bf::jstr(x.id) + ", \"contentType\": " + bf::jstr(x.content_type) + ", \"props\": " + props +
             ", \"deliveryCount\": " + std::to_string(x.delivery_count) + ", \"enqueuedMs\": " +
             std::to_string(x.enqueued_wall);
      if (bf::utf8_ok(x.body)) out += ", \"body\": " + bf::jstr(x.body) + "}";
      else out += ", \"bodyB64\": \"" + bf::b64(x.body) + "\"}";
    }
    out += "]";
    p.reply.send(200, {{"content-type", "application/json"}}, out);
    return true;
  }

  void retry_parked(Shard& sh, const std::string& key, double now = 0) {
    auto range = sh.parked.equal_range(key);
    if (range.first == range.second) return;
    Broker* b = nullptr;
    {
      std::shared_lock l(cfg_mu_);
      auto it = brokers_.find(key.substr(0, key.find('|')));
      if (it != brokers_.end()) b = it->second;
    }
    for (auto it = range.first; it != range.second;) {
      bool expired = now > 0 && now >= it->second.deadline;
      if (b && try_receive(b, it->second, expired)) it = sh.parked.erase(it);
      else ++it;
    }
  }
};

inline void BackingFront::Wake::on_event(uint32_t) {
  uint64_t v;
  while (::read(fd, &v, sizeof v) == (ssize_t)sizeof v) {
  }
  sh->on_wake();
}

}  // namespace tt
