// Native HTTP host for the Python services -- the Kestrel half of the ASP.NET Core equivalent.
//
// The reference's services run on Kestrel, whose socket I/O, HTTP parsing and connection
// management happen on native I/O threads while the application code runs on the managed
// thread pool.  AppHost does the same for a Python app process: one
// epoll thread (evhttp.hpp Loop/Server/Client) owns every socket of the process -- the app's
// listeners (TCP or Unix) and the keep-alive pools to the sidecar -- and the Python thread
// only runs route handlers.
//
//   loop thread                              Python thread (asyncio)
//   -----------                              -----------------------
//   parse request  --event(REQUEST)-->       eventfd readable -> drain() -> handler task
//   write response <--submit([respond])--   handler done
//   send request   <--submit([request])--   SDK call (await future)
//   parse response --event(RESPONSE)-->      drain() -> future.set_result
//
// Both directions are batched: a queue plus an eventfd that is signalled only when the queue
// goes from empty to non-empty, so a burst of N requests costs one wake-up on each side.
// The loop thread never touches Python objects (no GIL); conversion happens in drain(), which
// the Python thread calls.
//
// Native routes (add_route): a service may hand its hottest route to the host, the way the
// sidecar's data plane serves the hot Dapr routes for its Python control plane.  The loop
// thread then runs the whole exchange with the same native codec the Python handler calls, the
// same sidecar calls with the same headers, and the same answer; the Python thread only sees
// the route's log records (LOG events, written by its own logging sinks) and its request
// counters (route_stats, folded into the Prometheus registry).  What the native path does not
// decide goes to Python unchanged:
//   * bodies outside the codec's envelope, bad antiforgery tokens, other content types;
//   * sampled traces (the Python pipeline records their spans);
//   * a new trace the sampler picks, marked `x-tt-native: sample`.
// A sidecar call that fails is handed over too, marked `x-tt-native: fail <step> <status>
// <base64 body>` or `err <step> <errno>`: the Python handler raises the error the SDK would
// have raised, and the pipeline answers it as always.  The host drops that header from what
// clients send; web/native_host.py moves the host's own into `req.state["tt_native"]`.
#pragma once

#include <sys/eventfd.h>
#include <unistd.h>

#include <sys/random.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include <future>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_set>

#include "evhttp.hpp"
#include "formcodec.hpp"
#include "daprpb.hpp"
#include "h2.hpp"
#include "taskcodec.hpp"
#include "sweepcodec.hpp"
#include "textutil.hpp"

namespace tt::apphost {

using ev::HeaderList;
using ev::Message;

struct Event {
  enum Kind : int { REQUEST = 0, RESPONSE = 1, ERROR = 2, LOG = 3 };
  int kind = REQUEST;
  uint64_t id = 0;      // REQUEST: reply token; RESPONSE/ERROR: the client request id
  int server = 0;       // REQUEST: which listener group (one per Python HttpServer)
  int err = 0;          // ERROR: errno-like code; LOG: the level (Python logging's numbers)
  double t = 0;         // loop-thread monotonic time when the event was queued (ev::now_s)
  Message msg;          // LOG: method = logger name, body = message, target/reason = trace/span id
  std::string line;     // LOG: the finished JSON line, when the route has its sink's prefix
};

// Text the Python definitions hand a native route (a log template, a Location): "%s" slots
// filled in order from named fields of the request's task, "%%" a percent sign.  Compiled when
// the route is registered; a template the route cannot fill (another directive, a field it does
// not know, a slot count that differs from the fields) refuses the route -- Python serves it.
struct Template {
  enum Field { kId = 0, kName = 1, kAssignedTo = 2 };
  std::vector<std::string> lits;  // fields.size() + 1 literal pieces
  std::vector<int> fields;        // indices into the route's field names
  bool set = false;

  // `known`: the fields this route can fill, by name (default: a created task's)
  static Template compile(const std::string& text, const std::string& args,
                          const std::vector<std::string>& known = {"id", "name", "assigned_to"}) {
    Template t;
    t.set = true;
    std::vector<int> names;
    for (size_t a = 0; a < args.size();) {
      size_t b = args.find(',', a);
      std::string f = args.substr(a, b == std::string::npos ? std::string::npos : b - a);
      auto it = std::find(known.begin(), known.end(), f);
      if (it == known.end()) throw std::invalid_argument("native route template: unknown field " + f);
      names.push_back((int)(it - known.begin()));
      if (b == std::string::npos) break;
      a = b + 1;
    }
    std::string cur;
    for (size_t i = 0; i < text.size(); ++i) {
      if (text[i] != '%') {
        cur += text[i];
        continue;
      }
      char d = i + 1 < text.size() ? text[i + 1] : '\0';
      ++i;
      if (d == '%') {
        cur += '%';
      } else if (d == 's') {
        t.lits.push_back(std::move(cur));
        cur.clear();
        if (t.fields.size() == names.size()) throw std::invalid_argument("native route template: more slots than fields");
        t.fields.push_back(names[t.fields.size()]);
      } else {
        throw std::invalid_argument("native route template: only %s and %% are supported");
      }
    }
    t.lits.push_back(std::move(cur));
    if (t.fields.size() != names.size()) throw std::invalid_argument("native route template: fewer slots than fields");
    return t;
  }
  std::string render(const std::string& id, const std::string& name, const std::string& assigned_to) const {
    return render_with([&](int f) -> const std::string& { return f == kId ? id : f == kName ? name : assigned_to; });
  }
  template <class Value>
  std::string render_with(Value&& value) const {
    std::string out = lits[0];
    for (size_t i = 0; i < fields.size(); ++i) {
      out += value(fields[i]);
      out += lits[i + 1];
    }
    return out;
  }
};

// A page compiled by the Python side from its own Jinja template (services/frontend/rows.py):
// literal pieces around named slots, as a JSON array [lit, slot, lit, ..., lit].  The route
// only fills the slots; the markup is the template's.
struct Pieces {
  std::vector<std::string> lits;
  std::vector<int> slots;
  bool set = false;

  static Pieces parse(const std::string& json, const std::vector<std::string>& names) {
    Pieces p;
    tt::Value v = tt::parse(json);
    if (v.t != tt::Value::Array || v.items.size() % 2 != 1) throw std::invalid_argument("native route page: not pieces");
    for (size_t i = 0; i < v.items.size(); ++i) {
      const tt::Value& x = v.items[i];
      if (x.t != tt::Value::String) throw std::invalid_argument("native route page: a piece is not text");
      if (i % 2 == 0) {
        p.lits.push_back(x.s);
        continue;
      }
      auto it = std::find(names.begin(), names.end(), x.s);
      if (it == names.end()) throw std::invalid_argument("native route page: unknown slot " + x.s);
      p.slots.push_back((int)(it - names.begin()));
    }
    p.set = true;
    return p;
  }
  template <class Fill>
  void render(std::string& out, Fill&& fill) const {
    out += lits[0];
    for (size_t i = 0; i < slots.size(); ++i) {
      fill(slots[i], out);
      out += lits[i + 1];
    }
  }
};

// Jinja's autoescape (markupsafe.escape): & < > ' "
inline void html_escape_to(std::string& out, std::string_view s) {
  for (char c : s) {
    switch (c) {
      case '&': out += "&amp;"; break;
      case '<': out += "&lt;"; break;
      case '>': out += "&gt;"; break;
      case '\'': out += "&#39;"; break;
      case '"': out += "&#34;"; break;
      default: out += c;
    }
  }
}

// urllib.parse.quote (safe "/"): letters, digits, "_.-~" and "/" as is, every other byte %XX
inline void url_quote_to(std::string& out, std::string_view s) {
  static const char* hx = "0123456789ABCDEF";
  for (unsigned char c : s) {
    if (std::isalnum(c) || c == '_' || c == '.' || c == '-' || c == '~' || c == '/') {
      out += (char)c;
    } else {
      out += '%';
      out += hx[c >> 4];
      out += hx[c & 15];
    }
  }
}

// Request.query_get of web/http.py: parse_qsl (keep blank values, first value wins), the exact
// name, else the first name equal ignoring case; false when absent or not decodable.
inline bool query_param(std::string_view target, std::string_view name, std::string& out) {
  size_t q = target.find('?');
  if (q == std::string_view::npos) return false;
  std::string_view qs = target.substr(q + 1);
  std::vector<std::pair<std::string, std::string>> kv;
  for (size_t i = 0; i <= qs.size();) {
    size_t j = qs.find('&', i);
    if (j == std::string_view::npos) j = qs.size();
    std::string_view f = qs.substr(i, j - i);
    i = j + 1;
    if (f.empty()) continue;
    size_t eq = f.find('=');
    std::string k, v;
    if (!::formcodec::unquote(f.substr(0, eq), true, k)) return false;
    if (eq != std::string_view::npos && !::formcodec::unquote(f.substr(eq + 1), true, v)) return false;
    bool seen = false;
    for (auto& e : kv) seen = seen || e.first == k;
    if (!seen) kv.emplace_back(std::move(k), std::move(v));
  }
  for (auto& e : kv)
    if (e.first == name) return out = e.second, true;
  auto low = [](std::string_view x) {
    std::string r(x);
    for (auto& c : r) c = ::tt::ascii_lower(c);
    return r;
  };
  const std::string want = low(name);
  for (auto& e : kv)
    if (low(e.first) == want) return out = e.second, true;
  return false;
}

// web/http.py Request.cookies: ';'-separated, stripped, name=value, value unquoted, last wins
inline bool cookie_value(std::string_view cookie, std::string_view name, std::string& out) {
  bool have = false;
  std::string tmp;
  for (size_t i = 0; i <= cookie.size();) {
    size_t j = cookie.find(';', i);
    if (j == std::string_view::npos) j = cookie.size();
    std::string_view part = cookie.substr(i, j - i);
    i = j + 1;
    while (!part.empty() && (part.front() == ' ' || part.front() == '\t')) part.remove_prefix(1);
    while (!part.empty() && (part.back() == ' ' || part.back() == '\t')) part.remove_suffix(1);
    size_t eq = part.find('=');
    if (eq == std::string_view::npos || part.substr(0, eq) != name) continue;
    if (!::formcodec::unquote(part.substr(eq + 1), false, tmp)) return false;
    out = tmp;
    have = true;
  }
  return have;
}

// A route the loop thread serves itself (AppHost::add_route).
struct NativeRoute {
  enum Kind {
    kFrontendCreate = 1, kApiCreate = 2, kProcessorNotify = 3, kFrontendList = 4, kApiList = 5, kApiOverdue = 6,
    kApiMarkOverdue = 7, kApiGet = 8, kApiUpdate = 9, kApiComplete = 10, kApiDelete = 11,
    kFrontendEditGet = 12, kFrontendEdit = 13, kFrontendIndexPost = 14, kProcessorSweep = 15
  };
  // a path with an "{id}" segment (api/tasks/{id}[/markcomplete]) matches a canonical lower-case
  // GUID there (the route's key); other spellings (upper case, braces) are Python's
  bool pattern = false;
  int id = 0;
  int kind = 0;
  std::string method, path;
  ev::Endpoint sidecar;
  // protocol=grpc: the store and publish calls go to the sidecar's gRPC port (`sidecar` is
  // then that endpoint) as dapr.proto.runtime.v1.Dapr SaveState / PublishEvent /
  // QueryStateAlpha1 -- the transport of the reference's DaprClient for them
  // (TasksStoreManager.cs:35,61,155); the messages carry the component names below
  bool grpc = false;
  std::string store, pubsub, topic;
  std::string token;            // dapr-api-token, when the app has one
  double timeout_s = 60;
  double sample_rate = 1.0;     // the app tracer's rate for new traces
  // kFrontendCreate: the Create page's post -> invoke the API -> 302
  std::string af_key, af_cookie, id_cookie, invoke_target;
  // kApiCreate: POST api/tasks -> state save -> publish -> 201
  std::string save_target, publish_target, log_category;
  std::string log_prefix;  // '{"level":..,"role":..,"category":..' of the process's JSON sink, or ""
  // from the Python definitions: the answer's status, content type and Location; the log lines
  int status = 0;
  std::string content_type;
  Template location, log_save, log_publish, log_notify;
  // kFrontendList: GET Tasks/Index -> invoke GET api/tasks?createdBy= -> the page, compiled from
  // the Jinja templates (page slots: created_by, af_token, rows; row slots: task_id, task_name,
  // task_assigned_to, due -- one row per (isCompleted, isOverDue))
  std::string list_target;
  Pieces page, rows[4];
  // kApiList: GET api/tasks?createdBy= -> state query (the manager's query text around the
  // JSON-encoded creator) -> the TaskModel array newest first
  std::string query_target, query_prefix, query_suffix;
  // kApiOverdue: GET api/overduetasks[?limit=] -> the manager's range query (fields: the local
  // midnight, the page size) -> the TaskModel page oldest first + whether the store has more
  Template overdue_query, log_overdue;
  std::string page_default, more_header;
  // kApiMarkOverdue: POST api/overduetasks/markoverdue -> bulk get of the page's ids -> the
  // conditional mark (taskcodec conditional_mark) -> one log line per marked task -> ETag-guarded
  // bulk save, re-read and re-applied on a conflict (up to max_retries passes) -> 200
  std::string bulk_target;
  Template log_mark;
  int max_retries = 5, parallelism = 10;
  // kApiGet / kApiUpdate / kApiComplete / kApiDelete (TasksController.cs:26-75 over
  // TasksStoreManager.cs:40-99): the state read (get_target + key over HTTP), the ETag-guarded
  // save (save_target), the delete (delete_target + key), the assignee-change publish
  // (publish_target); `log_op`: the operation's log line (field: id), `missing`: the answer for a
  // task that is not there (404 / 400)
  std::string get_target, delete_target;
  Template log_op;
  int missing = 404;
  // kFrontendEditGet: GET Tasks/Edit/{id} -> invoke GET api/tasks/{id} -> the Edit page from the
  // template's pieces (slots af_token, task_id, task_name, task_assigned_to, due);
  // kFrontendEdit: POST Tasks/Edit/{id} -> invoke PUT api/tasks/{id} -> 302; kFrontendIndexPost:
  // POST Tasks/Index?handler=complete|delete&id= -> invoke PUT .../markcomplete | DELETE -> 302.
  // `invoke_target`: the API's invoke prefix (".../method/api/tasks/")
  Pieces edit_page;
  // kProcessorNotify: the tasksaved subscription in the notifier's log mode -> log line -> 200
  // kProcessorSweep: the cron job (ScheduledTasksManagerController.cs:19-46, services/processor/
  // app.py check_overdue_tasks_job) -> GET api/overduetasks[?limit=] through the sidecar -> the
  // page filtered and cut into chunks (taskcodec overdue_filter) -> concurrent POST markoverdue
  // per chunk -> the next page while the API reports more -> the job's JSON summary
  std::string sweep_get, sweep_mark;
  int sweep_page = 0, sweep_max_pages = 100000, sweep_chunk = 0, sweep_empty_limit = 3;
  Template log_triggered, log_retrieved, log_marking;
  std::vector<double> bounds;   // the request-latency histogram's buckets (seconds)
  ::taskcodec::Entropy rng;       // loop thread only

  struct Stat {
    uint64_t n = 0;
    double sum = 0;
    std::vector<uint64_t> buckets;  // bounds.size() + 1
  };
  std::mutex mu;
  std::map<int, Stat> stats;  // by status, since the last take

  void record(int status, double secs) {
    size_t b = (size_t)(std::lower_bound(bounds.begin(), bounds.end(), secs) - bounds.begin());
    std::lock_guard<std::mutex> g(mu);
    Stat& st = stats[status];
    if (st.buckets.empty()) st.buckets.assign(bounds.size() + 1, 0);
    ++st.n;
    st.sum += secs;
    ++st.buckets[b];
  }
};

class AppHost {
 public:
  AppHost() {
    ev::reserve_fd_table();  // no fd-table growth (RCU waits) once the I/O thread runs
    to_py_ = ::eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    auto w = std::make_shared<Waker>(*this);
    w->fd = ::eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    to_loop_ = w->fd;
    loop_.add(w, EPOLLIN);
  }
  ~AppHost() {
    stop();
    ::close(to_py_);
    if (trace_) std::fclose(trace_);
  }

  int event_fd() const { return to_py_; }

  void start() {
    if (thread_.joinable()) return;
    if (const char* p = std::getenv("TT_STALL_LOG"); p && *p) trace_ = std::fopen(p, "a");
    thread_ = std::thread([this] {
      pthread_setname_np(pthread_self(), "tt-apphost-io");  // per-thread CPU reports
      if (!trace_) {
        loop_.run();
        return;
      }
      // diagnostics: loop iterations > 100 ms apart and slow command batches
      ev::GapTracer gaps("apphost");
      gaps.attach(loop_);
      loop_.run([&gaps](double now) { gaps.tick(now); });
    });
  }

  void stop() {
    if (!thread_.joinable()) return;
    post([this] { loop_.stop(); });
    thread_.join();
  }

  // Bind a listener for server group `server`; returns the TCP port (0 for Unix sockets).
  // `cert` / `key` (PEM files): serve HTTPS on it (Kestrel's https endpoint).
  int listen(int server, const std::string& endpoint, const std::string& cert = "", const std::string& key = "") {
    auto ep = ev::Endpoint::parse(endpoint);
    std::shared_ptr<ev::TlsContext> tls;
    if (!cert.empty()) {
      ev::TlsConfig tc;
      tc.cert = cert;
      tc.key = key;
      tc.verify_peer = false;
      tls = std::make_shared<ev::TlsContext>(tc, true);
    }
    if (!thread_.joinable()) return listen_now(server, ep, tls);
    auto p = std::make_shared<std::promise<int>>();
    auto f = p->get_future();
    post([this, server, ep, p, tls] {
      try {
        p->set_value(listen_now(server, ep, tls));
      } catch (...) {
        p->set_exception(std::current_exception());
      }
    });
    return f.get();
  }

  // Stop accepting on every listener of `server` (open connections finish their requests).
  void close_server(int server) {
    post([this, server] {
      auto it = listeners_.find(server);
      if (it == listeners_.end()) return;
      for (auto& l : it->second)
        if (!l->dead) loop_.remove(l.get());
      listeners_.erase(it);
    });
  }

  // Close the connections `server` accepted (after its in-flight requests were answered).
  void close_connections(int server) {
    post([this, server] {
      auto it = conns_.find(server);
      if (it == conns_.end()) return;
      for (auto& w : it->second)
        if (auto c = w.lock())
          if (!c->dead) loop_.remove(c.get());
      conns_.erase(it);
    });
  }

  // A batch of respond/request operations from one Python loop iteration: one lock, at most
  // one wake-up of the loop thread.
  struct Op {
    bool is_request = false;
    bool is_grpc = false;  // a unary gRPC call: target = ":path", headers = metadata, body = message
    uint64_t id = 0;  // reply token or client request id
    int status = 0;
    std::string endpoint, method, target;
    HeaderList headers;
    std::string body;
    double timeout_s = 0;
  };
  void submit(std::vector<Op>&& ops) {
    post([this, ops = std::move(ops)]() mutable {
      for (auto& op : ops) {
        double t0 = trace_ ? ev::now_s() : 0;
        struct OpTimer {  // diagnostics: one slow operation inside a batch
          AppHost* h;
          double t0;
          bool req;
          ~OpTimer() {
            if (h->trace_ && ev::now_s() - t0 > 0.02) h->note(req ? "op-request-slow" : "op-respond-slow", (ev::now_s() - t0) * 1e3);
          }
        } timer{this, t0, op.is_request};
        if (!op.is_request) {
          auto it = replies_.find(op.id);
          if (it == replies_.end()) continue;
          auto r = std::move(it->second);
          replies_.erase(it);
          r.send(op.status, op.headers, op.body);
          continue;
        }
        uint64_t id = op.id;
        if (op.is_grpc) {
          // RESPONSE: status = grpc-status, headers = metadata + grpc-message, body = message
          grpc_.call(ev::Endpoint::parse(op.endpoint), std::move(op.target), op.headers, op.body, op.timeout_s,
                     [this, id](h2::GrpcResult&& r) {
                       Event e;
                       e.id = id;
                       if (r.err) {
                         e.kind = Event::ERROR;
                         e.err = r.err;
                       } else {
                         e.kind = Event::RESPONSE;
                         e.msg.status = r.status;
                         e.msg.headers = std::move(r.metadata);
                         e.msg.headers.emplace_back("grpc-message", std::move(r.message));
                         e.msg.body = std::move(r.payload);
                       }
                       emit(std::move(e));
                     });
          continue;
        }
        client_.request(ev::Endpoint::parse(op.endpoint), op.method, op.target, op.headers, op.body, op.timeout_s,
                        [this, id](ev::ClientResult&& r) {
                          Event e;
                          e.id = id;
                          if (r.err) {
                            e.kind = Event::ERROR;
                            e.err = r.err;
                          } else {
                            e.kind = Event::RESPONSE;
                            e.msg = std::move(r.resp);
                          }
                          emit(std::move(e));
                        });
      }
    });
  }

  // Called by the Python thread when event_fd() is readable.
  std::vector<Event> drain() {
    uint64_t v;
    while (::read(to_py_, &v, sizeof v) > 0) {
    }
    std::vector<Event> out;
    std::lock_guard<std::mutex> g(ev_mu_);
    out.swap(events_);
    wake_pending_ = false;
    return out;
  }

  size_t pending_replies() const { return pending_replies_.load() + native_inflight_.load(); }

  // Register a native route on listener group `server`; `cfg` holds the route's settings as
  // strings (see NativeRoute; web/native_host.py NativeHttpServer.native_route).  Returns its id.
  int add_route(int server, const std::string& kind, const std::map<std::string, std::string>& cfg,
                const std::vector<double>& bounds) {
    auto r = std::make_shared<NativeRoute>();
    auto get = [&](const char* k) {
      auto it = cfg.find(k);
      return it == cfg.end() ? std::string() : it->second;
    };
    if (kind == "frontend_create") r->kind = NativeRoute::kFrontendCreate;
    else if (kind == "api_create") r->kind = NativeRoute::kApiCreate;
    else if (kind == "processor_notify") r->kind = NativeRoute::kProcessorNotify;
    else if (kind == "frontend_list") r->kind = NativeRoute::kFrontendList;
    else if (kind == "api_list") r->kind = NativeRoute::kApiList;
    else if (kind == "api_overdue") r->kind = NativeRoute::kApiOverdue;
    else if (kind == "api_markoverdue") r->kind = NativeRoute::kApiMarkOverdue;
    else if (kind == "api_get") r->kind = NativeRoute::kApiGet;
    else if (kind == "api_update") r->kind = NativeRoute::kApiUpdate;
    else if (kind == "api_complete") r->kind = NativeRoute::kApiComplete;
    else if (kind == "api_delete") r->kind = NativeRoute::kApiDelete;
    else if (kind == "frontend_edit_get") r->kind = NativeRoute::kFrontendEditGet;
    else if (kind == "frontend_edit") r->kind = NativeRoute::kFrontendEdit;
    else if (kind == "frontend_index_post") r->kind = NativeRoute::kFrontendIndexPost;
    else if (kind == "processor_sweep") r->kind = NativeRoute::kProcessorSweep;
    else throw std::invalid_argument("unknown native route kind: " + kind);
    r->method = get("method");
    r->path = get("path");
    if (!get("sidecar").empty()) r->sidecar = ev::Endpoint::parse(get("sidecar"));
    r->token = get("token");
    if (!get("timeout").empty()) r->timeout_s = std::stod(get("timeout"));
    if (!get("sample_rate").empty()) r->sample_rate = std::stod(get("sample_rate"));
    r->af_key = get("af_key");
    r->af_cookie = get("af_cookie");
    r->id_cookie = get("id_cookie");
    r->invoke_target = get("invoke_target");
    r->save_target = get("save_target");
    r->publish_target = get("publish_target");
    r->log_category = get("log_category");
    r->log_prefix = get("log_prefix");
    r->bounds = bounds;
    if (get("protocol") == "grpc") {
      if (r->kind == NativeRoute::kFrontendCreate || r->kind == NativeRoute::kFrontendList ||
          r->kind == NativeRoute::kProcessorNotify || r->kind >= NativeRoute::kFrontendEditGet)  // sweep too
        throw std::invalid_argument("only the API's store routes speak gRPC");
      r->grpc = true;
      r->store = get("store");
      r->pubsub = get("pubsub");
      r->topic = get("topic");
      if (r->store.empty() || (r->kind == NativeRoute::kApiCreate && (r->pubsub.empty() || r->topic.empty())))
        throw std::invalid_argument("a gRPC route needs its store (and pubsub / topic)");
    } else if (!get("protocol").empty() && get("protocol") != "http") {
      throw std::invalid_argument("native route protocol must be http or grpc");
    }
    if (r->method.empty() || r->path.empty()) throw std::invalid_argument("a native route needs a method and a path");
    // every status, Location and log line comes from the Python definition: a route without
    // them is refused rather than answering with text of its own
    if (get("status").empty()) throw std::invalid_argument("a native route needs the handler's status");
    r->status = std::stoi(get("status"));
    r->content_type = get("content_type");
    if (r->kind == NativeRoute::kProcessorNotify) {
      r->log_notify = Template::compile(get("log_notify"), get("log_notify_args"));
    } else if (r->kind == NativeRoute::kFrontendList) {
      r->list_target = get("list_target");
      r->page = Pieces::parse(get("page"), {"created_by", "af_token", "rows"});
      const char* combos[4] = {"row_ff", "row_ft", "row_tf", "row_tt"};  // (isCompleted, isOverDue)
      for (int i = 0; i < 4; ++i)
        r->rows[i] = Pieces::parse(get(combos[i]), {"task_id", "task_name", "task_assigned_to", "due"});
      if (r->list_target.empty() || r->af_key.empty()) throw std::invalid_argument("frontend_list needs its target and key");
    } else if (r->kind == NativeRoute::kApiOverdue) {
      r->query_target = get("query_target");
      r->overdue_query = Template::compile(get("query"), get("query_args"), {"midnight", "page"});
      r->log_overdue = Template::compile(get("log_overdue"), get("log_overdue_args"), {"midnight", "page"});
      r->page_default = get("page_default");
      r->more_header = get("more_header");
      if (r->query_target.empty() || get("query").empty() || r->page_default.empty() || r->more_header.empty() ||
          get("log_overdue").empty())
        throw std::invalid_argument("api_overdue needs its query, page size, log template and header");
    } else if (r->kind == NativeRoute::kProcessorSweep) {
      r->sweep_get = get("overdue_target");
      r->sweep_mark = get("mark_target");
      r->more_header = get("more_header");
      r->sweep_page = std::stoi(get("page").empty() ? "0" : get("page"));
      if (!get("max_pages").empty()) r->sweep_max_pages = std::stoi(get("max_pages"));
      r->sweep_chunk = std::stoi(get("chunk").empty() ? "0" : get("chunk"));
      if (!get("empty_more_limit").empty()) r->sweep_empty_limit = std::stoi(get("empty_more_limit"));
      r->log_triggered = Template::compile(get("log_triggered"), "v", {"v"});
      r->log_retrieved = Template::compile(get("log_retrieved"), "v", {"v"});
      r->log_marking = Template::compile(get("log_marking"), "v", {"v"});
      if (r->sweep_get.empty() || r->sweep_mark.empty() || r->more_header.empty() || r->sweep_chunk <= 0 ||
          (r->sidecar.path.empty() && r->sidecar.host.empty()))
        throw std::invalid_argument("processor_sweep needs its targets, the more-results header and a chunk size");
    } else if (r->kind >= NativeRoute::kFrontendEditGet) {
      if (r->invoke_target.empty() || r->af_key.empty() || r->af_cookie.empty())
        throw std::invalid_argument("a frontend page route needs its invoke target and antiforgery settings");
      if (r->kind == NativeRoute::kFrontendEditGet)
        r->edit_page = Pieces::parse(get("page"), {"af_token", "task_id", "task_name", "task_assigned_to", "due"});
      if (r->kind != NativeRoute::kFrontendIndexPost) {
        if (r->path.find("{id}") == std::string::npos) throw std::invalid_argument("an Edit route needs an {id} path");
        r->pattern = true;
      }
      if (r->kind != NativeRoute::kFrontendEditGet) r->location = Template::compile(get("location"), "");
    } else if (r->kind >= NativeRoute::kApiGet && r->kind <= NativeRoute::kApiDelete) {
      r->get_target = get("get_target");
      r->delete_target = get("delete_target");
      r->log_op = Template::compile(get("log_op"), get("log_op_args"), {"id"});
      if (!get("max_retries").empty()) r->max_retries = std::stoi(get("max_retries"));
      if (!get("missing").empty()) r->missing = std::stoi(get("missing"));
      if (r->kind == NativeRoute::kApiUpdate) {
        r->log_publish = Template::compile(get("log_publish"), get("log_publish_args"));
        if (get("log_publish").empty() || r->publish_target.empty())
          throw std::invalid_argument("api_update needs the publish target and the manager's log template");
      }
      if (r->get_target.empty() || get("log_op").empty() ||
          ((r->kind == NativeRoute::kApiUpdate || r->kind == NativeRoute::kApiComplete) && r->save_target.empty()) ||
          (r->kind == NativeRoute::kApiDelete && r->delete_target.empty()) || r->path.find("{id}") == std::string::npos)
        throw std::invalid_argument("a task route needs its targets, its log template and an {id} path");
      if (r->grpc && r->store.empty()) throw std::invalid_argument("a gRPC task route needs its store");
      r->pattern = true;
    } else if (r->kind == NativeRoute::kApiMarkOverdue) {
      r->bulk_target = get("bulk_target");
      r->log_mark = Template::compile(get("log_mark"), get("log_mark_args"), {"id"});
      if (!get("max_retries").empty()) r->max_retries = std::stoi(get("max_retries"));
      if (!get("parallelism").empty()) r->parallelism = std::stoi(get("parallelism"));
      if (r->bulk_target.empty() || r->save_target.empty() || get("log_mark").empty() ||
          (!r->grpc && r->store.empty() && false))
        throw std::invalid_argument("api_markoverdue needs its bulk-get and save targets and its log template");
    } else if (r->kind == NativeRoute::kApiList) {
      r->query_target = get("query_target");
      r->query_prefix = get("query_prefix");
      r->query_suffix = get("query_suffix");
      if (r->query_target.empty() || r->query_prefix.empty()) throw std::invalid_argument("api_list needs its query");
    } else {
      r->location = Template::compile(get("location"), get("location_args"));
    }
    if (r->kind == NativeRoute::kApiCreate) {
      r->log_save = Template::compile(get("log_save"), get("log_save_args"));
      r->log_publish = Template::compile(get("log_publish"), get("log_publish_args"));
      if (get("log_save").empty() || get("log_publish").empty())
        throw std::invalid_argument("api_create needs the manager's log templates");
    }
    if (r->kind == NativeRoute::kProcessorNotify && get("log_notify").empty())
      throw std::invalid_argument("processor_notify needs the notifier's log template");
    auto p = std::make_shared<std::promise<int>>();
    auto f = p->get_future();
    post([this, server, r, p] {
      r->id = next_route_++;
      routes_[server].push_back(r);
      all_routes_.push_back(r);
      {
        std::lock_guard<std::mutex> g(routes_mu_);
        all_routes_snapshot_ = all_routes_;
      }
      p->set_value(r->id);
    });
    if (!thread_.joinable()) run_commands();
    return f.get();
  }

  struct RouteStat {
    int route = 0, status = 0;
    uint64_t n = 0;
    double sum = 0;
    std::vector<uint64_t> buckets;
  };
  // The native routes' request counts and latencies since the last call (then reset).
  std::vector<RouteStat> take_route_stats() {
    std::vector<std::shared_ptr<NativeRoute>> rs;
    {
      std::lock_guard<std::mutex> g(routes_mu_);
      rs = all_routes_snapshot_;
    }
    std::vector<RouteStat> out;
    for (auto& r : rs) {
      std::map<int, NativeRoute::Stat> st;
      {
        std::lock_guard<std::mutex> g(r->mu);
        st.swap(r->stats);
      }
      for (auto& [status, x] : st) out.push_back({r->id, status, x.n, x.sum, std::move(x.buckets)});
    }
    return out;
  }

 private:
  struct Waker : ev::IoObj {
    explicit Waker(AppHost& h) : host(h) {}
    AppHost& host;
    void on_event(uint32_t) override {
      uint64_t v;
      while (::read(fd, &v, sizeof v) > 0) {
      }
      host.run_commands();
    }
  };

  ev::Loop loop_;
  ev::Client client_{loop_};
  h2::GrpcClient grpc_{loop_};
  FILE* trace_ = nullptr;

  void note(const char* what, double ms, size_t n = 0) {
    std::fprintf(trace_, "{\"what\": \"%s\", \"ms\": %.2f, \"n\": %zu, \"pid\": %d, \"wall\": %.4f}\n", what, ms, n,
                 (int)::getpid(),
                 std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count());
    std::fflush(trace_);
  }
  std::thread thread_;
  int to_py_ = -1;
  int to_loop_ = -1;

  std::mutex cmd_mu_;
  std::vector<std::function<void()>> cmds_;
  std::mutex ev_mu_;
  std::vector<Event> events_;
  bool wake_pending_ = false, flush_armed_ = false;  // under ev_mu_

  // loop-thread state
  std::unordered_map<uint64_t, ev::Reply> replies_;
  uint64_t next_token_ = 1;
  std::atomic<size_t> pending_replies_{0};
  std::unordered_map<int, std::vector<std::shared_ptr<ev::IoObj>>> listeners_;
  std::unordered_map<int, std::vector<std::weak_ptr<ev::ServerConn>>> conns_;
  std::unordered_map<int, std::unique_ptr<ev::Handler>> handlers_;
  std::unordered_map<int, std::vector<std::shared_ptr<NativeRoute>>> routes_;  // loop thread
  std::vector<std::shared_ptr<NativeRoute>> all_routes_;                       // loop thread
  std::mutex routes_mu_;
  std::vector<std::shared_ptr<NativeRoute>> all_routes_snapshot_;  // for take_route_stats
  int next_route_ = 1;
  std::atomic<size_t> native_inflight_{0};
  uint64_t rng_s_[2] = {0, 0};

  // -- native routes ---------------------------------------------------------------------
  uint64_t next_random() {  // xorshift128+ (trace and span ids, the sampler's draw)
    if (rng_s_[0] == 0 && rng_s_[1] == 0) {
      if (getrandom(rng_s_, sizeof rng_s_, 0) != (ssize_t)sizeof rng_s_ || (rng_s_[0] | rng_s_[1]) == 0)
        rng_s_[0] = 0x9e3779b97f4a7c15ull ^ (uint64_t)ev::now_s();
    }
    uint64_t a = rng_s_[0];
    const uint64_t b = rng_s_[1];
    rng_s_[0] = b;
    a ^= a << 23;
    rng_s_[1] = a ^ b ^ (a >> 17) ^ (b >> 26);
    return rng_s_[1] + b;
  }
  static void hex_to(std::string& out, uint64_t v) {
    static const char* d = "0123456789abcdef";
    for (int i = 60; i >= 0; i -= 4) out += d[(v >> i) & 15];
  }
  std::string new_id(int words) {
    std::string s;
    s.reserve(16 * words);
    for (int i = 0; i < words; ++i) {
      uint64_t v = next_random();
      if (v == 0) v = 1;  // all-zero ids are invalid
      hex_to(s, v);
    }
    return s;
  }
  static const std::string* header(const Message& m, std::string_view name) {
    for (auto& kv : m.headers)
      if (kv.first == name) return &kv.second;
    return nullptr;
  }
  static bool is_hex(std::string_view v) {
    for (char c : v)
      if (!((c >= '0' && c <= '9') || (c >= 'a' && c <= 'f'))) return false;
    return true;
  }

  // The request's trace context, the way the Python middleware reads it
  // (telemetry/tracing.py parse_traceparent + Tracer.start_span).  0: serve natively in trace
  // `tid` (the route's span is new, unsampled); 1: the Python pipeline records this one;
  // 2: a new trace the sampler picked -- Python, marked so that it samples it.
  int trace_context(const NativeRoute& r, const Message& m, std::string& tid) {
    const std::string* tp = header(m, "traceparent");
    if (tp) {
      std::string_view v(*tp);
      while (!v.empty() && (v.front() == ' ' || v.front() == '\t')) v.remove_prefix(1);
      while (!v.empty() && (v.back() == ' ' || v.back() == '\t')) v.remove_suffix(1);
      // version(2)-trace(32)-span(16)-flags(2), lowercase hex; anything else goes to Python
      if (v.size() == 55 && v[2] == '-' && v[35] == '-' && v[52] == '-' && is_hex(v.substr(0, 2)) &&
          is_hex(v.substr(3, 32)) && is_hex(v.substr(36, 16)) && is_hex(v.substr(53, 2)) &&
          v.substr(3, 32) != std::string(32, '0') && v.substr(36, 16) != std::string(16, '0')) {
        int flags = ::formcodec::hexval(v[53]) * 16 + ::formcodec::hexval(v[54]);
        if (flags & 1) return 1;
        tid.assign(v.substr(3, 32));
        return 0;
      }
      return 1;
    }
    if (r.sample_rate >= 1.0) return 2;
    if (r.sample_rate > 0 && (double)(next_random() >> 11) * 0x1.0p-53 < r.sample_rate) return 2;
    tid = new_id(2);
    return 0;
  }

  struct NativeJob {
    std::shared_ptr<NativeRoute> route;
    Message req;  // kept for a hand-over to Python
    ev::Reply reply;
    int server = 0;
    double t0 = 0;
    std::string trace_id, span_id, traceparent;
    ev::HeaderList out_headers;  // traceparent, token, content-type: the SDK's unsampled call
    ev::HeaderList grpc_md;      // gRPC routes: traceparent, token (the SDK's call metadata)
    std::vector<std::string> pending;  // kApiMarkOverdue: the ids this pass reads
    int pass = 0;
    std::string key;                   // task routes: the {id} of the path
    ::taskcodec::Update upd;           // kApiUpdate: the bound body
    ev::HeaderList plain_headers;      // HTTP GET / DELETE: traceparent, token (no content type)
    ::taskcodec::Created task;
    struct Sweep {                     // kProcessorSweep: the job's loop state
      std::string run_at_iso, run_day;
      long long retrieved = 0, marked = 0, pages = 0, empty_more = 0;
      double t_query = 0, t_mark = 0, t_mark0 = 0;
      size_t outstanding = 0, failed_at = SIZE_MAX;
      ev::ClientResult failure;
      long long n_page = 0, n_kept = 0;
      std::string more;
    };
    std::shared_ptr<Sweep> sweep;
  };

  // the gRPC SDK's metadata on an unsampled call (sdk/grpc_client.py _call_encoded)
  static void grpc_metadata(NativeJob& j) {
    j.grpc_md.emplace_back("traceparent", j.traceparent);
    if (!j.route->token.empty()) j.grpc_md.emplace_back("dapr-api-token", j.route->token);
  }

  void log_event(const NativeRoute& r, const NativeJob& j, std::string message) {
    Event e;
    e.kind = Event::LOG;
    e.err = 20;  // logging.INFO
    if (!r.log_prefix.empty()) {  // telemetry/logging.py BufferedSink.write_fast's JSON line
      char ts[40];
      std::snprintf(ts, sizeof ts, ",\"ts\":%.6f,\"message\":",
                    std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count());
      e.line.reserve(r.log_prefix.size() + message.size() + 120);
      e.line = r.log_prefix;
      e.line += ts;
      tt::escape_to(e.line, message);
      e.line += ",\"traceId\":\"" + j.trace_id + "\",\"spanId\":\"" + j.span_id + "\"}\n";
    }
    e.msg.method = r.log_category;
    e.msg.target = j.trace_id;
    e.msg.reason = j.span_id;
    e.msg.body = std::move(message);
    emit(std::move(e));
  }

  void finish(NativeJob& j, int status, const ev::HeaderList& headers, std::string_view body = {}) {
    j.reply.send(status, headers, body);
    j.route->record(status, ev::now_s() - j.t0);
    native_inflight_.fetch_sub(1);
  }
  // The route cannot decide after all (an answer outside the page's shape): the request goes to
  // Python from scratch, which makes the same calls again (the list is a read).
  void decline(NativeJob& j) {
    to_python(j.server, std::move(j.req), std::move(j.reply));
    native_inflight_.fetch_sub(1);
  }

  // One task of GET api/tasks' answer as a Tasks/Index row (services/frontend/rows.py
  // RowRenderer._fields): false when it is outside the shape the compiled row covers.
  static bool render_row(const NativeRoute& r, const tt::Value& d, std::string& out) {
    if (d.t != tt::Value::Object) return false;
    const tt::Value *id = d.get("taskId"), *name = d.get("taskName"), *who = d.get("taskAssignedTo"),
                    *due = d.get("taskDueDate"), *done = d.get("isCompleted"), *over = d.get("isOverDue");
    if (!id || id->t != tt::Value::String || !name || name->t != tt::Value::String || !who ||
        who->t != tt::Value::String || !due || due->t != tt::Value::String || !done || done->t != tt::Value::Bool ||
        !over || over->t != tt::Value::Bool)
      return false;
    const std::string& g = id->s;  // the canonical lowercase GUID text
    if (g.size() != 36) return false;
    for (size_t i = 0; i < 36; ++i) {
      char c = g[i];
      bool dash = i == 8 || i == 13 || i == 18 || i == 23;
      if (dash ? c != '-' : !((c >= '0' && c <= '9') || (c >= 'a' && c <= 'f'))) return false;
    }
    // yyyy-MM-ddTHH:mm:ss[.f{1,7}][Z]: UTC or unspecified, the calendar day is the text's own
    const std::string& t = due->s;
    auto dig = [&](size_t a, size_t n) {
      if (a + n > t.size()) return false;
      for (size_t i = a; i < a + n; ++i)
        if (t[i] < '0' || t[i] > '9') return false;
      return true;
    };
    if (t.size() < 19 || !dig(0, 4) || t[4] != '-' || !dig(5, 2) || t[7] != '-' || !dig(8, 2) || t[10] != 'T' ||
        !dig(11, 2) || t[13] != ':' || !dig(14, 2) || t[16] != ':' || !dig(17, 2))
      return false;
    size_t k = 19;
    if (k < t.size() && t[k] == '.') {
      size_t f = k + 1;
      while (f < t.size() && t[f] >= '0' && t[f] <= '9') ++f;
      if (f - k - 1 < 1 || f - k - 1 > 7) return false;
      k = f;
    }
    if (k < t.size() && t[k] == 'Z') ++k;
    if (k != t.size()) return false;
    const Pieces& p = r.rows[(done->b ? 2 : 0) + (over->b ? 1 : 0)];
    p.render(out, [&](int slot, std::string& o) {
      switch (slot) {
        case 0: o += g; break;
        case 1: html_escape_to(o, name->s); break;
        case 2: html_escape_to(o, who->s); break;
        default: o.append(t, 8, 2), o += '-', o.append(t, 5, 2), o += '-', o.append(t, 0, 4);
      }
    });
    return true;
  }

  // kFrontendList (services/frontend/app.py tasks_index): the identity and antiforgery cookies,
  // the list through the sidecar, the page
  bool frontend_list(const std::shared_ptr<NativeJob>& j, const Message& m) {
    const NativeRoute& r = *j->route;
    const std::string* cookie = header(m, "cookie");
    std::string who, af;
    if (!cookie || !cookie_value(*cookie, r.id_cookie, who) || who.empty() || !cookie_value(*cookie, r.af_cookie, af) ||
        af.empty())
      return false;  // no identity (redirect) or a new antiforgery cookie to hand out: the page
    std::string target = r.list_target;
    url_quote_to(target, who);
    ev::HeaderList h{{"traceparent", j->traceparent}};
    if (!r.token.empty()) h.emplace_back("dapr-api-token", r.token);
    std::string token = ::formcodec::hmac_sha256_hex(r.af_key, af);
    native_inflight_.fetch_add(1);
    client_.request(r.sidecar, "GET", target, h, {}, r.timeout_s,
                    [this, j, who = std::move(who), token = std::move(token)](ev::ClientResult&& res) {
                      if (res.err || res.resp.status >= 300) return hand_over(*j, "invoke", res);
                      const NativeRoute& r = *j->route;
                      const std::string* ct = res.resp.header("content-type");
                      if (ct && !ct->empty() && ct->find("json") == std::string::npos) return decline(*j);
                      std::string rows_html;
                      if (!res.resp.body.empty()) {
                        tt::Value list;
                        try {
                          list = tt::parse(res.resp.body);
                        } catch (const std::exception&) {
                          return decline(*j);
                        }
                        if (list.t != tt::Value::Array) return decline(*j);
                        for (auto& d : list.items)
                          if (!render_row(r, d, rows_html)) return decline(*j);
                      }
                      std::string page;
                      page.reserve(rows_html.size() + 2048);
                      r.page.render(page, [&](int slot, std::string& o) {
                        if (slot == 0) html_escape_to(o, who);
                        else if (slot == 1) o += token;
                        else o += rows_html;
                      });
                      finish(*j, r.status, {{"Content-Type", r.content_type}}, page);
                    });
    return true;
  }

  // kApiOverdue (services/backend_api/app.py get_overdue + TasksStoreManager.overdue_page_json)
  bool api_overdue(const std::shared_ptr<NativeJob>& j, const Message& m) {
    const NativeRoute& r = *j->route;
    std::string page = r.page_default, limit;
    if (query_param(m.target, "limit", limit) && !limit.empty() && limit.size() < 10 &&
        std::all_of(limit.begin(), limit.end(), [](char c) { return c >= '0' && c <= '9'; }) && std::stol(limit) > 0)
      page = std::to_string(std::stol(limit));  // str.isdigit, then int(): leading zeros go
    std::time_t now = std::time(nullptr);
    std::tm lt{};
    localtime_r(&now, &lt);  // DateTime.Today: the local date (containers run in UTC)
    char mid[48];
    std::snprintf(mid, sizeof mid, "%04d-%02d-%02dT00:00:00", lt.tm_year + 1900, lt.tm_mon + 1, lt.tm_mday);
    const std::string midnight = mid;
    auto value = [&](int f) -> const std::string& { return f == 0 ? midnight : page; };
    log_event(r, *j, r.log_overdue.render_with(value));
    native_inflight_.fetch_add(1);
    std::string q = r.overdue_query.render_with(value);
    if (r.grpc) q = daprpb::query_state(r.store, q);
    // the query may take milliseconds (a GPU scan): an ordinary connection, not a pipelined one
    call_step(j, "query", r.query_target, std::move(q), false, [this, j](std::string&& body) {
      const NativeRoute& r = *j->route;
      std::string json, out;
      size_t count = 0;
      bool more = false;
      // the sidecar's answer read straight into the page (sweepcodec.hpp); else via its JSON
      if (!(r.grpc && ::taskcodec::query_pb_tasks(body, out, count, true, &more, false))) {
        if (r.grpc && !daprpb::query_response_json(body, json)) return decline(*j);
        if (!::taskcodec::query_tasks(r.grpc ? json : body, out, count, true, &more, false)) return decline(*j);
      }
      finish(*j, r.status, {{"Content-Type", r.content_type}, {r.more_header, more ? "true" : "false"}}, out);
    });
    return true;
  }

  // kApiMarkOverdue (services/backend_api/app.py mark_overdue + TasksStoreManager
  // mark_overdue_from_body / _mark_conditionally): the page's ids from the native binder, then
  // the conditional mark pass -- the same bulk get, codec, log lines and ETag-guarded bulk save.
  bool api_markoverdue(const std::shared_ptr<NativeJob>& j, const Message& m) {
    const std::string ctype = media_type(m);
    if (!ctype.empty() && ctype.find("json") == std::string::npos) return false;
    std::vector<std::string> ids;
    std::string unused;
    if (!::taskcodec::mark_overdue_ids(m.body, ids) && !::taskcodec::mark_overdue(m.body, ids, unused))
      return false;  // the general binder's
    std::unordered_set<std::string> seen;
    for (auto& id : ids)
      if (seen.insert(id).second) j->pending.push_back(id);  // dict.fromkeys: first occurrence
    native_inflight_.fetch_add(1);
    // the first pass starts once the request is the job's (serve_native moves it in on return)
    loop_.defer([this, j] { mark_pass(j); });
    return true;
  }
  void mark_pass(const std::shared_ptr<NativeJob>& j) {
    const NativeRoute& r = *j->route;
    if (j->pending.empty()) return finish(*j, r.status, {});
    if (j->pass++ >= r.max_retries) return decline(*j);  // kept conflicting: Python's ConcurrencyConflict
    std::string body;
    if (r.grpc) {
      body = daprpb::get_bulk_state(r.store, j->pending, r.parallelism);
    } else {  // sdk/client.py get_bulk_state_raw: {"keys":[..],"parallelism":N}, compact
      body = "{\"keys\":[";
      for (size_t i = 0; i < j->pending.size(); ++i) {
        if (i) body += ',';
        tt::escape_to(body, j->pending[i]);
      }
      body += "],\"parallelism\":" + std::to_string(r.parallelism) + "}";
    }
    call_step(j, "bulk", r.bulk_target, std::move(body), false, [this, j](std::string&& got) {
      const NativeRoute& r = *j->route;
      std::string json, bulk, save;
      std::vector<std::string> marked;
      size_t skipped = 0;
      // the bulk get's answer straight into the guarded save (sweepcodec.hpp); else via JSON
      if (!(r.grpc && ::taskcodec::conditional_mark_pb(got, r.store, save, marked, skipped))) {
        if (r.grpc && !daprpb::bulk_state_response_json(got, json)) return decline(*j);
        if (!::taskcodec::conditional_mark(r.grpc ? json : got, bulk, marked, skipped)) return decline(*j);
        if (!marked.empty() && r.grpc && !daprpb::save_state_bulk(r.store, bulk, save)) return decline(*j);
      }
      for (auto& id : marked) log_event(r, *j, r.log_mark.render_with([&](int) -> const std::string& { return id; }));
      if (marked.empty()) return finish(*j, r.status, {});
      j->pending = std::move(marked);
      call_step(
          j, "save", r.save_target, r.grpc ? std::move(save) : std::move(bulk), false,
          [this, j](std::string&&) { finish(*j, j->route->status, {}); },
          [this, j](int status) {  // lost a race on some of them: re-read and re-apply
            if (status != 409 && status != 412) return false;
            mark_pass(j);
            return true;
          });
    });
  }

  // kProcessorSweep (services/processor/app.py check_overdue_tasks_job): the same page loop,
  // filter, chunks, log lines and summary.  A failed call goes to Python as that call's error
  // (hand_over: "fail overdue|mark ..."); a page the native filter does not read goes to Python
  // with the loop's state ("resume <base64 JSON>"), which asks for that page again and goes on
  // from there -- nothing the job did is done twice.
  static std::string py_round2(double v) {  // repr(round(v, 2)) for the job's millisecond fields
    char b[64];
    std::snprintf(b, sizeof b, "%.2f", v);
    std::string s(b);
    while (s.size() > 1 && s.back() == '0' && s[s.size() - 2] != '.') s.pop_back();
    return s;
  }
  bool processor_sweep(const std::shared_ptr<NativeJob>& j, const Message&) {
    const NativeRoute& r = *j->route;
    auto st = std::make_shared<NativeJob::Sweep>();
    struct timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    const time_t sec = ts.tv_sec;
    const long us = ts.tv_nsec / 1000;
    std::tm tm{};
    gmtime_r(&sec, &tm);
    char d[40], t[40], f[40];
    std::snprintf(d, sizeof d, "%04d-%02d-%02d", tm.tm_year + 1900, tm.tm_mon + 1, tm.tm_mday);
    std::snprintf(t, sizeof t, "%02d:%02d:%02d", tm.tm_hour, tm.tm_min, tm.tm_sec);
    std::snprintf(f, sizeof f, ".%06ld", us);
    const std::string frac = us ? f : "";
    st->run_day = d;
    st->run_at_iso = std::string(d) + "T" + t + frac + "+00:00";  // datetime.isoformat()
    const std::string run_at_str = std::string(d) + " " + t + frac + "+00:00";  // str(datetime)
    j->sweep = st;
    native_inflight_.fetch_add(1);
    log_event(r, *j, r.log_triggered.render_with([&](int) -> const std::string& { return run_at_str; }));
    loop_.defer([this, j] { sweep_page(j); });
    return true;
  }
  void sweep_page(const std::shared_ptr<NativeJob>& j) {
    const NativeRoute& r = *j->route;
    auto& st = *j->sweep;
    st.pages += 1;
    const double t0 = ev::now_s();
    client_.request(r.sidecar, "GET", r.sweep_get, j->plain_headers, {}, r.timeout_s,
                    [this, j, t0](ev::ClientResult&& res) {
                      const NativeRoute& r = *j->route;
                      auto& st = *j->sweep;
                      st.t_query += ev::now_s() - t0;
                      if (res.err || res.resp.status >= 300) return hand_over(*j, "overdue", res);
                      size_t n_page = 0, n_kept = 0;
                      std::string kept;
                      std::vector<size_t> starts;
                      if (res.resp.body.empty() ||
                          !::taskcodec::overdue_filter(res.resp.body, st.run_day, n_page, n_kept, kept, &starts))
                        return sweep_resume(*j, true);  // Python's binder reads this page
                      st.retrieved += (long long)n_page;
                      const std::string n = std::to_string(n_page);
                      log_event(r, *j, r.log_retrieved.render_with([&](int) -> const std::string& { return n; }));
                      const std::string* more = res.resp.header(r.more_header);
                      st.more.clear();
                      if (more)
                        for (char c : *more) st.more += ::tt::ascii_lower(c);
                      st.n_page = (long long)n_page;
                      st.n_kept = (long long)n_kept;
                      if (!n_kept) return sweep_next(j);
                      const std::string k = std::to_string(n_kept);
                      log_event(r, *j, r.log_marking.render_with([&](int) -> const std::string& { return k; }));
                      // the chunks, as the module's tasks_overdue_filter_chunks cuts them
                      std::vector<std::string> parts;
                      const size_t body_end = kept.size() - 1;  // the closing ']'
                      const size_t chunk = (size_t)r.sweep_chunk;
                      for (size_t a = 0; a < starts.size(); a += chunk) {
                        const size_t b = std::min(starts.size(), a + chunk);
                        const size_t from = starts[a], to = b < starts.size() ? starts[b] - 1 : body_end;
                        std::string part;
                        part.reserve(to - from + 2);
                        part += '[';
                        part.append(kept, from, to - from);
                        part += ']';
                        parts.push_back(std::move(part));
                      }
                      st.outstanding = parts.size();
                      st.failed_at = SIZE_MAX;
                      st.t_mark0 = ev::now_s();
                      for (size_t i = 0; i < parts.size(); ++i)
                        client_.request(r.sidecar, "POST", r.sweep_mark, j->out_headers, parts[i], r.timeout_s,
                                        [this, j, i](ev::ClientResult&& res) {
                                          auto& st = *j->sweep;
                                          if ((res.err || res.resp.status >= 300) && i < st.failed_at) {
                                            st.failed_at = i;  // every call finishes; the first fails the job
                                            st.failure = std::move(res);
                                          }
                                          if (--st.outstanding) return;
                                          st.t_mark += ev::now_s() - st.t_mark0;
                                          if (st.failed_at != SIZE_MAX) return hand_over(*j, "mark", st.failure);
                                          st.marked += st.n_kept;
                                          sweep_next(j);
                                        },
                                        false);
                    });
  }
  // the loop's exit conditions after a page (the Python handler's, in its order)
  void sweep_next(const std::shared_ptr<NativeJob>& j) {
    const NativeRoute& r = *j->route;
    auto& st = *j->sweep;
    if (r.sweep_page <= 0) return sweep_done(j);
    if (!st.more.empty()) {
      if (st.more != "true" || (st.n_page && !st.n_kept)) return sweep_done(j);
      if (!st.n_page) {
        if (++st.empty_more >= r.sweep_empty_limit) return sweep_done(j);
        if (st.pages >= r.sweep_max_pages) return sweep_done(j);
        loop_.call_later(0.005 * (double)st.empty_more, [this, j] { sweep_page(j); });
        return;
      }
      st.empty_more = 0;
    } else if (st.n_page < r.sweep_page || !st.n_kept) {
      return sweep_done(j);
    }
    if (st.pages >= r.sweep_max_pages) return sweep_done(j);
    sweep_page(j);
  }
  void sweep_done(const std::shared_ptr<NativeJob>& j) {
    const NativeRoute& r = *j->route;
    const auto& st = *j->sweep;
    std::string out = "{\"runAt\":\"" + st.run_at_iso + "\",\"retrieved\":" + std::to_string(st.retrieved) +
                      ",\"markedOverdue\":" + std::to_string(st.marked) + ",\"pages\":" + std::to_string(st.pages) +
                      ",\"emptyMorePages\":" + std::to_string(st.empty_more) +
                      ",\"queryMs\":" + py_round2(st.t_query * 1e3) + ",\"markMs\":" + py_round2(st.t_mark * 1e3) + "}";
    finish(*j, r.status, {{"Content-Type", r.content_type}}, out);
  }
  // Python goes on from here: the page just read is asked for again (a GET), with the counts so far
  void sweep_resume(NativeJob& j, bool redo_page) {
    const auto& st = *j.sweep;
    char tq[40], tm[40];
    std::snprintf(tq, sizeof tq, "%.9f", st.t_query);
    std::snprintf(tm, sizeof tm, "%.9f", st.t_mark);
    std::string state = "{\"runAt\":\"" + st.run_at_iso + "\",\"retrieved\":" + std::to_string(st.retrieved) +
                        ",\"marked\":" + std::to_string(st.marked) +
                        ",\"pages\":" + std::to_string(st.pages - (redo_page ? 1 : 0)) +
                        ",\"emptyMore\":" + std::to_string(st.empty_more) + ",\"queryS\":" + tq +
                        ",\"markS\":" + tm + "}";
    j.req.headers.emplace_back("x-tt-native", "resume " + tt::text::base64(state));
    to_python(j.server, std::move(j.req), std::move(j.reply));
    native_inflight_.fetch_sub(1);
  }

  // kFrontendEditGet / kFrontendEdit / kFrontendIndexPost (services/frontend/app.py edit_get /
  // edit_post / tasks_index_post): the same cookies, antiforgery check and form binding
  // (formcodec.hpp), the same invoke through the sidecar, the same page or 302.  What they do not
  // decide -- no identity, a new antiforgery cookie, a bad token, a binding error, an answer
  // outside the page's shape, a failed invoke -- is the page's.
  bool frontend_page(const std::shared_ptr<NativeJob>& j, const Message& m) {
    const NativeRoute& r = *j->route;
    const std::string* cookie = header(m, "cookie");
    std::string_view path(m.target);
    path = path.substr(0, path.find('?'));
    if (r.kind == NativeRoute::kFrontendEditGet) {
      std::string who, af;
      if (!cookie || !cookie_value(*cookie, r.id_cookie, who) || who.empty() || !cookie_value(*cookie, r.af_cookie, af) ||
          af.empty())
        return false;  // a redirect to the landing page, or a new antiforgery cookie: the page's
      j->key = path_key(r.path, path);
      if (j->key.empty()) return false;
      std::string token = ::formcodec::hmac_sha256_hex(r.af_key, af);
      native_inflight_.fetch_add(1);
      client_.request(r.sidecar, "GET", r.invoke_target + j->key, j->plain_headers, {}, r.timeout_s,
                      [this, j, token = std::move(token)](ev::ClientResult&& res) {
                        if (res.err || res.resp.status >= 300) return hand_over(*j, "invoke", res);
                        std::string page;
                        if (!edit_page_html(*j->route, res.resp.body, token, j->key, page)) return decline(*j);
                        finish(*j, j->route->status, {{"Content-Type", j->route->content_type}}, page);
                      });
      return true;
    }
    const std::string_view ck = cookie ? std::string_view(*cookie) : std::string_view();
    std::string method = "PUT", target, body;
    if (r.kind == NativeRoute::kFrontendEdit) {
      std::string pid = path_key(r.path, path), id;
      if (pid.empty()) return false;
      if (::formcodec::edit_task(m.body, ck, r.af_key, r.af_cookie, pid, body, id) != ::formcodec::Verdict::kOk)
        return false;
      target = r.invoke_target + id;
    } else {
      if (::formcodec::index_post(m.body, ck, r.af_key, r.af_cookie) != ::formcodec::Verdict::kOk) return false;
      std::string handler, id;
      if (!query_param(m.target, "handler", handler) || !query_param(m.target, "id", id)) return false;
      for (auto& c : handler) c = ::tt::ascii_lower(c);
      if (!::taskcodec::is_guid36(id)) return false;  // is_guid's other spellings: the page's
      if (handler == "complete") target = r.invoke_target + id + "/markcomplete";
      else if (handler == "delete") method = "DELETE", target = r.invoke_target + id;
      else return false;  // an unknown handler: the page's 400
    }
    native_inflight_.fetch_add(1);
    auto done = [this, j](ev::ClientResult&& res) {
      if (res.err || res.resp.status >= 300) return hand_over(*j, "invoke", res);
      finish(*j, j->route->status, {{"Location", j->route->location.render({}, {}, {})}});
    };
    if (body.empty()) client_.request(r.sidecar, method, target, j->plain_headers, {}, r.timeout_s, std::move(done), false);
    else client_.request(r.sidecar, method, target, j->out_headers, body, r.timeout_s, std::move(done), false);
    return true;
  }

  // The Edit page for the API's TaskModel answer (edit_get's values: the id, name, assignee and
  // the due date's calendar day for the date input), or false outside the plain shape.
  static bool edit_page_html(const NativeRoute& r, const std::string& body, const std::string& token,
                             const std::string& key, std::string& out) {
    if (body.empty()) return false;  // no such task: the page's 404
    tt::Value d;
    try {
      d = tt::parse(body);
    } catch (const std::exception&) {
      return false;
    }
    if (d.t != tt::Value::Object) return false;
    const tt::Value *id = d.get("taskId"), *name = d.get("taskName"), *who = d.get("taskAssignedTo"),
                    *due = d.get("taskDueDate");
    if (!id || id->t != tt::Value::String || id->s != key || !name || name->t != tt::Value::String || !who ||
        who->t != tt::Value::String || !due || due->t != tt::Value::String)
      return false;
    // yyyy-MM-ddTHH:mm:ss[.f{1,7}][Z] (UTC or unspecified: the calendar day is the text's own)
    const std::string& t = due->s;
    auto dig = [&](size_t a, size_t n) {
      if (a + n > t.size()) return false;
      for (size_t i = a; i < a + n; ++i)
        if (t[i] < '0' || t[i] > '9') return false;
      return true;
    };
    if (t.size() < 19 || !dig(0, 4) || t[4] != '-' || !dig(5, 2) || t[7] != '-' || !dig(8, 2) || t[10] != 'T' ||
        !dig(11, 2) || t[13] != ':' || !dig(14, 2) || t[16] != ':' || !dig(17, 2))
      return false;
    size_t k = 19;
    if (k < t.size() && t[k] == '.') {
      size_t f = k + 1;
      while (f < t.size() && t[f] >= '0' && t[f] <= '9') ++f;
      if (f - k - 1 < 1 || f - k - 1 > 7) return false;
      k = f;
    }
    if (k < t.size() && t[k] == 'Z') ++k;
    if (k != t.size()) return false;
    out.reserve(8192);
    r.edit_page.render(out, [&](int slot, std::string& o) {
      switch (slot) {
        case 0: o += token; break;
        case 1: o += key; break;
        case 2: html_escape_to(o, name->s); break;
        case 3: html_escape_to(o, who->s); break;
        default: o.append(t, 0, 10);
      }
    });
    return true;
  }

  // The {id} of `path` under the route's `pattern` (one "{id}" segment), when it is a canonical
  // lower-case GUID -- the text uuid.UUID(...) prints back, so logs and keys agree; else "".
  static std::string path_key(std::string_view pattern, std::string_view path) {
    size_t at = pattern.find("{id}");
    if (at == std::string_view::npos) return {};
    std::string_view pre = pattern.substr(0, at), post = pattern.substr(at + 4);
    if (path.size() != pre.size() + 36 + post.size() || path.substr(0, pre.size()) != pre ||
        path.substr(pre.size() + 36) != post)
      return {};
    std::string_view g = path.substr(pre.size(), 36);
    for (size_t i = 0; i < 36; ++i) {
      char c = g[i];
      bool dash = i == 8 || i == 13 || i == 18 || i == 23;
      if (dash ? c != '-' : !((c >= '0' && c <= '9') || (c >= 'a' && c <= 'f'))) return {};
    }
    return std::string(g);
  }

  // kApiGet / kApiUpdate / kApiComplete / kApiDelete: the API's single-task routes
  // (services/backend_api/app.py get_task / put_task / mark_complete / delete_task over the
  // manager's get_task_json / update_task_from_body / mark_task_completed_fast / delete_task):
  // the same codec passes, sidecar calls, log lines and answers.
  bool api_task(const std::shared_ptr<NativeJob>& j, const Message& m) {
    const NativeRoute& r = *j->route;
    std::string_view path(m.target);
    path = path.substr(0, path.find('?'));
    j->key = path_key(r.path, path);
    if (j->key.empty()) return false;
    if (r.kind == NativeRoute::kApiUpdate) {
      const std::string ctype = media_type(m);
      if (!ctype.empty() && ctype.find("json") == std::string::npos) return false;
      if (!::taskcodec::bind_update(m.body, j->upd)) return false;  // the general binder's
    }
    log_event(r, *j, r.log_op.render_with([&](int) -> const std::string& { return j->key; }));
    native_inflight_.fetch_add(1);
    loop_.defer([this, j] { task_read(j); });  // once the request is the job's
    return true;
  }

  // The stored task with its ETag (HTTP GET state / gRPC GetState), then the route's step.
  void task_read(const std::shared_ptr<NativeJob>& j) {
    const NativeRoute& r = *j->route;
    if (r.kind != NativeRoute::kApiGet && r.kind != NativeRoute::kApiDelete && j->pass++ >= r.max_retries)
      return decline(*j);  // kept conflicting: Python's ConcurrencyConflict path decides
    auto then = [this, j](std::string&& data, std::string&& etag) {
      const NativeRoute& r = *j->route;
      if (data.empty()) return finish(*j, r.missing, {});
      switch (r.kind) {
        case NativeRoute::kApiGet: {
          std::string out;
          if (!::taskcodec::task_json(data, out)) return decline(*j);
          return finish(*j, r.status, {{"Content-Type", r.content_type}}, out);
        }
        case NativeRoute::kApiDelete: return task_delete(j, etag);
        default: return task_write(j, data, etag);
      }
    };
    if (r.grpc) {
      pb::Writer w;  // GetStateRequest {store_name = 1, key = 2}
      w.str(1, r.store);
      w.str(2, j->key);
      call_step(j, "get", r.get_target, std::move(w.s), false, [then](std::string&& msg) mutable {
        pb::Reader rd(msg);  // GetStateResponse {data = 1, etag = 2}
        uint32_t f, wt;
        std::string_view v, data, etag;
        while (rd.next(f, wt)) {
          if (f == 1 && wt == pb::LEN && rd.bytes(v)) data = v;
          else if (f == 2 && wt == pb::LEN && rd.bytes(v)) etag = v;
          else if (!rd.skip(wt)) break;
        }
        then(std::string(data), std::string(etag));
      });
      return;
    }
    client_.request(r.sidecar, "GET", r.get_target + j->key, j->plain_headers, {}, r.timeout_s,
                    [this, j, then](ev::ClientResult&& res) mutable {
                      if (res.err || res.resp.status >= 300) return hand_over(*j, "get", res);
                      const std::string* e = res.resp.header("etag");
                      then(res.resp.status == 204 ? std::string() : std::move(res.resp.body), e ? std::string(*e) : "");
                    });
  }

  // markcomplete / update: the edited document saved back under the ETag it was read with
  // (first-write), re-read and re-applied on a conflict; an update that changed the assignee
  // (compared like str.lower(); other than ASCII: Python decides) publishes the document.
  void task_write(const std::shared_ptr<NativeJob>& j, const std::string& data, const std::string& etag) {
    const NativeRoute& r = *j->route;
    const bool update = r.kind == NativeRoute::kApiUpdate;
    std::string doc, id, old;
    if (!::taskcodec::edit_task(data, update ? &j->upd : nullptr, !update, doc, id, old)) return decline(*j);
    bool publish = false;
    if (update) {
      int same = ::taskcodec::ascii_ieq(j->upd.assigned_to, old);
      if (same < 0) return decline(*j);
      publish = same == 0;
    }
    // TasksStoreManager._rmw_body: SidecarClient.save_state's body with the ETag and options
    std::string body = "[{\"key\":";
    tt::escape_to(body, j->key);
    if (!etag.empty()) {
      body += ",\"etag\":";
      tt::escape_to(body, etag);
    }
    body += ",\"options\":{\"concurrency\":\"first-write\"},\"value\":";
    body += doc;
    body += "}]";
    std::string msg;
    if (r.grpc && !daprpb::save_state_bulk(r.store, body, msg)) return decline(*j);
    auto saved = [this, j, publish, doc](std::string&&) {
      const NativeRoute& r = *j->route;
      if (!publish) return finish(*j, r.status, {});
      log_event(r, *j, r.log_publish.render(j->key, j->upd.name, j->upd.assigned_to));
      std::string pub = r.grpc ? daprpb::publish_event(r.pubsub, r.topic, doc, "application/json") : doc;
      call_step(j, "publish", r.publish_target, std::move(pub), true,
                [this, j](std::string&&) { finish(*j, j->route->status, {}); });
    };
    call_step(j, "save", r.save_target, r.grpc ? std::move(msg) : std::move(body), false, std::move(saved),
              [this, j](int status) {  // lost a race: re-read and re-apply
                if (status != 409 && status != 412) return false;
                task_read(j);
                return true;
              });
  }

  // delete: guarded by the ETag read; a concurrent change or delete (409 / 412) is fine -- the
  // task is gone or changed, as TasksStoreManager.delete_task treats it
  void task_delete(const std::shared_ptr<NativeJob>& j, const std::string& etag) {
    const NativeRoute& r = *j->route;
    if (r.grpc) {
      pb::Writer w, et;  // DeleteStateRequest {store_name = 1, key = 2, etag = 3 {value = 1}}
      w.str(1, r.store);
      w.str(2, j->key);
      if (!etag.empty()) {
        et.str(1, etag);
        w.len_field(3, et.s);
      }
      call_step(j, "delete", r.delete_target, std::move(w.s), false,
                [this, j](std::string&&) { finish(*j, j->route->status, {}); },
                [this, j](int status) {
                  if (status != 409 && status != 412) return false;
                  finish(*j, j->route->status, {});
                  return true;
                });
      return;
    }
    ev::HeaderList h = j->plain_headers;
    if (!etag.empty()) h.emplace_back("If-Match", etag);
    client_.request(r.sidecar, "DELETE", r.delete_target + j->key, h, {}, r.timeout_s,
                    [this, j](ev::ClientResult&& res) {
                      if (!res.err && (res.resp.status < 300 || res.resp.status == 409 || res.resp.status == 412))
                        return finish(*j, j->route->status, {});
                      hand_over(*j, "delete", res);
                    },
                    false);
  }

  // kApiList (services/backend_api/app.py get_tasks + TasksStoreManager.tasks_by_creator_json)
  bool api_list(const std::shared_ptr<NativeJob>& j, const Message& m) {
    const NativeRoute& r = *j->route;
    std::string who;
    if (!query_param(m.target, "createdBy", who) || who.empty()) return false;
    std::string body = r.query_prefix;
    tt::escape_to(body, who);
    body += r.query_suffix;
    native_inflight_.fetch_add(1);
    if (r.grpc) body = daprpb::query_state(r.store, body);
    call_step(j, "query", r.query_target, std::move(body), false, [this, j](std::string&& res) {
      const NativeRoute& r = *j->route;
      std::string json, out;
      size_t count = 0;
      bool more = false;
      if (!(r.grpc && ::taskcodec::query_pb_tasks(res, out, count, true, &more, true))) {
        if (r.grpc && !daprpb::query_response_json(res, json)) return decline(*j);
        if (!::taskcodec::query_tasks(r.grpc ? json : res, out, count, true, &more, true)) return decline(*j);
      }
      finish(*j, r.status, {{"Content-Type", r.content_type}}, out);
    });
    return true;
  }

  // A failed sidecar call: the request goes to Python with the result attached.
  void hand_over(NativeJob& j, const char* step, const ev::ClientResult& res) {
    std::string note;
    if (res.err) {
      note = std::string("err ") + step + " " + std::to_string(res.err);
    } else {
      note = std::string("fail ") + step + " " + std::to_string(res.resp.status) + " " + tt::text::base64(res.resp.body);
    }
    j.req.headers.emplace_back("x-tt-native", std::move(note));
    to_python(j.server, std::move(j.req), std::move(j.reply));
    native_inflight_.fetch_sub(1);
  }

  void to_python(int server, Message&& m, ev::Reply reply) {
    uint64_t token = next_token_++;
    replies_.emplace(token, std::move(reply));
    Event e;
    e.kind = Event::REQUEST;
    e.id = token;
    e.server = server;
    e.msg = std::move(m);
    emit(std::move(e));
  }

  // The content type as the Python request reads it (web/http.py Request.content_type).
  static std::string media_type(const Message& m) {
    const std::string* ct = header(m, "content-type");
    std::string v = ct ? ct->substr(0, ct->find(';')) : std::string();
    size_t a = v.find_first_not_of(" \t"), b = v.find_last_not_of(" \t");
    v = a == std::string::npos ? std::string() : v.substr(a, b - a + 1);
    for (auto& c : v) c = ::tt::ascii_lower(c);
    return v;
  }

  // kProcessorNotify: sdk/aspnet.py cloud_events_middleware (the envelope unwrapped by the same
  // native pass) + the log-mode TasksNotifierController (services/processor/app.py task_saved).
  bool notify(const std::shared_ptr<NativeRoute>& r, const Message& m, ev::Reply& reply, const std::string& tid) {
    double t0 = ev::now_s();
    std::string ctype = media_type(m);
    std::string_view data(m.body);
    ::taskcodec::Unwrapped u;
    if (ctype == "application/cloudevents+json" && !m.body.empty()) {
      if (!::taskcodec::unwrap_cloudevent(m.body, u)) return false;
      data = u.data;
      ctype = u.content_type.substr(0, u.content_type.find(';'));
      size_t a = ctype.find_first_not_of(" \t"), b = ctype.find_last_not_of(" \t");
      ctype = a == std::string::npos ? std::string() : ctype.substr(a, b - a + 1);
      for (auto& c : ctype) c = ::tt::ascii_lower(c);
    }
    if (!ctype.empty() && ctype.find("json") == std::string::npos) return false;
    std::string name;
    if (!::taskcodec::task_model_name(data, name)) return false;
    NativeJob j;
    j.trace_id = tid;
    j.span_id = new_id(1);
    std::string text = r->log_notify.render({}, name, {});
    log_event(*r, j, text);
    ev::HeaderList h;
    if (!r->content_type.empty()) h.emplace_back("Content-Type", r->content_type);
    reply.send(r->status, h, text);
    r->record(r->status, ev::now_s() - t0);
    return true;
  }

  // true: the route took the request (answered now or later); false: Python serves `m`
  // (possibly marked `x-tt-native: sample`).
  bool serve_native(const std::shared_ptr<NativeRoute>& r, int server, Message& m, ev::Reply& reply) {
    if (m.body.size() > (1u << 20)) return false;
    std::string tid;
    int tc = trace_context(*r, m, tid);
    if (tc == 1) return false;
    if (tc == 2) {
      m.headers.emplace_back("x-tt-native", "sample");
      return false;
    }
    if (r->kind == NativeRoute::kProcessorNotify) return notify(r, m, reply, tid);
    if (r->kind == NativeRoute::kFrontendList || r->kind == NativeRoute::kApiList ||
        r->kind == NativeRoute::kApiOverdue || r->kind == NativeRoute::kApiMarkOverdue ||
        (r->kind >= NativeRoute::kApiGet && r->kind <= NativeRoute::kProcessorSweep)) {
      auto j = std::make_shared<NativeJob>();
      j->route = r;
      j->server = server;
      j->t0 = ev::now_s();
      j->trace_id = std::move(tid);
      j->span_id = new_id(1);
      j->traceparent = "00-" + j->trace_id + "-" + j->span_id + "-00";
      j->out_headers.emplace_back("traceparent", j->traceparent);
      if (!r->token.empty()) j->out_headers.emplace_back("dapr-api-token", r->token);
      j->out_headers.emplace_back("Content-Type", "application/json");
      if (r->grpc) grpc_metadata(*j);
      j->plain_headers.emplace_back("traceparent", j->traceparent);
      if (!r->token.empty()) j->plain_headers.emplace_back("dapr-api-token", r->token);
      bool taken = r->kind == NativeRoute::kFrontendList     ? frontend_list(j, m)
                   : r->kind == NativeRoute::kApiList        ? api_list(j, m)
                   : r->kind == NativeRoute::kApiOverdue     ? api_overdue(j, m)
                   : r->kind == NativeRoute::kApiMarkOverdue ? api_markoverdue(j, m)
                   : r->kind == NativeRoute::kProcessorSweep ? processor_sweep(j, m)
                   : r->kind >= NativeRoute::kFrontendEditGet ? frontend_page(j, m)
                                                             : api_task(j, m);
      if (!taken) return false;
      j->req = std::move(m);
      j->reply = std::move(reply);
      return true;
    }
    auto j = std::make_shared<NativeJob>();
    if (r->kind == NativeRoute::kFrontendCreate) {
      const std::string* cookie = header(m, "cookie");
      std::string json;
      auto v = ::formcodec::create_task(m.body, cookie ? std::string_view(*cookie) : std::string_view(), r->af_key,
                                      r->af_cookie, r->id_cookie, json);
      if (v != ::formcodec::Verdict::kOk) return false;  // the page decides (binding errors, 400)
      j->task.task_json = std::move(json);
    } else {
      const std::string* ct = header(m, "content-type");
      if (ct && !ct->empty()) {
        std::string low(*ct);
        for (auto& c : low) c = ::tt::ascii_lower(c);
        if (low.find("json") == std::string::npos) return false;
      }
      if (!::taskcodec::create(m.body, r->rng, j->task)) return false;
    }
    j->route = r;
    j->server = server;
    j->t0 = ev::now_s();
    j->trace_id = std::move(tid);
    j->span_id = new_id(1);
    j->traceparent = "00-" + j->trace_id + "-" + j->span_id + "-00";
    j->out_headers.emplace_back("traceparent", j->traceparent);
    if (!r->token.empty()) j->out_headers.emplace_back("dapr-api-token", r->token);
    j->out_headers.emplace_back("Content-Type", "application/json");
    if (r->grpc) grpc_metadata(*j);
    j->req = std::move(m);
    j->reply = std::move(reply);
    native_inflight_.fetch_add(1);
    if (r->kind == NativeRoute::kFrontendCreate) {
      std::string body = std::move(j->task.task_json);
      client_.request(r->sidecar, "POST", r->invoke_target, j->out_headers, body, r->timeout_s,
                      [this, j](ev::ClientResult&& res) {
                        if (res.err || res.resp.status >= 300) return hand_over(*j, "invoke", res);
                        const NativeRoute& r = *j->route;
                        finish(*j, r.status, {{"Location", r.location.render({}, {}, {})}});
                      });
      return true;
    }
    log_event(*r, *j, r->log_save.render(j->task.id, j->task.name, j->task.assigned_to));
    // gRPC: SaveStateRequest{store, [StateItem{key, value}]} (sdk/grpc_client.py
    // encode_save_state); HTTP: the state API's body.  The save takes an ordinary connection:
    // the sidecar may hold it for seconds through the store's 429 retries, and a pipelined
    // connection would hold every answer queued behind it
    std::string save = r->grpc ? daprpb::save_state(r->store, j->task.id, j->task.task_json) : std::move(j->task.state_body);
    call_step(j, "save", r->save_target, std::move(save), false, [this, j](std::string&&) {
      const NativeRoute& r = *j->route;
      log_event(r, *j, r.log_publish.render(j->task.id, j->task.name, j->task.assigned_to));
      // the publishes ride the pipelined connections (ev::PipeConn): the broker answers at once,
      // and the creates of one loop iteration share a send(2) and the sidecar's answers a read
      std::string pub = r.grpc ? daprpb::publish_event(r.pubsub, r.topic, j->task.task_json, "application/json")
                               : j->task.task_json;
      call_step(j, "publish", r.publish_target, std::move(pub), true, [this, j](std::string&&) {
        const NativeRoute& r2 = *j->route;
        finish(*j, r2.status, {{"Location", r2.location.render(j->task.id, j->task.name, j->task.assigned_to)}});
      });
    });
    return true;
  }

  // -- the route's sidecar calls, over its protocol -----------------------------------------
  // One sidecar call of a native route: `target` is the HTTP API's path, or the RPC's :path
  // for a gRPC route (`body` its request message).  `done` gets the answer's body (HTTP) or the
  // response message (gRPC); a failure hands the request to Python with the step's result.
  // `pipelined`: an HTTP call that answers at once may share a pipelined connection.
  // `conflict` (optional): offered the HTTP status of a failed call first; true = it handled it.
  using StepDone = std::function<void(std::string&&)>;
  using StepConflict = std::function<bool(int)>;
  void call_step(const std::shared_ptr<NativeJob>& j, const char* step, const std::string& target, std::string body,
                 bool pipelined, StepDone done, StepConflict conflict = nullptr) {
    const NativeRoute& r = *j->route;
    if (r.grpc) {
      grpc_.call(r.sidecar, target, j->grpc_md, body, r.timeout_s,
                 [this, j, step, done = std::move(done), conflict = std::move(conflict)](h2::GrpcResult&& res) {
                   if (!res.err && res.status != 0 && conflict && conflict(grpc_http_status(res))) return;
                   if (res.err || res.status != 0) return grpc_hand_over(*j, step, res);
                   done(std::move(res.payload));
                 });
      return;
    }
    auto cb = [this, j, step, done = std::move(done), conflict = std::move(conflict)](ev::ClientResult&& res) {
      if (!res.err && res.resp.status >= 300 && conflict && conflict(res.resp.status)) return;
      if (res.err || res.resp.status >= 300) return hand_over(*j, step, res);
      done(std::move(res.resp.body));
    };
    if (pipelined) client_.request_pipelined(r.sidecar, "POST", target, j->out_headers, body, r.timeout_s, std::move(cb));
    else client_.request(r.sidecar, "POST", target, j->out_headers, body, r.timeout_s, std::move(cb), false);
  }

  // A failed gRPC call: the HTTP status the SDK's InvocationError carries (the sidecar's
  // dapr-http-status, else the gRPC code's HTTP equivalent: sdk/grpc_client.py _HTTP_OF) and
  // grpc-message as its body; transport errors go over as errno (sdk.client.native_route_failure
  // turns them into the SDK's 503 / 504).
  static int grpc_http_status(const h2::GrpcResult& res) {
    int http = 500;
    switch (res.status) {
      case 3: http = 400; break;
      case 16: http = 401; break;
      case 7: http = 403; break;
      case 5: http = 404; break;
      case 10: http = 409; break;
      case 8: http = 429; break;
      case 12: http = 501; break;
      case 14: http = 503; break;
      case 4: http = 504; break;
      default: break;
    }
    for (auto& kv : res.metadata)
      if (kv.first == "dapr-http-status") http = std::atoi(kv.second.c_str());
    return http;
  }
  void grpc_hand_over(NativeJob& j, const char* step, const h2::GrpcResult& res) {
    std::string note;
    if (res.err) {
      note = std::string("err ") + step + " " + std::to_string(res.err);
    } else {
      note = std::string("fail ") + step + " " + std::to_string(grpc_http_status(res)) + " " +
             tt::text::base64(res.message);
    }
    j.req.headers.emplace_back("x-tt-native", std::move(note));
    to_python(j.server, std::move(j.req), std::move(j.reply));
    native_inflight_.fetch_sub(1);
  }

  void post(std::function<void()> f) {
    bool was_empty;
    {
      std::lock_guard<std::mutex> g(cmd_mu_);
      was_empty = cmds_.empty();
      cmds_.push_back(std::move(f));
    }
    if (was_empty) {
      uint64_t one = 1;
      ssize_t n = ::write(to_loop_, &one, sizeof one);
      (void)n;
    }
  }

  void run_commands() {
    std::vector<std::function<void()>> cmds;
    {
      std::lock_guard<std::mutex> g(cmd_mu_);
      cmds.swap(cmds_);
    }
    double t0 = trace_ ? ev::now_s() : 0;
    for (auto& c : cmds) c();
    if (trace_ && ev::now_s() - t0 > 0.02) note("io-commands-slow", (ev::now_s() - t0) * 1e3, cmds.size());
    pending_replies_.store(replies_.size());
  }

  // Python is woken once per batch of events.  A finished log line (a native route's record on
  // the sink's fast path) is not waited for: it does not wake Python on its own but rides along
  // with the next request / response event, or goes up within kLogFlushS -- the native routes'
  // traffic then costs the Python thread a wake-up per flush, not per request.
  static constexpr double kLogFlushS = 0.005;
  void emit(Event&& e) {
    e.t = ev::now_s();
    const bool lazy = e.kind == Event::LOG && !e.line.empty();
    bool wake = false, arm = false;
    {
      std::lock_guard<std::mutex> g(ev_mu_);
      events_.push_back(std::move(e));
      if (!wake_pending_) {
        if (!lazy) wake = wake_pending_ = true;
        else if (!flush_armed_) arm = flush_armed_ = true;
      }
    }
    if (wake) wake_python();
    if (arm) {
      loop_.call_later(kLogFlushS, [this] {
        bool w = false;
        {
          std::lock_guard<std::mutex> g(ev_mu_);
          flush_armed_ = false;
          if (!events_.empty() && !wake_pending_) w = wake_pending_ = true;
        }
        if (w) wake_python();
      });
    }
  }
  void wake_python() {
    uint64_t one = 1;
    ssize_t n = ::write(to_py_, &one, sizeof one);
    (void)n;
  }

  int listen_now(int server, const ev::Endpoint& ep, std::shared_ptr<ev::TlsContext> tls = nullptr) {
    auto& h = handlers_[server];
    if (!h) {
      h = std::make_unique<ev::Handler>([this, server](Message&& m, ev::Reply reply) {
        // only the host marks requests: a client's own x-tt-native header never reaches Python
        for (size_t i = 0; i < m.headers.size(); ++i)
          if (m.headers[i].first == "x-tt-native") m.headers.erase(m.headers.begin() + (long)i--);
        auto rit = routes_.find(server);
        if (rit != routes_.end() && !rit->second.empty()) {
          std::string_view path(m.target);
          path = path.substr(0, path.find('?'));
          for (auto& r : rit->second)
            if (r->method == m.method && (r->pattern ? !path_key(r->path, path).empty() : r->path == path)) {
              if (serve_native(r, server, m, reply)) return;
              break;
            }
        }
        to_python(server, std::move(m), std::move(reply));
      });
    }
    std::shared_ptr<ev::IoObj> l;
    int port = ev::listen_on(loop_, ep, *h, false, &l, std::move(tls));
    std::static_pointer_cast<ev::Listener>(l)->on_accept = [this, server](const std::shared_ptr<ev::ServerConn>& c) {
      auto& v = conns_[server];
      if (v.size() >= 1024) {  // prune closed connections
        v.erase(std::remove_if(v.begin(), v.end(), [](const std::weak_ptr<ev::ServerConn>& w) {
                  auto p = w.lock();
                  return !p || p->dead;
                }), v.end());
      }
      v.push_back(c);
    };
    listeners_[server].push_back(l);
    return port;
  }
};

}  // namespace tt::apphost
