// ttloadgen: closed-loop HTTP/1.1 load generator on the native event loop (evhttp.hpp).
//
// Drives `--concurrency` keep-alive request streams round-robin over one or more targets
// (Unix sockets or TCP), in `--steps` steps of `--batch` requests.  With `--until-url` a
// step ends only when the JSON counter at that URL (field `--until-field`) has advanced by
// the batch size -- bench.py uses it to wait until the processor acknowledged every task.
// `--until-base N --until-stride M`: start from counter value N and require an advance of M per
// step (several generators sharing one subscription: M = ranks x batch).  `--until-url` may be
// repeated: the counter is then the sum over every URL (a partitioned broker, one per shard).
// Request bodies come from a file with one body per line (cycled); `--header "name: value"`
// (repeatable) adds request headers (the frontend entry sends its cookies).  Prints one JSON line:
// {"requests", "errors", "elapsed_s", "latency_ms": {"p50", "p99", "max"}}.
// `--follow`: a 3xx answer's Location is fetched next (GET, same target and headers) -- a
// browser following Create's redirect to the task list; its latency is reported apart
// ("follow_latency_ms", expected 200).  `--users N`: "{user}" in header values becomes
// u<k>@bench.local, k cycling over N users (per-user cookies: bounded task lists).
// `--duration S`: one step that stops issuing after S seconds; the --until-url counter must
// then advance by the number of requests issued.  "status_counts" counts answers by status.
// HTTPS targets: `--target https://127.0.0.1:port` with `--tls-ca ca.crt` verifies the server
// certificate (name / address) against that CA, the way a browser trusting it would; without
// `--tls-ca` the connection is encrypted but unverified.
// `--pause-after W` (one generator): after W steps (a warmup) print their JSON line, then wait for
// a line on stdin before the other steps; the final line covers only those.  The connections
// opened in the warmup (TLS handshakes included) carry the later steps, as a browser's would.
// `--threads T` (stepped mode): T generators on T event loops, each with its share of the
// in-flight window and of every step's batch; each waits for the counter to advance by the
// WHOLE batch, so the steps stay in lock-step.  One JSON line merges them.
//
//   ttloadgen --target unix:/path/a.sock --target unix:/path/b.sock 
//       --path /v1.0/invoke/api/method/api/tasks --bodies bodies.txt 
//       --concurrency 128 --batch 1024 --steps 20 --expect 201 
//       --until-url http://127.0.0.1:9000/servicebus/ns/counts?entity=... --until-field completed
#include <algorithm>
#include <cctype>
#include <functional>
#include <csignal>
#include <cstdio>
#include <fstream>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "evhttp.hpp"
#include "json.hpp"

using namespace tt;

namespace {

struct Opts {
  std::vector<ev::Endpoint> targets;
  std::string path = "/", method = "POST", ctype = "application/json", until_field = "completed";
  std::vector<std::string> until_urls;
  std::string tls_ca;
  std::vector<std::string> bodies{""};
  ev::HeaderList headers;
  int concurrency = 64, batch = 512, steps = 1, expect = 0, users = 0, threads = 1, pause_after = 0;
  int body_offset = 0;  // this generator's first body (a thread's share of the cycle)
  bool follow = false;
  double duration_s = 0;
  double until_timeout_s = 0;  // give up waiting for the counter after this long (0 = never)
  // shared environments (bench.py --shared-env): several generators drive one subscription, so
  // the counter's starting point and its advance per step are global, not this generator's own
  long long until_base = -1, until_stride = 0;
};

class Gen {
 public:
  Gen(ev::Loop& loop, Opts o) : loop_(loop), client_(loop), o_(std::move(o)) {
    if (!o_.tls_ca.empty()) {
      ev::TlsConfig tc;
      tc.ca = o_.tls_ca;
      tc.verify_peer = true;
      client_.set_tls(std::make_shared<ev::TlsContext>(tc, false));
    }
    hdrs_.emplace_back("content-type", o_.ctype);
    for (auto& h : o_.headers) {
      if (h.second.find("{user}") != std::string::npos) templated_ = true;
      hdrs_.push_back(h);
    }
    if (o_.duration_s > 0) {  // one open-ended step, closed by the clock
      o_.steps = 1;
      o_.batch = 1 << 30;
    }
    for (std::string u : o_.until_urls) {
      if (u.rfind("http://", 0) == 0) u = u.substr(7);
      auto slash = u.find('/');
      until_.emplace_back(ev::Endpoint::parse(u.substr(0, slash)), slash == std::string::npos ? "/" : u.substr(slash));
    }
  }

  void start() {
    t0_ = ev::now_s();
    if (until_.empty()) begin_step();
    else if (o_.until_base >= 0) {
      base_ = o_.until_base;
      begin_step();
    } else poll_counter([this](long long v) {
      base_ = v;
      begin_step();
    });
  }

  std::string report() const {
    std::vector<double> l = lat_;
    std::sort(l.begin(), l.end());
    auto pct = [&](double p) { return l.empty() ? 0.0 : l[std::min(l.size() - 1, (size_t)(l.size() * p))] * 1e3; };
    char buf[512];
    std::snprintf(buf, sizeof buf,
                  "{\"requests\": %lld, \"errors\": %lld, \"elapsed_s\": %.6f, \"latency_ms\": {\"p50\": %.3f, "
                  "\"p99\": %.3f, \"max\": %.3f}, \"first_error\": ",
                  done_total_, errors_, t1_ - t0_, pct(0.5), pct(0.99), l.empty() ? 0.0 : l.back() * 1e3);
    std::string s = buf;
    escape_to(s, first_error_);
    if (o_.follow) {
      std::vector<double> f = follow_lat_;
      std::sort(f.begin(), f.end());
      auto fp = [&](double p) { return f.empty() ? 0.0 : f[std::min(f.size() - 1, (size_t)(f.size() * p))] * 1e3; };
      std::snprintf(buf, sizeof buf, ", \"follow_requests\": %zu, \"follow_latency_ms\": {\"p50\": %.3f, \"p99\": %.3f, "
                    "\"max\": %.3f}", f.size(), fp(0.5), fp(0.99), f.empty() ? 0.0 : f.back() * 1e3);
      s += buf;
    }
    s += ", \"status_counts\": {";
    bool first = true;
    for (auto& kv : statuses_) {
      s += (first ? "\"" : ", \"") + std::to_string(kv.first) + "\": " + std::to_string(kv.second);
      first = false;
    }
    s += "}";
    // per step: [ms until the last create returned, ms until the step completed (counter reached)]
    s += ", \"steps_ms\": [";
    for (size_t i = 0; i < steps_.size(); ++i) {
      std::snprintf(buf, sizeof buf, "%s[%.2f, %.2f]", i ? ", " : "", steps_[i].first * 1e3, steps_[i].second * 1e3);
      s += buf;
    }
    return s + "]}";
  }
  long long errors() const { return errors_; }

  // Fold another generator's results into this one (--threads).
  void merge(const Gen& g) {
    lat_.insert(lat_.end(), g.lat_.begin(), g.lat_.end());
    follow_lat_.insert(follow_lat_.end(), g.follow_lat_.begin(), g.follow_lat_.end());
    for (auto& kv : g.statuses_) statuses_[kv.first] += kv.second;
    done_total_ += g.done_total_;
    errors_ += g.errors_;
    if (first_error_.empty()) first_error_ = g.first_error_;
    t0_ = std::min(t0_, g.t0_);
    t1_ = std::max(t1_, g.t1_);
    for (size_t i = 0; i < steps_.size() && i < g.steps_.size(); ++i) {  // a step lasts as long as its slowest share
      steps_[i].first = std::max(steps_[i].first, g.steps_[i].first);
      steps_[i].second = std::max(steps_[i].second, g.steps_[i].second);
    }
  }

  // The counter's current value (the sum over every --until-url), read on its own loop.
  static long long read_counter(const Opts& o) {
    ev::Loop loop;
    Opts q = o;
    q.steps = 0;
    Gen g(loop, q);
    long long out = -1;
    g.poll_counter([&](long long v) {
      out = v;
      loop.stop();
    });
    loop.run();
    return out;
  }

 private:
  ev::Loop& loop_;
  ev::Client client_;
  Opts o_;
  ev::HeaderList hdrs_;
  std::vector<std::pair<ev::Endpoint, std::string>> until_;
  double t0_ = 0, t1_ = 0;
  int step_ = 0;
  long long issued_ = 0, done_ = 0, done_total_ = 0, errors_ = 0, base_ = 0, ok_step_ = 0;
  double wait_t0_ = 0;
  size_t rr_ = 0;
  std::vector<double> lat_;
  std::string first_error_;
  std::vector<std::pair<double, double>> steps_;
  double step_t0_ = 0, step_creates_ = 0;
  bool templated_ = false, closed_ = false;
  std::vector<double> follow_lat_;
  std::map<int, long long> statuses_;
  long long user_rr_ = 0;

  ev::HeaderList headers_for(long long k) const {
    ev::HeaderList h = hdrs_;
    std::string u = "u" + std::to_string(o_.users > 0 ? k % o_.users : k) + "@bench.local";
    for (auto& kv : h)
      for (size_t at; (at = kv.second.find("{user}")) != std::string::npos;) kv.second.replace(at, 6, u);
    return h;
  }

  // the redirect's target on the same endpoint: "/path" or "scheme://host[:port]/path"
  static std::string location_path(const std::string& loc) {
    if (!loc.empty() && loc[0] == '/') return loc;
    auto p = loc.find("://");
    if (p == std::string::npos) return "/" + loc;
    auto slash = loc.find('/', p + 3);
    return slash == std::string::npos ? "/" : loc.substr(slash);
  }

  void begin_step() {
    if (step_t0_ > 0) steps_.emplace_back(step_creates_, ev::now_s() - step_t0_);
    if (o_.pause_after > 0 && step_ == o_.pause_after && step_ < o_.steps) pause();
    if (step_ == o_.steps) {
      t1_ = ev::now_s();
      loop_.stop();
      return;
    }
    issued_ = done_ = ok_step_ = 0;
    step_t0_ = ev::now_s();
    int n = std::min(o_.concurrency, o_.batch);
    for (int i = 0; i < n; ++i) issue();
  }

  // the warmup's line, then a blocking wait for the go line (nothing else runs on this loop);
  // the later steps' figures start from zero
  void pause() {
    t1_ = ev::now_s();
    std::printf("%s\n", report().c_str());
    std::fflush(stdout);
    char line[64];
    if (!std::fgets(line, sizeof line, stdin)) {  // the parent went away: stop here
      o_.steps = step_;
      return;
    }
    lat_.clear();
    follow_lat_.clear();
    statuses_.clear();
    steps_.clear();
    done_total_ = errors_ = 0;
    first_error_.clear();
    step_t0_ = 0;
    t0_ = ev::now_s();
  }

  void issue() {
    if (closed_ || issued_ >= o_.batch) return;
    if (o_.duration_s > 0 && ev::now_s() - step_t0_ >= o_.duration_s) {  // the clock closes the step
      closed_ = true;
      o_.batch = (int)std::min<long long>(issued_, 1 << 30);
      if (done_ == issued_) end_step();
      return;
    }
    long long i = issued_++;
    const ev::Endpoint& ep = o_.targets[rr_++ % o_.targets.size()];
    const std::string& body =
        o_.bodies[(size_t)((o_.body_offset + step_ * (long long)o_.batch + i) % (long long)o_.bodies.size())];
    double t = ev::now_s();
    auto hdrs = std::make_shared<ev::HeaderList>(templated_ ? headers_for(user_rr_++) : hdrs_);
    client_.request(ep, o_.method, o_.path, *hdrs, body, 60, [this, t, &ep, hdrs](ev::ClientResult&& r) {
      lat_.push_back(ev::now_s() - t);
      if (!r.err) statuses_[r.resp.status]++;
      bool bad = r.err || (o_.expect && r.resp.status != o_.expect);
      if (bad) note_error(r);
      else ok_step_++;
      const std::string* loc = r.err ? nullptr : r.resp.header("location");
      if (!bad && o_.follow && loc && r.resp.status >= 300 && r.resp.status < 400) {
        double t2 = ev::now_s();
        ev::HeaderList fh;
        for (auto& kv : *hdrs)
          if (kv.first != "content-type") fh.push_back(kv);
        client_.request(ep, "GET", location_path(*loc), fh, {}, 60, [this, t2](ev::ClientResult&& r2) {
          follow_lat_.push_back(ev::now_s() - t2);
          if (!r2.err) statuses_[r2.resp.status]++;
          if (r2.err || r2.resp.status != 200) note_error(r2);
          finish_one();
        });
        return;
      }
      finish_one();
    });
  }

  void note_error(const ev::ClientResult& r) {
    errors_++;
    if (first_error_.empty())
      first_error_ = r.err ? std::string("errno ") + std::to_string(r.err)
                           : "HTTP " + std::to_string(r.resp.status) + " " + r.resp.body.substr(0, 200);
  }

  void finish_one() {
    done_++;
    done_total_++;
    if (done_ == o_.batch || (closed_ && done_ == issued_)) end_step();
    else issue();
  }

  void end_step() {
    step_creates_ = ev::now_s() - step_t0_;
    // the counter advances once per request that succeeded (a failed create sends no message)
    base_ += o_.until_stride > 0 ? o_.until_stride : (o_.duration_s > 0 ? ok_step_ : o_.batch);
    wait_t0_ = ev::now_s();
    ++step_;
    if (until_.empty()) {
      begin_step();
      return;
    }
    wait_counter();
  }

  void wait_counter() {
    poll_counter([this](long long v) {
      if (v >= base_) begin_step();
      else if (o_.until_timeout_s > 0 && ev::now_s() - wait_t0_ > o_.until_timeout_s) {
        errors_++;
        if (first_error_.empty())
          first_error_ = "counter at " + std::to_string(v) + ", wanted " + std::to_string(base_) + " after " +
                         std::to_string((int)o_.until_timeout_s) + " s";
        t1_ = ev::now_s();
        loop_.stop();
      }
      // poll again right away: a timer would add up to its 1 ms granularity to every step's
      // measured duration (one counter read is ~50 us)
      else loop_.defer([this] { wait_counter(); });
    });
  }

  // the counter: the field summed over every --until-url, read concurrently
  void poll_counter(std::function<void(long long)> cb) {
    struct Sum {
      size_t left;
      long long total = 0;
      bool failed = false;
    };
    auto sum = std::make_shared<Sum>();
    sum->left = until_.size();
    for (auto& u : until_)
      client_.request(u.first, "GET", u.second, {}, {}, 30, [this, cb, sum](ev::ClientResult&& r) {
        long long v = -1;
        if (!r.err && r.resp.status == 200) {
          try {
            Value j = parse(r.resp.body);
            if (auto* f = j.get(o_.until_field); f && f->t == Value::Number) v = (long long)f->n;
          } catch (const std::exception&) {
          }
        }
        if (v < 0) sum->failed = true;
        else sum->total += v;
        if (--sum->left) return;
        if (sum->failed) {
          errors_++;
          if (first_error_.empty()) first_error_ = "counter poll failed";
          t1_ = ev::now_s();
          loop_.stop();
          return;
        }
        cb(sum->total);
      });
  }
};

// --session: the whole browser session of SURVEY §2.11's UI, one flow per user at a time (each
// in-flight slot owns user s<slot>, so its task list holds only its own flow's task):
//   POST /Tasks/Create (302) -> GET /Tasks/Index (200: the new task's id from its Edit link, the
//   list is newest first) -> GET /Tasks/Edit/{id} (200) -> POST /Tasks/Edit/{id} (302; a new name,
//   due date and assignee: the API publishes the assignee change) -> POST /Tasks/Index?handler=
//   complete&id= (302) -> POST /Tasks/Index?handler=delete&id= (302) -> GET /Tasks/Index (200)
// (Pages/Tasks/Create.cshtml.cs:30-51, Index.cshtml.cs:23-71, Edit.cshtml.cs:38-71).  `--batch` x
// `--steps` flows in all; the report has every page's latency percentiles (each slot's first flow,
// which opens its connection, is not in them).
class SessionGen {
 public:
  static constexpr int kPages = 7;
  static constexpr const char* kNames[kPages] = {"create", "list", "edit_get", "edit_post", "complete", "delete",
                                                 "list_after"};

  SessionGen(ev::Loop& loop, Opts o, std::string af_token) : loop_(loop), client_(loop), o_(std::move(o)),
                                                            token_(std::move(af_token)) {
    if (!o_.tls_ca.empty()) {
      ev::TlsConfig tc;
      tc.ca = o_.tls_ca;
      tc.verify_peer = true;
      client_.set_tls(std::make_shared<ev::TlsContext>(tc, false));
    }
    total_ = (long long)o_.batch * std::max(1, o_.steps);
  }

  void start() {
    t0_ = ev::now_s();
    int n = (int)std::min<long long>(o_.concurrency, total_);
    for (int s = 0; s < n; ++s) next_flow(s);
    if (n == 0) loop_.stop();
  }

  std::string report() const {
    char buf[512];
    std::snprintf(buf, sizeof buf, "{\"flows\": %lld, \"errors\": %lld, \"elapsed_s\": %.6f, \"pages\": {", done_,
                  errors_, t1_ - t0_);
    std::string s = buf;
    for (int p = 0; p < kPages; ++p) {
      std::vector<double> l = lat_[p];
      std::sort(l.begin(), l.end());
      auto pct = [&](double q) { return l.empty() ? 0.0 : l[std::min(l.size() - 1, (size_t)(l.size() * q))] * 1e3; };
      std::snprintf(buf, sizeof buf, "%s\"%s\": {\"n\": %zu, \"p50\": %.3f, \"p99\": %.3f, \"max\": %.3f}", p ? ", " : "",
                    kNames[p], l.size(), pct(0.5), pct(0.99), l.empty() ? 0.0 : l.back() * 1e3);
      s += buf;
    }
    s += "}, \"status_counts\": {";
    bool first = true;
    for (auto& kv : statuses_) {
      s += (first ? "\"" : ", \"") + std::to_string(kv.first) + "\": " + std::to_string(kv.second);
      first = false;
    }
    s += "}, \"first_error\": ";
    escape_to(s, first_error_);
    return s + "}";
  }
  long long errors() const { return errors_; }

 private:
  struct Flow {
    int slot = 0;
    long long n = 0;
    const ev::Endpoint* ep = nullptr;
    ev::HeaderList get_h, form_h;
    std::string id;
  };
  ev::Loop& loop_;
  ev::Client client_;
  Opts o_;
  std::string token_;
  long long total_ = 0, issued_ = 0, done_ = 0, errors_ = 0;
  size_t rr_ = 0;
  double t0_ = 0, t1_ = 0;
  std::vector<double> lat_[kPages];
  std::map<int, long long> statuses_;
  std::string first_error_;

  static std::string form_escape(const std::string& v) {
    static const char* hx = "0123456789ABCDEF";
    std::string o;
    for (unsigned char c : v) {
      if (std::isalnum(c) || c == '-' || c == '_' || c == '.') o += (char)c;
      else if (c == ' ') o += '+';
      else o += '%', o += hx[c >> 4], o += hx[c & 15];
    }
    return o;
  }

  void next_flow(int slot) {
    if (issued_ >= total_) {
      if (done_ == issued_ && t1_ == 0) {
        t1_ = ev::now_s();
        loop_.stop();
      }
      return;
    }
    auto f = std::make_shared<Flow>();
    f->slot = slot;
    f->n = issued_++;
    f->ep = &o_.targets[rr_++ % o_.targets.size()];
    const std::string user = "s" + std::to_string(slot) + "@bench.local";  // session users: their own lists
    for (auto h : o_.headers) {  // the cookies, with this slot's identity
      for (size_t at; (at = h.second.find("{user}")) != std::string::npos;) h.second.replace(at, 6, user);
      if (h.first != "content-type") f->get_h.push_back(h), f->form_h.push_back(h);
    }
    f->form_h.emplace_back("content-type", "application/x-www-form-urlencoded");
    const std::string& body = o_.bodies[(size_t)(f->n % (long long)o_.bodies.size())];
    page(f, 0, "POST", "/Tasks/Create", body, 302, [this, f](ev::ClientResult&) {
      page(f, 1, "GET", "/Tasks/Index", {}, 200, [this, f](ev::ClientResult& r) {
        const std::string& b = r.resp.body;
        size_t at = b.find("/Tasks/Edit/");
        if (at == std::string::npos || at + 12 + 36 > b.size()) return fail(f, "the new task is not on Tasks/Index");
        f->id = b.substr(at + 12, 36);
        page(f, 2, "GET", "/Tasks/Edit/" + f->id, {}, 200, [this, f](ev::ClientResult& r2) {
          if (r2.resp.body.find(f->id) == std::string::npos) return fail(f, "Tasks/Edit does not show the task");
          std::string n = std::to_string(f->n);
          std::string edit = "__RequestVerificationToken=" + form_escape(token_) + "&TaskUpdate.TaskId=" + f->id +
                             "&TaskUpdate.TaskName=" + form_escape("edited task " + n) +
                             "&TaskUpdate.TaskDueDate=2030-02-0" + std::to_string(1 + f->n % 9) +
                             "&TaskUpdate.TaskAssignedTo=" + form_escape("editor" + std::to_string(f->n % 7) + "@bench.local");
          page(f, 3, "POST", "/Tasks/Edit/" + f->id, edit, 302, [this, f](ev::ClientResult&) {
            std::string af = "__RequestVerificationToken=" + form_escape(token_);
            page(f, 4, "POST", "/Tasks/Index?handler=complete&id=" + f->id, af, 302, [this, f, af](ev::ClientResult&) {
              page(f, 5, "POST", "/Tasks/Index?handler=delete&id=" + f->id, af, 302, [this, f](ev::ClientResult&) {
                page(f, 6, "GET", "/Tasks/Index", {}, 200, [this, f](ev::ClientResult& r3) {
                  if (r3.resp.body.find(f->id) != std::string::npos) return fail(f, "the deleted task is still listed");
                  done_++;
                  next_flow(f->slot);
                });
              });
            });
          });
        });
      });
    });
  }

  void page(const std::shared_ptr<Flow>& f, int p, const char* method, const std::string& path, const std::string& body,
            int expect, std::function<void(ev::ClientResult&)> then) {
    double t = ev::now_s();
    client_.request(*f->ep, method, path, body.empty() && std::string(method) == "GET" ? f->get_h : f->form_h, body, 60,
                    [this, f, p, t, expect, then = std::move(then)](ev::ClientResult&& r) {
                      // each slot's first flow opens its connection (TLS handshake and all): kept
                      // out of the page percentiles, like a browser's already-open connection
                      if (f->n >= (long long)o_.concurrency) lat_[p].push_back(ev::now_s() - t);
                      if (!r.err) statuses_[r.resp.status]++;
                      if (r.err || r.resp.status != expect) {
                        std::string why = std::string(kNames[p]) + ": " +
                                          (r.err ? "errno " + std::to_string(r.err)
                                                 : "HTTP " + std::to_string(r.resp.status) + " " + r.resp.body.substr(0, 160));
                        return fail(f, why);
                      }
                      then(r);
                    });
  }

  void fail(const std::shared_ptr<Flow>& f, const std::string& why) {
    errors_++;
    if (first_error_.empty()) first_error_ = why;
    done_++;
    next_flow(f->slot);
  }
};
constexpr const char* SessionGen::kNames[];

}  // namespace

int main(int argc, char** argv) {
  Opts o;
  std::string session_token;  // --session <antiforgery token>: the browser-session mode
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) {
        std::fprintf(stderr, "missing value for %s\n", a.c_str());
        std::exit(2);
      }
      return argv[++i];
    };
    if (a == "--target") o.targets.push_back(ev::Endpoint::parse(next()));
    else if (a == "--path") o.path = next();
    else if (a == "--method") o.method = next();
    else if (a == "--content-type") o.ctype = next();
    else if (a == "--header") {
      std::string h = next();
      size_t c = h.find(':');
      if (c == std::string::npos) {
        std::fprintf(stderr, "--header wants \"name: value\"\n");
        return 2;
      }
      std::string name = h.substr(0, c), value = h.substr(c + 1);
      for (char& ch : name) ch = (char)std::tolower((unsigned char)ch);
      while (!value.empty() && value.front() == ' ') value.erase(0, 1);
      o.headers.emplace_back(name, value);
    }
    else if (a == "--concurrency") o.concurrency = std::max(1, std::atoi(next().c_str()));
    else if (a == "--batch") o.batch = std::max(1, std::atoi(next().c_str()));
    else if (a == "--steps") o.steps = std::max(0, std::atoi(next().c_str()));
    else if (a == "--expect") o.expect = std::atoi(next().c_str());
    else if (a == "--until-url") o.until_urls.push_back(next());
    else if (a == "--until-field") o.until_field = next();
    else if (a == "--tls-ca") o.tls_ca = next();
    else if (a == "--follow") o.follow = true;
    else if (a == "--users") o.users = std::max(0, std::atoi(next().c_str()));
    else if (a == "--duration") o.duration_s = std::atof(next().c_str());
    else if (a == "--until-timeout") o.until_timeout_s = std::atof(next().c_str());
    else if (a == "--until-base") o.until_base = std::atoll(next().c_str());
    else if (a == "--until-stride") o.until_stride = std::atoll(next().c_str());
    else if (a == "--threads") o.threads = std::max(1, std::atoi(next().c_str()));
    else if (a == "--pause-after") o.pause_after = std::max(0, std::atoi(next().c_str()));
    else if (a == "--session") session_token = next();
    else if (a == "--bodies") {
      std::ifstream in(next());
      o.bodies.clear();
      for (std::string line; std::getline(in, line);)
        if (!line.empty()) o.bodies.push_back(line);
      if (o.bodies.empty()) o.bodies.push_back("");
    } else {
      std::fprintf(stderr, "unknown option %s\n", a.c_str());
      return 2;
    }
  }
  if (o.targets.empty()) {
    std::fprintf(stderr, "at least one --target is required\n");
    return 2;
  }
  signal(SIGPIPE, SIG_IGN);
  if (!session_token.empty()) {
    ev::Loop loop;
    SessionGen g(loop, o, session_token);
    g.start();
    loop.run();
    std::printf("%s\n", g.report().c_str());
    return g.errors() ? 1 : 0;
  }
  int threads = std::min(o.threads, std::min(o.concurrency, o.batch));
  if (o.pause_after > 0 && (threads > 1 || o.duration_s > 0)) {
    std::fprintf(stderr, "--pause-after needs one stepped generator\n");
    return 2;
  }
  if (threads <= 1 || o.duration_s > 0 || o.follow) {  // one generator on this thread
    ev::Loop loop;
    Gen g(loop, o);
    g.start();
    loop.run();
    std::printf("%s\n", g.report().c_str());
    return g.errors() ? 1 : 0;
  }
  // --threads: every generator waits for the counter to advance by the whole batch per step
  if (!o.until_urls.empty() && o.until_base < 0) {
    o.until_base = Gen::read_counter(o);
    if (o.until_base < 0) {
      std::fprintf(stderr, "counter poll failed\n");
      return 1;
    }
  }
  if (o.until_stride <= 0) o.until_stride = o.batch;
  std::vector<std::unique_ptr<ev::Loop>> loops;
  std::vector<std::unique_ptr<Gen>> gens;
  for (int t = 0; t < threads; ++t) {
    Opts q = o;
    q.batch = o.batch / threads + (t < o.batch % threads ? 1 : 0);
    q.concurrency = std::max(1, o.concurrency / threads + (t < o.concurrency % threads ? 1 : 0));
    q.body_offset = t * (o.batch / threads);
    std::rotate(q.targets.begin(), q.targets.begin() + (t % q.targets.size()), q.targets.end());
    loops.push_back(std::make_unique<ev::Loop>());
    gens.push_back(std::make_unique<Gen>(*loops.back(), q));
  }
  std::vector<std::thread> th;
  for (int t = 0; t < threads; ++t)
    th.emplace_back([&, t] {
      gens[t]->start();
      loops[t]->run();
    });
  for (auto& x : th) x.join();
  for (int t = 1; t < threads; ++t) gens[0]->merge(*gens[t]);
  std::printf("%s\n", gens[0]->report().c_str());
  return gens[0]->errors() ? 1 : 0;
}
