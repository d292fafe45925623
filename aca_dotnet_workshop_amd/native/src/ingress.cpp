// ttingress: the Container Apps environment's HTTP ingress (the Envoy edge ACA puts in front
// of an app), native, on the epoll HTTP stack (evhttp.hpp) and OpenSSL (tls.hpp).
//
// Reference behaviour it reproduces:
// * external ingress (webapp-frontend-service.bicep:54-57): a public HTTPS listener
//   (`transport: auto`, a certificate issued by the environment CA) load-balancing over the
//   app's ready replicas; plain HTTP on a second listener is answered `301` to the HTTPS URL
//   unless `allowInsecure: true`, then it is proxied too;
// * internal ingress (webapi-backend-service.bicep:94-97): the environment-internal listener
//   (a Unix socket here) proxies, the public one answers `403` -- the module-2 check
//   (docs/aca/02-aca-comm/index.md:278);
// * revision traffic splitting (`traffic: [{revision, weight}]`): a weighted draw picks the
//   revision, then the least-loaded replica of it (fewest requests in flight, ties rotated);
// * a request that fails before anything reached a replica (refused connect) moves on to the
//   next replica; one that failed after the replica may have acted on it is retried only when
//   its method is idempotent -- a createTask POST answers 502 rather than being replayed.
//
// Layout: `threads` event loops, each with its own keep-alive upstream pools, share the public
// port through SO_REUSEPORT (the kernel spreads client connections over them); loop 0 also
// serves the internal socket, the plain-HTTP listener and the control socket.  The control
// plane (platform/ingress.py) pushes the replica set with `PUT /backends` and reads
// `GET /stats`; the in-flight / request / failure totals are also kept in a small shared
// memory file (`statsFile`) the controller's autoscaler (`http` scale rule) reads without a
// round trip.
//
//   ttingress <config.json>
//   {"app": "...", "external": true, "public": "127.0.0.1:0", "tls": {"cert": "...", "key": "..."},
//    "insecure": "127.0.0.1:0", "allowInsecure": false, "internal": "unix:/x/app.ingress.sock",
//    "control": "unix:/x/app.ingress-ctl.sock", "threads": 2, "statsFile": "...", "portFile": "...",
//    "backends": [{"revision": "app--r1", "url": "http://127.0.0.1:8080"}], "weights": {"app--r1": 100}}
#include <fcntl.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/prctl.h>
#include <sys/signalfd.h>
#include <sys/stat.h>

#include <algorithm>
#include <atomic>
#include <fstream>
#include <mutex>
#include <random>
#include <sstream>
#include <thread>

#include "evhttp.hpp"
#include "json.hpp"
#include "pcsample.hpp"
#include "textutil.hpp"

using namespace tt;
using ev::Endpoint;
using ev::HeaderList;
using ev::Message;
using ev::Reply;
using text::json_str;

namespace {

// ------------------------------------------------------------------------------ routes
struct Replica {
  std::string revision, url;
  Endpoint ep;
  std::atomic<int64_t> inflight{0};
  std::atomic<uint64_t> requests{0}, failures{0};
};

// One immutable snapshot of the replica set; swapped whole by the control plane.
struct Routes {
  std::vector<std::shared_ptr<Replica>> replicas;
  std::vector<std::string> revisions;                  // sorted, distinct
  std::vector<std::vector<Replica*>> by_revision;      // parallel to `revisions`
  std::vector<std::pair<std::string, int>> weights;    // revision -> percent
};

// The shared counters (`statsFile`): what the autoscaler and `status` read.
struct SharedStats {
  uint64_t magic;  // "TTINGRS1"
  std::atomic<int64_t> inflight;
  std::atomic<uint64_t> requests, failures, forbidden, redirects;
};
constexpr uint64_t kStatsMagic = 0x315352474e495454ull;

class Ingress {
 public:
  explicit Ingress(const Value& cfg) {
    app_ = cfg.get("app") && cfg.get("app")->t == Value::String ? cfg.get("app")->s : "app";
    external_ = cfg.get("external") && cfg.get("external")->t == Value::Bool && cfg.get("external")->b;
    if (auto* a = cfg.get("allowInsecure"); a && a->t == Value::Bool) allow_insecure_ = a->b;
    stats_ = map_stats(cfg.get("statsFile") && cfg.get("statsFile")->t == Value::String ? cfg.get("statsFile")->s
                                                                                       : std::string());
    std::atomic_store(&routes_, std::shared_ptr<const Routes>(std::make_shared<Routes>()));
    if (cfg.get("backends")) set_routes(cfg);
  }

  const std::string& app() const { return app_; }
  bool external() const { return external_; }
  bool allow_insecure() const { return allow_insecure_; }
  SharedStats& stats() { return *stats_; }
  int public_port = 0;
  bool tls = false;

  std::shared_ptr<const Routes> routes() const { return std::atomic_load(&routes_); }

  // `{"backends": [{"revision", "url"}], "weights": {revision: percent}}`; replicas that stay
  // keep their counters (in-flight requests against them are still counted down).
  void set_routes(const Value& v) {
    std::lock_guard<std::mutex> g(mu_);
    auto old = routes();
    auto r = std::make_shared<Routes>();
    if (auto* bs = v.get("backends"); bs && bs->t == Value::Array)
      for (auto& b : bs->items) {
        auto* rev = b.get("revision");
        auto* url = b.get("url");
        if (!rev || !url || rev->t != Value::String || url->t != Value::String) continue;
        std::shared_ptr<Replica> keep;
        for (auto& o : old->replicas)
          if (o->revision == rev->s && o->url == url->s) keep = o;
        if (!keep) {
          keep = std::make_shared<Replica>();
          keep->revision = rev->s;
          keep->url = url->s;
          keep->ep = Endpoint::parse(url->s);
        }
        r->replicas.push_back(keep);
      }
    for (auto& x : r->replicas)
      if (std::find(r->revisions.begin(), r->revisions.end(), x->revision) == r->revisions.end())
        r->revisions.push_back(x->revision);
    std::sort(r->revisions.begin(), r->revisions.end());
    r->by_revision.resize(r->revisions.size());
    for (auto& x : r->replicas) {
      size_t i = (size_t)(std::find(r->revisions.begin(), r->revisions.end(), x->revision) - r->revisions.begin());
      r->by_revision[i].push_back(x.get());
    }
    if (auto* w = v.get("weights"); w && w->t == Value::Object)
      for (size_t i = 0; i < w->keys.size(); ++i)
        if (w->items[i].t == Value::Number) r->weights.emplace_back(w->keys[i], (int)w->items[i].n);
    std::atomic_store(&routes_, std::shared_ptr<const Routes>(std::move(r)));
  }

  std::string stats_json() const {
    auto r = routes();
    std::string s = "{\"app\":" + json_str(app_) + ",\"external\":" + (external_ ? "true" : "false") +
                    ",\"native\":true,\"inflight\":" + std::to_string(stats_->inflight.load()) +
                    ",\"requests\":" + std::to_string(stats_->requests.load()) +
                    ",\"failures\":" + std::to_string(stats_->failures.load()) +
                    ",\"forbidden\":" + std::to_string(stats_->forbidden.load()) +
                    ",\"redirects\":" + std::to_string(stats_->redirects.load()) + ",\"backends\":[";
    for (size_t i = 0; i < r->replicas.size(); ++i) {
      auto& x = *r->replicas[i];
      s += (i ? ",{" : "{") + std::string("\"revision\":") + json_str(x.revision) + ",\"url\":" + json_str(x.url) +
           ",\"inflight\":" + std::to_string(x.inflight.load()) + ",\"requests\":" +
           std::to_string(x.requests.load()) + ",\"failures\":" + std::to_string(x.failures.load()) + "}";
    }
    s += "],\"weights\":{";
    for (size_t i = 0; i < r->weights.size(); ++i)
      s += (i ? "," : "") + json_str(r->weights[i].first) + ":" + std::to_string(r->weights[i].second);
    return s + "}}";
  }

 private:
  std::string app_;
  bool external_ = false, allow_insecure_ = false;
  std::shared_ptr<const Routes> routes_;
  std::mutex mu_;
  SharedStats* stats_ = nullptr;

  static SharedStats* map_stats(const std::string& path) {
    void* p = MAP_FAILED;
    if (!path.empty()) {
      int fd = ::open(path.c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0644);
      if (fd >= 0 && ::ftruncate(fd, 4096) == 0)
        p = ::mmap(nullptr, 4096, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
      if (fd >= 0) ::close(fd);
    }
    if (p == MAP_FAILED) p = ::mmap(nullptr, 4096, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    auto* s = new (p) SharedStats();
    s->magic = kStatsMagic;
    return s;
  }
};

bool idempotent(std::string_view m) {
  return m == "GET" || m == "HEAD" || m == "OPTIONS" || m == "PUT" || m == "DELETE";
}

std::string problem_json(int status, std::string_view detail) {
  return "{\"type\":\"https://tools.ietf.org/html/rfc9110#section-15." + std::to_string(status / 100) +
         "\",\"title\":" + json_str(ev::reason_phrase(status)) + ",\"status\":" + std::to_string(status) +
         ",\"detail\":" + json_str(detail) + "}";
}

void send_problem(const Reply& r, int status, std::string_view detail) {
  r.send(status, {{"content-type", "application/problem+json; charset=utf-8"}}, problem_json(status, detail));
}

// ------------------------------------------------------------------------------ one loop
class Worker {
 public:
  Worker(Ingress& ing, int index) : ing_(ing), client_(loop_), rng_(0x9e3779b97f4a7c15ull * (uint64_t)(index + 1)) {
    public_ = [this](Message&& m, Reply r) { on_public(std::move(m), std::move(r)); };
    internal_ = [this](Message&& m, Reply r) { forward(std::move(m), std::move(r)); };
    insecure_ = [this](Message&& m, Reply r) {
      if (ing_.allow_insecure()) forward(std::move(m), std::move(r));
      else redirect(m, r);
    };
  }
  ev::Loop& loop() { return loop_; }
  ev::Handler public_, internal_, insecure_, control_;

 private:
  Ingress& ing_;
  ev::Loop loop_;
  ev::Client client_;
  std::mt19937_64 rng_;
  uint64_t rr_ = 0;

  void on_public(Message&& m, Reply r) {
    if (m.method == "GET" && m.target == "/.tt/ingress") {
      r.json(200, ing_.stats_json());
      return;
    }
    if (!ing_.external()) {  // internal ingress: not reachable from outside the environment
      ing_.stats().forbidden.fetch_add(1, std::memory_order_relaxed);
      send_problem(r, 403, ing_.app() + " has internal ingress only");
      return;
    }
    forward(std::move(m), std::move(r));
  }

  void redirect(const Message& m, const Reply& r) {
    ing_.stats().redirects.fetch_add(1, std::memory_order_relaxed);
    std::string host = "127.0.0.1";
    if (auto* h = m.header("host"); h && !h->empty()) {
      host = *h;
      auto c = host.rfind(':');
      if (c != std::string::npos && host.find(']', c) == std::string::npos) host.resize(c);
    }
    r.send(301, {{"location", "https://" + host + ":" + std::to_string(ing_.public_port) + m.target}}, {});
  }

  // Up to three replicas, in the order to try them: a weighted draw picks the revision
  // (`traffic` weights), the least-loaded replica of it goes first, then the rest of that
  // revision and then the other revisions, each rotated so ties spread.
  void pick(const Routes& rt, Replica* out[3], int& n) {
    n = 0;
    if (rt.replicas.empty()) return;
    size_t first = 0;
    int total = 0;
    for (auto& w : rt.weights)
      if (w.second > 0 && std::find(rt.revisions.begin(), rt.revisions.end(), w.first) != rt.revisions.end())
        total += w.second;
    if (total > 0) {
      int x = (int)(rng_() % (uint64_t)total), acc = 0;
      for (auto& w : rt.weights) {
        auto it = std::find(rt.revisions.begin(), rt.revisions.end(), w.first);
        if (w.second <= 0 || it == rt.revisions.end()) continue;
        acc += w.second;
        if (x < acc) {
          first = (size_t)(it - rt.revisions.begin());
          break;
        }
      }
    }
    uint64_t rot = rr_++;
    for (size_t k = 0; k < rt.revisions.size() && n < 3; ++k) {
      size_t ri = k == 0 ? first : (k <= first ? k - 1 : k);
      auto& reps = rt.by_revision[ri];
      size_t m = reps.size();
      if (!m) continue;
      size_t start = (size_t)(rot % m), best = start;
      if (k == 0) {
        int64_t low = reps[start]->inflight.load(std::memory_order_relaxed);
        for (size_t j = 1; j < m; ++j) {
          size_t i = (start + j) % m;
          int64_t f = reps[i]->inflight.load(std::memory_order_relaxed);
          if (f < low) low = f, best = i;
        }
      }
      out[n++] = reps[best];
      for (size_t j = 0; j < m && n < 3; ++j) {
        size_t i = (best + 1 + j) % m;
        if (i != best) out[n++] = reps[i];
      }
    }
  }

  struct Call {
    Message req;
    Reply reply;
    HeaderList headers;
    std::shared_ptr<const Routes> routes;  // keeps the picked replicas alive
    Replica* order[3];
    int n = 0, next = 0;
    int last_err = 0;
  };

  void forward(Message&& m, Reply r) {
    auto& st = ing_.stats();
    st.requests.fetch_add(1, std::memory_order_relaxed);
    auto c = std::make_shared<Call>();
    c->routes = ing_.routes();
    pick(*c->routes, c->order, c->n);
    if (c->n == 0) {
      st.failures.fetch_add(1, std::memory_order_relaxed);
      send_problem(r, 503, ing_.app() + " has no replicas");
      return;
    }
    c->headers.reserve(m.headers.size() + 2);
    for (auto& h : m.headers)
      if (!ev::is_hop_header(h.first) && h.first != "x-forwarded-for" && h.first != "x-forwarded-proto")
        c->headers.push_back(std::move(h));
    c->headers.emplace_back("x-forwarded-for", m.peer.empty() ? std::string("local") : m.peer);
    c->headers.emplace_back("x-forwarded-proto", m.tls ? "https" : "http");
    c->req = std::move(m);
    c->reply = std::move(r);
    st.inflight.fetch_add(1, std::memory_order_relaxed);
    attempt(std::move(c));
  }

  void attempt(std::shared_ptr<Call> c) {
    Replica* rep = c->order[c->next++];
    rep->inflight.fetch_add(1, std::memory_order_relaxed);
    rep->requests.fetch_add(1, std::memory_order_relaxed);
    const Message& q = c->req;
    client_.request(rep->ep, q.method, q.target, c->headers, q.body, 120.0, [this, c, rep](ev::ClientResult&& res) {
      rep->inflight.fetch_sub(1, std::memory_order_relaxed);
      auto& st = ing_.stats();
      if (!res.err) {
        st.inflight.fetch_sub(1, std::memory_order_relaxed);
        c->reply.send(res.resp.status, res.resp.headers, res.resp.body);
        return;
      }
      rep->failures.fetch_add(1, std::memory_order_relaxed);
      c->last_err = res.err;
      // refused / no such socket: nothing reached the replica, any method may go elsewhere;
      // otherwise it may already have acted on the request -- only idempotent ones are replayed
      bool undelivered = res.err == ECONNREFUSED || res.err == ENOENT || res.err == EAGAIN;
      if (!undelivered && !idempotent(c->req.method)) {
        st.inflight.fetch_sub(1, std::memory_order_relaxed);
        st.failures.fetch_add(1, std::memory_order_relaxed);
        send_problem(c->reply, 502, ing_.app() + " replica failed mid-request: " + errno_name(res.err));
        return;
      }
      if (c->next < c->n && !c->reply.abandoned()) {
        attempt(c);
        return;
      }
      st.inflight.fetch_sub(1, std::memory_order_relaxed);
      st.failures.fetch_add(1, std::memory_order_relaxed);
      send_problem(c->reply, 503, "no healthy replica for " + ing_.app() + ": " + errno_name(c->last_err));
    }, /*retry_stale=*/idempotent(q.method));  // a POST a replica may have read is never re-sent
  }

  static std::string errno_name(int e) {
    switch (e) {
      case ECONNREFUSED: return "connection refused";
      case ENOENT: return "no such socket";
      case ETIMEDOUT: return "timed out";
      case ECONNRESET: return "connection reset";
      case EPIPE: return "broken pipe";
      case EIO: return "connection closed mid-response";
      case EPROTO: return "protocol error";
      default: return "errno " + std::to_string(e);
    }
  }
};

class SignalIo : public ev::IoObj {
 public:
  SignalIo(const sigset_t& s, std::function<void()> on) : on_(std::move(on)) {
    fd = signalfd(-1, &s, SFD_NONBLOCK | SFD_CLOEXEC);
  }
  void on_event(uint32_t) override {
    signalfd_siginfo si;
    while (read(fd, &si, sizeof si) == (ssize_t)sizeof si) on_();
  }

 private:
  std::function<void()> on_;
};

const std::string* opt_str(const Value& cfg, const char* k) {
  auto* v = cfg.get(k);
  return v && v->t == Value::String && !v->s.empty() ? &v->s : nullptr;
}

}  // namespace

int main(int argc, char** argv) {
  pcsample::start();  // TT_PC_SAMPLE diagnostics
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s <config.json>\n", argv[0]);
    return 2;
  }
  prctl(PR_SET_PDEATHSIG, SIGTERM);  // the controller owns our lifetime
  signal(SIGPIPE, SIG_IGN);
  sigset_t sigs;
  sigemptyset(&sigs);
  sigaddset(&sigs, SIGTERM);
  sigaddset(&sigs, SIGINT);
  sigprocmask(SIG_BLOCK, &sigs, nullptr);  // before any thread starts: every thread inherits the mask
  std::ifstream in(argv[1]);
  std::stringstream ss;
  ss << in.rdbuf();
  Value cfg;
  try {
    cfg = parse(ss.str());
  } catch (const std::exception& e) {
    std::fprintf(stderr, "ingress: bad config %s: %s\n", argv[1], e.what());
    return 2;
  }
  ev::reserve_fd_table();
  Ingress ing(cfg);
  int nthreads = 1;
  if (auto* t = cfg.get("threads"); t && t->t == Value::Number) nthreads = std::max(1, std::min(64, (int)t->n));
  std::vector<std::unique_ptr<Worker>> workers;
  for (int i = 0; i < nthreads; ++i) workers.push_back(std::make_unique<Worker>(ing, i));
  Worker& w0 = *workers[0];
  w0.control_ = [&ing](Message&& m, Reply r) {
    if (m.method == "GET" && (m.target == "/stats" || m.target == "/.tt/ingress")) return r.json(200, ing.stats_json());
    if ((m.method == "PUT" || m.method == "POST") && m.target == "/backends") {
      try {
        ing.set_routes(parse(m.body));
      } catch (const std::exception& e) {
        return send_problem(r, 400, e.what());
      }
      return r.empty(204);
    }
    send_problem(r, 404, "unknown ingress control route");
  };
  int insecure_port = 0;
  try {
    std::shared_ptr<ev::TlsContext> tls;
    if (auto* t = cfg.get("tls"); t && t->t == Value::Object && opt_str(*t, "cert")) {
      ev::TlsConfig tc;
      tc.cert = *opt_str(*t, "cert");
      tc.key = opt_str(*t, "key") ? *opt_str(*t, "key") : tc.cert;
      tc.verify_peer = false;  // browsers present no client certificate
      tls = std::make_shared<ev::TlsContext>(tc, true);
      ing.tls = true;
    }
    Endpoint pub = Endpoint::parse(opt_str(cfg, "public") ? *opt_str(cfg, "public") : std::string("127.0.0.1:0"));
    ing.public_port = ev::listen_on(w0.loop(), pub, w0.public_, nthreads > 1, nullptr, tls, true);
    pub.port = ing.public_port;
    for (int i = 1; i < nthreads; ++i)  // the same port on every loop: the kernel spreads connections
      ev::listen_on(workers[i]->loop(), pub, workers[i]->public_, true, nullptr, tls, true);
    if (auto* p = opt_str(cfg, "insecure"); p && tls)
      insecure_port = ev::listen_on(w0.loop(), Endpoint::parse(*p), w0.insecure_, false, nullptr, nullptr, true);
    if (auto* p = opt_str(cfg, "internal")) ev::listen_on(w0.loop(), Endpoint::parse(*p), w0.internal_);
    if (auto* p = opt_str(cfg, "control")) ev::listen_on(w0.loop(), Endpoint::parse(*p), w0.control_);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "ingress: %s\n", e.what());
    return 1;
  }
  std::atomic<bool> stopping{false};
  w0.loop().add(std::make_shared<SignalIo>(sigs, [&] { stopping = true; }), EPOLLIN);
  if (auto* pf = opt_str(cfg, "portFile")) {
    std::string tmp = *pf + ".tmp";
    std::ofstream(tmp) << "{\"public\":" << ing.public_port << ",\"insecure\":" << insecure_port
                       << ",\"tls\":" << (ing.tls ? "true" : "false") << ",\"threads\":" << nthreads
                       << ",\"pid\":" << getpid() << "}";
    std::rename(tmp.c_str(), pf->c_str());
  }
  std::vector<std::thread> threads;
  for (int i = 1; i < nthreads; ++i) {
    ev::Loop* lp = &workers[i]->loop();
    threads.emplace_back([lp, &stopping] {
      lp->run([lp, &stopping](double) {
        if (stopping.load()) lp->stop();
      });
    });
  }
  ev::GapTracer gaps("ingress");
  gaps.attach(w0.loop());
  w0.loop().run([&](double t) {
    gaps.tick(t);
    if (stopping.load()) w0.loop().stop();
  });
  for (auto& t : threads) t.join();
  pcsample::dump("ingress");
  return 0;
}
