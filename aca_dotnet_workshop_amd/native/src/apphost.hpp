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
#pragma once

#include <sys/eventfd.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <future>
#include <mutex>
#include <thread>

#include "evhttp.hpp"
#include "h2.hpp"

namespace tt::apphost {

using ev::HeaderList;
using ev::Message;

struct Event {
  enum Kind : int { REQUEST = 0, RESPONSE = 1, ERROR = 2 };
  int kind = REQUEST;
  uint64_t id = 0;      // REQUEST: reply token; RESPONSE/ERROR: the client request id
  int server = 0;       // REQUEST: which listener group (one per Python HttpServer)
  int err = 0;          // ERROR: errno-like code
  double t = 0;         // loop-thread monotonic time when the event was queued (ev::now_s)
  Message msg;
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
      if (!trace_) {
        loop_.run();
        return;
      }
      // diagnostics: loop iterations > 100 ms apart and slow command batches
      ev::GapTracer gaps("apphost");
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
    return out;
  }

  size_t pending_replies() const { return pending_replies_.load(); }

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

  // loop-thread state
  std::unordered_map<uint64_t, ev::Reply> replies_;
  uint64_t next_token_ = 1;
  std::atomic<size_t> pending_replies_{0};
  std::unordered_map<int, std::vector<std::shared_ptr<ev::IoObj>>> listeners_;
  std::unordered_map<int, std::vector<std::weak_ptr<ev::ServerConn>>> conns_;
  std::unordered_map<int, std::unique_ptr<ev::Handler>> handlers_;

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

  void emit(Event&& e) {
    e.t = ev::now_s();
    bool was_empty;
    {
      std::lock_guard<std::mutex> g(ev_mu_);
      was_empty = events_.empty();
      events_.push_back(std::move(e));
    }
    if (was_empty) {
      uint64_t one = 1;
      ssize_t n = ::write(to_py_, &one, sizeof one);
      (void)n;
    }
  }

  int listen_now(int server, const ev::Endpoint& ep, std::shared_ptr<ev::TlsContext> tls = nullptr) {
    auto& h = handlers_[server];
    if (!h) {
      h = std::make_unique<ev::Handler>([this, server](Message&& m, ev::Reply reply) {
        uint64_t token = next_token_++;
        replies_.emplace(token, std::move(reply));
        Event e;
        e.kind = Event::REQUEST;
        e.id = token;
        e.server = server;
        e.msg = std::move(m);
        emit(std::move(e));
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
