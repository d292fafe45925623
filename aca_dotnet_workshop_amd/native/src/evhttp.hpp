// Single-threaded epoll event loop + HTTP/1.1 server and pooled client, used by the native
// sidecar data plane (dataplane.cpp).
//
// * Loop        -- epoll (level-triggered), deferred destruction, coarse timer sweep.
// * MsgParser   -- incremental HTTP/1.1 parser for requests and responses (Content-Length and
//                  chunked bodies, keep-alive, pipelining).
// * Server      -- listeners (TCP and Unix sockets) and connections that dispatch parsed
//                  requests to a handler and write responses back in request order.
// * Client      -- keep-alive connection pools per upstream endpoint (Unix socket or TCP), with
//                  one transparent retry when a reused idle connection turns out to be stale.
//
// Everything runs on one thread; handlers complete asynchronously through Reply objects that
// hold only weak references, so a downstream connection may close while its upstream call is
// still in flight.
#pragma once

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <sys/resource.h>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <string_view>
#include <unordered_map>
#include <utility>
#include <vector>

#include "httpparse.hpp"
#include "tls.hpp"

namespace tt::ev {

inline double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

inline void set_nonblock(int fd) { fcntl(fd, F_SETFL, fcntl(fd, F_GETFL, 0) | O_NONBLOCK); }

// Local (unix) stream sockets carry whole pages of query results and bulk saves (200-300 KB)
// between the apps, the sidecars and the backing.  The default send buffer (net.core.wmem_default,
// ~208 KB) splits such a message over several event-loop turns of a busy reader; asking for more
// gets the kernel's maximum (wmem_max, doubled), enough for one message in one write.
inline void widen_local_sndbuf(int fd) {
  int sz = 4 << 20;
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &sz, sizeof sz);
}

// TCP connections (the sidecars' mutual-TLS mesh, the ingress): no Nagle delay.  With
// TT_TCP_BUF_KB=<n> (an A/B switch; default 0 = the kernel's autotuning) also fixed send and
// receive buffers of n KB, so a whole page of query results fits in one write.
inline void tune_tcp(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  static const int kb = [] {
    const char* v = std::getenv("TT_TCP_BUF_KB");
    return v && *v ? std::max(0, std::atoi(v)) : 0;
  }();
  if (kb > 0) {
    int sz = kb << 10;
    setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &sz, sizeof sz);
    setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &sz, sizeof sz);
  }
}

// ------------------------------------------------------------------------------ loop
struct IoObj : std::enable_shared_from_this<IoObj> {
  int fd = -1;
  bool dead = false;
  virtual ~IoObj() {
    if (fd >= 0) ::close(fd);
  }
  virtual void on_event(uint32_t ev) = 0;
  virtual void on_tick(double /*now*/) {}
  // Output queued during this loop iteration goes out here, once, after every event, deferred
  // call and timer of the iteration has had its turn (Loop::want_flush).
  virtual void on_flush() {}
  bool flush_queued = false;
};

class Loop {
 public:
  Loop() : ep_(epoll_create1(EPOLL_CLOEXEC)) {}
  ~Loop() { ::close(ep_); }

  void add(const std::shared_ptr<IoObj>& o, uint32_t ev) {
    epoll_event e{};
    e.events = ev;
    e.data.ptr = o.get();
    epoll_ctl(ep_, EPOLL_CTL_ADD, o->fd, &e);
    objs_[o.get()] = o;
  }
  void mod(IoObj* o, uint32_t ev) {
    epoll_event e{};
    e.events = ev;
    e.data.ptr = o;
    epoll_ctl(ep_, EPOLL_CTL_MOD, o->fd, &e);
  }
  // Unregister now, destroy after the current dispatch batch (events for it may be pending).
  void remove(IoObj* o) {
    if (o->dead) return;
    o->dead = true;
    epoll_ctl(ep_, EPOLL_CTL_DEL, o->fd, nullptr);
    auto it = objs_.find(o);
    if (it != objs_.end()) {
      graveyard_.push_back(std::move(it->second));
      objs_.erase(it);
    }
  }
  void defer(std::function<void()> f) { deferred_.push_back(std::move(f)); }
  // Write `o`'s queued output at the end of this iteration: the responses (or pipelined
  // requests) one connection collects while the iteration's events are handled leave in one
  // send(2), not one each.
  void want_flush(IoObj* o) {
    if (o->dead) return;
    if (!defer_flushes()) {  // the default: every write goes out at once
      o->on_flush();
      return;
    }
    if (o->flush_queued) return;
    o->flush_queued = true;
    flush_.push_back(o);
  }
  void call_later(double delay_s, std::function<void()> f) { timers_.emplace(now_s() + delay_s, std::move(f)); }
  void stop() { running_ = false; }
  bool running() const { return running_; }
  size_t live_objects() const { return objs_.size(); }

  void run(const std::function<void(double)>& tick = nullptr) {
    epoll_event evs[256];
    double last_tick = now_s();
    while (running_) {
      int timeout_ms = 50;
      if (!deferred_.empty() || !flush_.empty()) timeout_ms = 0;
      else if (!timers_.empty()) {
        double dt = timers_.begin()->first - now_s();
        timeout_ms = dt <= 0 ? 0 : std::min(50, (int)(dt * 1000.0) + 1);
      }
      int n = epoll_wait(ep_, evs, 256, timeout_ms);
      const double t_wake = iter_hook_ ? now_s() : 0.0;
      for (int i = 0; i < n; ++i) {
        auto* o = static_cast<IoObj*>(evs[i].data.ptr);
        if (!o->dead) o->on_event(evs[i].events);
        // a long batch of events does not hold back what the first ones produced: the queued
        // output leaves every kFlushEvery events (batching without adding a whole iteration of
        // latency to every hop)
        if ((i + 1) % kFlushEvery == 0 && !flush_.empty()) run_flushes();
      }
      while (!deferred_.empty()) {
        auto d = std::move(deferred_);
        deferred_.clear();
        for (auto& f : d) f();
      }
      double t = now_s();
      while (!timers_.empty() && timers_.begin()->first <= t) {
        auto f = std::move(timers_.begin()->second);
        timers_.erase(timers_.begin());
        f();
      }
      run_flushes();
      if (t - last_tick >= 0.05) {
        last_tick = t;
        std::vector<std::shared_ptr<IoObj>> snapshot;
        snapshot.reserve(objs_.size());
        for (auto& kv : objs_) snapshot.push_back(kv.second);
        for (auto& o : snapshot)
          if (!o->dead) o->on_tick(t);
        if (tick) tick(t);
        run_flushes();  // what the ticks queued (timeouts answered), before the graveyard empties
      }
      graveyard_.clear();
      if (iter_hook_) iter_hook_(t_wake, now_s(), n);
    }
  }
  static constexpr int kFlushEvery = 8;
  // TT_DEFER_FLUSH=1: hold each connection's output to the end of the event batch (at most
  // kFlushEvery events).  Fewer sends, but every hop's answer waits for the batch: on the
  // headline that cost more throughput (69.5 k vs 73.4 k tasks/s, profiles/r5_dataplane.md)
  // than the sends it saved, so writes go out at once unless asked.
  static bool defer_flushes() {
    static const bool on = [] {
      const char* v = std::getenv("TT_DEFER_FLUSH");
      return v && v[0] == '1';
    }();
    return on;
  }
  // Queued flushes, then the deferred calls they caused, until both are empty.  The objects
  // are alive: a removed one waits in the graveyard until the iteration's end.
  void run_flushes() {
    while (!flush_.empty()) {
      auto f = std::move(flush_);
      flush_.clear();
      for (IoObj* o : f) {
        o->flush_queued = false;
        if (!o->dead) o->on_flush();
      }
      while (!deferred_.empty()) {
        auto d = std::move(deferred_);
        deferred_.clear();
        for (auto& g : d) g();
      }
    }
  }
  // Diagnostics: called after every iteration with (woke, done, events) -- GapTracer::attach.
  void set_iter_hook(std::function<void(double, double, int)> f) { iter_hook_ = std::move(f); }

 private:
  int ep_;
  bool running_ = true;
  std::unordered_map<IoObj*, std::shared_ptr<IoObj>> objs_;
  std::vector<std::shared_ptr<IoObj>> graveyard_;
  std::vector<std::function<void()>> deferred_;
  std::vector<IoObj*> flush_;
  std::multimap<double, std::function<void()>> timers_;
  std::function<void(double, double, int)> iter_hook_;
};

// Diagnostics: with TT_STALL_LOG=<file>, a loop's tick reports iterations more than 100 ms
// apart (the thread was blocked or not scheduled) as JSON lines; attached to its loop, it also
// reports every iteration that stayed busy (handlers, deferred work, timers) longer than
// TT_STALL_MS (default 100) ms.
inline double stall_threshold_s() {
  static const double s = [] {
    const char* p = std::getenv("TT_STALL_MS");
    double ms = p && *p ? std::atof(p) : 100.0;
    return (ms > 0 ? ms : 100.0) / 1e3;
  }();
  return s;
}

class GapTracer {
 public:
  explicit GapTracer(const char* who) : who_(who), min_busy_(stall_threshold_s()) {
    if (const char* p = std::getenv("TT_STALL_LOG"); p && *p) f_ = std::fopen(p, "a");
  }
  ~GapTracer() {
    if (hooked_) hooked_->set_iter_hook(nullptr);  // the loop may outlive this tracer
    if (f_) std::fclose(f_);
  }
  void tick(double now) {
    if (f_ && last_ > 0 && now - last_ > 0.1)
      std::fprintf(f_, "{\"what\": \"loop-gap\", \"who\": \"%s\", \"ms\": %.2f, \"pid\": %d, \"wall\": %.4f}\n", who_,
                   (now - last_) * 1e3, (int)::getpid(),
                   std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count()),
          std::fflush(f_);
    last_ = now;
  }
  void attach(Loop& loop) {
    if (!f_) return;
    hooked_ = &loop;
    loop.set_iter_hook([this](double woke, double done, int n) {
      if (done - woke > min_busy_)
        std::fprintf(f_, "{\"what\": \"loop-busy\", \"who\": \"%s\", \"ms\": %.2f, \"events\": %d, \"pid\": %d, \"wall\": %.4f}\n",
                     who_, (done - woke) * 1e3, n, (int)::getpid(),
                     std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count()),
            std::fflush(f_);
    });
  }

 private:
  const char* who_;
  double min_busy_;
  Loop* hooked_ = nullptr;
  FILE* f_ = nullptr;
  double last_ = 0;
};

// Grow this process's file-descriptor table once, up front.  The kernel expands the table in
// powers of two as descriptors are allocated, and in a multi-threaded process every expansion
// waits for an RCU grace period (expand_fdtable -> synchronize_rcu), which on a large busy host
// takes 100+ ms -- measured as 90-175 ms socket()/connect() calls stalling a whole event loop.
// Call before starting I/O threads (or any time: it is one expansion instead of several).
inline void reserve_fd_table(int want = 1 << 16) {
  rlimit rl{};
  if (getrlimit(RLIMIT_NOFILE, &rl) != 0) return;
  long top = std::min<long>((long)rl.rlim_cur, want) - 1;
  if (top < 64) return;
  int src = ::open("/dev/null", O_RDONLY | O_CLOEXEC);
  if (src < 0) return;
  int d = ::dup2(src, (int)top);  // allocates the slot -> table sized to cover `top`
  if (d >= 0) ::close(d);
  ::close(src);
}

inline FILE* stall_log() {  // TT_STALL_LOG, shared by the diagnostics below (nullptr when unset)
  static FILE* f = [] {
    const char* p = std::getenv("TT_STALL_LOG");
    return p && *p ? std::fopen(p, "a") : nullptr;
  }();
  return f;
}

inline void stall_note(const char* what, double ms, long n = 0) {
  if (FILE* f = stall_log()) {
    std::fprintf(f, "{\"what\": \"%s\", \"ms\": %.2f, \"n\": %ld, \"pid\": %d}\n", what, ms, n, (int)::getpid());
    std::fflush(f);
  }
}

// ------------------------------------------------------------------------------ messages
using HeaderList = std::vector<std::pair<std::string, std::string>>;

struct Message {
  // request: method/target; response: status/reason
  std::string method, target, reason;
  int status = 0;
  bool http10 = false;
  HeaderList headers;  // lower-cased names
  std::string body;
  // server side over TLS: SAN names of the verified client certificate (shared by the
  // connection's requests)
  std::shared_ptr<const std::string> tls_peer;
  bool tls = false;      // server side: arrived over TLS
  std::string peer;      // server side, listeners with `record_peer`: the client's IP address

  const std::string* header(std::string_view name) const {
    for (auto& h : headers)
      if (h.first == name) return &h.second;
    return nullptr;
  }
  bool keep_alive() const {
    auto* c = header("connection");
    if (!c) return !http10;
    std::string v = *c;
    for (auto& ch : v) ch = ascii_lower(ch);
    if (v.find("close") != std::string::npos) return false;
    if (http10) return v.find("keep-alive") != std::string::npos;
    return true;
  }
};

class MsgParser {
 public:
  enum Result { NEED_MORE, DONE, ERROR };
  explicit MsgParser(bool request) : request_(request) {}
  void expect_no_body() { no_body_ = true; }  // response to HEAD
  std::string error;
  // Set when a request head carrying "Expect: 100-continue" was parsed and its body is still
  // pending; the server answers "100 Continue" once and clears it.
  bool continue_wanted = false;

  // Consume bytes from buf[off..]; returns DONE with `out` filled when a full message is in.
  Result feed(const std::string& buf, size_t& off, Message& out) {
    while (true) {
      switch (st_) {
        case HEAD: {
          size_t e = buf.find("\r\n\r\n", off);
          if (e == std::string::npos) {
            if (buf.size() - off > kMaxHead) return fail("header section too large");
            return NEED_MORE;
          }
          try {
            auto h = parse_head(std::string_view(buf).substr(off, e - off));
            if (request_) {
              msg_.method = std::move(h.a);
              msg_.target = std::move(h.b);
              msg_.http10 = h.c == "HTTP/1.0";
            } else {
              msg_.http10 = h.a == "HTTP/1.0";
              msg_.status = std::atoi(h.b.c_str());
              msg_.reason = std::move(h.c);
            }
            msg_.headers = std::move(h.headers);
          } catch (const std::exception& ex) {
            return fail(ex.what());
          }
          off = e + 4;
          if (request_) {
            auto* ex = msg_.header("expect");
            if (ex && (*ex == "100-continue" || *ex == "100-Continue")) continue_wanted = true;
          }
          auto* te = msg_.header("transfer-encoding");
          auto* cl = msg_.header("content-length");
          bool bodyless = no_body_ || (!request_ && (msg_.status == 204 || msg_.status == 304 || msg_.status < 200));
          if (bodyless) {
            st_ = FINISH;
          } else if (te && te->find("chunked") != std::string::npos) {
            st_ = CHUNK_SIZE;
          } else if (cl) {
            char* end = nullptr;
            long long n = std::strtoll(cl->c_str(), &end, 10);
            if (n < 0 || end == cl->c_str()) return fail("bad content-length");
            if ((size_t)n > kMaxBody) return fail("body too large");
            remaining_ = (size_t)n;
            // one allocation for a body that arrives over several reads (bounded: the length
            // is the peer's claim until the bytes come)
            if (remaining_ > buf.size() - off) msg_.body.reserve(std::min<size_t>(remaining_, 4u << 20));
            st_ = remaining_ ? BODY : FINISH;
          } else if (request_) {
            st_ = FINISH;
          } else {
            st_ = UNTIL_CLOSE;  // response without length: body runs to EOF
          }
          break;
        }
        case BODY: {
          size_t take = std::min(remaining_, buf.size() - off);
          msg_.body.append(buf, off, take);
          off += take;
          remaining_ -= take;
          if (remaining_) return NEED_MORE;
          st_ = FINISH;
          break;
        }
        case CHUNK_SIZE: {
          size_t e = buf.find("\r\n", off);
          if (e == std::string::npos) return buf.size() - off > 1024 ? fail("bad chunk header") : NEED_MORE;
          // chunk-size = 1*HEXDIG [ ";" ext ]: parse by hand so an over-long size cannot
          // saturate/wrap and a line without digits is not read as the last chunk
          size_t p = off, digits = 0, size = 0;
          for (; p < e; ++p, ++digits) {
            char c = buf[p];
            int v = c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10
                  : c >= 'A' && c <= 'F' ? c - 'A' + 10 : -1;
            if (v < 0) break;
            if (size > (kMaxBody >> 4)) return fail("body too large");  // next shift would exceed the cap
            size = (size << 4) | (size_t)v;
          }
          if (!digits) return fail("bad chunk header");
          if (p < e && buf[p] != ';' && buf[p] != ' ' && buf[p] != '\t') return fail("bad chunk header");
          off = e + 2;
          if (size > kMaxBody - msg_.body.size()) return fail("body too large");
          remaining_ = size;
          st_ = remaining_ ? CHUNK_DATA : TRAILERS;
          break;
        }
        case CHUNK_DATA: {
          size_t take = std::min(remaining_, buf.size() - off);
          msg_.body.append(buf, off, take);
          off += take;
          remaining_ -= take;
          if (remaining_) return NEED_MORE;
          st_ = CHUNK_CRLF;
          break;
        }
        case CHUNK_CRLF:
          if (buf.size() - off < 2) return NEED_MORE;
          if (buf[off] != '\r' || buf[off + 1] != '\n') return fail("bad chunk terminator");
          off += 2;
          st_ = CHUNK_SIZE;
          break;
        case TRAILERS: {
          size_t e = buf.find("\r\n", off);
          if (e == std::string::npos) return NEED_MORE;
          bool empty = e == off;
          off = e + 2;
          if (empty) st_ = FINISH;
          break;
        }
        case UNTIL_CLOSE:
          msg_.body.append(buf, off, std::string::npos);
          off = buf.size();
          return NEED_MORE;
        case FINISH:
          out = std::move(msg_);
          reset();
          return DONE;
      }
    }
  }
  // EOF from the peer: completes a read-until-close response.
  bool finish_on_eof(Message& out) {
    if (st_ != UNTIL_CLOSE) return false;
    out = std::move(msg_);
    reset();
    return true;
  }
  bool idle() const { return st_ == HEAD && msg_.headers.empty(); }

 private:
  static constexpr size_t kMaxHead = 64 * 1024;
  static constexpr size_t kMaxBody = 256ull * 1024 * 1024;
  enum St { HEAD, BODY, CHUNK_SIZE, CHUNK_DATA, CHUNK_CRLF, TRAILERS, UNTIL_CLOSE, FINISH } st_ = HEAD;
  bool request_;
  bool no_body_ = false;
  size_t remaining_ = 0;
  Message msg_;
  Result fail(const char* m) {
    error = m;
    return ERROR;
  }
  void reset() {
    msg_ = Message();
    st_ = HEAD;
    remaining_ = 0;
    no_body_ = false;
  }
};

inline const char* reason_phrase(int s) {
  switch (s) {
    case 100: return "Continue";
    case 200: return "OK";
    case 201: return "Created";
    case 202: return "Accepted";
    case 204: return "No Content";
    case 301: return "Moved Permanently";
    case 302: return "Found";
    case 303: return "See Other";
    case 304: return "Not Modified";
    case 307: return "Temporary Redirect";
    case 308: return "Permanent Redirect";
    case 400: return "Bad Request";
    case 401: return "Unauthorized";
    case 403: return "Forbidden";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 409: return "Conflict";
    case 412: return "Precondition Failed";
    case 413: return "Payload Too Large";
    case 415: return "Unsupported Media Type";
    case 422: return "Unprocessable Entity";
    case 429: return "Too Many Requests";
    case 501: return "Not Implemented";
    case 500: return "Internal Server Error";
    case 502: return "Bad Gateway";
    case 503: return "Service Unavailable";
    case 504: return "Gateway Timeout";
    default: return "Status";
  }
}

inline bool is_hop_header(std::string_view k) {
  return k == "connection" || k == "keep-alive" || k == "transfer-encoding" || k == "content-length" ||
         k == "upgrade" || k == "te" || k == "trailer" || k == "proxy-authorization" || k == "host" ||
         k == "expect";
}

// Serialize a response; hop-by-hop headers in `headers` are dropped, framing is ours.
inline void write_response(std::string& out, int status, const HeaderList& headers, std::string_view body,
                           bool head_request, bool close) {
  out += "HTTP/1.1 ";
  out += std::to_string(status);
  out += ' ';
  out += reason_phrase(status);
  out += "\r\n";
  for (auto& h : headers) {
    if (is_hop_header(h.first)) continue;
    out += h.first;
    out += ": ";
    out += h.second;
    out += "\r\n";
  }
  if (status != 204 && status != 304) {
    out += "content-length: ";
    out += std::to_string(body.size());
    out += "\r\n";
  }
  if (close) out += "connection: close\r\n";
  out += "\r\n";
  if (!head_request && status != 204 && status != 304) out.append(body);
}

// Whether a read loop on level-triggered epoll can stop after a read of `n` bytes into a
// `cap`-byte buffer without another (failing, EAGAIN) read: plain sockets -- a short read
// drained the socket; TLS -- a record shorter than the 16 KB maximum with nothing left in
// OpenSSL's buffer (a full record means more of a large message is probably queued).  Bytes
// still in the kernel make epoll report the socket again.
inline bool read_done(const TlsIo* tls, size_t n, size_t cap) {
  if (!tls) return n < cap;
  return n < 16384 && !tls->pending();
}

// ------------------------------------------------------------------------------ endpoints
struct Endpoint {
  bool unix_socket = true;
  std::string path;  // unix
  std::string host;  // tcp
  int port = 0;
  // TLS: 0 plain, 1 mutual TLS with the mesh context (peer certificate must name `tls_name`),
  // 2 https verified by the mesh CA, 3 https without verification (`--app-ssl` dev certificates)
  int tls = 0;
  std::string tls_name;
  std::string key() const {
    std::string k = unix_socket ? "unix:" + path : host + ":" + std::to_string(port);
    return tls ? "tls" + std::to_string(tls) + ":" + tls_name + "@" + k : k;
  }

  // "unix:/path/to.sock[:]" | "http://host:port" | "tcp:host:port" | "host:port" |
  // "https://host:port" | "https+insecure://host:port" | "mtls:<peer-name>@<any of these>"
  static Endpoint parse(std::string s) {
    if (s.rfind("mtls:", 0) == 0) {
      size_t at = s.find('@');
      Endpoint e = parse(at == std::string::npos ? std::string() : s.substr(at + 1));
      e.tls = 1;
      e.tls_name = s.substr(5, at == std::string::npos ? std::string::npos : at - 5);
      return e;
    }
    if (s.rfind("https://", 0) == 0 || s.rfind("https+insecure://", 0) == 0) {
      bool insecure = s[5] == '+';
      Endpoint e = parse("http://" + s.substr(insecure ? 17 : 8));
      e.tls = insecure ? 3 : 2;
      e.tls_name = e.host;
      return e;
    }
    Endpoint e;
    if (s.rfind("unix:", 0) == 0) {
      s = s.substr(5);
      if (!s.empty() && s.back() == ':') s.pop_back();
      e.path = s;
      return e;
    }
    if (s.rfind("http://", 0) == 0) s = s.substr(7);
    if (s.rfind("tcp:", 0) == 0) s = s.substr(4);
    while (!s.empty() && s.back() == '/') s.pop_back();
    auto c = s.rfind(':');
    e.unix_socket = false;
    e.host = c == std::string::npos ? s : s.substr(0, c);
    e.port = c == std::string::npos ? 80 : std::atoi(s.c_str() + c + 1);
    if (e.host == "localhost") e.host = "127.0.0.1";
    return e;
  }
};

// ------------------------------------------------------------------------------ server
class Server;
class ServerConn;

// Completes one request; safe to call after the connection went away.
class Reply {
 public:
  // An in-process completion (e.g. a gRPC call translated into an API request).
  using Sink = std::function<void(int status, const HeaderList& headers, std::string_view body)>;
  Reply() = default;
  Reply(std::weak_ptr<ServerConn> c, uint64_t seq, bool head) : conn_(std::move(c)), seq_(seq), head_(head) {}
  explicit Reply(Sink sink) : sink_(std::make_shared<Sink>(std::move(sink))) {}
  void send(int status, const HeaderList& headers, std::string_view body) const;
  void json(int status, std::string_view body) const {
    send(status, {{"content-type", "application/json"}}, body);
  }
  void empty(int status) const { send(status, {}, {}); }
  // The client is gone (connection closed, or the peer shut down its side): a parked long
  // poll must not take messages for it.
  bool abandoned() const;

 private:
  std::weak_ptr<ServerConn> conn_;
  uint64_t seq_ = 0;
  bool head_ = false;
  std::shared_ptr<Sink> sink_;
};

using Handler = std::function<void(Message&&, Reply)>;

class ServerConn : public IoObj {
 public:
  ServerConn(Loop& loop, int fd, Handler& h, const TlsContext* tls = nullptr, bool record_peer = false)
      : loop_(loop), handler_(h), parser_(true), record_peer_(record_peer) {
    this->fd = fd;
    if (tls) tls_ = std::make_unique<TlsIo>(*tls, fd);
  }

  void on_event(uint32_t ev) override {
    // over TLS, writability may be what a pending handshake / read step waits for
    if (!peer_closed_ && ((ev & (EPOLLIN | EPOLLHUP | EPOLLERR)) || (tls_ && (ev & EPOLLOUT)))) {
      char buf[65536];
      while (true) {
        ssize_t n = io_recv(buf, sizeof buf);
        if (n > 0) {
          in_.append(buf, (size_t)n);
          if (short_read((size_t)n, sizeof buf)) break;
          continue;
        }
        if (n == 0) {
          peer_closed_ = true;
          break;
        }
        if (errno == EAGAIN || errno == EWOULDBLOCK) break;
        if (errno == EINTR) continue;
        close_now();
        return;
      }
      parse();
      if (dead) return;
      if (peer_closed_) {
        if (pending_.empty() && out_off_ == out_.size()) {
          close_now();
          return;
        }
        update_interest();  // stop polling a half-closed socket; finish writing what is pending
      }
    }
    if ((ev & EPOLLOUT) || (tls_ && out_off_ < out_.size())) flush();
    else if (tls_) update_interest();
  }

  bool peer_gone() const { return dead || peer_closed_; }

  void respond(uint64_t seq, int status, const HeaderList& headers, std::string_view body, bool head_request) {
    if (dead || seq < head_seq_) return;
    size_t idx = (size_t)(seq - head_seq_);
    if (idx >= pending_.size() || pending_[idx].ready) return;
    Slot& sl = pending_[idx];
    if (idx == 0) {
      // the oldest answer owed goes straight into the output buffer (which keeps its capacity):
      // no slot allocation and no second copy
      const bool close_after = sl.close_after;
      write_response(out_, status, headers, body, head_request, close_after);
      if (close_after) close_after_write_ = true;
      pending_.pop_front();
      ++head_seq_;
    } else {
      sl.wire.reserve(body.size() + 256);
      write_response(sl.wire, status, headers, body, head_request, sl.close_after);
      sl.ready = true;
    }
    drain();
    // resume a pipeline that was paused at its depth limit
    if (!dead && !parsing_ && !close_after_write_ && in_off_ < in_.size()) parse();
  }

 private:
  struct Slot {
    bool ready = false;
    bool close_after = false;
    std::string wire;
  };
  Loop& loop_;
  Handler& handler_;
  MsgParser parser_;
  std::string in_;
  size_t in_off_ = 0;
  std::string out_;
  size_t out_off_ = 0;
  std::deque<Slot> pending_;
  uint64_t head_seq_ = 0;
  bool peer_closed_ = false;
  bool close_after_write_ = false;
  bool parsing_ = false;
  uint32_t interest_ = EPOLLIN;
  std::unique_ptr<TlsIo> tls_;
  std::shared_ptr<const std::string> tls_peer_;
  bool record_peer_ = false;
  std::string peer_;

  ssize_t io_recv(char* buf, size_t n) { return tls_ ? tls_->recv(buf, n) : ::recv(fd, buf, n, 0); }
  ssize_t io_send(const char* p, size_t n) { return tls_ ? tls_->send(p, n) : ::send(fd, p, n, MSG_NOSIGNAL); }
  bool short_read(size_t n, size_t cap) const { return read_done(tls_.get(), n, cap); }

  const std::string& peer_ip() {
    if (peer_.empty()) {
      sockaddr_storage ss{};
      socklen_t len = sizeof ss;
      char buf[INET6_ADDRSTRLEN] = "local";
      if (::getpeername(fd, (sockaddr*)&ss, &len) == 0) {
        if (ss.ss_family == AF_INET) inet_ntop(AF_INET, &((sockaddr_in*)&ss)->sin_addr, buf, sizeof buf);
        else if (ss.ss_family == AF_INET6) inet_ntop(AF_INET6, &((sockaddr_in6*)&ss)->sin6_addr, buf, sizeof buf);
      }
      peer_ = buf;
    }
    return peer_;
  }

  void drain() {
    while (!pending_.empty() && pending_.front().ready) {
      out_ += pending_.front().wire;
      if (pending_.front().close_after) close_after_write_ = true;
      pending_.pop_front();
      ++head_seq_;
    }
    // the answers a read's pipelined requests produce while it is parsed leave together, in
    // one send at the end of parse(); others go at once (or with the batch, TT_DEFER_FLUSH=1)
    if (!parsing_) loop_.want_flush(this);
  }
  void on_flush() override { flush(); }

  void parse() {
    parsing_ = true;
    while (!dead && !close_after_write_ && pending_.size() < 64) {
      Message m;
      auto r = parser_.feed(in_, in_off_, m);
      if (parser_.continue_wanted) {  // client waits for this before sending the body
        parser_.continue_wanted = false;
        if (r == MsgParser::NEED_MORE && pending_.empty()) {
          out_ += "HTTP/1.1 100 Continue\r\n\r\n";
          flush();
          if (dead) return;
        }
      }
      if (r == MsgParser::NEED_MORE) break;
      if (r == MsgParser::ERROR) {
        std::string w;
        write_response(w, 400, {{"content-type", "text/plain"}}, parser_.error, false, true);
        pending_.push_back(Slot{true, true, std::move(w)});
        in_off_ = in_.size();
        drain();
        break;
      }
      if (tls_) {
        if (!tls_peer_) tls_peer_ = std::make_shared<const std::string>(tls_->peer_names());
        m.tls = true;
        m.tls_peer = tls_peer_;
      }
      if (record_peer_) m.peer = peer_ip();
      bool ka = m.keep_alive();
      bool head = m.method == "HEAD";
      uint64_t seq = head_seq_ + pending_.size();
      pending_.push_back(Slot{});
      if (!ka) pending_.back().close_after = true, stop_reading_ = true;
      auto self = std::static_pointer_cast<ServerConn>(shared_from_this());
      handler_(std::move(m), Reply(self, seq, head));
      if (stop_reading_) break;
    }
    parsing_ = false;
    if (dead) return;
    if (in_off_ > 0 && (in_off_ == in_.size() || in_off_ > 65536)) {
      in_.erase(0, in_off_);
      in_off_ = 0;
    }
    if (out_off_ < out_.size()) loop_.want_flush(this);  // what the parsed requests answered at once
  }
  bool stop_reading_ = false;

  void update_interest() {
    bool out = tls_ ? tls_->want_write : out_off_ < out_.size();
    uint32_t want = (peer_closed_ || stop_reading_ ? 0u : (uint32_t)EPOLLIN) | (out ? (uint32_t)EPOLLOUT : 0u);
    if (want != interest_) {
      interest_ = want;
      loop_.mod(this, want);
    }
  }

  void flush() {
    while (out_off_ < out_.size()) {
      ssize_t n = io_send(out_.data() + out_off_, out_.size() - out_off_);
      if (n > 0) {
        out_off_ += (size_t)n;
        continue;
      }
      if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
      if (n < 0 && errno == EINTR) continue;
      close_now();
      return;
    }
    if (out_off_ == out_.size()) {
      out_.clear();
      out_off_ = 0;
      if ((close_after_write_ || peer_closed_) && pending_.empty()) {
        close_now();
        return;
      }
    }
    update_interest();
  }

  void close_now() { loop_.remove(this); }
};

inline bool Reply::abandoned() const {
  if (sink_) return false;
  auto c = conn_.lock();
  return !c || c->peer_gone();
}

inline void Reply::send(int status, const HeaderList& headers, std::string_view body) const {
  if (sink_) {
    (*sink_)(status, headers, body);
    return;
  }
  if (auto c = conn_.lock()) c->respond(seq_, status, headers, body, head_);
}

class Listener : public IoObj {
 public:
  Listener(Loop& loop, int fd, Handler& h, std::shared_ptr<TlsContext> tls = nullptr, bool record_peer = false)
      : loop_(loop), handler_(h), tls_(std::move(tls)), record_peer_(record_peer) {
    this->fd = fd;
    sockaddr_storage ss{};
    socklen_t len = sizeof ss;
    unix_ = ::getsockname(fd, (sockaddr*)&ss, &len) == 0 && ss.ss_family == AF_UNIX;
  }
  void on_event(uint32_t) override {
    while (true) {
      int c = ::accept4(fd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (c < 0) {
        if (errno == EINTR) continue;
        return;  // EAGAIN or transient error (EMFILE ...): try again on the next readiness event
      }
      if (unix_) widen_local_sndbuf(c);
      else tune_tcp(c);
      if (hand_off && hand_off(c)) continue;  // another loop serves it
      std::shared_ptr<ServerConn> conn;
      try {
        conn = std::make_shared<ServerConn>(loop_, c, handler_, tls_.get(), record_peer_);
      } catch (const std::exception&) {
        ::close(c);
        continue;
      }
      loop_.add(conn, EPOLLIN);
      if (on_accept) on_accept(conn);
    }
  }
  // optional: observe accepted connections (the app host closes them when its server stops)
  std::function<void(const std::shared_ptr<ServerConn>&)> on_accept;
  // optional: give an accepted socket to another loop (true: taken; it calls adopt() there)
  std::function<bool(int fd)> hand_off;

 private:
  bool unix_ = false;
  Loop& loop_;
  Handler& handler_;
  std::shared_ptr<TlsContext> tls_;
  bool record_peer_;
};

// Serve an accepted socket on `loop` (a Listener's hand_off, on the receiving loop's thread).
inline void adopt(Loop& loop, int fd, Handler& h) {
  std::shared_ptr<ServerConn> conn;
  try {
    conn = std::make_shared<ServerConn>(loop, fd, h);
  } catch (const std::exception&) {
    ::close(fd);
    return;
  }
  loop.add(conn, EPOLLIN);
}

// Bind + listen on `ep`; returns the socket, and the bound port in `port` (tcp) or 0 (unix).
// Throws on failure.  `reuseport`: several loops (threads) bind the same TCP port and the
// kernel spreads incoming connections over them.
inline int bind_listen(const Endpoint& ep, bool reuseport, int& port) {
  int fd;
  port = 0;
  if (ep.unix_socket) {
    fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    sockaddr_un a{};
    a.sun_family = AF_UNIX;
    if (ep.path.size() >= sizeof a.sun_path) {
      ::close(fd);
      throw std::runtime_error("unix socket path too long: " + ep.path);
    }
    std::strcpy(a.sun_path, ep.path.c_str());
    ::unlink(ep.path.c_str());
    if (::bind(fd, (sockaddr*)&a, sizeof a) != 0) {
      int e = errno;
      ::close(fd);
      throw std::runtime_error("bind " + ep.path + ": " + strerror(e));
    }
  } else {
    fd = ::socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    if (reuseport) setsockopt(fd, SOL_SOCKET, SO_REUSEPORT, &one, sizeof one);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)ep.port);
    inet_pton(AF_INET, ep.host.c_str(), &a.sin_addr);
    if (::bind(fd, (sockaddr*)&a, sizeof a) != 0) {
      int e = errno;
      ::close(fd);
      throw std::runtime_error("bind " + ep.key() + ": " + strerror(e));
    }
    socklen_t len = sizeof a;
    getsockname(fd, (sockaddr*)&a, &len);
    port = ntohs(a.sin_port);
  }
  if (::listen(fd, 1024) != 0) {
    int e = errno;
    ::close(fd);
    throw std::runtime_error(std::string("listen: ") + strerror(e));
  }
  return fd;
}

// Returns the bound port (tcp) or 0 (unix); throws on failure.
// `tls`: serve HTTPS (with `verify_peer`: mutual TLS) on this listener.
// `record_peer`: messages carry the client's address (`Message::peer`; a proxy's X-Forwarded-For).
inline int listen_on(Loop& loop, const Endpoint& ep, Handler& h, bool reuseport = false,
                     std::shared_ptr<IoObj>* listener_out = nullptr, std::shared_ptr<TlsContext> tls = nullptr,
                     bool record_peer = false) {
  int port = 0;
  int fd = bind_listen(ep, reuseport, port);
  auto l = std::make_shared<Listener>(loop, fd, h, std::move(tls), record_peer);
  loop.add(l, EPOLLIN);
  if (listener_out) *listener_out = l;
  return port;
}

// ------------------------------------------------------------------------------ client
struct ClientResult {
  int err = 0;  // 0 = ok; otherwise errno-like (ECONNREFUSED, ENOENT, ETIMEDOUT, ECONNRESET ...)
  Message resp;
};
using ClientCallback = std::function<void(ClientResult&&)>;

class Client;

class ClientConn : public IoObj {
 public:
  ClientConn(Loop& loop, Client& owner, std::string key) : loop_(loop), owner_(owner), key_(std::move(key)), parser_(false) {}
  bool reused = false;
  bool connecting = false;

  void start(std::string&& wire, bool head, double deadline, ClientCallback&& cb) {
    out_ = std::move(wire);
    out_off_ = 0;
    cb_ = std::move(cb);
    deadline_ = deadline;
    got_bytes_ = false;
    busy_ = true;
    if (head) parser_.expect_no_body();
    if (!connecting) flush();
  }
  void on_event(uint32_t ev) override;
  void on_tick(double now) override {
    if (busy_ && deadline_ > 0 && now > deadline_) fail(ETIMEDOUT);
    else if (!busy_ && now - idle_since_ > 30.0) loop_.remove(this);  // idle pool entry aged out
  }
  bool busy() const { return busy_; }
  std::string wire_copy;  // kept for the stale-connection retry
  // An idle connection whose peer already closed it (FIN or RST queued, not yet seen by the
  // loop): not reused.  Pending bytes (a TLS session ticket) say nothing either way: kept.
  bool peer_gone() const {
    char b;
    ssize_t n = ::recv(fd, &b, 1, MSG_PEEK | MSG_DONTWAIT);
    return n == 0 || (n < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR);
  }
  bool head_req = false;
  std::unique_ptr<TlsIo> tls_;

  ssize_t io_recv(char* buf, size_t n) { return tls_ ? tls_->recv(buf, n) : ::recv(fd, buf, n, 0); }
  ssize_t io_send(const char* p, size_t n) { return tls_ ? tls_->send(p, n) : ::send(fd, p, n, MSG_NOSIGNAL); }
  bool short_read(size_t n, size_t cap) const { return read_done(tls_.get(), n, cap); }

 private:
  friend class Client;
  Loop& loop_;
  Client& owner_;
  std::string key_;
  MsgParser parser_;
  std::string in_;
  size_t in_off_ = 0;
  std::string out_;
  size_t out_off_ = 0;
  ClientCallback cb_;
  double deadline_ = 0;
  double idle_since_ = 0;
  bool busy_ = false;
  bool got_bytes_ = false;
  bool want_out_ = false;

  void flush();
  void fail(int err);
  void finish(Message&& m, bool keep);
};

// A pipelined connection (HTTP/1.1 pipelining) to a local peer that answers in order -- an
// evhttp ServerConn: a sidecar's API, the backing's front.  The requests issued during one loop
// iteration leave in one send(2) at its end (Loop::want_flush), their answers come back in as
// few reads, and the peer answers a batch with one write (ServerConn::drain): the per-exchange
// system calls of the busiest hops (app -> sidecar -> store) shrink with the load.  A failure
// fails every request in flight on it: none is re-sent (the peer may have acted on it).
class PipeConn : public IoObj {
 public:
  PipeConn(Loop& loop, Client& owner, std::string key) : loop_(loop), owner_(owner), key_(std::move(key)), parser_(false) {}
  size_t inflight() const { return q_.size(); }
  double idle_since() const { return q_.empty() ? idle_since_ : 0.0; }
  void send(std::string&& wire, double deadline, ClientCallback&& cb) {
    if (out_off_ == out_.size()) {
      out_ = std::move(wire);
      out_off_ = 0;
    } else {
      out_ += wire;
    }
    q_.push_back(Pending{std::move(cb), deadline});
    loop_.want_flush(this);
  }
  // the peer closed an idle connection (FIN or RST queued, not yet seen by the loop)
  bool peer_gone() const {
    char b;
    ssize_t n = ::recv(fd, &b, 1, MSG_PEEK | MSG_DONTWAIT);
    return n == 0 || (n < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR);
  }
  void on_event(uint32_t ev) override;
  void on_flush() override;
  void on_tick(double now) override {
    for (auto& p : q_)
      if (p.deadline > 0 && now > p.deadline) {
        fail_all(ETIMEDOUT);  // the answers behind it cannot be told apart any more
        return;
      }
    if (q_.empty() && now - idle_since_ > 30.0) fail_all(0);  // idle pool entry aged out
  }

 private:
  struct Pending {
    ClientCallback cb;
    double deadline;
  };
  Loop& loop_;
  Client& owner_;
  std::string key_;
  MsgParser parser_;
  std::string in_, out_;
  size_t in_off_ = 0, out_off_ = 0;
  std::deque<Pending> q_;
  double idle_since_ = now_s();
  bool want_out_ = false;
  void fail_all(int err);
};

class Client {
 public:
  explicit Client(Loop& loop) : loop_(loop) {}

  // Mutual-TLS identity for "mtls:" endpoints (and the CA that verifies "https://" ones).
  void set_tls(std::shared_ptr<TlsContext> mesh) { mesh_tls_ = std::move(mesh); }

  // Issue `method target` with `headers`/`body` to `ep`; `cb` runs on completion or failure.
  // `retry_stale`: a reused keep-alive connection that fails with a reset / broken pipe is
  // retried once on a new one.  That is only safe when re-sending cannot repeat an action: pass
  // false for a non-idempotent request whose peer may have read it before resetting.
  void request(const Endpoint& ep, std::string_view method, std::string_view target, const HeaderList& headers,
               std::string_view body, double timeout_s, ClientCallback cb, bool retry_stale = true) {
    std::string w;
    w.reserve(body.size() + 512);
    w.append(method);
    w += ' ';
    w.append(target);
    w += " HTTP/1.1\r\nhost: ";
    w += ep.unix_socket ? "localhost" : ep.host + ":" + std::to_string(ep.port);
    w += "\r\n";
    for (auto& h : headers) {
      if (is_hop_header(h.first)) continue;
      w += h.first;
      w += ": ";
      w += h.second;
      w += "\r\n";
    }
    w += "content-length: ";
    w += std::to_string(body.size());
    w += "\r\n\r\n";
    w.append(body);
    dispatch(ep, std::move(w), method == "HEAD", timeout_s, std::move(cb), retry_stale);
  }

  // `request` over a pipelined connection (PipeConn) when `ep` is a local socket: for peers
  // that answer in order (evhttp servers) and requests that answer quickly -- a slow one holds
  // up the answers queued behind it.  No stale-connection retry (a long-idle connection is
  // checked before reuse instead).  Other endpoints take `request`.
  void request_pipelined(const Endpoint& ep, std::string_view method, std::string_view target,
                         const HeaderList& headers, std::string_view body, double timeout_s, ClientCallback cb) {
    static const bool enabled = [] {  // TT_PIPELINE=0: the ordinary connections (A/B switch)
      const char* v = std::getenv("TT_PIPELINE");
      return !(v && v[0] == '0');
    }();
    if (!enabled || !ep.unix_socket || ep.tls || method == "HEAD") {
      request(ep, method, target, headers, body, timeout_s, std::move(cb), false);
      return;
    }
    std::string w;
    w.reserve(body.size() + 256 + target.size());
    w.append(method);
    w += ' ';
    w.append(target);
    w += " HTTP/1.1\r\nhost: localhost\r\n";
    for (auto& h : headers) {
      if (is_hop_header(h.first)) continue;
      w += h.first;
      w += ": ";
      w += h.second;
      w += "\r\n";
    }
    w += "content-length: ";
    w += std::to_string(body.size());
    w += "\r\n\r\n";
    w.append(body);
    double deadline = timeout_s > 0 ? now_s() + timeout_s : 0;
    auto c = pipe_for(ep);
    if (!c) {  // could not connect now: the ordinary path (it retries a full backlog, reports errors)
      dispatch(ep, std::move(w), false, timeout_s, std::move(cb), false);
      return;
    }
    c->send(std::move(w), deadline, std::move(cb));
    ++pipelined_;
  }
  // A pipelined connection flushed its batch: the next iteration's requests go to the next one
  // (the peer's accept spread them over its loops).
  void pipe_flushed(const std::string& key) {
    auto it = pipes_.find(key);
    if (it != pipes_.end()) it->second.cur = (it->second.cur + 1) % kPipeConns;
  }
  void pipe_closed(PipeConn* c, const std::string& key) {
    auto it = pipes_.find(key);
    if (it == pipes_.end()) return;
    for (auto& p : it->second.conns)
      if (p.get() == c) p.reset();
  }
  uint64_t pipelined() const { return pipelined_; }
  // new outbound connections, by transport (a TLS one costs a handshake): how often the pools
  // had no idle connection to hand out
  uint64_t connects() const { return connects_; }
  uint64_t tls_connects() const { return tls_connects_; }

  void release(const std::shared_ptr<ClientConn>& c) {
    auto& v = idle_[c->key_];
    if (v.size() < 256) {
      c->idle_since_ = now_s();
      v.push_back(c);
    } else {
      loop_.remove(c.get());
    }
  }
  void forget(ClientConn* c) {
    auto it = idle_.find(c->key_);
    if (it == idle_.end()) return;
    auto& v = it->second;
    for (size_t i = 0; i < v.size(); ++i)
      if (v[i].get() == c) {
        v.erase(v.begin() + (long)i);
        break;
      }
  }
  Loop& loop() { return loop_; }

  void dispatch(const Endpoint& ep, std::string&& wire, bool head, double timeout_s, ClientCallback&& cb,
                bool allow_retry) {
    std::string key = ep.key();
    std::shared_ptr<ClientConn> c;
    auto& v = idle_[key];
    while (!v.empty()) {
      c = v.back();
      v.pop_back();
      // without the stale retry, first make sure the peer has not closed it meanwhile
      if (!c->dead && (allow_retry || !c->peer_gone())) break;
      loop_.remove(c.get());
      c.reset();
    }
    double deadline = timeout_s > 0 ? now_s() + timeout_s : 0;
    if (c) {
      c->reused = true;
    } else {
      int err = 0;
      double tc = stall_log() ? now_s() : 0;
      c = connect(ep, key, err);
      if (tc > 0 && now_s() - tc > 0.02) stall_note("client-connect-slow", (now_s() - tc) * 1e3, err);
      if (!c && err == EAGAIN && (deadline == 0 || now_s() < deadline)) {
        // Unix listener backlog full: try again shortly instead of blocking the loop in connect()
        auto ep_copy = ep;
        loop_.call_later(0.0005, [this, ep_copy, wire = std::move(wire), head, timeout_s, cb = std::move(cb),
                                  allow_retry, deadline]() mutable {
          double left = deadline > 0 ? deadline - now_s() : 0;
          dispatch(ep_copy, std::move(wire), head, deadline > 0 ? std::max(left, 1e-3) : timeout_s, std::move(cb),
                   allow_retry);
        });
        return;
      }
      if (!c) {
        loop_.defer([cb = std::move(cb), err]() mutable {
          ClientResult r;
          r.err = err;
          cb(std::move(r));
        });
        return;
      }
    }
    if (allow_retry && c->reused) {
      // a reused keep-alive connection may have been closed by the peer: retry once on a new one
      auto ep_copy = ep;
      auto wire_copy = wire;
      ClientCallback inner = [this, ep_copy, wire_copy = std::move(wire_copy), head, timeout_s,
                              cb = std::move(cb)](ClientResult&& r) mutable {
        if (r.err == ECONNRESET || r.err == EPIPE) {
          dispatch(ep_copy, std::move(wire_copy), head, timeout_s, std::move(cb), false);
          return;
        }
        cb(std::move(r));
      };
      double ts = stall_log() ? now_s() : 0;
      c->start(std::move(wire), head, deadline, std::move(inner));
      if (ts > 0 && now_s() - ts > 0.02) stall_note("client-start-slow", (now_s() - ts) * 1e3, 1);
    } else {
      double ts = stall_log() ? now_s() : 0;
      c->start(std::move(wire), head, deadline, std::move(cb));
      if (ts > 0 && now_s() - ts > 0.02) stall_note("client-start-slow", (now_s() - ts) * 1e3, 0);
    }
  }

 private:
  Loop& loop_;
  std::unordered_map<std::string, std::vector<std::shared_ptr<ClientConn>>> idle_;
  std::shared_ptr<TlsContext> mesh_tls_, insecure_tls_, system_tls_;
  // pipelined connections per endpoint: a few, one per loop iteration in turn, each holding at
  // most kPipeDepth requests in flight
  static constexpr size_t kPipeConns = 4, kPipeDepth = 64;
  struct PipeGroup {
    std::shared_ptr<PipeConn> conns[kPipeConns];
    size_t cur = 0;
  };
  std::unordered_map<std::string, PipeGroup> pipes_;
  uint64_t pipelined_ = 0, connects_ = 0, tls_connects_ = 0;

  std::shared_ptr<PipeConn> pipe_for(const Endpoint& ep) {
    std::string key = ep.key();
    auto& g = pipes_[key];
    for (size_t tries = 0; tries < kPipeConns; ++tries) {
      auto& c = g.conns[g.cur];
      if (c && (c->dead || (c->idle_since() > 0 && now_s() - c->idle_since() > 1.0 && c->peer_gone()))) {
        auto gone = c;
        c.reset();
        if (!gone->dead) loop_.remove(gone.get());
      }
      if (!c) {
        int fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
        if (fd < 0) return nullptr;
        widen_local_sndbuf(fd);
        sockaddr_un a{};
        a.sun_family = AF_UNIX;
        std::strncpy(a.sun_path, ep.path.c_str(), sizeof a.sun_path - 1);
        if (::connect(fd, (sockaddr*)&a, sizeof a) != 0) {
          ::close(fd);
          return nullptr;
        }
        c = std::make_shared<PipeConn>(loop_, *this, key);
        c->fd = fd;
        loop_.add(c, EPOLLIN);
      }
      if (c->inflight() < kPipeDepth) return c;
      g.cur = (g.cur + 1) % kPipeConns;
    }
    return nullptr;
  }

  const TlsContext* tls_for(const Endpoint& ep) {
    if (ep.tls == 1) return mesh_tls_.get();
    if (ep.tls == 2 && mesh_tls_) return mesh_tls_.get();
    if (ep.tls == 2) {
      if (!system_tls_) {
        TlsConfig c;
        c.verify_peer = false;  // no trust store configured: encrypt, but only the mesh CA can verify
        system_tls_ = std::make_shared<TlsContext>(c, false);
      }
      return system_tls_.get();
    }
    if (!insecure_tls_) {
      TlsConfig c;
      c.verify_peer = false;
      insecure_tls_ = std::make_shared<TlsContext>(c, false);
    }
    return insecure_tls_.get();
  }

  std::shared_ptr<ClientConn> connect(const Endpoint& ep, const std::string& key, int& err) {
    const TlsContext* tctx = nullptr;
    ++connects_;
    if (ep.tls) {
      ++tls_connects_;
      tctx = tls_for(ep);
      if (!tctx) {  // "mtls:" endpoint but this process has no mesh identity
        err = EPROTO;
        return nullptr;
      }
    }
    int fd;
    bool in_progress = false;
    if (ep.unix_socket) {
      // non-blocking: a local connect completes at once, or fails with EAGAIN while the
      // listener's accept queue is full -- the caller retries then, rather than parking the
      // whole event loop in connect() until the peer gets round to accept()
      fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
      widen_local_sndbuf(fd);
      sockaddr_un a{};
      a.sun_family = AF_UNIX;
      std::strncpy(a.sun_path, ep.path.c_str(), sizeof a.sun_path - 1);
      if (::connect(fd, (sockaddr*)&a, sizeof a) != 0) {
        err = errno == EWOULDBLOCK ? EAGAIN : errno;
        ::close(fd);
        return nullptr;
      }
    } else {
      fd = ::socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
      tune_tcp(fd);
      sockaddr_in a{};
      a.sin_family = AF_INET;
      a.sin_port = htons((uint16_t)ep.port);
      inet_pton(AF_INET, ep.host.c_str(), &a.sin_addr);
      if (::connect(fd, (sockaddr*)&a, sizeof a) != 0) {
        if (errno != EINPROGRESS) {
          err = errno;
          ::close(fd);
          return nullptr;
        }
        in_progress = true;
      }
    }
    auto c = std::make_shared<ClientConn>(loop_, *this, key);
    c->fd = fd;
    if (tctx) c->tls_ = std::make_unique<TlsIo>(*tctx, fd, ep.tls == 3 ? std::string() : ep.tls_name);
    c->connecting = in_progress;
    loop_.add(c, in_progress ? (EPOLLOUT | EPOLLIN) : EPOLLIN);
    if (in_progress) c->want_out_ = true;
    return c;
  }
};

inline void ClientConn::on_event(uint32_t ev) {
  if (connecting && (ev & (EPOLLOUT | EPOLLERR | EPOLLHUP))) {
    int e = 0;
    socklen_t l = sizeof e;
    getsockopt(fd, SOL_SOCKET, SO_ERROR, &e, &l);
    if (e != 0) {
      fail(e);
      return;
    }
    connecting = false;
  }
  if ((ev & (EPOLLIN | EPOLLHUP | EPOLLERR)) || (tls_ && !connecting && (ev & EPOLLOUT))) {
    char buf[65536];
    bool eof = false;
    while (true) {
      ssize_t n = io_recv(buf, sizeof buf);
      if (n > 0) {
        in_.append(buf, (size_t)n);
        got_bytes_ = true;
        if (short_read((size_t)n, sizeof buf)) break;
        continue;
      }
      if (n == 0) {
        eof = true;
        break;
      }
      if (errno == EAGAIN || errno == EWOULDBLOCK) break;
      if (errno == EINTR) continue;
      fail(got_bytes_ ? EIO : ECONNRESET);
      return;
    }
    if (busy_ && !in_.empty()) {
      Message m;
      auto r = parser_.feed(in_, in_off_, m);
      if (r == MsgParser::DONE) {
        bool keep = !eof && m.keep_alive() && in_off_ == in_.size();
        finish(std::move(m), keep);
        return;
      }
      if (r == MsgParser::ERROR) {
        fail(EPROTO);
        return;
      }
    }
    if (eof) {
      Message m;
      if (busy_ && parser_.finish_on_eof(m)) {
        finish(std::move(m), false);
        return;
      }
      if (busy_) fail(got_bytes_ ? EIO : ECONNRESET);
      else {
        owner_.forget(this);
        loop_.remove(this);
      }
      return;
    }
  }
  if (!dead && busy_ && ((ev & EPOLLOUT) || (tls_ && out_off_ < out_.size()))) flush();
  else if (!dead && tls_) flush();  // re-evaluate write interest (handshake progress)
}

inline void ClientConn::flush() {
  while (out_off_ < out_.size()) {
    ssize_t n = io_send(out_.data() + out_off_, out_.size() - out_off_);
    if (n > 0) {
      out_off_ += (size_t)n;
      continue;
    }
    if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
    if (n < 0 && errno == EINTR) continue;
    fail(tls_ ? EPROTO : errno == EPIPE ? EPIPE : ECONNRESET);
    return;
  }
  // over TLS a pending write may be waiting for the handshake's next read, not writability
  bool need_out = tls_ ? tls_->want_write : out_off_ < out_.size();
  if (need_out != want_out_) {
    want_out_ = need_out;
    loop_.mod(this, need_out ? (EPOLLIN | EPOLLOUT) : EPOLLIN);
  }
  if (out_off_ >= out_.size()) {
    out_.clear();
    out_off_ = 0;
  }
}

inline void ClientConn::fail(int err) {
  auto self = shared_from_this();  // keep alive through the callback
  busy_ = false;
  owner_.forget(this);
  loop_.remove(this);
  if (cb_) {
    auto cb = std::move(cb_);
    cb_ = nullptr;
    ClientResult r;
    r.err = err;
    cb(std::move(r));
  }
}

inline void ClientConn::finish(Message&& m, bool keep) {
  auto self = std::static_pointer_cast<ClientConn>(shared_from_this());
  busy_ = false;
  in_.erase(0, in_off_);
  in_off_ = 0;
  auto cb = std::move(cb_);
  cb_ = nullptr;
  if (keep) owner_.release(self);
  else loop_.remove(this);
  ClientResult r;
  r.resp = std::move(m);
  cb(std::move(r));
}

inline void PipeConn::on_flush() {
  while (out_off_ < out_.size()) {
    ssize_t n = ::send(fd, out_.data() + out_off_, out_.size() - out_off_, MSG_NOSIGNAL);
    if (n > 0) {
      out_off_ += (size_t)n;
      continue;
    }
    if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
    if (n < 0 && errno == EINTR) continue;
    fail_all(errno == EPIPE ? EPIPE : ECONNRESET);
    return;
  }
  bool need_out = out_off_ < out_.size();
  if (need_out != want_out_) {
    want_out_ = need_out;
    loop_.mod(this, need_out ? (EPOLLIN | EPOLLOUT) : EPOLLIN);
  }
  if (!need_out) {
    out_.clear();
    out_off_ = 0;
  }
  owner_.pipe_flushed(key_);
}

inline void PipeConn::on_event(uint32_t ev) {
  auto self = shared_from_this();  // alive through the callbacks
  if (ev & (EPOLLIN | EPOLLHUP | EPOLLERR)) {
    char buf[65536];
    bool eof = false;
    while (true) {
      ssize_t n = ::recv(fd, buf, sizeof buf, 0);
      if (n > 0) {
        in_.append(buf, (size_t)n);
        if ((size_t)n < sizeof buf) break;
        continue;
      }
      if (n == 0) {
        eof = true;
        break;
      }
      if (errno == EAGAIN || errno == EWOULDBLOCK) break;
      if (errno == EINTR) continue;
      fail_all(ECONNRESET);
      return;
    }
    while (in_off_ < in_.size()) {
      if (q_.empty()) {  // an answer nobody asked for: the stream is out of step
        fail_all(EPROTO);
        return;
      }
      Message m;
      auto r = parser_.feed(in_, in_off_, m);
      if (r == MsgParser::NEED_MORE) break;
      if (r == MsgParser::ERROR) {
        fail_all(EPROTO);
        return;
      }
      bool keep = m.keep_alive();
      Pending p = std::move(q_.front());
      q_.pop_front();
      if (q_.empty()) idle_since_ = now_s();
      ClientResult res;
      res.resp = std::move(m);
      if (!keep) {  // the peer closes after this answer: the requests behind it were not read
        auto cb = std::move(p.cb);
        fail_all(ECONNRESET);
        cb(std::move(res));
        return;
      }
      p.cb(std::move(res));  // may queue more requests here (answered in later reads)
      if (dead) return;
    }
    if (in_off_ > 0 && (in_off_ == in_.size() || in_off_ > 65536)) {
      in_.erase(0, in_off_);
      in_off_ = 0;
    }
    if (eof) {
      fail_all(q_.empty() ? 0 : EIO);
      return;
    }
  }
  if (!dead && (ev & EPOLLOUT)) on_flush();
}

inline void PipeConn::fail_all(int err) {
  auto self = shared_from_this();
  owner_.pipe_closed(this, key_);
  loop_.remove(this);
  if (q_.empty()) return;
  // answered from the loop, never from inside the caller's request_pipelined (a send can fail
  // at once): callers may still be setting up around the call
  auto q = std::make_shared<std::deque<Pending>>(std::move(q_));
  q_.clear();
  loop_.defer([q, err] {
    for (auto& p : *q) {
      ClientResult r;
      r.err = err ? err : ECONNRESET;
      p.cb(std::move(r));
    }
  });
}

}  // namespace tt::ev
