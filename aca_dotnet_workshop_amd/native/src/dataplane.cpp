// ttsidecar-dataplane: the native data plane of the sidecar runtime (daprd equivalent).
//
// The Python sidecar (sidecar/runtime.py) stays the control plane: it loads components,
// resolves secrets, runs subscriptions / bindings / cron and serves every API.  When the
// native data plane is enabled it hands the public sidecar sockets to this process and
// listens on a private socket instead.  This process answers the hot, request-per-task part
// of the API in C++ and forwards everything else to the Python control plane unchanged:
//
//   POST|GET|...  /v1.0/invoke/{appId}/method/{*path}   service invocation (self or peer)
//   POST|PUT      /v1.0/state/{store}                   save (backing cosmos / redis stores)
//   GET|DELETE    /v1.0/state/{store}/{key}             get / delete
//   POST          /v1.0/state/{store}/bulk              bulk get (per-shard fan-out, raw values)
//   POST|PUT      /v1.0-alpha1/state/{store}/query      query (forwarded to the backing planner)
//   POST|PUT      /v1.0/publish/{pubsub}/{*topic}        publish (backing service bus / redis)
//   internal endpoint                                   peer sidecar -> this app
//   GET /metrics                                        Python's exposition + ours
//
// Semantics mirror the Python handlers (sidecar/runtime.py h_invoke/_invoke/h_internal/
// h_state_save/h_state_get/h_state_delete/h_publish) including error codes, ETag handling,
// key prefixes, CloudEvent envelopes and W3C trace propagation; tests run the same API suite
// against both planes (tests/test_dataplane.py).  Reference behaviour: the Dapr HTTP API as
// used in docs/aca/03-aca-dapr-integration, 04-aca-dapr-stateapi, 05-aca-dapr-pubsubapi.
//
// Usage: ttsidecar-dataplane <config.json>   (written by the Python sidecar)
#include <signal.h>
#include <sys/prctl.h>
#include <sys/signalfd.h>
#include <sys/stat.h>
#include <dirent.h>

#include <cstdio>
#include <ctime>
#include <fstream>
#include <map>
#include <random>
#include <sstream>

#include "evhttp.hpp"
#include "daprpb.hpp"
#include "h2.hpp"
#include "json.hpp"
#include "pb.hpp"
#include "pcsample.hpp"
#include "textutil.hpp"

using namespace tt;
using ev::ClientResult;
using ev::Endpoint;
using ev::HeaderList;
using ev::Message;
using ev::Reply;
using namespace tt::text;

namespace {

// ------------------------------------------------------------------------------ utilities
std::mt19937_64& rng() {
  static std::mt19937_64 r{std::random_device{}() ^ ((uint64_t)getpid() << 32)};
  return r;
}

std::string hex_u64(uint64_t v, int digits = 16) {
  static const char* d = "0123456789abcdef";
  std::string s((size_t)digits, '0');
  for (int i = digits - 1; i >= 0; --i, v >>= 4) s[(size_t)i] = d[v & 15];
  return s;
}

std::string uuid4() {
  uint64_t a = rng()(), b = rng()();
  a = (a & 0xFFFFFFFFFFFF0FFFull) | 0x0000000000004000ull;
  b = (b & 0x3FFFFFFFFFFFFFFFull) | 0x8000000000000000ull;
  std::string h = hex_u64(a) + hex_u64(b);
  return h.substr(0, 8) + "-" + h.substr(8, 4) + "-" + h.substr(12, 4) + "-" + h.substr(16, 4) + "-" + h.substr(20);
}

std::string utc_now_iso() {  // 2024-05-01T12:34:56.123456Z (models/dotnet.py format_datetime)
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  tm t;
  gmtime_r(&ts.tv_sec, &t);
  char buf[64];
  std::snprintf(buf, sizeof buf, "%04d-%02d-%02dT%02d:%02d:%02d.%06ldZ", t.tm_year + 1900, t.tm_mon + 1, t.tm_mday,
                t.tm_hour, t.tm_min, t.tm_sec, ts.tv_nsec / 1000);
  return buf;
}

double wall_now() {
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return (double)ts.tv_sec + ts.tv_nsec / 1e9;
}

std::string error_json(std::string_view code, std::string_view msg) {
  return "{\"errorCode\":" + json_str(code) + ",\"message\":" + json_str(msg) + "}";
}

// ws_end / skip_value: tt:: (json.hpp), shared with the backing front

bool valid_json(std::string_view s) { return tt::valid(s); }  // compact(): tt::compact

// The string value of a top-level key of a valid JSON object (the CloudEvent's traceparent),
// found by scanning, without building the object; false when absent or not a plain string (a
// key or value with escapes is decoded by the full parser instead).
bool top_level_string(std::string_view json, std::string_view key, std::string& out) {
  const char* p = tt::ws_end(json.data(), json.data() + json.size());
  const char* e = json.data() + json.size();
  if (p >= e || *p != '{') return false;
  p = tt::ws_end(p + 1, e);
  while (p < e && *p == '"') {
    const char* k = p + 1;
    const char* q = tt::skip_value(p, e);  // past the key's closing quote
    std::string_view name(k, (size_t)(q - 1 - k));
    p = tt::ws_end(q, e);
    if (p >= e || *p != ':') return false;
    p = tt::ws_end(p + 1, e);
    const char* v = p;
    p = tt::skip_value(p, e);
    if (name.find('\\') != std::string_view::npos) {  // an escaped key: the parser decides
      try {
        Value obj = parse(json);
        const Value* x = obj.get(key);
        if (!x || x->t != Value::String) return false;
        out = x->s;
        return true;
      } catch (const std::exception&) {
        return false;
      }
    }
    if (name == key) {
      if (*v != '"') return false;
      std::string_view lit(v + 1, (size_t)(p - 1 - (v + 1)));
      if (lit.find('\\') != std::string_view::npos) {
        try {
          out = parse(std::string_view(v, (size_t)(p - v))).s;
        } catch (const std::exception&) {
          return false;
        }
      } else {
        out.assign(lit);
      }
      return true;
    }
    p = tt::ws_end(p, e);
    if (p < e && *p == ',') p = tt::ws_end(p + 1, e);
  }
  return false;
}

std::string errno_text(int e) {
  switch (e) {
    case ETIMEDOUT: return "timeout";
    case ECONNREFUSED: return "connection refused";
    case ENOENT: return "no such socket";
    case ECONNRESET: return "connection closed";
    case EPROTO: return "malformed upstream response";
    default: return std::string(strerror(e));
  }
}

const std::string* opt_str(const Value& cfg, const char* k) {
  auto* v = cfg.get(k);
  return v && v->t == Value::String ? &v->s : nullptr;
}

// ------------------------------------------------------------------------------ tracing
void hex16(uint64_t v, char* out) {  // 16 lowercase hex digits, no terminator
  static const char* d = "0123456789abcdef";
  for (int i = 15; i >= 0; --i, v >>= 4) out[i] = d[v & 15];
}

// Span ids in fixed buffers: starting a span (every natively handled request) allocates nothing.
struct SpanCtx {
  char trace_id[32], span_id[16], parent_id[16];
  bool has_parent = false, sampled = false;
  double start_wall = 0, t0 = 0;
  std::string_view tid() const { return {trace_id, 32}; }
  std::string_view sid() const { return {span_id, 16}; }
  std::string_view pid() const { return {parent_id, 16}; }
  std::string traceparent() const {
    std::string s;
    s.reserve(55);
    s.append("00-", 3).append(trace_id, 32).append(1, '-').append(span_id, 16).append(sampled ? "-01" : "-00", 3);
    return s;
  }
};

bool parse_traceparent(const std::string* v, SpanCtx& out) {
  if (!v) return false;
  std::string_view s(*v);
  // 00-<32 hex>-<16 hex>-<2 hex>
  if (s.size() < 55 || s[2] != '-' || s[35] != '-' || s[52] != '-') return false;
  bool tz = true, pz = true;
  for (size_t i = 3; i < 35; ++i) {
    if (hexv(s[i]) < 0) return false;
    tz = tz && s[i] == '0';
  }
  for (size_t i = 36; i < 52; ++i) {
    if (hexv(s[i]) < 0) return false;
    pz = pz && s[i] == '0';
  }
  if (tz || pz) return false;
  int f1 = hexv(s[53]), f2 = hexv(s[54]);
  if (f1 < 0 || f2 < 0) return false;
  std::memcpy(out.trace_id, s.data() + 3, 32);
  std::memcpy(out.parent_id, s.data() + 36, 16);
  out.has_parent = true;
  out.sampled = ((f1 * 16 + f2) & 1) != 0;
  return true;
}

class Tracer {
 public:
  void init(const Value& cfg) {
    if (auto* d = opt_str(cfg, "dir")) dir_ = *d;
    if (auto* r = cfg.get("sampleRate"); r && r->t == Value::Number) rate_ = r->n;
    if (auto* r = opt_str(cfg, "role")) role_ = *r;
    if (auto* i = opt_str(cfg, "instance")) instance_ = *i;
    if (auto* f = opt_str(cfg, "file")) path_ = *f;
    if (auto* fe = cfg.get("flushEach"); fe && fe->t == Value::Bool) flush_each_ = fe->b;
    if (!dir_.empty() && path_.empty()) {
      mkdir(dir_.c_str(), 0755);
      std::string safe = role_;
      for (auto& c : safe)
        if (c == '/') c = '_';
      stem_ = dir_ + "/spans-" + safe + "-" + std::to_string(getpid()) + "-";
      path_ = stem_;  // non-empty: tracing on; the file is per UTC day (log retention prunes days)
    }
  }
  SpanCtx start(const std::string* traceparent) {
    SpanCtx s;
    if (!parse_traceparent(traceparent, s)) {
      hex16(rng()(), s.trace_id);
      hex16(rng()(), s.trace_id + 16);
      s.has_parent = false;
      s.sampled = rate_ >= 1.0 || std::uniform_real_distribution<double>(0, 1)(rng()) < rate_;
    }
    hex16(rng()(), s.span_id);
    if (s.sampled) s.start_wall = wall_now();  // only recorded spans carry a timestamp
    s.t0 = ev::now_s();
    return s;
  }
  void end(const SpanCtx& s, const std::string& name, int status, const std::vector<std::pair<std::string, std::string>>& attrs) {
    if (!s.sampled || path_.empty()) return;
    char dur[32];
    std::snprintf(dur, sizeof dur, "%.3f", (ev::now_s() - s.t0) * 1000.0);
    char ts[32];
    std::snprintf(ts, sizeof ts, "%.6f", s.start_wall);
    std::string l = "{\"type\":\"span\",\"role\":" + json_str(role_) + ",\"instance\":" + json_str(instance_) +
                    ",\"name\":" + json_str(name) + ",\"kind\":\"server\",\"traceId\":\"" + std::string(s.tid()) +
                    "\",\"spanId\":\"" + std::string(s.sid()) + "\",\"parentId\":" +
                    (s.has_parent ? "\"" + std::string(s.pid()) + "\"" : std::string("null")) + ",\"ts\":" + ts +
                    ",\"durationMs\":" + dur + ",\"status\":\"" + (status >= 500 ? "error" : "ok") +
                    "\",\"attributes\":{\"http.status\":" + std::to_string(status);
    for (auto& a : attrs) l += "," + json_str(a.first) + ":" + json_str(a.second);
    l += "},\"plane\":\"native\"}\n";
    buf_ += l;
    if (flush_each_ || buf_.size() > 64 * 1024) flush();
  }
  void flush() {
    if (buf_.empty() || path_.empty()) return;
    std::string path = path_;
    if (!stem_.empty()) {
      time_t t = time(nullptr);
      struct tm g;
      gmtime_r(&t, &g);
      char day[16];
      std::strftime(day, sizeof day, "%Y%m%d", &g);
      path = stem_ + day + ".jsonl";
    }
    if (FILE* f = std::fopen(path.c_str(), "a")) {
      std::fwrite(buf_.data(), 1, buf_.size(), f);
      std::fclose(f);
    }
    buf_.clear();
  }

 private:
  std::string dir_, path_, stem_, role_ = "sidecar", instance_;
  double rate_ = 1.0;
  bool flush_each_ = false;
  std::string buf_;
};

// ------------------------------------------------------------------------------ registry
// Same records the Python NameResolver writes: <dir>/<appId>/<instance>.json with
// {"endpoint": ..., "pid": ...}; dead pids are skipped; results cached 0.5 s; round-robin.
class Resolver {
 public:
  std::string dir;
  std::vector<std::string> candidates(const std::string& app) {
    auto& e = cache_[app];
    double t = ev::now_s();
    if (t - e.at > 0.5) {
      e.eps.clear();
      e.at = t;
      std::string d = dir + "/" + app;
      if (DIR* dh = opendir(d.c_str())) {
        std::vector<std::string> files;
        while (dirent* de = readdir(dh)) {
          std::string n = de->d_name;
          if (n.size() > 5 && n[0] != '.' && n.compare(n.size() - 5, 5, ".json") == 0) files.push_back(n);
        }
        closedir(dh);
        std::sort(files.begin(), files.end());
        for (auto& f : files) {
          std::ifstream in(d + "/" + f);
          std::stringstream ss;
          ss << in.rdbuf();
          try {
            Value rec = parse(ss.str());
            auto* ep = rec.get("endpoint");
            auto* pid = rec.get("pid");
            if (!ep || ep->t != Value::String) continue;
            if (pid && pid->t == Value::Number && kill((pid_t)pid->n, 0) != 0 && errno == ESRCH) continue;
            e.eps.push_back(ep->s);
          } catch (const std::exception&) {
          }
        }
      }
    }
    if (e.eps.size() <= 1) return e.eps;
    size_t n = e.rr++ % e.eps.size();
    std::vector<std::string> out(e.eps.begin() + (long)n, e.eps.end());
    out.insert(out.end(), e.eps.begin(), e.eps.begin() + (long)n);
    return out;
  }
  void invalidate(const std::string& app) { cache_.erase(app); }

 private:
  struct Entry {
    double at = -1;
    std::vector<std::string> eps;
    size_t rr = 0;
  };
  std::map<std::string, Entry> cache_;
};

// ------------------------------------------------------------------------------ data plane
// A partitioned store or broker (backing/shards.py): the collection and the topics are split
// over several backing processes, one per rank, and a document or message lives on the shard
// its partition key hashes to (FNV-1a 64 of the key's bytes, modulo the shard count; the
// Python side computes the same hash).  No shard list: one backing.
inline uint64_t fnv1a64(std::string_view s) {
  uint64_t h = 14695981039346656037ull;
  for (unsigned char c : s) {
    h ^= c;
    h *= 1099511628211ull;
  }
  return h;
}
struct Store {
  Endpoint backing;
  std::vector<Endpoint> shards;
  std::string coll_path;  // /cosmos/<acct>/<db>/<coll>
  std::string prefix;
  HeaderList auth;
  size_t shard_of(std::string_view full_key) const { return shards.empty() ? 0 : fnv1a64(full_key) % shards.size(); }
  const Endpoint& ep(size_t shard) const { return shards.empty() ? backing : shards[shard]; }
};
struct Bus {
  Endpoint backing;
  std::vector<Endpoint> shards;
  std::string ns;
  HeaderList auth;
  const Endpoint& ep(std::string_view partition_key) const {
    return shards.empty() ? backing : shards[fnv1a64(partition_key) % shards.size()];
  }
};
inline std::vector<Endpoint> shard_list(const Value& s) {
  std::vector<Endpoint> out;
  if (auto* sh = s.get("shards"); sh && sh->t == Value::Array)
    for (auto& u : sh->items)
      if (u.t == Value::String) out.push_back(Endpoint::parse(u.s));
  if (out.size() == 1) out.clear();
  return out;
}

bool is_invoke_hop(const std::string& k) {  // sidecar/runtime.py _HOP + traceparent
  return ev::is_hop_header(k) || k == "dapr-api-token" || k == "dapr-app-id" || k == "traceparent";
}

class DataPlane {
 public:
  DataPlane(ev::Loop& loop, const Value& cfg) : loop_(loop), client_(loop) {
    app_id_ = *opt_str(cfg, "appId");
    if (auto* a = opt_str(cfg, "app")) {
      app_ = Endpoint::parse(*a);
      has_app_ = true;
    }
    if (auto* t = opt_str(cfg, "appToken")) app_token_ = *t;
    if (auto* t = opt_str(cfg, "apiToken")) api_token_ = *t;
    if (auto* t = opt_str(cfg, "meshToken")) mesh_token_ = *t;
    if (auto* t = cfg.get("mtls"); t && t->t == Value::Object) {
      // mutual TLS with peer sidecars: our workload certificate for both directions
      ev::TlsConfig tc;
      tc.cert = *opt_str(*t, "cert");
      tc.key = *opt_str(*t, "key");
      tc.ca = *opt_str(*t, "ca");
      mesh_server_tls = std::make_shared<ev::TlsContext>(tc, true);
      client_.set_tls(std::make_shared<ev::TlsContext>(tc, false));
    }
    if (auto* r = opt_str(cfg, "registryDir")) resolver_.dir = *r;
    fallback_ = Endpoint::parse(*opt_str(cfg, "fallback"));
    if (auto* v = cfg.get("invokeNative"); v && v->t == Value::Bool) invoke_native_ = v->b;
    if (auto* v = cfg.get("appTimeout"); v && v->t == Value::Number) app_timeout_ = v->n;
    if (auto* v = cfg.get("apiLogging"); v && v->t == Value::Bool) api_logging_ = v->b;
    if (auto* tr = cfg.get("trace")) tracer_.init(*tr);
    if (auto* st = cfg.get("stores"); st && st->t == Value::Object)
      for (size_t i = 0; i < st->keys.size(); ++i) {
        const Value& s = st->items[i];
        Store x;
        x.backing = Endpoint::parse(*opt_str(s, "backing"));
        x.coll_path = "/cosmos/" + quote_all(*opt_str(s, "account")) + "/" + quote_all(*opt_str(s, "db")) + "/" +
                      quote_all(*opt_str(s, "coll"));
        x.prefix = *opt_str(s, "prefix");
        x.auth = auth_headers(s);
        x.shards = shard_list(s);
        stores_[st->keys[i]] = std::move(x);
      }
    if (auto* ps = cfg.get("pubsubs"); ps && ps->t == Value::Object)
      for (size_t i = 0; i < ps->keys.size(); ++i) {
        const Value& s = ps->items[i];
        Bus b;
        b.backing = Endpoint::parse(*opt_str(s, "backing"));
        b.ns = *opt_str(s, "ns");
        b.auth = auth_headers(s);
        b.shards = shard_list(s);
        buses_[ps->keys[i]] = std::move(b);
      }
  }

  ev::Handler api_handler() {
    return [this](Message&& m, Reply r) { on_api(std::move(m), std::move(r)); };
  }
  ev::Handler internal_handler() {
    return [this](Message&& m, Reply r) { on_internal(std::move(m), std::move(r)); };
  }
  ev::Handler control_handler() {
    return [this](Message&& m, Reply r) { on_control(std::move(m), std::move(r)); };
  }
  void flush() {
    flush_api_log();
    tracer_.flush();
  }
  size_t inflight() const { return inflight_; }
  void tick(double now) {
    flush_api_log();
    for (auto& c : consumers_) c->tick(now);
  }
  void begin_stop() {
    for (auto& c : consumers_) c->stop();
  }
  bool drained() const {
    if (inflight_) return false;
    for (auto& c : consumers_)
      if (!c->drained()) return false;
    return true;
  }

 private:
  ev::Loop& loop_;
  ev::Client client_;
  Tracer tracer_;
  Resolver resolver_;
  std::string app_id_, app_token_, api_token_, mesh_token_;

 public:
  std::shared_ptr<ev::TlsContext> mesh_server_tls;  // internal listeners (mutual TLS), when configured
  const std::string& app_id() const { return app_id_; }

 private:
  Endpoint app_, fallback_;
  bool has_app_ = false, invoke_native_ = true, api_logging_ = false;
  double app_timeout_ = 300;
  std::map<std::string, Store> stores_;
  std::map<std::string, Bus> buses_;
  std::map<std::string, uint64_t> counters_;
  std::map<std::pair<std::string, int>, uint64_t> op_counts_;  // (op, status): no label string per request
  size_t inflight_ = 0;

  static HeaderList auth_headers(const Value& s) {
    HeaderList h;
    if (auto* i = opt_str(s, "identity"); i && !i->empty()) h.emplace_back("x-tt-identity", *i);
    if (auto* k = opt_str(s, "key"); k && !k->empty()) h.emplace_back("x-tt-key", *k);
    return h;
  }

  // Dapr's enableApiLogging: one JSON line per API call on stderr (the replica's log stream),
  // same shape as telemetry/logging.py JsonFormatter.
  // Appended straight into the batch buffer (no temporaries: three of these per created task on
  // the API's sidecar).
  void api_log(const std::string& name, int status, const SpanCtx& span) {
    char buf[96];
    std::snprintf(buf, sizeof buf, " status=%d duration_ms=%.3f app_id=", status, (ev::now_s() - span.t0) * 1e3);
    auto sp = name.find(' ');
    std::string& msg = api_log_msg_;
    msg.assign("HTTP API Called method=");
    msg.append(name, 0, sp);
    msg += " path=";
    if (sp != std::string::npos) msg.append(name, sp + 1, std::string::npos);
    msg += buf;
    msg += app_id_;
    if (api_log_role_.empty()) api_log_role_ = json_str(app_id_ + ".sidecar");
    char ts[32];
    std::snprintf(ts, sizeof ts, "%.6f", wall_now());
    std::string& b = api_log_buf_;
    b += "{\"ts\":";
    b += ts;
    b += ",\"level\":\"INFO\",\"role\":";
    b += api_log_role_;
    b += ",\"category\":\"sidecar.http-info\",\"message\":";
    escape_to(b, msg);
    b += ",\"traceId\":\"";
    b += span.tid();
    b += "\",\"spanId\":\"";
    b += span.sid();
    b += "\",\"plane\":\"native\"}\n";
    if (b.size() >= 32768) flush_api_log();
  }
  std::string api_log_msg_, api_log_role_;
  // The lines go out in batches: when 32 KB have gathered and on every loop tick (<= ~50 ms),
  // one write(2) for many API calls instead of one per call on the unbuffered stderr.
  void flush_api_log() {
    if (api_log_buf_.empty()) return;
    std::fwrite(api_log_buf_.data(), 1, api_log_buf_.size(), stderr);
    api_log_buf_.clear();
  }
  std::string api_log_buf_;

  void count(const std::string& op, int status) {
    op_counts_[{op, status}]++;
  }

  // Wrap a Reply so every natively handled request gets a span, a counter and in-flight accounting.
  struct Done {
    DataPlane* dp;
    Reply rep;
    SpanCtx span;
    std::string name, op;
    std::vector<std::pair<std::string, std::string>> attrs;
    void send(int status, const HeaderList& h, std::string_view body) {
      rep.send(status, h, body);
      if (dp->api_logging_) dp->api_log(name, status, span);
      dp->tracer_.end(span, name, status, attrs);
      dp->count(op, status);
      dp->inflight_--;
    }
    void json(int status, std::string_view body) { send(status, {{"content-type", "application/json"}}, body); }
    void error(int status, std::string_view code, std::string_view msg) { json(status, error_json(code, msg)); }
  };
  std::shared_ptr<Done> begin(const Message& m, Reply&& r, std::string op, std::string_view path) {
    inflight_++;
    auto d = std::make_shared<Done>();
    d->dp = this;
    d->rep = std::move(r);
    d->span = tracer_.start(m.header("traceparent"));
    d->name = m.method + " " + std::string(path.substr(0, 80));
    d->op = std::move(op);
    return d;
  }

  static void split_target(const std::string& target, std::string& path, std::string& qs) {
    auto q = target.find('?');
    path = target.substr(0, q);
    qs = q == std::string::npos ? "" : target.substr(q + 1);
  }

  // ---------------------------------------------------------------- pub/sub consumer
  // Competing consumer on one subscription entity: the native counterpart of
  // sidecar/pubsub.py Consumer + runtime.py _make_delivery/_make_dead_letter.  Prefetches up
  // to `prefetch` messages under peek-lock, runs at most `max_conc` app deliveries at once,
  // renews locks of running deliveries, settles outcomes in batches (success -> complete,
  // retry -> abandon, drop -> dead-letter or forward to the deadLetterTopic).
  struct SubSpec {
    std::string name, pubsub, topic, route, entity, ns, dlt;
    Endpoint backing;
    HeaderList auth;
    int lock_ms = 60000, prefetch = 64, max_conc = 32, retry_delay_ms = 0;
    bool raw = false;
  };
  class Consumer {
   public:
    Consumer(DataPlane& dp, SubSpec s) : s_(std::move(s)), dp_(dp) { next_renew_ = ev::now_s() + renew_period(); }
    SubSpec s_;
    uint64_t delivered = 0, succeeded = 0, retried = 0, dropped = 0, errors = 0;

    void start() { pump(); }
    void stop() {
      stopping_ = true;
      while (!queued_.empty()) {  // prefetched but never delivered: give them back
        abandon_.emplace_back(queued_.front().token, 0);
        locked_.erase(queued_.front().token);
        queued_.pop_front();
      }
      schedule_flush();
    }
    // An outstanding long-poll receive is not waited for (its messages' locks simply expire).
    bool drained() const { return running_ == 0 && !settling_ && pending_empty(); }
    void tick(double now) {
      if (!stopping_ && !receiving_ && retry_at_ > 0 && now >= retry_at_) {
        retry_at_ = 0;
        pump();
      }
      if (now >= next_renew_) {
        next_renew_ = now + renew_period();
        if (!locked_.empty() && !stopping_) renew();
      }
    }
    std::string stats_json() const {
      return "{\"delivered\":" + std::to_string(delivered) + ",\"succeeded\":" + std::to_string(succeeded) +
             ",\"retried\":" + std::to_string(retried) + ",\"dropped\":" + std::to_string(dropped) +
             ",\"errors\":" + std::to_string(errors) + ",\"plane\":\"native\"}";
    }

   private:
    struct Msg {
      std::string token, id, body, ctype;
      long long delivery_count = 0;
    };
    DataPlane& dp_;
    std::deque<Msg> queued_;
    std::map<std::string, int> locked_;  // tokens we hold (queued + running)
    int running_ = 0;
    bool receiving_ = false, stopping_ = false, settling_ = false, flush_scheduled_ = false;
    double retry_at_ = 0, backoff_ = 0.1, next_renew_ = 0;
    std::vector<std::string> complete_;
    std::vector<std::pair<std::string, int>> abandon_;
    std::vector<std::pair<std::string, std::string>> deadletter_;

    double renew_period() const { return std::max(s_.lock_ms / 3000.0, 0.05); }
    bool pending_empty() const { return complete_.empty() && abandon_.empty() && deadletter_.empty(); }
    std::string sb_path(const std::string& tail) const { return "/servicebus/" + quote_all(s_.ns) + tail; }

    void pump() {
      if (stopping_ || receiving_) return;
      int room = s_.prefetch - (int)locked_.size();
      if (room <= 0) return;
      receiving_ = true;
      std::string q = "?entity=" + quote_all(s_.entity) + "&max=" + std::to_string(std::min(room, 256)) +
                      "&lockMs=" + std::to_string(s_.lock_ms) + "&waitMs=2000";
      dp_.client_.request(s_.backing, "POST", sb_path("/receive" + q), s_.auth, {}, 32.0,
                          [this](ClientResult&& res) { on_received(std::move(res)); });
    }

    void on_received(ClientResult&& res) {
      receiving_ = false;
      if (res.err || res.resp.status != 200) {
        if (!stopping_) {
          std::fprintf(stderr, "dataplane: %s: receive failed (%s); retrying in %.1fs\n", s_.name.c_str(),
                       res.err ? errno_text(res.err).c_str() : ("HTTP " + std::to_string(res.resp.status)).c_str(),
                       backoff_);
          retry_at_ = ev::now_s() + backoff_;
          backoff_ = std::min(backoff_ * 2, 5.0);
        }
        return;
      }
      backoff_ = 0.1;
      try {
        Value arr = parse(res.resp.body);
        for (auto& v : arr.items) {
          Msg m;
          if (auto* t = v.get("lockToken")) m.token = t->s;
          if (auto* t = v.get("id")) m.id = t->s;
          if (auto* t = v.get("contentType"); t && t->t == Value::String) m.ctype = t->s;
          if (auto* t = v.get("deliveryCount"); t && t->t == Value::Number) m.delivery_count = (long long)t->n;
          if (auto* b = v.get("bodyB64"); b && b->t == Value::String) m.body = unbase64(b->s);
          else if (auto* b = v.get("body"); b && b->t == Value::String) m.body = b->s;
          if (stopping_) {
            abandon_.emplace_back(m.token, 0);
            continue;
          }
          locked_[m.token] = 1;
          queued_.push_back(std::move(m));
        }
      } catch (const std::exception& e) {
        std::fprintf(stderr, "dataplane: %s: bad receive payload: %s\n", s_.name.c_str(), e.what());
      }
      start_deliveries();
      if (stopping_) schedule_flush();
      pump();
    }

    void start_deliveries() {
      while (!queued_.empty() && running_ < s_.max_conc) {
        Msg m = std::move(queued_.front());
        queued_.pop_front();
        running_++;
        delivered++;
        deliver(std::move(m));
      }
    }

    // Build the delivery request exactly like runtime.py _make_delivery.
    void deliver(Msg&& m) {
      std::string body = std::move(m.body);
      std::string ctype = m.ctype.empty() ? "application/json" : m.ctype;
      SpanCtx span;
      bool is_ce = false;
      std::string parent_tp;
      if (ctype.rfind("application/cloudevents", 0) == 0 && valid_json(body)) {
        // the envelope's traceparent by scanning it: no value tree per delivery
        is_ce = true;
        top_level_string(body, "traceparent", parent_tp);
      }
      if (!is_ce && !s_.raw) {
        std::string base = lower(ctype.substr(0, ctype.find(';')));
        std::string ce = "{\"specversion\":\"1.0\",\"id\":" + json_str(m.id.empty() ? uuid4() : m.id) +
                         ",\"source\":\"unknown\",\"type\":\"com.dapr.event.sent\",\"datacontenttype\":" +
                         json_str(base.empty() ? "application/json" : base) + ",\"topic\":" + json_str(s_.topic) +
                         ",\"pubsubname\":" + json_str(s_.pubsub) + ",\"time\":\"" + utc_now_iso() + "\"";
        if (base.find("json") != std::string::npos && !body.empty() && valid_json(body)) ce += ",\"data\":" + compact(body);
        else if (base.find("json") != std::string::npos && body.empty()) ce += ",\"data\":null";
        else if (base.rfind("text/", 0) == 0 || base.find("json") != std::string::npos || body.empty())
          ce += ",\"data\":" + json_str(body);
        else ce += ",\"data_base64\":\"" + base64(body) + "\"";
        ce += "}";
        body = std::move(ce);
        is_ce = true;
      }
      span = dp_.tracer_.start(parent_tp.empty() ? nullptr : &parent_tp);
      HeaderList h;
      h.emplace_back("content-type", is_ce && !s_.raw ? "application/cloudevents+json" : ctype);
      h.emplace_back("traceparent", span.traceparent());
      h.emplace_back("pubsubname", s_.pubsub);
      h.emplace_back("topic", s_.topic);
      std::string token = m.token;
      long long dc = m.delivery_count;
      std::string raw_body = body;  // kept for a dead-letter-topic forward
      std::string out_ct = h[0].second;
      dp_.call_app("POST", "/" + s_.route, std::move(h), std::move(body),
                   [this, token, span, dc, raw_body = std::move(raw_body), out_ct](ClientResult&& res) mutable {
                     int outcome = 1;  // 0 success, 1 retry, 2 drop
                     int status = res.err ? 0 : res.resp.status;
                     if (res.err) {
                       errors++;
                     } else if (status >= 200 && status < 300) {
                       outcome = 0;
                       auto* ct = res.resp.header("content-type");
                       if (!res.resp.body.empty() && ct && ct->find("json") != std::string::npos) {
                         try {
                           Value v = parse(res.resp.body);
                           if (auto* st = v.get("status"); st && st->t == Value::String) {
                             std::string u = st->s;
                             for (auto& c : u) c = (char)std::toupper((unsigned char)c);
                             outcome = u == "RETRY" ? 1 : u == "DROP" ? 2 : 0;
                           }
                         } catch (const std::exception&) {
                         }
                       }
                     } else if (status == 404) {
                       outcome = 2;
                     }
                     dp_.tracer_.end(span, "pubsub/" + s_.topic, outcome == 0 ? status : 500,
                                     {{"messaging.delivery_count", std::to_string(dc)}});
                     dp_.count("deliver", outcome == 0 ? 200 : outcome == 1 ? 503 : 404);
                     finish(token, outcome, raw_body, out_ct);
                   });
    }

    void finish(const std::string& token, int outcome, const std::string& body, const std::string& ctype) {
      running_--;
      if (outcome == 0) {
        succeeded++;
        complete_.push_back(token);
        locked_.erase(token);
      } else if (outcome == 1) {
        retried++;
        abandon_.emplace_back(token, s_.retry_delay_ms);
        locked_.erase(token);
      } else {
        dropped++;
        if (!s_.dlt.empty()) {
          forward_dead_letter(token, body, ctype);
        } else {
          deadletter_.emplace_back(token, "dropped by application");
          locked_.erase(token);
        }
      }
      schedule_flush();
      start_deliveries();
      pump();
    }

    void forward_dead_letter(const std::string& token, const std::string& body, const std::string& ctype) {
      HeaderList h = s_.auth;
      h.emplace_back("content-type", ctype);
      running_++;  // the forward keeps the message "in flight"
      dp_.client_.request(s_.backing, "POST", sb_path("/topics/" + quote_all(s_.dlt) + "/messages"), h, body, 60,
                          [this, token](ClientResult&& res) {
                            running_--;
                            if (!res.err && res.resp.status < 300) complete_.push_back(token);
                            else deadletter_.emplace_back(token, "dropped by application");
                            locked_.erase(token);
                            schedule_flush();
                          });
    }

    void schedule_flush() {
      if (flush_scheduled_) return;
      flush_scheduled_ = true;
      dp_.loop_.defer([this] {
        flush_scheduled_ = false;
        flush();
      });
    }

    void flush() {
      if (settling_ || pending_empty()) return;
      std::string b = "{\"entity\":" + json_str(s_.entity) + ",\"complete\":[";
      for (size_t i = 0; i < complete_.size(); ++i) b += (i ? "," : "") + json_str(complete_[i]);
      b += "],\"abandon\":[";
      for (size_t i = 0; i < abandon_.size(); ++i)
        b += (i ? ",{\"token\":" : "{\"token\":") + json_str(abandon_[i].first) + ",\"delayMs\":" +
             std::to_string(abandon_[i].second) + "}";
      b += "],\"deadletter\":[";
      for (size_t i = 0; i < deadletter_.size(); ++i)
        b += (i ? ",{\"token\":" : "{\"token\":") + json_str(deadletter_[i].first) + ",\"reason\":" +
             json_str(deadletter_[i].second) + "}";
      b += "]}";
      complete_.clear();
      abandon_.clear();
      deadletter_.clear();
      settling_ = true;
      HeaderList h = s_.auth;
      h.emplace_back("content-type", "application/json");
      dp_.client_.request(s_.backing, "POST", sb_path("/settle"), h, b, 60, [this](ClientResult&& res) {
        settling_ = false;
        if (res.err || res.resp.status >= 300)  // locks expire and the broker redelivers (at-least-once)
          std::fprintf(stderr, "dataplane: %s: settle failed\n", s_.name.c_str());
        if (!pending_empty()) flush();
      });
    }

    void renew() {
      std::string b = "{\"entity\":" + json_str(s_.entity) + ",\"renew\":[";
      size_t i = 0;
      for (auto& kv : locked_)
        b += (i++ ? ",{\"token\":" : "{\"token\":") + json_str(kv.first) + ",\"lockMs\":" + std::to_string(s_.lock_ms) + "}";
      b += "]}";
      HeaderList h = s_.auth;
      h.emplace_back("content-type", "application/json");
      dp_.client_.request(s_.backing, "POST", sb_path("/settle"), h, b, 60, [](ClientResult&&) {});
    }
  };
  std::vector<std::unique_ptr<Consumer>> consumers_;

  // Control socket (private to the Python control plane): start consumers, report stats.
  void on_control(Message&& m, Reply r) {
    std::string path, qs;
    split_target(m.target, path, qs);
    if (path == "/subscribe" && m.method == "POST") {
      try {
        Value v = parse(m.body);
        SubSpec s;
        auto str = [&](const char* k) { auto* x = opt_str(v, k); return x ? *x : std::string(); };
        auto num = [&](const char* k, int d) { auto* x = v.get(k); return x && x->t == Value::Number ? (int)x->n : d; };
        s.name = str("name");
        s.pubsub = str("pubsub");
        s.topic = str("topic");
        s.route = str("route");
        s.entity = str("entity");
        s.ns = str("ns");
        s.dlt = str("deadLetterTopic");
        s.backing = Endpoint::parse(str("backing"));
        s.auth = auth_headers(v);
        s.lock_ms = num("lockMs", 60000);
        s.prefetch = std::max(1, num("prefetch", 64));
        s.max_conc = std::max(1, num("maxConcurrent", 32));
        s.retry_delay_ms = num("retryDelayMs", 0);
        if (auto* x = v.get("raw"); x && x->t == Value::Bool) s.raw = x->b;
        consumers_.push_back(std::make_unique<Consumer>(*this, std::move(s)));
        consumers_.back()->start();
        r.empty(204);
      } catch (const std::exception& e) {
        r.json(400, error_json("ERR_MALFORMED_REQUEST", e.what()));
      }
      return;
    }
    if (path == "/stats" && m.method == "GET") {
      std::string b = "{\"consumers\":{";
      for (size_t i = 0; i < consumers_.size(); ++i)
        b += (i ? "," : "") + json_str(consumers_[i]->s_.name) + ":" + consumers_[i]->stats_json();
      b += "},\"inflight\":" + std::to_string(inflight_) + "}";
      r.json(200, b);
      return;
    }
    r.json(404, error_json("ERR_NOT_FOUND", "no such control route"));
  }

  // ---------------------------------------------------------------- routing
  void on_api(Message&& m, Reply r) {
    std::string path, qs;
    split_target(m.target, path, qs);
    if (!api_token_.empty() && path.rfind("/v1.0/healthz", 0) != 0) {
      auto* t = m.header("dapr-api-token");
      if (!t || *t != api_token_) {
        r.json(401, error_json("ERR_API_TOKEN", "invalid api token"));
        return;
      }
    }
    std::vector<std::string_view> seg;
    {
      std::string_view p(path);
      size_t i = 1;
      while (i <= p.size()) {
        size_t j = p.find('/', i);
        if (j == std::string_view::npos) j = p.size();
        seg.push_back(p.substr(i, j - i));
        i = j + 1;
      }
    }
    if (seg.size() == 4 && (lower(seg[0]) == "v1.0-alpha1" || lower(seg[0]) == "v1.0-beta1") &&
        lower(seg[1]) == "state" && lower(seg[3]) == "query" && (m.method == "POST" || m.method == "PUT")) {
      auto it = stores_.find(unquote(seg[2]));
      // state query: straight to the backing's query planner; a partitioned store's
      // cross-partition query fans out and merges here (two phases: sort keys, then the page)
      if (it != stores_.end()) {
        if (it->second.shards.empty()) state_query(std::move(m), std::move(r), it->second, path);
        else state_query_sharded(std::move(m), std::move(r), it->second, path);
        return;
      }
    }
    if (seg.size() >= 2 && lower(seg[0]) == "v1.0") {
      std::string s1 = lower(seg[1]);
      if (s1 == "invoke" && seg.size() >= 4 && lower(seg[3]) == "method" && invoke_native_) {
        size_t off = (size_t)(seg[3].data() + seg[3].size() + 1 - path.data());
        std::string method_path = off <= path.size() ? path.substr(off) : "";
        std::string target = unquote(seg[2]);
        target = target.substr(0, target.find('.'));
        invoke(std::move(m), std::move(r), target, method_path, qs, path);
        return;
      }
      if (s1 == "state" && seg.size() >= 3) {
        std::string store = unquote(seg[2]);
        auto it = stores_.find(store);
        if (it != stores_.end()) {
          if (seg.size() == 3 && (m.method == "POST" || m.method == "PUT")) {
            state_save(std::move(m), std::move(r), store, it->second, path);
            return;
          }
          if (seg.size() == 4 && m.method == "GET") {
            state_get(std::move(m), std::move(r), it->second, unquote(seg[3]), path);
            return;
          }
          if (seg.size() == 4 && (m.method == "POST" || m.method == "PUT") && lower(seg[3]) == "bulk") {
            state_bulk_get(std::move(m), std::move(r), it->second, path);
            return;
          }
          if (seg.size() == 4 && m.method == "DELETE") {
            state_delete(std::move(m), std::move(r), it->second, unquote(seg[3]), path);
            return;
          }
        }
      }
      if (s1 == "publish" && seg.size() >= 4 && (m.method == "POST" || m.method == "PUT")) {
        std::string name = unquote(seg[2]);
        size_t off = (size_t)(seg[3].data() - path.data());
        std::string topic = unquote(std::string_view(path).substr(off));
        auto it = buses_.find(name);
        if (it != buses_.end() && !topic.empty() && publish(m, r, name, topic, it->second, qs, path)) return;
      }
    }
    if (path == "/metrics" && m.method == "GET") {
      metrics(std::move(m), std::move(r));
      return;
    }
    forward_to_control_plane(std::move(m), std::move(r));
  }

  // Everything the native plane does not own goes to the Python control plane verbatim.
  void forward_to_control_plane(Message&& m, Reply r, std::function<void(std::string&)> amend = nullptr) {
    HeaderList h;
    for (auto& kv : m.headers)
      if (!ev::is_hop_header(kv.first)) h.push_back(kv);
    client_.request(fallback_, m.method, m.target, h, m.body, 0,
                    [r, amend = std::move(amend)](ClientResult&& res) {
                      if (res.err) {
                        r.json(503, error_json("ERR_SIDECAR_CONTROL_PLANE", "control plane unreachable: " + errno_text(res.err)));
                        return;
                      }
                      if (amend) amend(res.resp.body);
                      r.send(res.resp.status, res.resp.headers, res.resp.body);
                    });
  }

  void metrics(Message&& m, Reply r) {
    std::string extra = "# HELP sidecar_native_requests_total requests served by the native data plane\n"
                        "# TYPE sidecar_native_requests_total counter\n";
    std::map<std::string, uint64_t> all = counters_;
    for (auto& kv : op_counts_)
      all["app=\"" + app_id_ + "\",op=\"" + kv.first.first + "\",status=\"" + std::to_string(kv.first.second) + "\""] +=
          kv.second;
    for (auto& kv : all) extra += "sidecar_native_requests_total{" + kv.first + "} " + std::to_string(kv.second) + "\n";
    extra += "# HELP sidecar_mtls_handshake_rejected_total mesh TLS handshakes this sidecar refused\n"
             "# TYPE sidecar_mtls_handshake_rejected_total counter\n"
             "sidecar_mtls_handshake_rejected_total{app=\"" + app_id_ + "\"} " +
             std::to_string(ev::tls_server_handshake_rejects.load(std::memory_order_relaxed)) + "\n";
    extra += "# HELP sidecar_pipelined_requests_total requests sent over pipelined local connections "
             "(store and broker calls to the backing's Unix socket)\n"
             "# TYPE sidecar_pipelined_requests_total counter\n"
             "sidecar_pipelined_requests_total{app=\"" + app_id_ + "\"} " + std::to_string(client_.pipelined()) + "\n";
    extra += "# HELP sidecar_client_connects_total outbound connections opened (the pools had none idle); "
             "tls: with a TLS handshake\n"
             "# TYPE sidecar_client_connects_total counter\n"
             "sidecar_client_connects_total{app=\"" + app_id_ + "\",transport=\"any\"} " +
             std::to_string(client_.connects()) + "\n" +
             "sidecar_client_connects_total{app=\"" + app_id_ + "\",transport=\"tls\"} " +
             std::to_string(client_.tls_connects()) + "\n";
    extra += "# HELP sidecar_partitioned_query_rows_total cross-partition state queries: sort-key entries the "
             "shards sent (phase keys) and documents fetched for the merged pages (phase documents)\n"
             "# TYPE sidecar_partitioned_query_rows_total counter\n"
             "sidecar_partitioned_query_rows_total{app=\"" + app_id_ + "\",phase=\"keys\"} " +
             std::to_string(keys_moved_) + "\nsidecar_partitioned_query_rows_total{app=\"" + app_id_ +
             "\",phase=\"documents\"} " + std::to_string(rows_fetched_) + "\n";
    forward_to_control_plane(std::move(m), std::move(r), [extra](std::string& body) { body += extra; });
  }

  // ---------------------------------------------------------------- invoke
  // The request's end-to-end headers, moved out of `m` (its headers are not read afterwards).
  HeaderList fwd_headers(Message& m, const std::string& traceparent, bool drop_mesh) {
    HeaderList h;
    h.reserve(m.headers.size() + 3);
    for (auto& kv : m.headers) {
      if (is_invoke_hop(kv.first)) continue;
      if (drop_mesh && kv.first == "tt-mesh-token") continue;
      h.push_back(std::move(kv));
    }
    h.emplace_back("traceparent", traceparent);
    return h;
  }

  static void relay(Done& d, ClientResult& res) {
    d.send(res.resp.status, res.resp.headers, res.resp.body);
  }

  void invoke(Message&& m, Reply&& r, const std::string& target, const std::string& method_path,
              const std::string& qs, const std::string& path) {
    auto d = begin(m, std::move(r), "invoke", path);
    d->attrs.emplace_back("invoke.target", target);
    HeaderList h = fwd_headers(m, d->span.traceparent(), false);
    h.emplace_back("dapr-caller-app-id", app_id_);
    std::string tgt = "/" + method_path + (qs.empty() ? "" : "?" + qs);
    if (target == app_id_) {
      call_app(m.method, tgt, std::move(h), std::move(m.body), [d, target](ClientResult&& res) {
        if (res.err) {
          d->error(500, "ERR_DIRECT_INVOKE", "failed to invoke, id: " + target + ", err: " + errno_text(res.err));
          return;
        }
        relay(*d, res);
      });
      return;
    }
    auto cands = resolver_.candidates(target);
    if (cands.empty()) {
      resolver_.invalidate(target);
      cands = resolver_.candidates(target);
    }
    if (cands.empty()) {
      d->error(500, "ERR_DIRECT_INVOKE", "failed to resolve address for app-id '" + target + "'");
      return;
    }
    if (!mesh_token_.empty()) h.emplace_back("tt-mesh-token", mesh_token_);
    if (cands.size() > 3) cands.resize(3);
    call_peer(std::make_shared<PeerCall>(PeerCall{d, target, m.method, tgt, std::move(h), std::move(m.body),
                                                  std::move(cands), 0}));
  }

  struct PeerCall {
    std::shared_ptr<Done> d;
    std::string target, method, path;
    HeaderList headers;
    std::string body;
    std::vector<std::string> cands;
    size_t i;
  };
  void call_peer(std::shared_ptr<PeerCall> pc) {
    Endpoint ep = Endpoint::parse(pc->cands[pc->i]);
    client_.request(ep, pc->method, pc->path, pc->headers, pc->body, app_timeout_, [this, pc](ClientResult&& res) {
      if (res.err == ECONNREFUSED || res.err == ENOENT || res.err == ECONNRESET) {
        resolver_.invalidate(pc->target);  // replica went away: try the next one
        if (++pc->i < pc->cands.size()) {
          call_peer(pc);
          return;
        }
      }
      if (res.err) {
        pc->d->error(500, "ERR_DIRECT_INVOKE", "failed to invoke, id: " + pc->target + ", err: " + errno_text(res.err));
        return;
      }
      relay(*pc->d, res);
    });
  }

  void call_app(const std::string& method, const std::string& target, HeaderList&& h, std::string&& body,
                ev::ClientCallback cb) {
    if (!has_app_) {
      loop_.defer([cb = std::move(cb)]() mutable {
        ClientResult r;
        r.err = ECONNREFUSED;
        cb(std::move(r));
      });
      return;
    }
    if (!app_token_.empty()) h.emplace_back("dapr-api-token", app_token_);
    client_.request(app_, method, target, h, body, app_timeout_, std::move(cb));
  }

  void on_internal(Message&& m, Reply r) {
    if (mesh_server_tls) {
      // mutual TLS: the caller proved an environment workload identity; the app-id it claims
      // must be one its certificate names (no spoofed dapr-caller-app-id)
      auto* c = m.header("dapr-caller-app-id");
      if (!m.tls || (c && !(m.tls_peer && names_include(*m.tls_peer, *c)))) {
        r.json(403, error_json("ERR_MESH_AUTH", "caller identity not proven by its mTLS certificate"));
        return;
      }
    }
    if (!mesh_token_.empty()) {
      auto* t = m.header("tt-mesh-token");
      if (!t || *t != mesh_token_) {
        r.json(403, error_json("ERR_MESH_AUTH", "sidecar-to-sidecar call not authenticated"));
        return;
      }
    }
    std::string path, qs;
    split_target(m.target, path, qs);
    auto d = begin(m, std::move(r), "internal", path);
    if (auto* c = m.header("dapr-caller-app-id")) d->attrs.emplace_back("caller", *c);
    HeaderList h = fwd_headers(m, d->span.traceparent(), true);  // dapr-caller-app-id goes along
    std::string app_id = app_id_;
    call_app(m.method, m.target, std::move(h), std::move(m.body), [d, app_id](ClientResult&& res) {
      if (res.err) {
        d->error(502, "ERR_APP_CHANNEL", "app " + app_id + " unreachable: " + errno_text(res.err));
        return;
      }
      relay(*d, res);
    });
  }

  static bool names_include(const std::string& csv, const std::string& name) {
    size_t p = 0;
    while (p <= csv.size()) {
      size_t e = csv.find(',', p);
      if (e == std::string::npos) e = csv.size();
      if (csv.compare(p, e - p, name) == 0) return true;
      p = e + 1;
    }
    return false;
  }

  // ---------------------------------------------------------------- state
  struct Item {
    std::string key, value, etag;
    bool first_write = false;
    long long ttl_ms = 0;
  };

  // Parse the Dapr save-state body: [{"key","value","etag","options":{"concurrency"},"metadata":{"ttlInSeconds"}}]
  static bool parse_items(const std::string& body, std::vector<Item>& items, std::string& err) {
    if (!valid_json(body)) {
      err = "request body is not valid JSON";
      return false;
    }
    const char* p = ws_end(body.data(), body.data() + body.size());
    const char* e = body.data() + body.size();
    if (p >= e || *p != '[') {
      err = "request body must be an array of state items";
      return false;
    }
    ++p;
    while (true) {
      p = ws_end(p, e);
      if (p < e && *p == ']') break;
      if (p >= e || *p != '{') {
        err = "state item without key";
        return false;
      }
      Item it;
      bool have_value = false;
      ++p;
      while (true) {
        p = ws_end(p, e);
        if (*p == '}') {
          ++p;
          break;
        }
        const char* ks = p;
        p = skip_value(p, e);
        std::string_view ktok(ks, (size_t)(p - ks));
        std::string k = ktok.size() >= 2 && ktok.find('\\') == std::string_view::npos
                            ? std::string(ktok.substr(1, ktok.size() - 2))  // plain key: no unescaping
                            : parse(ktok).s;
        p = ws_end(p, e) + 1;  // ':'
        p = ws_end(p, e);
        const char* vs = p;
        p = skip_value(p, e);
        std::string_view raw(vs, (size_t)(p - vs));
        if (k == "key") {
          if (raw.size() >= 2 && raw.front() == '"' && raw.find('\\') == std::string_view::npos) {
            it.key.assign(raw.data() + 1, raw.size() - 2);
          } else {
            Value v = parse(raw);
            if (v.t == Value::String) it.key = v.s;
          }
        } else if (k == "value") {
          it.value = compact(raw);
          have_value = true;
        } else if (k == "etag") {
          Value v = parse(raw);
          if (v.t == Value::String) it.etag = v.s;
          else if (auto* x = v.get("value"); x && x->t == Value::String) it.etag = x->s;
        } else if (k == "options") {
          Value v = parse(raw);
          if (auto* c = v.get("concurrency"); c && c->t == Value::String) it.first_write = c->s == "first-write";
        } else if (k == "metadata") {
          Value v = parse(raw);
          if (auto* t = v.get("ttlInSeconds")) {
            double s = t->t == Value::Number ? t->n : t->t == Value::String ? std::atof(t->s.c_str()) : 0.0;
            it.ttl_ms = (long long)(s * 1000);
          }
        }
        p = ws_end(p, e);
        if (*p == ',') ++p;
      }
      if (it.key.empty()) {
        err = "state item without key";
        return false;
      }
      if (!have_value) it.value = "null";
      items.push_back(std::move(it));
      p = ws_end(p, e);
      if (*p == ',') ++p;
    }
    return true;
  }

  // Requests to the state store retry throttled answers (429, provisioned RU/s exhausted) after
  // the store's x-ms-retry-after-ms, like the Cosmos SDK under Dapr's state.azure.cosmosdb:
  // at most 9 retries and 30 s of accumulated waiting, then the 429 is the caller's.
  struct StoreCall {
    Endpoint ep;
    std::string method, target, body;
    HeaderList headers;
    ev::ClientCallback cb;
    int attempt = 0;
    double waited = 0.0;
    bool pipeline = true;
  };

  // `pipeline`: over the pipelined connections (ev::Client::request_pipelined) -- every store
  // call but the queries, which can take milliseconds and would hold up the answers behind them
  void store_request(const Endpoint& ep, std::string method, std::string target, HeaderList h, std::string body,
                     ev::ClientCallback cb, bool pipeline = true) {
    auto c = std::make_shared<StoreCall>();
    c->pipeline = pipeline;
    c->ep = ep;
    c->method = std::move(method);
    c->target = std::move(target);
    c->headers = std::move(h);
    c->body = std::move(body);
    c->cb = std::move(cb);
    store_send(std::move(c));
  }

  void store_send(std::shared_ptr<StoreCall> c) {
    StoreCall& k = *c;
    auto on_done = [this, c](ClientResult&& res) {
      if (!res.err && res.resp.status == 429 && c->attempt < 9) {
        const std::string* ra = res.resp.header("x-ms-retry-after-ms");
        double delay = ra ? std::strtod(ra->c_str(), nullptr) / 1000.0 : 0.1;
        delay = std::min(std::max(delay, 0.001), 5.0);
        if (c->waited + delay <= 30.0) {
          count("state.throttled_retry", 429);
          c->attempt++;
          c->waited += delay;
          // the store reserved this call a slot: the retry presents its ticket and is admitted
          // there without a second charge (DocStore::charge), so waiters do not collide again
          auto& hs = c->headers;
          hs.erase(std::remove_if(hs.begin(), hs.end(), [](const auto& h) { return h.first == "x-tt-ru-ticket"; }),
                   hs.end());
          if (const std::string* t = res.resp.header("x-tt-ru-ticket")) hs.emplace_back("x-tt-ru-ticket", *t);
          loop_.call_later(delay, [this, c] { store_send(c); });
          return;
        }
      }
      c->cb(std::move(res));
    };
    if (k.pipeline) client_.request_pipelined(k.ep, k.method, k.target, k.headers, k.body, 60, std::move(on_done));
    else client_.request(k.ep, k.method, k.target, k.headers, k.body, 60, std::move(on_done));
  }

  void state_save(Message&& m, Reply&& r, const std::string& name, const Store& s, const std::string& path) {
    auto d = begin(m, std::move(r), "state.save", path);
    std::vector<Item> items;
    std::string err;
    if (!parse_items(m.body, items, err)) {
      d->error(400, "ERR_MALFORMED_REQUEST", err);
      return;
    }
    auto done = [d, name](ClientResult&& res) {
      if (!res.err && (res.resp.status == 409 || res.resp.status == 412)) {
        d->error(409, "ERR_STATE_SAVE", "failed saving state in state store " + name + ": state save: HTTP " +
                                            std::to_string(res.resp.status) + " " + res.resp.body.substr(0, 200));
        return;
      }
      if (res.err || res.resp.status >= 300) {
        d->error(500, "ERR_STATE_SAVE", "failed saving state in state store " + name + ": " +
                                            (res.err ? errno_text(res.err) : "HTTP " + std::to_string(res.resp.status)));
        return;
      }
      d->send(204, {}, {});
    };
    if (items.empty()) {
      d->send(204, {}, {});
      return;
    }
    HeaderList h = s.auth;
    h.emplace_back("content-type", "application/json");
    if (s.shards.empty()) {
      save_on(s, 0, h, items, std::move(done));
      return;
    }
    // partitioned: one request per shard the items hash to, answered when all have answered
    // (a bulk save is not atomic in Dapr either; the worst status wins)
    std::map<size_t, std::vector<Item>> by_shard;
    for (auto& it : items) by_shard[s.shard_of(full_key(s, it.key))].push_back(std::move(it));
    if (by_shard.size() == 1) {
      save_on(s, by_shard.begin()->first, h, by_shard.begin()->second, std::move(done));
      return;
    }
    struct Join {
      size_t left;
      ClientResult worst;
      bool have = false;
      ev::ClientCallback done;
    };
    auto j = std::make_shared<Join>();
    j->left = by_shard.size();
    j->done = std::move(done);
    for (auto& kv : by_shard)
      save_on(s, kv.first, h, kv.second, [j](ClientResult&& res) {
        auto rank = [](const ClientResult& r) {
          return r.err ? 3 : (r.resp.status == 409 || r.resp.status == 412) ? 2 : r.resp.status >= 300 ? 1 : 0;
        };
        if (!j->have || rank(res) > rank(j->worst)) {
          j->worst = std::move(res);
          j->have = true;
        }
        if (--j->left == 0) j->done(std::move(j->worst));
      });
  }

  void save_on(const Store& s, size_t shard, HeaderList h, std::vector<Item>& items, ev::ClientCallback done) {
    if (items.size() == 1) {
      Item& it = items[0];
      if (!it.etag.empty()) h.emplace_back("if-match", it.etag);
      if (it.first_write) h.emplace_back("x-tt-first-write", "1");
      if (it.ttl_ms) h.emplace_back("x-tt-ttl-ms", std::to_string(it.ttl_ms));
      store_request(s.ep(shard), "PUT", s.coll_path + "/docs/" + quote_all(full_key(s, it.key)), std::move(h), it.value,
                    std::move(done));
      return;
    }
    std::string body = "[";
    for (size_t i = 0; i < items.size(); ++i) {
      auto& it = items[i];
      if (i) body += ',';
      // a value that is a JSON object/array/number/literal goes in as itself (the body was
      // validated and it.value is its compact text): the store parses it once, no escaping
      // here and no unescaping there; a JSON string value travels as JSON text in a string
      const bool as_text = it.value.empty() || it.value[0] == '"';
      body += "{\"key\":" + json_str(full_key(s, it.key)) + ",\"value\":" + (as_text ? json_str(it.value) : it.value) +
              ",\"etag\":" + (it.etag.empty() ? std::string("null") : json_str(it.etag)) +
              ",\"firstWrite\":" + (it.first_write ? "true" : "false") + ",\"ttlMs\":" + std::to_string(it.ttl_ms) + "}";
    }
    body += "]";
    // a bulk save takes the store a millisecond or two: not on the pipelined connections, where
    // the single saves queued behind it would wait for it
    store_request(s.ep(shard), "POST", s.coll_path + "/bulkset", std::move(h), std::move(body), std::move(done), false);
  }

  static std::string full_key(const Store& s, const std::string& key) {
    if (s.prefix.empty() && key.find("||") != std::string::npos) return key;
    return s.prefix + key;
  }

  void state_get(Message&& m, Reply&& r, const Store& s, const std::string& key, const std::string& path) {
    auto d = begin(m, std::move(r), "state.get", path);
    const std::string fk = full_key(s, key);
    store_request(s.ep(s.shard_of(fk)), "GET", s.coll_path + "/docs/" + quote_all(fk), s.auth, {},
                    [d](ClientResult&& res) {
                      if (res.err || (res.resp.status != 200 && res.resp.status != 404)) {
                        d->error(500, "ERR_STATE_GET", "state get: " + (res.err ? errno_text(res.err)
                                                                               : "HTTP " + std::to_string(res.resp.status)));
                        return;
                      }
                      if (res.resp.status == 404) {
                        d->send(204, {}, {});
                        return;
                      }
                      const std::string* et = res.resp.header("etag");
                      d->send(200, {{"etag", et ? *et : ""}, {"content-type", "application/json"}}, res.resp.body);
                    });
  }

  // POST /v1.0/state/{store}/bulk {"keys": [...]}: one bulkget per shard the keys hash to,
  // answered in request order as [{"key", "data", "etag"} | {"key"}] -- the stored JSON goes
  // through as raw slices (the read half of the API's conditional markoverdue).
  struct BulkGet {
    std::vector<std::string> keys, full;  // as asked / with the store's key prefix
    std::vector<std::string> bodies;      // the shards' answers (the slices below point into them)
    std::unordered_map<std::string, std::pair<std::string_view, std::string>> found;  // full key -> data, etag
    size_t left = 0;
    bool failed = false;
    std::string error;
  };

  static bool scan_bulkget(const std::string& body, BulkGet& bg) {
    const char* p = tt::ws_end(body.data(), body.data() + body.size());
    const char* e = body.data() + body.size();
    if (p >= e || *p != '[') return false;
    ++p;
    while (true) {
      p = tt::ws_end(p, e);
      if (p < e && *p == ']') return true;
      if (p >= e || *p != '{') return false;
      ++p;
      std::string key, etag;
      std::string_view data;
      while (true) {
        p = tt::ws_end(p, e);
        if (p < e && *p == '}') {
          ++p;
          break;
        }
        const char* ks = p;
        p = tt::skip_value(p, e);
        std::string_view name(ks, (size_t)(p - ks));
        p = tt::ws_end(p, e);
        if (p >= e || *p != ':') return false;
        const char* vs = tt::ws_end(p + 1, e);
        p = tt::skip_value(vs, e);
        std::string_view val(vs, (size_t)(p - vs));
        try {
          if (name == "\"key\"") key = tt::parse(val).s;
          else if (name == "\"etag\"") etag = tt::parse(val).s;
          else if (name == "\"data\"") data = val;
        } catch (const std::exception&) {
          return false;
        }
        p = tt::ws_end(p, e);
        if (p < e && *p == ',') ++p;
      }
      if (!data.empty()) bg.found[key] = {data, std::move(etag)};
      p = tt::ws_end(p, e);
      if (p < e && *p == ',') ++p;
    }
  }

  // One bulkget per shard the full keys hash to; `done` runs once every shard has answered,
  // with bg->found filled (or bg->failed).
  void fetch_docs(const Store& s, const std::shared_ptr<BulkGet>& bg, std::function<void()> done) {
    std::map<size_t, std::vector<size_t>> by_shard;
    for (size_t i = 0; i < bg->full.size(); ++i) by_shard[s.shards.empty() ? 0 : s.shard_of(bg->full[i])].push_back(i);
    if (by_shard.empty()) {
      done();
      return;
    }
    bg->left = by_shard.size();
    bg->bodies.resize(by_shard.size());
    auto fin = std::make_shared<std::function<void()>>(std::move(done));
    HeaderList h = s.auth;
    h.emplace_back("content-type", "application/json");
    size_t slot = 0;
    for (auto& kv : by_shard) {
      std::string body = "{\"keys\":[";
      for (size_t j = 0; j < kv.second.size(); ++j) body += (j ? "," : "") + json_str(bg->full[kv.second[j]]);
      body += "]}";
      store_request(s.ep(kv.first), "POST", s.coll_path + "/bulkget", h, std::move(body),
                    [bg, slot, fin](ClientResult&& res) {
                      if (res.err || res.resp.status != 200) {
                        bg->failed = true;
                        if (bg->error.empty())
                          bg->error = res.err ? errno_text(res.err) : "HTTP " + std::to_string(res.resp.status);
                      } else {
                        bg->bodies[slot] = std::move(res.resp.body);
                        if (!scan_bulkget(bg->bodies[slot], *bg)) bg->failed = true, bg->error = "unreadable bulkget";
                      }
                      if (--bg->left == 0) (*fin)();
                    },
                    bg->keys.size() <= 16);  // a large bulk get is not pipelined either (see bulkset)
      ++slot;
    }
  }

  void state_bulk_get(Message&& m, Reply&& r, const Store& s, const std::string& path) {
    auto d = begin(m, std::move(r), "state.bulkget", path);
    auto bg = std::make_shared<BulkGet>();
    try {
      Value v = parse(m.body.empty() ? std::string("{}") : m.body);
      const Value* ks = v.get("keys");
      if (ks && ks->t == Value::Array)
        for (auto& k : ks->items) {
          if (k.t != Value::String) throw std::runtime_error("keys must be strings");
          bg->keys.push_back(k.s);
          bg->full.push_back(full_key(s, k.s));
        }
    } catch (const std::exception& ex) {
      d->error(400, "ERR_MALFORMED_REQUEST", std::string("bulk get: ") + ex.what());
      return;
    }
    fetch_docs(s, bg, [d, bg] {
      if (bg->failed) {
        d->error(500, "ERR_STATE_BULK_GET", "bulk get: " + bg->error);
        return;
      }
      std::string out = "[";
      for (size_t i = 0; i < bg->keys.size(); ++i) {
        out += i ? ",{\"key\":" : "{\"key\":";
        out += json_str(bg->keys[i]);
        auto it = bg->found.find(bg->full[i]);
        if (it != bg->found.end()) {
          out += ",\"data\":";
          out.append(it->second.first);
          out += ",\"etag\":" + json_str(it->second.second);
        }
        out += '}';
      }
      out += ']';
      d->send(200, {{"content-type", "application/json"}}, out);
    });
  }

  // ---------------------------------------------------------------- cross-partition query
  // A partitioned store's state query (backing/shards.py semantics, natively): every shard
  // still holding matches answers its own sorted page as SORT KEYS only (`?project=sortkeys`:
  // key, etag and the values at the sort paths); the pages are k-way merged on those values
  // (the store's JSON order, ties in shard order); then only the merged page's documents are
  // fetched, one bulkget per shard.  At N shards a page of `limit` moves N x limit small key
  // entries plus `limit` documents, not N x limit documents.  The continuation token is the
  // shards' offsets ("p1." + url-safe base64 of a JSON array; null = exhausted), the same one
  // the Python plane issues.
  struct ShardPage {
    std::vector<std::string> keys;        // without the store's key prefix
    std::vector<std::vector<Value>> sort;  // sort values per result
    bool more = false;
    bool present = false;  // asked (offset not null)
    long long next = -1;   // the shard's own continuation (its position after the page), when numeric
  };
  struct XQuery {
    std::vector<std::pair<std::string, bool>> sort;  // path, desc
    size_t limit = 0;
    std::vector<long long> offsets;  // -1 = exhausted
    std::vector<ShardPage> pages;
    size_t left = 0;
    bool failed = false;
    int fail_status = 500;
    std::string error;
  };

  static std::string b64url(std::string_view in) {
    std::string o = base64(in);
    for (char& c : o) c = c == '+' ? '-' : c == '/' ? '_' : c;
    while (!o.empty() && o.back() == '=') o.pop_back();
    return o;
  }
  static std::string unb64url(std::string_view in) {
    std::string t(in);
    for (char& c : t) c = c == '-' ? '+' : c == '_' ? '/' : c;
    return unbase64(t);
  }
  static bool decode_xtoken(const std::string& tok, size_t n, std::vector<long long>& offs) {
    offs.assign(n, 0);
    if (tok.empty()) return true;
    if (tok.rfind("p1.", 0) != 0) return false;
    try {
      Value v = parse(unb64url(std::string_view(tok).substr(3)));
      if (v.t != Value::Array || v.items.size() != n) return false;
      for (size_t i = 0; i < n; ++i) {
        const Value& x = v.items[i];
        if (x.t == Value::Null) offs[i] = -1;
        else if (x.t == Value::Number && x.n >= 0 && x.n == (double)(long long)x.n) offs[i] = (long long)x.n;
        else return false;
      }
    } catch (const std::exception&) {
      return false;
    }
    return true;
  }

  void state_query_sharded(Message&& m, Reply&& r, const Store& s, const std::string& path) {
    auto d = begin(m, std::move(r), "state.query", path);
    auto x = std::make_shared<XQuery>();
    const size_t n = s.shards.size();
    Value q;
    std::string token;
    try {
      q = parse(m.body.empty() ? std::string("{}") : m.body);
      if (q.t != Value::Object) throw std::runtime_error("query must be a JSON object");
      if (const Value* sv = q.get_ci("sort"); sv && sv->t == Value::Array)
        for (auto& e : sv->items) {
          const Value* k = e.get_ci("key");
          if (!k || k->t != Value::String) throw std::runtime_error("sort entry needs a string key");
          const Value* o = e.get_ci("order");
          x->sort.emplace_back(k->s, o && o->t == Value::String && lower(o->s) == "desc");
        }
      if (Value* pg = const_cast<Value*>(q.get_ci("page")); pg && pg->t == Value::Object) {
        if (const Value* l = pg->get_ci("limit"); l && l->t == Value::Number && l->n > 0) x->limit = (size_t)l->n;
        if (const Value* t = pg->get_ci("token"); t && t->t == Value::String) token = t->s;
      }
    } catch (const std::exception& ex) {
      d->error(400, "ERR_STATE_QUERY", std::string("state query: ") + ex.what());
      return;
    }
    if (!decode_xtoken(token, n, x->offsets)) {
      d->error(400, "ERR_STATE_QUERY", "state query: invalid continuation token for a partitioned collection");
      return;
    }
    x->pages.resize(n);
    // the shard's sub-query: the same filter and sort, its own offset as the token
    auto sub_query = [&](long long off) {
      Value sub = q;
      Value page;
      page.t = Value::Object;
      if (x->limit) page.keys.push_back("limit"), page.items.push_back(Value::number((double)x->limit));
      if (off > 0) page.keys.push_back("token"), page.items.push_back(Value::string(std::to_string(off)));
      for (size_t i = 0; i < sub.keys.size(); ++i)
        if (lower(sub.keys[i]) == "page") {
          sub.keys.erase(sub.keys.begin() + (long)i);
          sub.items.erase(sub.items.begin() + (long)i);
          break;
        }
      if (!page.keys.empty()) sub.keys.push_back("page"), sub.items.push_back(std::move(page));
      return dump(sub);
    };
    std::string target = s.coll_path + "/query?project=sortkeys";
    if (!s.prefix.empty()) target += "&prefix=" + quote_all(s.prefix);
    HeaderList h = s.auth;
    h.emplace_back("content-type", "application/json");
    for (size_t i = 0; i < n; ++i)
      if (x->offsets[i] >= 0) x->left++;
    if (x->left == 0) {  // every shard exhausted
      d->send(200, {{"content-type", "application/json"}}, "{\"results\":[]}");
      return;
    }
    for (size_t i = 0; i < n; ++i) {
      if (x->offsets[i] < 0) continue;
      x->pages[i].present = true;
      store_request(s.ep(i), "POST", target, h, sub_query(x->offsets[i]), [this, d, x, i, &s](ClientResult&& res) {
        if (res.err || res.resp.status != 200) {
          if (!x->failed) {
            x->failed = true;
            x->fail_status = (!res.err && res.resp.status == 400) ? 400 : 500;
            x->error = res.err ? errno_text(res.err)
                               : "HTTP " + std::to_string(res.resp.status) + " " + res.resp.body.substr(0, 300);
          }
        } else {
          try {
            Value v = parse(res.resp.body);
            ShardPage& pg = x->pages[i];
            if (const Value* t = v.get("token"); t && t->t == Value::String && !t->s.empty()) {
              pg.more = true;
              char* end = nullptr;
              long long nx = std::strtoll(t->s.c_str(), &end, 10);
              if (end && *end == 0 && nx >= 0) pg.next = nx;
            }
            if (const Value* rs = v.get("results"); rs && rs->t == Value::Array)
              for (auto& it : rs->items) {
                const Value* k = it.get("key");
                const Value* sv = it.get("sort");
                if (!k || k->t != Value::String) continue;
                pg.keys.push_back(k->s);
                pg.sort.push_back(sv && sv->t == Value::Array ? sv->items : std::vector<Value>());
              }
            keys_moved_ += pg.keys.size();
          } catch (const std::exception& ex) {
            x->failed = true;
            x->error = std::string("unreadable shard page: ") + ex.what();
          }
        }
        if (--x->left == 0) merge_and_fetch(d, x, s);
      }, false);
    }
  }

  void merge_and_fetch(const std::shared_ptr<Done>& d, const std::shared_ptr<XQuery>& x, const Store& s) {
    if (x->failed) {
      d->error(x->fail_status, "ERR_STATE_QUERY", "state query: " + x->error);
      return;
    }
    const size_t n = x->pages.size();
    std::vector<size_t> pos(n, 0), used(n, 0);
    static const Value kNull;
    auto less = [&](size_t a, size_t b) {  // shard a's head before shard b's head
      const auto& va = x->pages[a].sort[pos[a]];
      const auto& vb = x->pages[b].sort[pos[b]];
      for (size_t k = 0; k < x->sort.size(); ++k) {
        int c = compare(k < va.size() ? va[k] : kNull, k < vb.size() ? vb[k] : kNull);
        if (c) return x->sort[k].second ? c > 0 : c < 0;
      }
      return a < b;
    };
    auto bg = std::make_shared<BulkGet>();
    std::vector<size_t> order_shard;  // the merged page, as (shard) per entry; keys in bg
    // a k-way PAGED merge: once a shard that has more matches (it sent a continuation) runs out
    // of this page's entries, its unfetched ones may sort before anything left here -- the
    // merged page ends there (a shard can send a short page: its mirror skipped stale rows)
    auto starved = [&] {
      for (size_t i = 0; i < n; ++i)
        if (x->pages[i].more && pos[i] >= x->pages[i].keys.size()) return true;
      return false;
    };
    while ((!x->limit || bg->full.size() < x->limit) && !starved()) {
      size_t best = n;
      for (size_t i = 0; i < n; ++i) {
        if (pos[i] >= x->pages[i].keys.size()) continue;
        if (x->sort.empty()) {  // unsorted: shard order
          best = i;
          break;
        }
        if (best == n || less(i, best)) best = i;
      }
      if (best == n) break;
      bg->keys.push_back(x->pages[best].keys[pos[best]]);
      bg->full.push_back(full_key(s, bg->keys.back()));
      ++pos[best];
      ++used[best];
    }
    // next offsets: a shard is exhausted when it said so and every result it gave was used
    std::string tok;
    if (x->limit) {
      bool any = false;
      std::string arr = "[";
      for (size_t i = 0; i < n; ++i) {
        if (i) arr += ',';
        const ShardPage& pg = x->pages[i];
        if (!pg.present || (!pg.more && used[i] == pg.keys.size())) {
          arr += "null";
        } else {  // a fully used page resumes where the shard said (past any rows it skipped)
          bool all = used[i] == pg.keys.size();
          arr += std::to_string(all && pg.next >= 0 ? pg.next : x->offsets[i] + (long long)used[i]);
          any = true;
        }
      }
      arr += ']';
      if (any) tok = "p1." + b64url(arr);
    }
    rows_fetched_ += bg->full.size();
    fetch_docs(s, bg, [d, bg, tok] {
      if (bg->failed) {
        d->error(500, "ERR_STATE_QUERY", "state query: " + bg->error);
        return;
      }
      std::string out = "{\"results\":[";
      bool first = true;
      for (size_t i = 0; i < bg->keys.size(); ++i) {
        auto it = bg->found.find(bg->full[i]);
        if (it == bg->found.end()) continue;  // deleted between the two phases
        out += first ? "{\"key\":" : ",{\"key\":";
        first = false;
        out += json_str(bg->keys[i]);
        out += ",\"data\":";
        out.append(it->second.first);
        out += ",\"etag\":" + json_str(it->second.second);
        out += '}';
      }
      out += ']';
      if (!tok.empty()) out += ",\"token\":" + json_str(tok);
      out += '}';
      d->send(200, {{"content-type", "application/json"}}, out);
    });
  }
  uint64_t keys_moved_ = 0, rows_fetched_ = 0;

  // sidecar/runtime.py h_state_query: the filter goes to the backing's query route (hash
  // indexes / GPU columnar planner there) with the store's key prefix; 400 from the backing is
  // the caller's filter, anything else a store failure.
  void state_query(Message&& m, Reply&& r, const Store& s, const std::string& path) {
    auto d = begin(m, std::move(r), "state.query", path);
    std::string target = s.coll_path + "/query";
    if (!s.prefix.empty()) target += "?prefix=" + quote_all(s.prefix);
    HeaderList h = s.auth;
    h.emplace_back("content-type", "application/json");
    if (d->span.sampled) {  // the store's spans join the trace, with when this hop sent (CLOCK_MONOTONIC s)
      h.emplace_back("traceparent", d->span.traceparent());
      char t[32];
      std::snprintf(t, sizeof t, "%.6f", ev::now_s());
      h.emplace_back("x-tt-sent-mono", t);
    }
    store_request(s.backing, "POST", target, h, m.body.empty() ? std::string("{}") : m.body,
                    [d](ClientResult&& res) {
                      if (!res.err && res.resp.status == 200) {
                        if (d->span.sampled) {  // the return path, from the store's monotonic stamps
                          const double now = ev::now_s();
                          for (auto [attr, hdr] : {std::pair{"store_handler_end_to_sidecar_ms", "x-tt-handler-end-mono"},
                                                   std::pair{"store_front_rx_to_sidecar_ms", "x-tt-front-rx-mono"}})
                            if (const std::string* t = res.resp.header(hdr)) {
                              char b[32];
                              std::snprintf(b, sizeof b, "%.3f", (now - std::strtod(t->c_str(), nullptr)) * 1e3);
                              d->attrs.emplace_back(attr, b);
                            }
                        }
                        d->send(200, {{"content-type", "application/json"}}, res.resp.body);
                        return;
                      }
                      int status = (!res.err && res.resp.status == 400) ? 400 : 500;
                      d->error(status, "ERR_STATE_QUERY",
                               "state query: " + (res.err ? errno_text(res.err)
                                                          : "HTTP " + std::to_string(res.resp.status) + " " +
                                                                res.resp.body.substr(0, 300)));
                    },
                    false);
  }

  void state_delete(Message&& m, Reply&& r, const Store& s, const std::string& key, const std::string& path) {
    auto d = begin(m, std::move(r), "state.delete", path);
    HeaderList h = s.auth;
    if (auto* im = m.header("if-match"); im && !im->empty()) h.emplace_back("if-match", *im);
    const std::string fk = full_key(s, key);
    store_request(s.ep(s.shard_of(fk)), "DELETE", s.coll_path + "/docs/" + quote_all(fk), h, {},
                    [d](ClientResult&& res) {
                      if (!res.err && (res.resp.status == 409 || res.resp.status == 412)) {
                        d->error(409, "ERR_STATE_DELETE", "state delete: HTTP " + std::to_string(res.resp.status) +
                                                              " " + res.resp.body.substr(0, 200));
                        return;
                      }
                      if (res.err || (res.resp.status != 204 && res.resp.status != 404)) {
                        d->error(500, "ERR_STATE_DELETE", "state delete: " + (res.err ? errno_text(res.err)
                                                                                     : "HTTP " + std::to_string(res.resp.status)));
                        return;
                      }
                      d->send(204, {}, {});
                    });
  }

  // ---------------------------------------------------------------- publish
  // Returns false when the request should go to the control plane (rare envelope shapes).
  bool publish(Message& m, Reply& r, const std::string& name, const std::string& topic, const Bus& b,
               const std::string& qs, const std::string& path) {
    std::map<std::string, std::string> meta;
    for (size_t i = 0; i <= qs.size() && !qs.empty();) {
      size_t j = qs.find('&', i);
      if (j == std::string::npos) j = qs.size();
      std::string_view kv(qs.data() + i, j - i);
      size_t eq = kv.find('=');
      std::string k = unquote(kv.substr(0, eq), true);
      std::string v = eq == std::string_view::npos ? "" : unquote(kv.substr(eq + 1), true);
      if (k.rfind("metadata.", 0) == 0) meta[k.substr(9)] = v;
      i = j + 1;
    }
    const std::string* ct = m.header("content-type");
    std::string ctype = ct && !ct->empty() ? *ct : "application/json";
    std::string base = lower(ctype.substr(0, ctype.find(';')));
    while (!base.empty() && base.back() == ' ') base.pop_back();
    while (!base.empty() && base.front() == ' ') base.erase(0, 1);
    bool raw = lower(meta.count("rawPayload") ? meta["rawPayload"] : "") == "true";
    if (!raw && base == "application/cloudevents+json") return false;
    bool is_json = base.find("json") != std::string::npos;
    bool json_body = is_json && !m.body.empty() && valid_json(m.body);
    bool as_string = !json_body && (is_json || base.rfind("text/", 0) == 0 || m.body.empty());
    if (!raw && as_string && !valid_utf8(m.body)) return false;  // Python decodes with replacement chars
    auto d = begin(m, std::move(r), "publish", path);
    d->attrs.emplace_back("topic", topic);
    std::string body, out_ct, event_id;
    if (raw) {
      body = std::move(m.body);
      out_ct = ctype;
    } else {
      std::string tp = d->span.traceparent();
      event_id = uuid4();
      body = "{\"specversion\":\"1.0\",\"id\":\"" + event_id + "\",\"source\":" + json_str(app_id_) +
             ",\"type\":\"com.dapr.event.sent\",\"datacontenttype\":" + json_str(base.empty() ? "application/json" : base) +
             ",\"topic\":" + json_str(topic) + ",\"pubsubname\":" + json_str(name) + ",\"time\":\"" + utc_now_iso() + "\"";
      if (is_json) {
        if (m.body.empty()) body += ",\"data\":null";
        else if (json_body) body += ",\"data\":" + compact(m.body);
        else body += ",\"data\":" + json_str(m.body);
      } else if (base.rfind("text/", 0) == 0 || m.body.empty()) {
        body += ",\"data\":" + json_str(m.body);
      } else {
        body += ",\"data_base64\":\"" + base64(m.body) + "\"";
      }
      body += ",\"traceparent\":\"" + tp + "\",\"traceid\":\"" + tp + "\"}";
      out_ct = "application/cloudevents+json";
    }
    HeaderList h = b.auth;
    h.emplace_back("content-type", out_ct);
    std::string props;
    for (auto& kv : meta) {
      if (kv.first == "ttlInSeconds" || kv.first == "rawPayload") continue;
      props += (props.empty() ? "{" : ",") + json_str(kv.first) + ":" + json_str(kv.second);
    }
    if (!props.empty()) h.emplace_back("x-tt-props", props + "}");
    if (meta.count("ttlInSeconds")) {
      long long ttl = (long long)(std::atof(meta["ttlInSeconds"].c_str()) * 1000);
      if (ttl) h.emplace_back("x-tt-ttl-ms", std::to_string(ttl));
    }
    // partitioned broker: the message's partitionKey metadata (Service Bus partitioning), else
    // its CloudEvent id, picks the shard
    // (an empty partitionKey is no key: backing/shards.py routes it by the message id too)
    const std::string pkey = meta.count("partitionKey") && !meta["partitionKey"].empty() ? meta["partitionKey"]
                             : event_id.empty()                                          ? uuid4()
                                                                                         : event_id;
    client_.request_pipelined(b.ep(pkey), "POST", "/servicebus/" + quote_all(b.ns) + "/topics/" + quote_all(topic) + "/messages", h,
                    body, 60, [d, name, topic](ClientResult&& res) {
                      if (res.err || res.resp.status >= 300) {
                        d->error(500, "ERR_PUBSUB_PUBLISH_MESSAGE",
                                 "error when publish to topic " + topic + " in pubsub " + name + ": " +
                                     (res.err ? errno_text(res.err)
                                              : "publish: HTTP " + std::to_string(res.resp.status) + " " +
                                                    res.resp.body.substr(0, 200)));
                        return;
                      }
                      d->send(204, {}, {});
                    });
    return true;
  }

  // ---------------------------------------------------------------- gRPC API
  // dapr.proto.runtime.v1.Dapr over HTTP/2 (h2.hpp): the hot unary RPCs of the reference's
  // DaprClient -- SaveState / GetState / DeleteState / QueryStateAlpha1 / PublishEvent /
  // InvokeService / InvokeBinding (Backend.Api Services/TasksStoreManager.cs:35-155, Processor
  // ExternalTasksProcessorController.cs:33-43) -- are decoded here and run through on_api as
  // the equivalent HTTP API request, so both protocols share one implementation of the
  // semantics (ETags, key prefixes, CloudEvents, tracing, API token).  Every other RPC goes to
  // the control plane's /_tt/grpc/{Method} route, which runs sidecar/grpc_api.py's handler for
  // it.  Errors map HTTP statuses onto gRPC codes exactly like grpc_api.py (_CODES, _fail).
 public:
  h2::GrpcHandler grpc_handler() {
    return [this](h2::GrpcCall&& c, h2::GrpcReply r) { on_grpc(std::move(c), std::move(r)); };
  }

 private:
  static int grpc_code(int http) {
    switch (http) {
      case 400: return 3;   // INVALID_ARGUMENT
      case 401: return 16;  // UNAUTHENTICATED
      case 403: return 7;   // PERMISSION_DENIED
      case 404: return 5;   // NOT_FOUND
      case 405: case 501: return 12;  // UNIMPLEMENTED
      case 409: return 10;  // ABORTED
      case 429: return 8;   // RESOURCE_EXHAUSTED
      case 500: return 13;  // INTERNAL
      case 502: case 503: return 14;  // UNAVAILABLE
      case 504: return 4;   // DEADLINE_EXCEEDED
      default: return http >= 400 ? 2 : 0;  // UNKNOWN
    }
  }
  static void grpc_fail(const h2::GrpcReply& r, int status, std::string_view body, const std::string& what) {
    std::string msg;
    try {
      Value js = parse(body);
      if (js.t == Value::Object) {
        const Value* c = js.get("errorCode");
        const Value* m = js.get("message");
        msg = (c && c->t == Value::String ? c->s : std::string()) + ": " +
              (m && m->t == Value::String ? m->s : dump(js));
      } else {
        msg = dump(js);
      }
    } catch (const std::exception&) {
      msg = std::string(body.substr(0, 500));
    }
    r.error(grpc_code(status), what + ": " + msg, {{"dapr-http-status", std::to_string(status)}});
  }
  // A value carried as bytes on the gRPC side, as the HTTP API's JSON body expects it
  // (grpc_api.py _json_or_text): JSON text embedded as JSON, else a string, else base64.
  static std::string json_or_text(std::string_view raw) {
    if (raw.empty()) return "null";
    if (valid_json(raw)) return compact(raw);
    if (valid_utf8(raw)) return json_str(raw);
    return json_str(base64(raw));
  }
  static std::string meta_qs(const std::vector<std::pair<std::string, std::string>>& meta) {
    std::string qs;
    for (auto& kv : meta) qs += (qs.empty() ? "?" : "&") + quote_all("metadata." + kv.first) + "=" + quote_all(kv.second);
    return qs;
  }
  static std::string quote_path(std::string_view s) {  // quote each '/'-separated segment
    std::string o;
    size_t i = 0;
    while (true) {
      size_t j = s.find('/', i);
      o += quote_all(s.substr(i, j == std::string_view::npos ? std::string_view::npos : j - i));
      if (j == std::string_view::npos) break;
      o += '/';
      i = j + 1;
    }
    return o;
  }
  // Runs a translated request through the HTTP API pipeline; `done` gets the HTTP result.
  using HttpDone = std::function<void(int, const HeaderList&, std::string_view)>;
  void grpc_http(const h2::GrpcCall& c, std::string method, std::string target, std::string body,
                 std::string ctype, HeaderList extra, HttpDone done) {
    Message m;
    m.method = std::move(method);
    m.target = std::move(target);
    for (auto& kv : c.metadata)
      if (kv.first == "dapr-api-token" || kv.first == "traceparent" || kv.first == "tracestate" ||
          kv.first.rfind("dapr-", 0) == 0)
        m.headers.push_back(kv);
    if (!ctype.empty()) m.headers.emplace_back("content-type", std::move(ctype));
    for (auto& kv : extra) m.headers.push_back(std::move(kv));
    m.headers.emplace_back("content-length", std::to_string(body.size()));
    m.body = std::move(body);
    on_api(std::move(m), Reply(std::move(done)));
  }

  struct StateItemPb {
    std::string key, value, etag;
    bool has_etag = false;
    std::vector<std::pair<std::string, std::string>> meta;
    uint64_t concurrency = 0, consistency = 0;
  };
  static bool decode_state_item(std::string_view s, StateItemPb& it) {
    pb::Reader r(s);
    uint32_t f, wt;
    std::string_view v;
    while (r.next(f, wt)) {
      if (f == 1 && wt == pb::LEN && r.bytes(v)) it.key.assign(v);
      else if (f == 2 && wt == pb::LEN && r.bytes(v)) it.value.assign(v);
      else if (f == 3 && wt == pb::LEN && r.bytes(v)) {  // Etag {value = 1}
        it.has_etag = true;
        pb::Reader er(v);
        uint32_t ef, ewt;
        std::string_view ev;
        while (er.next(ef, ewt))
          if (ef == 1 && ewt == pb::LEN && er.bytes(ev)) it.etag.assign(ev);
          else if (!er.skip(ewt)) break;
        if (!er.ok) return false;
      } else if (f == 4 && wt == pb::LEN && r.bytes(v)) {
        std::string k, val;
        if (!pb::map_entry(v, k, val)) return false;
        it.meta.emplace_back(std::move(k), std::move(val));
      } else if (f == 5 && wt == pb::LEN && r.bytes(v)) {  // StateOptions {concurrency = 1, consistency = 2}
        pb::Reader orr(v);
        uint32_t of, owt;
        uint64_t x;
        while (orr.next(of, owt))
          if ((of == 1 || of == 2) && owt == pb::VARINT && orr.varint(x)) (of == 1 ? it.concurrency : it.consistency) = x;
          else if (!orr.skip(owt)) break;
        if (!orr.ok) return false;
      } else if (!r.skip(wt)) {
        break;
      }
    }
    return r.ok;
  }
  static std::string state_item_json(const StateItemPb& it) {
    std::string o = "{\"key\":" + json_str(it.key) + ",\"value\":" + json_or_text(it.value);
    if (it.has_etag) o += ",\"etag\":" + json_str(it.etag);
    if (!it.meta.empty()) {
      o += ",\"metadata\":{";
      for (size_t i = 0; i < it.meta.size(); ++i)
        o += (i ? "," : "") + json_str(it.meta[i].first) + ":" + json_str(it.meta[i].second);
      o += "}";
    }
    std::string opts;
    if (it.concurrency == 1 || it.concurrency == 2)
      opts += std::string("\"concurrency\":\"") + (it.concurrency == 1 ? "first-write" : "last-write") + "\"";
    if (it.consistency == 1 || it.consistency == 2)
      opts += std::string(opts.empty() ? "" : ",") + "\"consistency\":\"" +
              (it.consistency == 1 ? "eventual" : "strong") + "\"";
    if (!opts.empty()) o += ",\"options\":{" + opts + "}";
    return o + "}";
  }

  void on_grpc(h2::GrpcCall&& c, h2::GrpcReply r) {
    static constexpr std::string_view kSvc = "/dapr.proto.runtime.v1.Dapr/";
    if (c.path.compare(0, kSvc.size(), kSvc) != 0) {
      r.error(12, "unknown service: " + c.path);
      return;
    }
    std::string rpc = c.path.substr(kSvc.size());
    counters_["app=\"" + app_id_ + "\",op=\"grpc." + rpc + "\",status=\"call\""]++;
    pb::Reader rd(c.message);
    uint32_t f, wt;
    std::string_view v;
    auto fail_decode = [&] { r.error(3, rpc + ": malformed request message"); };
    auto empty_ok = [r, rpc](int status, const HeaderList&, std::string_view body) {
      if (status >= 300) grpc_fail(r, status, body, rpc);
      else r.ok({});
    };

    if (rpc == "SaveState") {
      std::string store, items = "[";
      bool first = true;
      while (rd.next(f, wt)) {
        if (f == 1 && wt == pb::LEN && rd.bytes(v)) store.assign(v);
        else if (f == 2 && wt == pb::LEN && rd.bytes(v)) {
          StateItemPb it;
          if (!decode_state_item(v, it)) return fail_decode();
          items += (first ? "" : ",") + state_item_json(it);
          first = false;
        } else if (!rd.skip(wt)) break;
      }
      if (!rd.ok) return fail_decode();
      grpc_http(c, "POST", "/v1.0/state/" + quote_all(store), items + "]", "application/json", {}, empty_ok);
      return;
    }
    if (rpc == "GetState") {
      std::string store, key;
      std::vector<std::pair<std::string, std::string>> meta;
      while (rd.next(f, wt)) {
        if (f == 1 && wt == pb::LEN && rd.bytes(v)) store.assign(v);
        else if (f == 2 && wt == pb::LEN && rd.bytes(v)) key.assign(v);
        else if (f == 4 && wt == pb::LEN && rd.bytes(v)) {
          std::string k, val;
          if (!pb::map_entry(v, k, val)) return fail_decode();
          meta.emplace_back(std::move(k), std::move(val));
        } else if (!rd.skip(wt)) break;
      }
      if (!rd.ok) return fail_decode();
      grpc_http(c, "GET", "/v1.0/state/" + quote_all(store) + "/" + quote_all(key) + meta_qs(meta), {}, {}, {},
                [r, rpc](int status, const HeaderList& h, std::string_view body) {
                  if (status >= 300) return grpc_fail(r, status, body, rpc);
                  pb::Writer w;  // GetStateResponse {data = 1, etag = 2}
                  if (status == 200) {
                    w.str(1, body);
                    for (auto& kv : h)
                      if (kv.first == "etag") w.str(2, kv.second);
                  }
                  r.ok(w.s);
                });
      return;
    }
    if (rpc == "DeleteState") {
      std::string store, key, etag;
      std::vector<std::pair<std::string, std::string>> meta;
      while (rd.next(f, wt)) {
        if (f == 1 && wt == pb::LEN && rd.bytes(v)) store.assign(v);
        else if (f == 2 && wt == pb::LEN && rd.bytes(v)) key.assign(v);
        else if (f == 3 && wt == pb::LEN && rd.bytes(v)) {
          pb::Reader er(v);
          uint32_t ef, ewt;
          std::string_view ev;
          while (er.next(ef, ewt))
            if (ef == 1 && ewt == pb::LEN && er.bytes(ev)) etag.assign(ev);
            else if (!er.skip(ewt)) break;
          if (!er.ok) return fail_decode();
        } else if (f == 5 && wt == pb::LEN && rd.bytes(v)) {
          std::string k, val;
          if (!pb::map_entry(v, k, val)) return fail_decode();
          meta.emplace_back(std::move(k), std::move(val));
        } else if (!rd.skip(wt)) break;
      }
      if (!rd.ok) return fail_decode();
      HeaderList extra;
      if (!etag.empty()) extra.emplace_back("if-match", etag);
      grpc_http(c, "DELETE", "/v1.0/state/" + quote_all(store) + "/" + quote_all(key) + meta_qs(meta), {}, {},
                std::move(extra), empty_ok);
      return;
    }
    if (rpc == "QueryStateAlpha1") {
      std::string store, query;
      std::vector<std::pair<std::string, std::string>> meta;
      while (rd.next(f, wt)) {
        if (f == 1 && wt == pb::LEN && rd.bytes(v)) store.assign(v);
        else if (f == 2 && wt == pb::LEN && rd.bytes(v)) query.assign(v);
        else if (f == 3 && wt == pb::LEN && rd.bytes(v)) {
          std::string k, val;
          if (!pb::map_entry(v, k, val)) return fail_decode();
          meta.emplace_back(std::move(k), std::move(val));
        } else if (!rd.skip(wt)) break;
      }
      if (!rd.ok) return fail_decode();
      grpc_http(c, "POST", "/v1.0-alpha1/state/" + quote_all(store) + "/query" + meta_qs(meta), std::move(query),
                "application/json", {}, [r, rpc](int status, const HeaderList&, std::string_view body) {
                  if (status >= 300) return grpc_fail(r, status, body, rpc);
                  std::string fast;
                  if (tt::daprpb::query_response_pb(body, fast)) return r.ok(fast);
                  pb::Writer w;  // QueryStateResponse {results = 1 {key, data, etag, error}, token = 2, metadata = 3}
                  try {
                    Value js = body.empty() ? Value() : parse(body);
                    if (const Value* res = js.get("results"); res && res->t == Value::Array)
                      for (auto& it : res->items) {
                        pb::Writer e;
                        auto sv = [&](const char* k) -> std::string {
                          const Value* x = it.get(k);
                          return x && x->t == Value::String ? x->s : std::string();
                        };
                        e.str(1, sv("key"));
                        if (const Value* d = it.get("data"); d && d->t != Value::Null) e.str(2, dump(*d));
                        e.str(3, sv("etag"));
                        e.str(4, sv("error"));
                        w.len_field(1, e.s);
                      }
                    if (const Value* t = js.get("token"); t && t->t == Value::String) w.str(2, t->s);
                    if (const Value* md = js.get("metadata"); md && md->t == Value::Object)
                      for (size_t i = 0; i < md->keys.size(); ++i)
                        w.map_entry(3, md->keys[i], md->items[i].t == Value::String ? md->items[i].s : dump(md->items[i]));
                  } catch (const std::exception& ex) {
                    return r.error(13, rpc + ": malformed query response: " + ex.what());
                  }
                  r.ok(w.s);
                });
      return;
    }
    if (rpc == "GetBulkState") {
      std::string store, body = "{\"keys\":[";
      uint64_t parallelism = 0;
      bool first = true;
      std::vector<std::pair<std::string, std::string>> meta;
      while (rd.next(f, wt)) {
        if (f == 1 && wt == pb::LEN && rd.bytes(v)) store.assign(v);
        else if (f == 2 && wt == pb::LEN && rd.bytes(v)) {
          body += first ? "" : ",";
          body += json_str(v);
          first = false;
        } else if (f == 3 && wt == pb::VARINT && rd.varint(parallelism)) {
        } else if (f == 4 && wt == pb::LEN && rd.bytes(v)) {
          std::string k, val;
          if (!pb::map_entry(v, k, val)) return fail_decode();
          meta.emplace_back(std::move(k), std::move(val));
        } else if (!rd.skip(wt)) break;
      }
      if (!rd.ok) return fail_decode();
      body += "],\"parallelism\":" + std::to_string(parallelism ? parallelism : 10) + "}";
      grpc_http(c, "POST", "/v1.0/state/" + quote_all(store) + "/bulk" + meta_qs(meta), std::move(body),
                "application/json", {}, [r, rpc](int status, const HeaderList&, std::string_view res) {
                  if (status >= 300) return grpc_fail(r, status, res, rpc);
                  // GetBulkStateResponse {items = 1: BulkStateItem {key, data, etag, error}}
                  pb::Writer w;
                  try {
                    Value js = res.empty() ? Value() : parse(res);
                    if (js.t == Value::Array)
                      for (auto& it : js.items) {
                        pb::Writer e;
                        auto sv = [&](const char* k) -> std::string {
                          const Value* x = it.get(k);
                          return x && x->t == Value::String ? x->s : std::string();
                        };
                        e.str(1, sv("key"));
                        if (const Value* d = it.get("data"); d && d->t != Value::Null) e.str(2, dump(*d));
                        e.str(3, sv("etag"));
                        e.str(4, sv("error"));
                        w.len_field(1, e.s);
                      }
                  } catch (const std::exception& ex) {
                    return r.error(13, rpc + ": malformed bulk-get response: " + ex.what());
                  }
                  r.ok(w.s);
                });
      return;
    }
    if (rpc == "PublishEvent") {
      std::string pubsub, topic, data, ctype;
      std::vector<std::pair<std::string, std::string>> meta;
      while (rd.next(f, wt)) {
        if (f == 1 && wt == pb::LEN && rd.bytes(v)) pubsub.assign(v);
        else if (f == 2 && wt == pb::LEN && rd.bytes(v)) topic.assign(v);
        else if (f == 3 && wt == pb::LEN && rd.bytes(v)) data.assign(v);
        else if (f == 4 && wt == pb::LEN && rd.bytes(v)) ctype.assign(v);
        else if (f == 5 && wt == pb::LEN && rd.bytes(v)) {
          std::string k, val;
          if (!pb::map_entry(v, k, val)) return fail_decode();
          meta.emplace_back(std::move(k), std::move(val));
        } else if (!rd.skip(wt)) break;
      }
      if (!rd.ok) return fail_decode();
      grpc_http(c, "POST", "/v1.0/publish/" + quote_all(pubsub) + "/" + quote_path(topic) + meta_qs(meta),
                std::move(data), ctype.empty() ? "application/json" : ctype, {}, empty_ok);
      return;
    }
    if (rpc == "InvokeService") {
      std::string id, method, qs, ctype, data;
      uint64_t verb = 0;
      bool has_data = false;
      while (rd.next(f, wt)) {
        if (f == 1 && wt == pb::LEN && rd.bytes(v)) id.assign(v);
        else if (f == 3 && wt == pb::LEN && rd.bytes(v)) {  // InvokeRequest
          pb::Reader ir(v);
          uint32_t g, gwt;
          std::string_view x;
          while (ir.next(g, gwt)) {
            if (g == 1 && gwt == pb::LEN && ir.bytes(x)) method.assign(x);
            else if (g == 2 && gwt == pb::LEN && ir.bytes(x)) {  // google.protobuf.Any {type_url = 1, value = 2}
              has_data = true;
              pb::Reader ar(x);
              uint32_t a, awt;
              std::string_view y;
              while (ar.next(a, awt))
                if (a == 2 && awt == pb::LEN && ar.bytes(y)) data.assign(y);
                else if (!ar.skip(awt)) break;
              if (!ar.ok) return fail_decode();
            } else if (g == 3 && gwt == pb::LEN && ir.bytes(x)) ctype.assign(x);
            else if (g == 4 && gwt == pb::LEN && ir.bytes(x)) {  // HTTPExtension {verb = 1, querystring = 2}
              pb::Reader hr(x);
              uint32_t hf, hwt;
              std::string_view y;
              uint64_t n;
              while (hr.next(hf, hwt))
                if (hf == 1 && hwt == pb::VARINT && hr.varint(n)) verb = n;
                else if (hf == 2 && hwt == pb::LEN && hr.bytes(y)) qs.assign(y);
                else if (!hr.skip(hwt)) break;
              if (!hr.ok) return fail_decode();
            } else if (!ir.skip(gwt)) break;
          }
          if (!ir.ok) return fail_decode();
        } else if (!rd.skip(wt)) break;
      }
      if (!rd.ok) return fail_decode();
      static const char* kVerbs[] = {"NONE", "GET", "HEAD", "POST", "PUT", "DELETE", "CONNECT", "OPTIONS", "TRACE", "PATCH"};
      std::string http_method = verb == 0 || verb > 9 ? "POST" : kVerbs[verb];
      size_t s = method.find_first_not_of('/');
      std::string target = "/v1.0/invoke/" + quote_all(id) + "/method/" + (s == std::string::npos ? "" : method.substr(s)) +
                           (qs.empty() ? "" : "?" + qs);
      if (ctype.empty() && has_data) ctype = "application/json";
      std::string what = "InvokeService " + id + "/" + method;
      grpc_http(c, http_method, target, std::move(data), ctype, {},
                [r, what](int status, const HeaderList& h, std::string_view body) {
                  if (status >= 300) return grpc_fail(r, status, body, what);
                  pb::Writer any, w;  // InvokeResponse {data = 1 (Any {value = 2}), content_type = 2}
                  any.str(2, body);
                  w.len_field(1, any.s);
                  for (auto& kv : h)
                    if (kv.first == "content-type") w.str(2, kv.second);
                  r.ok(w.s);
                });
      return;
    }
    // everything else: the control plane runs grpc_api.py's handler on the raw message
    grpc_http(c, "POST", "/_tt/grpc/" + quote_all(rpc), std::move(c.message), "application/grpc+proto", {},
              [r, rpc](int status, const HeaderList& h, std::string_view body) {
                const std::string* gs = nullptr;
                const std::string* gm = nullptr;
                HeaderList trailers;
                for (auto& kv : h) {
                  if (kv.first == "grpc-status") gs = &kv.second;
                  else if (kv.first == "grpc-message") gm = &kv.second;
                  else if (kv.first == "dapr-http-status") trailers.push_back(kv);
                }
                if (!gs) {  // the HTTP pipeline refused it before the handler (e.g. the API token)
                  if (status >= 300) return grpc_fail(r, status, body, rpc);
                  return r.error(13, rpc + ": control plane gave no gRPC status");
                }
                int code = std::atoi(gs->c_str());
                if (code == 0) return r.ok(body);
                r.error(code, gm ? unquote(*gm) : std::string(), trailers);
              });
  }
};

// ------------------------------------------------------------------------------ signals
class SignalIo : public ev::IoObj {
 public:
  explicit SignalIo(std::function<void()> on) : on_(std::move(on)) {
    sigset_t s;
    sigemptyset(&s);
    sigaddset(&s, SIGTERM);
    sigaddset(&s, SIGINT);
    sigprocmask(SIG_BLOCK, &s, nullptr);
    fd = signalfd(-1, &s, SFD_NONBLOCK | SFD_CLOEXEC);
  }
  void on_event(uint32_t) override {
    signalfd_siginfo si;
    while (read(fd, &si, sizeof si) == (ssize_t)sizeof si) on_();
  }

 private:
  std::function<void()> on_;
};

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s <config.json>\n", argv[0]);
    return 2;
  }
  prctl(PR_SET_PDEATHSIG, SIGTERM);  // the Python control plane owns our lifetime
  signal(SIGPIPE, SIG_IGN);
  pcsample::start();  // TT_PC_SAMPLE diagnostics
  std::ifstream in(argv[1]);
  std::stringstream ss;
  ss << in.rdbuf();
  Value cfg;
  try {
    cfg = parse(ss.str());
  } catch (const std::exception& e) {
    std::fprintf(stderr, "dataplane: bad config %s: %s\n", argv[1], e.what());
    return 2;
  }
  ev::Loop loop;
  DataPlane dp(loop, cfg);
  ev::Handler api = dp.api_handler();
  ev::Handler internal = dp.internal_handler();
  ev::Handler control = dp.control_handler();
  h2::GrpcHandler grpc = dp.grpc_handler();
  std::string ports = "{";
  try {
    int http_port = 0;
    if (auto* l = cfg.get("listen"); l && l->t == Value::Array)
      for (auto& x : l->items) {
        int p = ev::listen_on(loop, Endpoint::parse(x.s), api);
        if (p) http_port = p;
      }
    ports += "\"http\":" + std::to_string(http_port);
    std::string internal_ep;
    if (auto* l = cfg.get("internal"); l && l->t == Value::Array)
      for (auto& x : l->items) {
        Endpoint ep = Endpoint::parse(x.s);
        int p = ev::listen_on(loop, ep, internal, false, nullptr, dp.mesh_server_tls);
        if (internal_ep.empty()) {
          internal_ep = ep.unix_socket ? "unix:" + ep.path + ":" : "http://127.0.0.1:" + std::to_string(p);
          if (dp.mesh_server_tls) internal_ep = "mtls:" + dp.app_id() + "@" + internal_ep;
        }
      }
    if (auto* c = opt_str(cfg, "control")) ev::listen_on(loop, Endpoint::parse(*c), control);
    int grpc_port = 0;
    if (auto* l = cfg.get("grpcListen"); l && l->t == Value::Array)
      for (auto& x : l->items) {
        int p = h2::listen_grpc(loop, Endpoint::parse(x.s), grpc);
        if (p) grpc_port = p;
      }
    ports += ",\"grpc\":" + std::to_string(grpc_port);
    ports += ",\"internal\":" + json_str(internal_ep) + ",\"pid\":" + std::to_string(getpid()) + "}";
  } catch (const std::exception& e) {
    std::fprintf(stderr, "dataplane: %s\n", e.what());
    return 1;
  }
  bool stopping = false;
  double stop_deadline = 0;
  loop.add(std::make_shared<SignalIo>([&] {
             if (stopping) return;
             stopping = true;
             stop_deadline = ev::now_s() + 5.0;
             dp.begin_stop();
           }),
           EPOLLIN);
  if (auto* pf = opt_str(cfg, "portFile")) {
    std::string tmp = *pf + ".tmp";
    std::ofstream(tmp) << ports;
    std::rename(tmp.c_str(), pf->c_str());
  }
  double last_flush = ev::now_s();
  ev::GapTracer gaps("dataplane");
  gaps.attach(loop);
  loop.run([&](double t) {
    gaps.tick(t);
    if (t - last_flush > 1.0) {
      dp.flush();
      last_flush = t;
    }
    dp.tick(t);
    if (stopping && (dp.drained() || t > stop_deadline)) loop.stop();
  });
  dp.flush();
  pcsample::dump(("dataplane " + dp.app_id()).c_str());  // the profile names its app
  return 0;
}
