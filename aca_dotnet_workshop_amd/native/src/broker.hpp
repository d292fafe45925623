// Native message broker: the engine behind the Service Bus topic/subscription, Storage
// Queue and Redis Streams emulation.
//
// Semantics mirrored from the reference's platform dependencies (SURVEY.md §2.4 D2-D4,
// §5 "Failure detection"):
//   * topics fan out to named subscriptions (the processor's subscription is named after
//     its app-id, reference bicep/modules/service-bus.bicep:55-58); replicas of one app
//     are competing consumers on that subscription (KEDA scale-out);
//   * peek-lock receive with a lock duration; complete / abandon(+delay) / dead-letter /
//     renew; an expired lock makes the message visible again (at-least-once);
//   * delivery count per message, MaxDeliveryCount (default 10) -> dead-letter queue;
//   * per-message TTL, scheduled (delayed) enqueue, message ids;
//   * queue-length metrics (active / scheduled / locked / dead-letter) consumed by the
//     KEDA-style scaler (reference processor-backend-service.bicep:159-183);
//   * optional durability through the same append-only log as the document store.
#pragma once

#include <chrono>
#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "applog.hpp"

namespace tt {

inline int64_t mono_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
inline int64_t wall_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::system_clock::now().time_since_epoch()).count();
}

struct Message {
  uint64_t seq = 0;
  std::string id;
  std::string body;
  std::string content_type;
  std::string props;  // JSON object text (application properties)
  int64_t enqueued_wall = 0;
  int64_t visible_at = 0;  // mono ms
  int64_t expires_at = 0;  // mono ms, 0 = never
  uint32_t delivery_count = 0;
  std::string lock_token;
  int64_t locked_until = 0;
  std::string dl_reason;
};
using MsgPtr = std::shared_ptr<Message>;

struct Received {
  std::string lock_token;
  uint64_t seq;
  std::string id;
  std::string body;
  std::string content_type;
  std::string props;
  uint32_t delivery_count;
  int64_t enqueued_wall;
};

struct QueueOptions {
  int64_t lock_ms = 60000;
  uint32_t max_delivery = 10;
  int64_t default_ttl_ms = 0;
  bool dead_letter_on_expiry = false;
};

class Queue {
 public:
  std::string path;
  QueueOptions opt;
  std::map<uint64_t, MsgPtr> ready;
  std::multimap<int64_t, MsgPtr> delayed;
  std::unordered_map<std::string, MsgPtr> locked;
  std::multimap<int64_t, std::string> lock_expiry;
  std::deque<MsgPtr> dlq;
  uint64_t n_enqueued = 0, n_completed = 0, n_dead = 0, n_received = 0, n_expired = 0;

  void enqueue(MsgPtr m, int64_t now) {
    ++n_enqueued;
    if (m->visible_at > now) delayed.emplace(m->visible_at, m);
    else ready.emplace(m->seq, m);
  }

  // Move due delayed messages to ready; release expired locks.
  void tick(int64_t now) {
    while (!delayed.empty() && delayed.begin()->first <= now) {
      MsgPtr m = delayed.begin()->second;
      delayed.erase(delayed.begin());
      ready.emplace(m->seq, m);
    }
    while (!lock_expiry.empty() && lock_expiry.begin()->first <= now) {
      std::string tok = lock_expiry.begin()->second;
      lock_expiry.erase(lock_expiry.begin());
      auto it = locked.find(tok);
      if (it == locked.end() || it->second->locked_until > now) continue;  // completed or renewed
      MsgPtr m = it->second;
      locked.erase(it);
      release(m, now, "MaxDeliveryCountExceeded");
    }
  }

  void release(MsgPtr m, int64_t now, const char* reason) {
    m->lock_token.clear();
    m->locked_until = 0;
    if (opt.max_delivery && m->delivery_count >= opt.max_delivery) {
      dead_letter(m, reason);
      return;
    }
    if (m->visible_at > now) delayed.emplace(m->visible_at, m);
    else ready.emplace(m->seq, m);
  }

  void dead_letter(MsgPtr m, const std::string& reason) {
    m->dl_reason = reason;
    m->lock_token.clear();
    dlq.push_back(m);
    ++n_dead;
  }
};

class Broker {
 public:
  explicit Broker(const std::string& path = "", int fsync_mode = 0) : rng_(std::random_device{}()) {
    if (!path.empty()) {
      log_.open(path, fsync_mode);
      replaying_ = true;
      log_.replay([this](char kind, std::vector<std::string_view>& f) { apply_log(kind, f); });
      replaying_ = false;
    }
  }

  // ----------------------------------------------------------------- topology
  void create_queue(const std::string& name, const QueueOptions& o) {
    std::lock_guard<std::mutex> g(mu_);
    auto& q = queues_[name];
    q.path = name;
    q.opt = o;
  }

  void create_topic(const std::string& topic) {
    std::lock_guard<std::mutex> g(mu_);
    topics_[topic];
  }

  void create_subscription(const std::string& topic, const std::string& sub, const QueueOptions& o) {
    std::lock_guard<std::mutex> g(mu_);
    auto& t = topics_[topic];
    auto it = t.find(sub);
    if (it == t.end()) {
      std::string p = topic + "/subscriptions/" + sub;
      auto& q = t[sub];
      q.path = p;
      q.opt = o;
      if (!replaying_) log_.append('S', {topic, sub, AppLog::pod(o.lock_ms), AppLog::pod(o.max_delivery),
                                         AppLog::pod(o.default_ttl_ms)});
    } else {
      it->second.opt = o;
    }
  }

  bool delete_entity(const std::string& path) {
    std::lock_guard<std::mutex> g(mu_);
    if (queues_.erase(path)) return true;
    auto [topic, sub] = split(path);
    auto t = topics_.find(topic);
    if (t == topics_.end()) return false;
    if (sub.empty()) { topics_.erase(t); return true; }
    return t->second.erase(sub) > 0;
  }

  std::vector<std::string> subscriptions(const std::string& topic) {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<std::string> out;
    auto t = topics_.find(topic);
    if (t != topics_.end())
      for (auto& [n, _] : t->second) out.push_back(n);
    return out;
  }

  std::vector<std::string> entities() {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<std::string> out;
    for (auto& [n, _] : queues_) out.push_back(n);
    for (auto& [t, subs] : topics_) {
      out.push_back(t);
      for (auto& [s, _] : subs) out.push_back(t + "/subscriptions/" + s);
    }
    return out;
  }

  // ----------------------------------------------------------------- send
  // Publish to a topic: fan out to every subscription.  Returns sequence number
  // (0 when the topic has no subscriptions and the message is discarded).
  uint64_t publish(const std::string& topic, const std::string& body, const std::string& ctype,
                   const std::string& props, const std::string& id, int64_t ttl_ms, int64_t delay_ms) {
    std::lock_guard<std::mutex> g(mu_);
    auto& t = topics_[topic];
    uint64_t seq = ++seq_;
    int64_t now = mono_ms();
    std::string mid = id.empty() ? new_id() : id;
    for (auto& [name, q] : t) {
      auto m = make(seq, mid, body, ctype, props, ttl_ms ? ttl_ms : q.opt.default_ttl_ms, delay_ms, now);
      q.enqueue(m, now);
    }
    if (!t.empty()) log_msg('P', topic, seq, mid, body, ctype, props);
    total_published_++;
    return t.empty() ? 0 : seq;
  }

  uint64_t send(const std::string& queue, const std::string& body, const std::string& ctype,
                const std::string& props, const std::string& id, int64_t ttl_ms, int64_t delay_ms) {
    std::lock_guard<std::mutex> g(mu_);
    auto& q = queue_locked(queue);
    uint64_t seq = ++seq_;
    int64_t now = mono_ms();
    std::string mid = id.empty() ? new_id() : id;
    q.enqueue(make(seq, mid, body, ctype, props, ttl_ms ? ttl_ms : q.opt.default_ttl_ms, delay_ms, now), now);
    log_msg('Q', queue, seq, mid, body, ctype, props);
    total_published_++;
    return seq;
  }

  // ----------------------------------------------------------------- receive
  std::vector<Received> receive(const std::string& path, size_t max_messages, int64_t lock_ms) {
    std::lock_guard<std::mutex> g(mu_);
    Queue* q = find(path, true);
    std::vector<Received> out;
    if (!q) return out;
    int64_t now = mono_ms();
    q->tick(now);
    int64_t lms = lock_ms > 0 ? lock_ms : q->opt.lock_ms;
    while (out.size() < max_messages && !q->ready.empty()) {
      MsgPtr m = q->ready.begin()->second;
      q->ready.erase(q->ready.begin());
      if (m->expires_at && m->expires_at <= now) {
        ++q->n_expired;
        if (q->opt.dead_letter_on_expiry) q->dead_letter(m, "TTLExpiredException");
        continue;
      }
      m->delivery_count++;
      m->lock_token = new_token();
      m->locked_until = now + lms;
      q->locked.emplace(m->lock_token, m);
      q->lock_expiry.emplace(m->locked_until, m->lock_token);
      q->n_received++;
      out.push_back({m->lock_token, m->seq, m->id, m->body, m->content_type, m->props, m->delivery_count,
                     m->enqueued_wall});
    }
    return out;
  }

  bool complete(const std::string& path, const std::string& token) {
    std::lock_guard<std::mutex> g(mu_);
    Queue* q = find(path, false);
    if (!q) return false;
    auto it = q->locked.find(token);
    if (it == q->locked.end()) return false;
    uint64_t seq = it->second->seq;
    q->locked.erase(it);
    q->n_completed++;
    if (log_.is_open()) log_.append('C', {path, AppLog::pod(seq)});
    return true;
  }

  bool abandon(const std::string& path, const std::string& token, int64_t delay_ms) {
    std::lock_guard<std::mutex> g(mu_);
    Queue* q = find(path, false);
    if (!q) return false;
    auto it = q->locked.find(token);
    if (it == q->locked.end()) return false;
    MsgPtr m = it->second;
    q->locked.erase(it);
    int64_t now = mono_ms();
    m->visible_at = now + std::max<int64_t>(0, delay_ms);
    q->release(m, now, "MaxDeliveryCountExceeded");
    if (!m->dl_reason.empty() && log_.is_open()) log_.append('C', {path, AppLog::pod(m->seq)});
    return true;
  }

  bool dead_letter(const std::string& path, const std::string& token, const std::string& reason) {
    std::lock_guard<std::mutex> g(mu_);
    Queue* q = find(path, false);
    if (!q) return false;
    auto it = q->locked.find(token);
    if (it == q->locked.end()) return false;
    MsgPtr m = it->second;
    q->locked.erase(it);
    q->dead_letter(m, reason);
    if (log_.is_open()) log_.append('C', {path, AppLog::pod(m->seq)});
    return true;
  }

  bool renew(const std::string& path, const std::string& token, int64_t lock_ms) {
    std::lock_guard<std::mutex> g(mu_);
    Queue* q = find(path, false);
    if (!q) return false;
    auto it = q->locked.find(token);
    if (it == q->locked.end()) return false;
    int64_t now = mono_ms();
    it->second->locked_until = now + (lock_ms > 0 ? lock_ms : q->opt.lock_ms);
    q->lock_expiry.emplace(it->second->locked_until, token);
    return true;
  }

  // Drain up to `max` dead-lettered messages (receive from `<path>/$deadletterqueue`).
  std::vector<std::tuple<uint64_t, std::string, std::string, std::string, uint32_t>> drain_dead_letters(
      const std::string& path, size_t max) {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<std::tuple<uint64_t, std::string, std::string, std::string, uint32_t>> out;
    Queue* q = find(path, false);
    if (!q) return out;
    while (out.size() < max && !q->dlq.empty()) {
      MsgPtr m = q->dlq.front();
      q->dlq.pop_front();
      out.emplace_back(m->seq, m->id, m->body, m->dl_reason, m->delivery_count);
    }
    return out;
  }

  // active, scheduled, locked, dead-letter, enqueued, completed, received
  std::tuple<size_t, size_t, size_t, size_t, uint64_t, uint64_t, uint64_t> counts(const std::string& path) {
    std::lock_guard<std::mutex> g(mu_);
    Queue* q = find(path, false);
    if (!q) return {0, 0, 0, 0, 0, 0, 0};
    q->tick(mono_ms());
    return {q->ready.size(), q->delayed.size(), q->locked.size(), q->dlq.size(), q->n_enqueued, q->n_completed,
            q->n_received};
  }

  // Topic-level active count: sum over subscriptions (what the KEDA scaler reads when
  // pointed at a topic + subscription it reads that subscription only).
  size_t purge(const std::string& path) {
    std::lock_guard<std::mutex> g(mu_);
    Queue* q = find(path, false);
    if (!q) return 0;
    size_t n = q->ready.size() + q->delayed.size();
    q->ready.clear();
    q->delayed.clear();
    return n;
  }

  uint64_t total_published() {
    std::lock_guard<std::mutex> g(mu_);
    return total_published_;
  }

  // group commit (AppLog fsync_mode 2): a writer's mark after its write, and the wait for the
  // sync that covers it (the backing front answers from the callback; Python callers block)
  bool group_commit() const { return log_.group(); }
  uint64_t log_mark() const { return log_.mark(); }
  void after_durable(uint64_t mark, std::function<void()> cb) { log_.after_durable(mark, std::move(cb)); }
  void wait_durable() { log_.wait_durable(); }
  AppLog::CommitStats commit_stats() { return log_.commit_stats(); }

 private:
  static std::pair<std::string, std::string> split(const std::string& path) {
    auto pos = path.find("/subscriptions/");
    if (pos == std::string::npos) return {path, ""};
    return {path.substr(0, pos), path.substr(pos + 15)};
  }

  Queue& queue_locked(const std::string& name) {
    auto it = queues_.find(name);
    if (it != queues_.end()) return it->second;
    auto& q = queues_[name];
    q.path = name;
    return q;
  }

  Queue* find(const std::string& path, bool create) {
    auto [topic, sub] = split(path);
    if (sub.empty()) {
      auto it = queues_.find(path);
      if (it != queues_.end()) return &it->second;
      if (!create) return nullptr;
      return &queue_locked(path);
    }
    auto& t = topics_[topic];
    auto it = t.find(sub);
    if (it != t.end()) return &it->second;
    if (!create) return nullptr;
    auto& q = t[sub];
    q.path = path;
    if (!replaying_ && log_.is_open()) log_.append('S', {topic, sub, AppLog::pod(q.opt.lock_ms),
                                                        AppLog::pod(q.opt.max_delivery), AppLog::pod(q.opt.default_ttl_ms)});
    return &q;
  }

  MsgPtr make(uint64_t seq, const std::string& id, const std::string& body, const std::string& ctype,
              const std::string& props, int64_t ttl_ms, int64_t delay_ms, int64_t now) {
    auto m = std::make_shared<Message>();
    m->seq = seq;
    m->id = id;
    m->body = body;
    m->content_type = ctype;
    m->props = props;
    m->enqueued_wall = wall_ms();
    m->visible_at = now + std::max<int64_t>(0, delay_ms);
    m->expires_at = ttl_ms > 0 ? now + ttl_ms : 0;
    return m;
  }

  std::string new_token() {
    uint64_t a = rng_(), b = rng_();
    char buf[40];
    std::snprintf(buf, sizeof buf, "%016llx%016llx", (unsigned long long)a, (unsigned long long)b);
    return buf;
  }
  std::string new_id() {
    uint64_t a = rng_(), b = rng_();
    char buf[40];
    std::snprintf(buf, sizeof buf, "%08llx-%04llx-4%03llx-%04llx-%012llx", (unsigned long long)(a >> 32),
                  (unsigned long long)((a >> 16) & 0xffff), (unsigned long long)(a & 0xfff),
                  (unsigned long long)(0x8000 | ((b >> 48) & 0x3fff)), (unsigned long long)(b & 0xffffffffffffULL));
    return buf;
  }

  void log_msg(char kind, const std::string& entity, uint64_t seq, const std::string& id, const std::string& body,
               const std::string& ctype, const std::string& props) {
    if (!log_.is_open() || replaying_) return;
    log_.append(kind, {entity, AppLog::pod(seq), id, body, ctype, props});
  }

  void apply_log(char kind, std::vector<std::string_view>& f) {
    int64_t now = mono_ms();
    if (kind == 'S' && f.size() == 5) {
      QueueOptions o;
      std::memcpy(&o.lock_ms, f[2].data(), 8);
      std::memcpy(&o.max_delivery, f[3].data(), 4);
      std::memcpy(&o.default_ttl_ms, f[4].data(), 8);
      auto& q = topics_[std::string(f[0])][std::string(f[1])];
      q.path = std::string(f[0]) + "/subscriptions/" + std::string(f[1]);
      q.opt = o;
    } else if ((kind == 'P' || kind == 'Q') && f.size() == 6) {
      uint64_t seq;
      std::memcpy(&seq, f[1].data(), 8);
      seq_ = std::max(seq_, seq);
      std::string entity(f[0]);
      if (kind == 'P') {
        for (auto& [name, q] : topics_[entity]) {
          q.enqueue(make(seq, std::string(f[2]), std::string(f[3]), std::string(f[4]), std::string(f[5]), 0, 0, now), now);
          pending_[q.path][seq] = true;
        }
      } else {
        auto& q = queue_locked(entity);
        q.enqueue(make(seq, std::string(f[2]), std::string(f[3]), std::string(f[4]), std::string(f[5]), 0, 0, now), now);
      }
    } else if (kind == 'C' && f.size() == 2) {
      uint64_t seq;
      std::memcpy(&seq, f[1].data(), 8);
      Queue* q = find(std::string(f[0]), false);
      if (q) q->ready.erase(seq);
    }
  }

  std::mutex mu_;
  std::map<std::string, Queue> queues_;
  std::map<std::string, std::map<std::string, Queue>> topics_;
  std::unordered_map<std::string, std::map<uint64_t, bool>> pending_;
  AppLog log_;
  bool replaying_ = false;
  uint64_t seq_ = 0;
  uint64_t total_published_ = 0;
  std::mt19937_64 rng_;
};

}  // namespace tt
