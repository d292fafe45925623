// Append-only record log shared by the document store and the broker.
//
// Record: [u32 total_len][u8 kind][fields...] where every field is [u32 len][bytes].
// Writes go straight to the fd (one write(2) per record) so a process crash never loses
// an acknowledged mutation; fsync_mode=1 additionally fdatasync()s each record.  A batch
// (BatchScope: a bulk write acknowledged as a whole) collects its records and writes them with
// one write(2) when the scope ends, before the caller acknowledges.
//
// fsync_mode=2 is group commit: a host crash never loses an acknowledged mutation either, but
// the records are not synced one by one under the engine's lock.  A committer thread
// fdatasync()s everything written so far, and a writer that must acknowledge durably waits for
// the sync that covers its record: `mark()` after the write, then `after_durable(mark, cb)`
// (the backing front answers from `cb`) or `wait_durable(mark)` (blocking callers).  Writes that
// arrive while a sync is in flight share the next one, so the syncs per second stay bounded by
// the device's sync latency, not by the write rate (Cosmos and Service Bus acknowledge a write
// once it is durable; this is how a log-structured store gets that at 100k writes/s).
#pragma once

#include <fcntl.h>
#include <pthread.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <functional>
#include <future>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <string_view>
#include <thread>
#include <vector>

namespace tt {

class AppLog {
 public:
  AppLog() = default;
  AppLog(const AppLog&) = delete;
  AppLog& operator=(const AppLog&) = delete;
  ~AppLog() {
    stop_committer();
    close();
  }

  bool open(const std::string& path, int fsync_mode) {
    path_ = path;
    fsync_ = fsync_mode;
    open_fd();
    if (fsync_ == 2 && !gc_thread_.joinable()) gc_thread_ = std::thread([this] { commit_loop(); });
    return true;
  }
  bool is_open() const { return fd_ >= 0; }
  uint64_t bytes() const { return bytes_; }
  const std::string& path() const { return path_; }

  void close() {
    std::lock_guard<std::mutex> f(fd_mu_);
    if (fd_ >= 0) { ::close(fd_); fd_ = -1; }
  }

  // -- group commit (fsync_mode 2) -----------------------------------------------------------
  bool group() const { return fsync_ == 2 && fd_ >= 0; }
  // Bytes written through this log so far (every record, compaction aside): a writer's mark.
  uint64_t mark() const { return written_.load(std::memory_order_acquire); }
  // `cb` runs (on the committer thread, or here when already durable) once everything up to
  // `mark` is on the device.
  void after_durable(uint64_t mark, std::function<void()> cb) {
    if (!group() || synced_.load(std::memory_order_acquire) >= mark) {
      cb();
      return;
    }
    {
      std::lock_guard<std::mutex> l(gc_mu_);
      waiters_.emplace(mark, std::move(cb));
      gc_want_ = true;
    }
    gc_cv_.notify_one();
  }
  void wait_durable(uint64_t mark) {
    if (!group() || synced_.load(std::memory_order_acquire) >= mark) return;
    std::promise<void> done;
    auto f = done.get_future();
    after_durable(mark, [&done] { done.set_value(); });
    f.wait();
  }
  void wait_durable() { wait_durable(mark()); }
  struct CommitStats {
    uint64_t syncs, acks, written, synced;
    double sync_ms_total, sync_ms_max;
  };
  CommitStats commit_stats() {
    std::lock_guard<std::mutex> l(gc_mu_);
    return {gc_syncs_, gc_acks_, mark(), synced_.load(), gc_sync_s_ * 1e3, gc_sync_max_s_ * 1e3};
  }

  static void put_field(std::string& rec, std::string_view f) {
    uint32_t n = (uint32_t)f.size();
    rec.append(reinterpret_cast<const char*>(&n), 4);
    rec.append(f.data(), f.size());
  }
  template <class T>
  static std::string_view pod(const T& v) { return std::string_view(reinterpret_cast<const char*>(&v), sizeof(T)); }

  void append(char kind, const std::vector<std::string_view>& fields) {
    if (fd_ < 0) return;
    std::string rec;
    rec.resize(5);
    rec[4] = kind;
    for (auto f : fields) put_field(rec, f);
    uint32_t total = (uint32_t)rec.size();
    std::memcpy(&rec[0], &total, 4);
    if (batching_) {
      batch_ += rec;
      return;
    }
    write_all(rec);
  }

  // Records appended while a BatchScope is alive go out in one write(2) when it ends.
  class BatchScope {
   public:
    explicit BatchScope(AppLog& log) : log_(log) { log_.batching_ = true; }
    ~BatchScope() noexcept(false) {
      log_.batching_ = false;
      if (log_.batch_.empty()) return;
      std::string b;
      b.swap(log_.batch_);
      if (std::uncaught_exceptions() == 0) {
        log_.write_all(b);
        return;
      }
      try {  // unwinding already: keep what was applied, do not throw a second time
        log_.write_all(b);
      } catch (...) {
      }
    }
    BatchScope(const BatchScope&) = delete;
    BatchScope& operator=(const BatchScope&) = delete;

   private:
    AppLog& log_;
  };

  // Replays every complete record; a torn tail (crash mid-write) is truncated.
  void replay(const std::function<void(char, std::vector<std::string_view>&)>& fn) {
    if (fd_ < 0) return;
    std::string data;
    data.resize(bytes_);
    size_t off = 0;
    while (off < data.size()) {
      ssize_t r = ::pread(fd_, &data[off], data.size() - off, (off_t)off);
      if (r <= 0) break;
      off += (size_t)r;
    }
    size_t pos = 0;
    std::vector<std::string_view> fields;
    while (pos + 5 <= off) {
      uint32_t total;
      std::memcpy(&total, &data[pos], 4);
      if (total < 5 || pos + total > off) break;
      char kind = data[pos + 4];
      fields.clear();
      size_t p = pos + 5, end = pos + total;
      bool ok = true;
      while (p < end) {
        if (p + 4 > end) { ok = false; break; }
        uint32_t n;
        std::memcpy(&n, &data[p], 4);
        p += 4;
        if (p + n > end) { ok = false; break; }
        fields.emplace_back(&data[p], n);
        p += n;
      }
      if (!ok) break;
      fn(kind, fields);
      pos = end;
    }
    if (pos < bytes_) {
      if (::ftruncate(fd_, (off_t)pos) == 0) bytes_ = pos;
    }
  }

  // Atomically replace the log with the records produced by `writer`.
  void rewrite(const std::function<void(AppLog&)>& writer) {
    if (fd_ < 0) return;
    std::string tmp = path_ + ".compact";
    AppLog out;
    ::unlink(tmp.c_str());
    out.open(tmp, 0);
    writer(out);
    ::fdatasync(out.fd_);
    out.close();
    {
      std::lock_guard<std::mutex> f(fd_mu_);  // the committer never syncs a closed descriptor
      if (::rename(tmp.c_str(), path_.c_str()) != 0) throw std::runtime_error("log compaction rename failed");
      if (fd_ >= 0) ::close(fd_);
      fd_ = -1;
      open_fd_locked();
    }
    if (fsync_ == 2) {  // the compacted file was synced whole: every record so far is durable
      {
        std::lock_guard<std::mutex> l(gc_mu_);
        gc_want_ = true;
      }
      gc_cv_.notify_one();
    }
  }

  void sync() {
    std::lock_guard<std::mutex> f(fd_mu_);
    if (fd_ >= 0) ::fdatasync(fd_);
  }

 private:
  // TT_STALL_LOG=<file> (diagnostics): a write(2) slower than TT_STALL_MS (default 100) ms is
  // reported as a JSON line -- the caller holds its engine's mutex meanwhile.
  static FILE* stall_file(double& min_s) {
    static double th = [] {
      const char* p = std::getenv("TT_STALL_MS");
      double ms = p && *p ? std::atof(p) : 100.0;
      return (ms > 0 ? ms : 100.0) / 1e3;
    }();
    static FILE* f = [] {
      const char* p = std::getenv("TT_STALL_LOG");
      return p && *p ? std::fopen(p, "a") : nullptr;
    }();
    min_s = th;
    return f;
  }

  void write_all(const std::string& rec) {
    double min_s;
    FILE* stall = stall_file(min_s);
    auto t0 = stall ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point{};
    size_t off = 0;
    while (off < rec.size()) {
      ssize_t w = ::write(fd_, rec.data() + off, rec.size() - off);
      if (w < 0) {
        if (errno == EINTR) continue;
        throw std::runtime_error(std::string("log write failed: ") + std::strerror(errno));
      }
      off += (size_t)w;
    }
    bytes_ += rec.size();
    written_.fetch_add(rec.size(), std::memory_order_release);
    if (fsync_ == 1) ::fdatasync(fd_);
    if (stall) {
      double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (s > min_s) {
        double wall = std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
        std::fprintf(stall, "{\"what\": \"log-write\", \"ms\": %.2f, \"bytes\": %zu, \"log\": \"%s\", \"pid\": %d, \"wall\": %.4f}\n",
                     s * 1e3, rec.size(), path_.c_str(), (int)::getpid(), wall);
        std::fflush(stall);
      }
    }
  }

  void open_fd() {
    std::lock_guard<std::mutex> f(fd_mu_);
    open_fd_locked();
  }
  void open_fd_locked() {
    fd_ = ::open(path_.c_str(), O_RDWR | O_CREAT | O_APPEND | O_CLOEXEC, 0644);
    if (fd_ < 0) throw std::runtime_error("cannot open log " + path_ + ": " + std::strerror(errno));
    struct stat st;
    if (::fstat(fd_, &st) == 0) bytes_ = (uint64_t)st.st_size;
  }

  // The committer: sync what has been written, release the writers it covers; writes that land
  // during a sync wait for the next one (one fdatasync per batch, not per record).
  void commit_loop() {
    pthread_setname_np(pthread_self(), "tt-log-commit");
    std::unique_lock<std::mutex> l(gc_mu_);
    // TT_LOG_COMMIT_DELAY_US (default 100): once a writer waits, more writers may join the same
    // sync for this long (PostgreSQL's commit_delay) -- one fdatasync per ~delay x write rate
    // records instead of one per handful, at the cost of this much latency per acknowledgement
    static const auto delay = [] {
      const char* v = std::getenv("TT_LOG_COMMIT_DELAY_US");
      return std::chrono::microseconds(v && *v ? std::max(0L, std::atol(v)) : 100L);
    }();
    while (true) {
      gc_cv_.wait(l, [this] { return gc_stop_ || gc_want_; });
      if (gc_stop_ && waiters_.empty()) return;
      if (delay.count() > 0 && !gc_stop_) gc_cv_.wait_for(l, delay, [this] { return gc_stop_; });
      gc_want_ = false;
      l.unlock();
      const uint64_t target = written_.load(std::memory_order_acquire);
      const auto t0 = std::chrono::steady_clock::now();
      {
        std::lock_guard<std::mutex> f(fd_mu_);
        if (fd_ >= 0) ::fdatasync(fd_);
      }
      const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      uint64_t prev = synced_.load();
      while (prev < target && !synced_.compare_exchange_weak(prev, target)) {
      }
      std::vector<std::function<void()>> ready;
      l.lock();
      ++gc_syncs_;
      gc_sync_s_ += s;
      gc_sync_max_s_ = std::max(gc_sync_max_s_, s);
      auto end = waiters_.upper_bound(target);
      for (auto it = waiters_.begin(); it != end; ++it) ready.push_back(std::move(it->second));
      waiters_.erase(waiters_.begin(), end);
      gc_acks_ += ready.size();
      if (!waiters_.empty()) gc_want_ = true;  // written after this sync's snapshot
      l.unlock();
      for (auto& f : ready) f();
      l.lock();
    }
  }
  void stop_committer() {
    if (!gc_thread_.joinable()) return;
    {
      std::lock_guard<std::mutex> l(gc_mu_);
      gc_stop_ = true;
      gc_want_ = true;
    }
    gc_cv_.notify_one();
    gc_thread_.join();
  }

  int fd_ = -1;
  int fsync_ = 0;
  uint64_t bytes_ = 0;
  std::string path_;
  bool batching_ = false;
  std::string batch_;
  std::mutex fd_mu_;  // fd_ between the writers' compaction and the committer's fdatasync
  std::atomic<uint64_t> written_{0}, synced_{0};
  std::mutex gc_mu_;
  std::condition_variable gc_cv_;
  std::multimap<uint64_t, std::function<void()>> waiters_;
  std::thread gc_thread_;
  bool gc_stop_ = false, gc_want_ = false;
  uint64_t gc_syncs_ = 0, gc_acks_ = 0;
  double gc_sync_s_ = 0, gc_sync_max_s_ = 0;
};

}  // namespace tt
