// Append-only record log shared by the document store and the broker.
//
// Record: [u32 total_len][u8 kind][fields...] where every field is [u32 len][bytes].
// Writes go straight to the fd (one write(2) per record) so a process crash never loses
// an acknowledged mutation; fsync_mode=1 additionally fdatasync()s each record.  A batch
// (BatchScope: a bulk write acknowledged as a whole) collects its records and writes them with
// one write(2) when the scope ends, before the caller acknowledges.
#pragma once

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <functional>
#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

namespace tt {

class AppLog {
 public:
  AppLog() = default;
  AppLog(const AppLog&) = delete;
  AppLog& operator=(const AppLog&) = delete;
  ~AppLog() { close(); }

  bool open(const std::string& path, int fsync_mode) {
    path_ = path;
    fsync_ = fsync_mode;
    fd_ = ::open(path.c_str(), O_RDWR | O_CREAT | O_APPEND | O_CLOEXEC, 0644);
    if (fd_ < 0) throw std::runtime_error("cannot open log " + path + ": " + std::strerror(errno));
    struct stat st;
    if (::fstat(fd_, &st) == 0) bytes_ = (uint64_t)st.st_size;
    return true;
  }
  bool is_open() const { return fd_ >= 0; }
  uint64_t bytes() const { return bytes_; }
  const std::string& path() const { return path_; }

  void close() {
    if (fd_ >= 0) { ::close(fd_); fd_ = -1; }
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
    if (::rename(tmp.c_str(), path_.c_str()) != 0) throw std::runtime_error("log compaction rename failed");
    close();
    open(path_, fsync_);
  }

  void sync() { if (fd_ >= 0) ::fdatasync(fd_); }

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

  int fd_ = -1;
  int fsync_ = 0;
  uint64_t bytes_ = 0;
  std::string path_;
  bool batching_ = false;
  std::string batch_;
};

}  // namespace tt
