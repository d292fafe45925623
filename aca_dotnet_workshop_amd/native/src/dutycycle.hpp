// CPU duty cycle for replicas without a writable cgroup (platform/limits.py, mode `watchdog`):
// the native counterpart of the controller's Python tick, on its own thread.
//
// A replica is a process group (sidecar + native data plane + app).  Every `period / 8` the
// thread sums the CPU time of every thread of the replica's processes from
// /proc/<pid>/task/<tid>/schedstat (nanoseconds; descriptors kept open, one pread each), and:
//   * once the replica has used `cpu x period` in the current period -> SIGSTOP the group;
//   * at the next period boundary -> SIGCONT, with any overrun carried as debt (quota unused in
//     one period does not carry over; an overrun is paid off in the next).
// Period boundaries are kept on an absolute CLOCK_MONOTONIC schedule (clock_nanosleep with
// TIMER_ABSTIME), independent of how busy the controller's Python threads are -- a stopped
// replica resumes on time -- and the process / thread lists are re-read every 500 ms
// (children via /proc/<pid>/task/<tid>/children, so the app and the data plane a sidecar
// started are counted).  The same semantics as Linux CFS bandwidth control (`cpu.max`) at a
// finer period; CFS itself is used whenever a cgroup can be written.
#pragma once

#include <dirent.h>
#include <fcntl.h>
#include <signal.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace tt {

class DutyCycle {
 public:
  struct Stats {
    uint64_t throttled_periods = 0;
    double cpu_seconds = 0;
    double stopped_seconds = 0;
    bool stopped = false;
  };

  explicit DutyCycle(double period_s) : period_ns_((int64_t)(period_s * 1e9)) {
    if (period_ns_ < 1000000) period_ns_ = 1000000;
  }
  ~DutyCycle() { stop(); }

  void add(const std::string& name, int pid, double cpu) {
    std::lock_guard<std::mutex> g(mu_);
    auto& r = reps_[name];
    r.pid = pid;
    r.cpu = cpu;
    refresh(r);
    r.period_start = now_ns();
    r.period_used = read_used(r);
  }

  void remove(const std::string& name) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = reps_.find(name);
    if (it == reps_.end()) return;
    if (it->second.stopped) ::killpg(it->second.pid, SIGCONT);
    close_all(it->second);
    reps_.erase(it);
  }

  void start() {
    if (running_.exchange(true)) return;
    th_ = std::thread([this] {
      pthread_setname_np(pthread_self(), "tt-dutycycle");
      run();
    });
  }

  void stop() {
    if (!running_.exchange(false)) return;
    if (th_.joinable()) th_.join();
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : reps_)
      if (kv.second.stopped) ::killpg(kv.second.pid, SIGCONT), kv.second.stopped = false;
  }

  std::map<std::string, Stats> stats() {
    std::lock_guard<std::mutex> g(mu_);
    std::map<std::string, Stats> out;
    for (auto& kv : reps_) {
      Stats s;
      s.throttled_periods = kv.second.throttled;
      s.cpu_seconds = kv.second.total_ns / 1e9;
      s.stopped_seconds = kv.second.stopped_ns / 1e9;
      s.stopped = kv.second.stopped;
      out[kv.first] = s;
    }
    return out;
  }

  double period_s() const { return period_ns_ / 1e9; }

 private:
  struct Thread {
    int fd = -1;
    int64_t last = -1;
  };
  struct Rep {
    int pid = 0;
    double cpu = 0;
    std::map<std::pair<int, int>, Thread> threads;  // (pid, tid)
    int64_t total_ns = 0;     // CPU used since added (deltas: an exited thread keeps its share)
    int64_t period_start = 0, period_used = 0;
    int64_t refreshed = 0;
    bool stopped = false;
    int64_t stopped_at = 0, stopped_ns = 0;
    uint64_t throttled = 0;
  };

  int64_t period_ns_;
  std::mutex mu_;
  std::map<std::string, Rep> reps_;
  std::atomic<bool> running_{false};
  std::thread th_;

  static int64_t now_ns() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (int64_t)ts.tv_sec * 1000000000LL + ts.tv_nsec;
  }

  static void list_tree(int pid, std::vector<int>& out, int depth = 0) {
    if (depth > 16) return;
    out.push_back(pid);
    std::string dir = "/proc/" + std::to_string(pid) + "/task";
    DIR* d = ::opendir(dir.c_str());
    if (!d) return;
    std::vector<int> kids;
    while (dirent* e = ::readdir(d)) {
      if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
      std::string f = dir + "/" + e->d_name + "/children";
      FILE* fp = std::fopen(f.c_str(), "r");
      if (!fp) continue;
      int c;
      while (std::fscanf(fp, "%d", &c) == 1) kids.push_back(c);
      std::fclose(fp);
    }
    ::closedir(d);
    for (int k : kids) list_tree(k, out, depth + 1);
  }

  void refresh(Rep& r) {
    std::vector<int> pids;
    list_tree(r.pid, pids);
    std::map<std::pair<int, int>, bool> seen;
    bool first = r.threads.empty();
    for (int p : pids) {
      std::string dir = "/proc/" + std::to_string(p) + "/task";
      DIR* d = ::opendir(dir.c_str());
      if (!d) continue;
      while (dirent* e = ::readdir(d)) {
        if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
        int tid = std::atoi(e->d_name);
        auto key = std::make_pair(p, tid);
        seen[key] = true;
        if (r.threads.count(key)) continue;
        std::string f = dir + "/" + e->d_name + "/schedstat";
        int fd = ::open(f.c_str(), O_RDONLY | O_CLOEXEC);
        if (fd < 0) continue;
        Thread t;
        t.fd = fd;
        // a thread found after the first read started inside the window: it counts from zero
        t.last = first ? -1 : 0;
        r.threads[key] = t;
      }
      ::closedir(d);
    }
    for (auto it = r.threads.begin(); it != r.threads.end();) {
      if (!seen.count(it->first)) {
        ::close(it->second.fd);
        it = r.threads.erase(it);
      } else {
        ++it;
      }
    }
    r.refreshed = now_ns();
  }

  static void close_all(Rep& r) {
    for (auto& kv : r.threads) ::close(kv.second.fd);
    r.threads.clear();
  }

  int64_t read_used(Rep& r) {
    char buf[128];
    for (auto it = r.threads.begin(); it != r.threads.end();) {
      ssize_t n = ::pread(it->second.fd, buf, sizeof buf - 1, 0);
      if (n <= 0) {
        ::close(it->second.fd);
        it = r.threads.erase(it);
        continue;
      }
      buf[n] = 0;
      int64_t v = std::strtoll(buf, nullptr, 10);
      if (it->second.last >= 0 && v > it->second.last) r.total_ns += v - it->second.last;
      it->second.last = v;
      ++it;
    }
    return r.total_ns;
  }

  void tick(int64_t now) {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : reps_) {
      Rep& r = kv.second;
      if (now - r.refreshed >= 500000000LL) refresh(r);
      int64_t used = read_used(r);
      if (now - r.period_start >= period_ns_) {
        int64_t quota = (int64_t)(r.cpu * (double)(now - r.period_start));
        int64_t overrun = std::max<int64_t>(0, (used - r.period_used) - quota);
        r.period_used = used - overrun;
        r.period_start = now;
        if (r.stopped) {
          ::killpg(r.pid, SIGCONT);
          r.stopped = false;
          r.stopped_ns += now - r.stopped_at;
        }
        continue;
      }
      if (!r.stopped && used - r.period_used >= (int64_t)(r.cpu * (double)period_ns_)) {
        ::killpg(r.pid, SIGSTOP);
        r.stopped = true;
        r.stopped_at = now;
        r.throttled++;
      }
    }
  }

  void run() {
    const int64_t step = std::max<int64_t>(period_ns_ / 8, 250000);
    int64_t next = now_ns();
    while (running_.load()) {
      next += step;
      timespec ts{(time_t)(next / 1000000000LL), (long)(next % 1000000000LL)};
      while (clock_nanosleep(CLOCK_MONOTONIC, TIMER_ABSTIME, &ts, nullptr) == EINTR) {
      }
      int64_t now = now_ns();
      if (now - next > 4 * step) next = now;  // fell behind (suspended): do not burst
      tick(now);
    }
  }
};

}  // namespace tt
