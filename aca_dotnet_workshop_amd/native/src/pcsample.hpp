// Self-profiling by PC sampling, for the standalone native executables (data plane, ingress).
//
// TT_PC_SAMPLE=<file>: a SIGPROF per millisecond of the process's CPU time (coarsened to the
// kernel's tick: CPU-time timers are checked there) records the
// interrupted program counter in a preallocated buffer (the handler only stores a word); at
// exit the PCs are resolved with dladdr into "samples share module symbol" lines, busiest
// first, written to <file>.<pid>.  perf is not in the image, and gprof sees neither the shared libraries (libssl, libc)
// nor the kernel: here a sample taken in a system call lands on the libc wrapper that made it,
// so the profile splits the process's time into its own code, each library, and each syscall.
// Executables are linked with -rdynamic so their own functions resolve too.
#pragma once

#include <cxxabi.h>
#include <dlfcn.h>
#include <signal.h>
#include <sys/time.h>
#include <ucontext.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

namespace tt::pcsample {

constexpr size_t kCap = 1 << 22;  // 4 M samples: ~70 CPU-minutes at 1 kHz
inline uintptr_t* g_pcs = nullptr;
inline std::atomic<size_t> g_n{0};
inline std::string* g_path = nullptr;

inline void on_prof(int, siginfo_t*, void* ctx) {
  auto* uc = static_cast<ucontext_t*>(ctx);
  size_t i = g_n.fetch_add(1, std::memory_order_relaxed);
  if (i < kCap) g_pcs[i] = (uintptr_t)uc->uc_mcontext.gregs[REG_RIP];
}

// Starts sampling when TT_PC_SAMPLE is set; call once from main before any thread starts.
inline void start() {
  const char* p = std::getenv("TT_PC_SAMPLE");
  if (!p || !*p) return;
  g_path = new std::string(p);
  g_pcs = static_cast<uintptr_t*>(std::calloc(kCap, sizeof(uintptr_t)));
  if (!g_pcs) return;
  struct sigaction sa {};
  sa.sa_sigaction = on_prof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGPROF, &sa, nullptr);
  itimerval t{};
  t.it_interval.tv_usec = 1000;
  t.it_value.tv_usec = 1000;
  setitimer(ITIMER_PROF, &t, nullptr);
}

// Stops sampling and writes the flat profile to <TT_PC_SAMPLE>.<pid>.
inline void dump(const char* who) {
  if (!g_pcs || !g_path) return;
  itimerval off{};
  setitimer(ITIMER_PROF, &off, nullptr);
  signal(SIGPROF, SIG_IGN);
  size_t n = std::min(g_n.load(), kCap);
  std::map<std::pair<std::string, std::string>, size_t> by_sym;
  std::map<uintptr_t, std::pair<std::string, std::string>> cache;
  for (size_t i = 0; i < n; ++i) {
    uintptr_t pc = g_pcs[i];
    auto it = cache.find(pc);
    if (it == cache.end()) {
      Dl_info di{};
      std::string mod = "?", sym = "?";
      if (dladdr(reinterpret_cast<void*>(pc), &di)) {
        if (di.dli_fname) {
          mod = di.dli_fname;
          size_t slash = mod.rfind('/');
          if (slash != std::string::npos) mod = mod.substr(slash + 1);
        }
        if (di.dli_sname) {
          int st = 0;
          char* dm = abi::__cxa_demangle(di.dli_sname, nullptr, nullptr, &st);
          sym = st == 0 && dm ? dm : di.dli_sname;
          std::free(dm);
          if (sym.size() > 160) sym = sym.substr(0, 160);
        }
      }
      it = cache.emplace(pc, std::make_pair(mod, sym)).first;
    }
    ++by_sym[it->second];
  }
  std::vector<std::pair<size_t, std::pair<std::string, std::string>>> rows;
  std::map<std::string, size_t> by_mod;
  for (auto& [k, c] : by_sym) {
    rows.emplace_back(c, k);
    by_mod[k.first] += c;
  }
  std::sort(rows.begin(), rows.end(), [](auto& a, auto& b) { return a.first > b.first; });
  FILE* f = std::fopen((*g_path + "." + std::to_string(getpid())).c_str(), "w");
  if (!f) return;
  // one sample per timer expiry: 1 ms of CPU is asked for, but the kernel checks CPU-time timers
  // on its tick, so at HZ=100 a sample stands for ~10 ms -- shares are what to read
  std::fprintf(f, "== %s pid %d: %zu samples\n-- by module\n", who, (int)getpid(), n);
  for (auto& [m, c] : by_mod) std::fprintf(f, "%8zu %5.1f%%  %s\n", c, n ? 100.0 * c / n : 0.0, m.c_str());
  std::fprintf(f, "-- by symbol (top 60)\n");
  for (size_t i = 0; i < rows.size() && i < 60; ++i)
    std::fprintf(f, "%8zu %5.1f%%  %-24s %s\n", rows[i].first, n ? 100.0 * rows[i].first / n : 0.0,
                 rows[i].second.first.c_str(), rows[i].second.second.c_str());
  std::fclose(f);
}

}  // namespace tt::pcsample
