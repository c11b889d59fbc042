#include "cpuprof.h"

#include <dirent.h>
#include <dlfcn.h>
#include <signal.h>
#include <sys/time.h>
#include <time.h>
#include <ucontext.h>

#include <cstdlib>

#include <algorithm>
#include <atomic>
#include <map>
#include <mutex>

namespace sca::prof {
namespace {

std::mutex g_mu;                 // start / stop
uintptr_t* g_pcs = nullptr;      // samples (program counters)
size_t g_cap = 0;
std::atomic<size_t> g_n{0};
std::atomic<bool> g_on{false};
struct sigaction g_old {};
std::vector<timer_t> g_timers;   // one CPU-time timer per thread alive at start()

// Per-thread CPU-time clock of thread `tid` (linux/posix-timers.h:
// MAKE_THREAD_CPUCLOCK(tid, CPUCLOCK_SCHED)).
clockid_t thread_cpu_clock(pid_t tid) { return clockid_t((~unsigned(tid) << 3) | 4 | 2); }

void on_sigprof(int, siginfo_t*, void* uc) {
  if (!g_on.load(std::memory_order_relaxed)) return;
  const size_t i = g_n.fetch_add(1, std::memory_order_relaxed);
  if (i >= g_cap) return;
  const auto* ctx = static_cast<const ucontext_t*>(uc);
#if defined(__x86_64__)
  g_pcs[i] = uintptr_t(ctx->uc_mcontext.gregs[REG_RIP]);
#else
  (void)ctx;
  g_pcs[i] = 0;
#endif
}

}  // namespace

bool start(int hz, size_t max_samples) {
  std::lock_guard<std::mutex> g(g_mu);
  if (g_on.load() || hz <= 0) return false;
  delete[] g_pcs;
  g_pcs = new uintptr_t[max_samples];
  g_cap = max_samples;
  g_n.store(0);
  struct sigaction sa {};
  sa.sa_sigaction = on_sigprof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  if (sigaction(SIGPROF, &sa, &g_old) != 0) return false;
  g_on.store(true);
  // A process-wide ITIMER_PROF coalesces expirations while its signal is
  // pending, so with many busy threads most samples are lost: arm one
  // CPU-time timer per thread instead, each signalling its own thread.
  itimerspec its{};
  its.it_interval.tv_nsec = std::max(1000L, 1000000000L / hz);
  its.it_value = its.it_interval;
  if (DIR* d = opendir("/proc/self/task")) {
    while (dirent* e = readdir(d)) {
      const int tid = std::atoi(e->d_name);
      if (tid <= 0) continue;
      sigevent sev{};
      sev.sigev_notify = SIGEV_THREAD_ID;
      sev.sigev_signo = SIGPROF;
      sev._sigev_un._tid = tid;
      timer_t t;
      if (timer_create(thread_cpu_clock(tid), &sev, &t) != 0) continue;
      if (timer_settime(t, 0, &its, nullptr) != 0) {
        timer_delete(t);
        continue;
      }
      g_timers.push_back(t);
    }
    closedir(d);
  }
  if (g_timers.empty()) {
    g_on.store(false);
    sigaction(SIGPROF, &g_old, nullptr);
    return false;
  }
  return true;
}

std::vector<std::pair<std::pair<std::string, uint64_t>, uint64_t>> stop() {
  std::lock_guard<std::mutex> g(g_mu);
  std::vector<std::pair<std::pair<std::string, uint64_t>, uint64_t>> out;
  if (!g_on.load()) return out;
  for (timer_t t : g_timers) timer_delete(t);
  g_timers.clear();
  g_on.store(false);
  sigaction(SIGPROF, &g_old, nullptr);
  const size_t n = std::min(g_n.load(), g_cap);
  std::map<uintptr_t, uint64_t> by_pc;
  for (size_t i = 0; i < n; ++i) by_pc[g_pcs[i]]++;
  std::map<std::pair<std::string, uint64_t>, uint64_t> agg;
  for (const auto& kv : by_pc) {
    Dl_info info{};
    if (kv.first && dladdr(reinterpret_cast<void*>(kv.first), &info) && info.dli_fname)
      agg[{info.dli_fname, uint64_t(kv.first - uintptr_t(info.dli_fbase))}] += kv.second;
    else
      agg[{"", uint64_t(kv.first)}] += kv.second;
  }
  out.assign(agg.begin(), agg.end());
  std::sort(out.begin(), out.end(), [](const auto& a, const auto& b) { return a.second > b.second; });
  return out;
}

}  // namespace sca::prof
