#include "cpuprof.h"

#include <dirent.h>
#include <dlfcn.h>
#include <execinfo.h>
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
// Sample buffer: allocated once at its maximum size and never freed or
// resized, so a SIGPROF handler still running from a previous session can
// only ever write inside it.  The handler bounds every store by kMaxWords
// with the depth it read itself, whatever start() publishes meanwhile.
constexpr size_t kMaxWords = size_t(1) << 22;  // 32 MiB of program counters
std::atomic<uintptr_t*> g_pcs{nullptr};
std::atomic<size_t> g_cap{0};
std::atomic<size_t> g_n{0};
std::atomic<bool> g_on{false};
std::atomic<int> g_depth{1};     // frames per sample: 1 = the interrupted PC only
std::vector<timer_t> g_timers;   // one CPU-time timer per thread alive at start()

// Per-thread CPU-time clock of thread `tid` (linux/posix-timers.h:
// MAKE_THREAD_CPUCLOCK(tid, CPUCLOCK_SCHED)).
clockid_t thread_cpu_clock(pid_t tid) { return clockid_t((~unsigned(tid) << 3) | 4 | 2); }

void on_sigprof(int, siginfo_t*, void* uc) {
  if (!g_on.load(std::memory_order_acquire)) return;
  uintptr_t* pcs = g_pcs.load(std::memory_order_relaxed);
  const size_t depth = size_t(g_depth.load(std::memory_order_relaxed));
  const size_t i = g_n.fetch_add(1, std::memory_order_relaxed);
  if (pcs == nullptr || i >= g_cap.load(std::memory_order_relaxed) || (i + 1) * depth > kMaxWords) return;
  uintptr_t* rec = pcs + i * depth;
  const auto* ctx = static_cast<const ucontext_t*>(uc);
#if defined(__x86_64__)
  rec[0] = uintptr_t(ctx->uc_mcontext.gregs[REG_RIP]);
#else
  (void)ctx;
  rec[0] = 0;
#endif
  if (depth > 1) {
    // Callers through the DWARF unwinder (libgcc, preloaded by start()):
    // frames [0, 1] are this handler and the signal trampoline.
    void* fr[34];
    const int n = backtrace(fr, std::min(34, int(depth) + 2));
    for (int d = 1; d < int(depth); ++d) rec[d] = d + 1 < n ? uintptr_t(fr[d + 1]) - 1 : 0;
  }
}

}  // namespace

bool start(int hz, size_t max_samples, int depth) {
  std::lock_guard<std::mutex> g(g_mu);
  if (g_on.load() || hz <= 0) return false;
  depth = std::max(1, std::min(depth, 32));
  if (depth > 1) {  // load the unwinder outside signal context
    void* fr[4];
    (void)backtrace(fr, 4);
  }
  if (g_pcs.load() == nullptr) g_pcs.store(new uintptr_t[kMaxWords]);  // once; never freed
  g_depth.store(depth);
  g_cap.store(std::min(max_samples, kMaxWords / size_t(depth)));
  g_n.store(0);
  struct sigaction sa {};
  sa.sa_sigaction = on_sigprof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  // The handler stays installed after stop() (a no-op while g_on is false):
  // restoring SIGPROF's default action could let a sample signal still pending
  // at stop() terminate the process.
  if (sigaction(SIGPROF, &sa, nullptr) != 0) return false;
  g_on.store(true, std::memory_order_release);  // publishes buffer, depth and cap to the handler
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
    return false;
  }
  return true;
}

Profile stop() {
  std::lock_guard<std::mutex> g(g_mu);
  Profile out;
  if (!g_on.load()) return out;
  for (timer_t t : g_timers) timer_delete(t);
  g_timers.clear();
  g_on.store(false);
  const size_t n = std::min(g_n.load(), g_cap.load());
  const int depth = g_depth.load();
  out.depth = depth;
  const uintptr_t* pcs = g_pcs.load();
  std::map<uintptr_t, Loc> locs;
  auto loc = [&](uintptr_t pc) -> const Loc& {
    auto it = locs.find(pc);
    if (it != locs.end()) return it->second;
    Loc l;
    Dl_info info{};
    if (pc && dladdr(reinterpret_cast<void*>(pc), &info) && info.dli_fname) {
      l.module = info.dli_fname;
      l.offset = uint64_t(pc - uintptr_t(info.dli_fbase));
    } else {
      l.offset = uint64_t(pc);
    }
    return locs.emplace(pc, std::move(l)).first->second;
  };
  std::map<std::vector<uintptr_t>, uint64_t> stacks;
  for (size_t i = 0; i < n; ++i) {
    const uintptr_t* rec = pcs + i * size_t(depth);
    stacks[std::vector<uintptr_t>(rec, rec + depth)]++;
  }
  for (const auto& kv : stacks) {
    Sample smp;
    smp.count = kv.second;
    for (uintptr_t pc : kv.first) smp.frames.push_back(loc(pc));
    out.samples.push_back(std::move(smp));
  }
  std::sort(out.samples.begin(), out.samples.end(), [](const Sample& a, const Sample& b) { return a.count > b.count; });
  return out;
}

}  // namespace sca::prof
