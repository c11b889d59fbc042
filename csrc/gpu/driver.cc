#include "driver.h"

#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <map>

namespace sca::gpu {

namespace {

// Idle-spin permits shared by every driver of the process: a multi-GPU
// deployment otherwise keeps two spinning threads per GPU on the CPU share
// the front end needs.  SCA_MAX_SPINNERS, default 16 (profiles/r03h_frontend_fp32,
// profiles/r03r_head/spin_ab).
std::atomic<int> g_spinners{0};
int max_spinners() {
  static const int m = [] {
    const char* e = std::getenv("SCA_MAX_SPINNERS");
    return e ? std::max(0, std::atoi(e)) : 16;
  }();
  return m;
}
struct SpinPermit {
  bool ok;
  SpinPermit() : ok(g_spinners.fetch_add(1, std::memory_order_relaxed) < max_spinners()) {
    if (!ok) g_spinners.fetch_sub(1, std::memory_order_relaxed);
  }
  ~SpinPermit() {
    if (ok) g_spinners.fetch_sub(1, std::memory_order_relaxed);
  }
};

using clk = std::chrono::steady_clock;

}  // namespace

std::shared_ptr<DeviceDriver> DeviceDriver::acquire(int device, bool shared) {
  static const bool per_unit = [] {
    const char* e = std::getenv("SCA_DRIVER_PER_UNIT");
    return e && e[0] == '1';
  }();
  if (!shared || per_unit) return std::make_shared<DeviceDriver>(device);
  static std::mutex m;
  static std::map<int, std::weak_ptr<DeviceDriver>> reg;
  std::lock_guard<std::mutex> g(m);
  auto& w = reg[device];
  auto d = w.lock();
  if (!d) {
    d = std::make_shared<DeviceDriver>(device);
    w = d;
  }
  return d;
}

DeviceDriver::DeviceDriver(int device) : device_(device) {
  if (device == kAsyncCpuDriver) {
    const char* e = std::getenv("SCA_ASYNC_INLINE_HANDOFF");
    inline_handoff_ = !e || std::atoi(e) != 0;
  } else {
    // GPU pumps post responses themselves by default: the hand-off thread's
    // spin cost a CPU the front end needs (headline A/B, profiles/r05l_inline:
    // server -0.8 CPU, +3% REST, p99 0.23 vs 0.24-0.44 ms)
    const char* e = std::getenv("SCA_INLINE_HANDOFF");
    inline_handoff_ = e ? std::atoi(e) != 0 : device >= 0;
  }
  if (const char* e = std::getenv("SCA_IDLE_SPIN_US")) idle_spin_us_ = std::max(0, std::atoi(e));
  ho_spin_us_ = idle_spin_us_;
  if (const char* e = std::getenv("SCA_HANDOFF_SPIN_US")) ho_spin_us_ = std::max(0, std::atoi(e));
  ho_th_ = std::thread([this] { handoff_loop(); });
  pump_th_ = std::thread([this] { pump_loop(); });
}

DeviceDriver::~DeviceDriver() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
    version_.fetch_add(1, std::memory_order_release);  // the pump re-reads membership and sees stop_
  }
  cv_.notify_all();
  if (pump_th_.joinable()) pump_th_.join();
  {
    std::lock_guard<std::mutex> g(ho_mu_);
    ho_stop_ = true;
  }
  ho_cv_.notify_all();
  if (ho_th_.joinable()) ho_th_.join();
  for (auto* p : inline_spare_) delete p;
}

int DeviceDriver::units() const {
  std::lock_guard<std::mutex> g(mu_);
  return int(units_.size());
}

void DeviceDriver::add(BatchedUnit* u) {
  {
    std::lock_guard<std::mutex> g(mu_);
    units_.push_back(u);
    version_.fetch_add(1, std::memory_order_release);
  }
  cv_.notify_all();
}

void DeviceDriver::remove(BatchedUnit* u) {
  std::unique_lock<std::mutex> lk(mu_);
  if (std::find(units_.begin(), units_.end(), u) == units_.end()) return;
  removing_.push_back(u);
  version_.fetch_add(1, std::memory_order_release);
  cv_.notify_all();
  cv_removed_.wait(lk, [&] { return std::find(units_.begin(), units_.end(), u) == units_.end(); });
}

void DeviceDriver::wake() {
  { std::lock_guard<std::mutex> g(mu_); }
  cv_.notify_all();
}

bool DeviceDriver::any_queued(const std::vector<BatchedUnit*>& us) const {
  for (auto* u : us)
    if (u->has_queued()) return true;
  return false;
}

// Pump thread: a leaving unit is drained here, off the caller's thread, so
// the pump never races its own state: its taken requests are launched, every
// batch in flight completes, and a fence through the hand-off queue confirms
// every response was posted before remove() returns.
void DeviceDriver::retire(const std::vector<BatchedUnit*>& gone) {
  for (auto* u : gone) {
    u->finish_all();
    BatchedUnit::Handoff f;
    f.unit = u;
    f.fence = true;
    uint64_t ticket;
    {
      std::lock_guard<std::mutex> g(ho_mu_);
      ticket = ++ho_fences_pushed_;
      ho_q_.push_back(std::move(f));
      ho_pending_.store(true, std::memory_order_release);
    }
    ho_cv_.notify_all();
    std::unique_lock<std::mutex> lk(ho_mu_);
    ho_fence_cv_.wait(lk, [&] { return ho_fences_done_ >= ticket; });
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto* u : gone) {
      units_.erase(std::remove(units_.begin(), units_.end(), u), units_.end());
      removing_.erase(std::remove(removing_.begin(), removing_.end(), u), removing_.end());
    }
    version_.fetch_add(1, std::memory_order_release);
  }
  cv_removed_.notify_all();
}

void DeviceDriver::pump_loop() {
  if (device_ >= 0) (void)hipSetDevice(device_);
  std::vector<BatchedUnit*> us;
  uint64_t seen = ~uint64_t(0);
  int spins = 0;
  clk::time_point wait_start{};
  while (true) {
    // ---- membership (rare): leaving units are drained first
    if (version_.load(std::memory_order_acquire) != seen) {
      std::vector<BatchedUnit*> gone;
      {
        std::lock_guard<std::mutex> g(mu_);
        seen = version_.load(std::memory_order_acquire);
        us = units_;
        gone = removing_;
        if (stop_ && units_.empty()) break;
      }
      if (!gone.empty()) {
        retire(gone);
        continue;
      }
    }
    // ---- one round over every unit
    const bool watch = spins >= 512 || (spins & 31) == 0;  // the hang watchdog's clock reads
    bool progress = false, busy = false;
    for (auto* u : us) {
      bool b = false;
      progress |= u->pump(watch, b);
      busy |= b;
    }
    if (progress) {
      spins = 0;
      continue;
    }
    if (!busy) {
      // Idle.  Brief spin first: a closed-loop caller's next request usually
      // arrives within tens of microseconds, and a condition-variable wake-up
      // costs about that much again.
      if (idle_spin_us_ > 0 && !any_queued(us)) {
        SpinPermit permit;
        const auto until = clk::now() + std::chrono::microseconds(idle_spin_us_);
        // (the clock is read every 32 pauses: a vDSO clock_gettime per pause
        // was ~10% of the serving process's CPU with several units spinning)
        for (unsigned n = 1; permit.ok && !any_queued(us) &&
                             version_.load(std::memory_order_relaxed) == seen;
             ++n) {
          _mm_pause();
          if ((n & 31) == 0 && clk::now() >= until) break;
        }
      }
      if (!any_queued(us) && version_.load(std::memory_order_acquire) == seen) {
        std::unique_lock<std::mutex> lk(mu_);
        sleeping_.store(true, std::memory_order_seq_cst);
        // Pairs with BatchedUnit::submit_item's queued_n_ increment + notify():
        // either we see the item or the submitter sees us asleep and wakes us.
        cv_.wait(lk, [&] {
          return stop_ || version_.load(std::memory_order_acquire) != seen || any_queued(units_);
        });
        sleeping_.store(false, std::memory_order_relaxed);
      }
      spins = 0;
      continue;
    }
    bool launchable = false;  // new work for a unit with a free slot: the next round launches it
    for (auto* u : us) launchable |= u->has_queued() && !u->ps_.free_list.empty();
    if (launchable) continue;
    // ---- busy, nothing finished yet
    bool spin = false;
    BatchedUnit* only = nullptr;
    int n_busy = 0;
    for (auto* u : us) {
      spin |= u->spin_wait();
      if (!u->ps_.inflight.empty() || !u->ps_.pending.empty()) {
        only = u;
        ++n_busy;
      }
    }
    if (!spin) {  // low-CPU mode: block on the oldest batch when one unit alone is busy
      if (!(n_busy == 1 && only->block_on_oldest())) std::this_thread::sleep_for(std::chrono::microseconds(20));
      continue;
    }
    // Spin through the usual 10-50 us round trip; back off if the GPU is slow
    // so a long kernel does not burn a core (and CPU quota) for nothing.
    if (spins++ == 0) wait_start = clk::now();
    if (spins < 512) {
      _mm_pause();
    } else if (clk::now() - wait_start < std::chrono::microseconds(200)) {
      std::this_thread::yield();
    } else {
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }
}

void DeviceDriver::push_handoff(BatchedUnit::Handoff&& h) {
  if (inline_handoff_ && !h.fence) {  // (pump thread)
    h.unit->post_responses(h, inline_spare_);
    h.unit = nullptr;
    std::lock_guard<std::mutex> g(ho_mu_);
    ho_free_.push_back(std::move(h));
    return;
  }
  bool wake;
  {
    std::lock_guard<std::mutex> g(ho_mu_);
    ho_q_.push_back(std::move(h));
    wake = ho_sleeping_;
  }
  ho_pending_.store(true, std::memory_order_release);
  if (wake) ho_cv_.notify_one();
}

BatchedUnit::Handoff DeviceDriver::take_free_handoff() {
  std::lock_guard<std::mutex> g(ho_mu_);
  if (ho_free_.empty()) return BatchedUnit::Handoff();
  BatchedUnit::Handoff h = std::move(ho_free_.back());
  ho_free_.pop_back();
  return h;
}

// Hand-off thread: groups each completed batch's requests by front-end
// executor and posts them (eventfd wake-ups), off the pump thread, which only
// launches and reaps batches.
void DeviceDriver::handoff_loop() {
  std::vector<BatchedUnit::Handoff> batch;
  std::vector<BatchedUnit::Parcel*> spare;
  while (true) {
    uint64_t fences = 0;
    {
      std::unique_lock<std::mutex> lk(ho_mu_);
      for (auto& h : batch) {  // emptied below: capacity goes back
        if (h.fence) continue;
        h.unit = nullptr;
        ho_free_.push_back(std::move(h));
      }
      batch.clear();
      if (ho_q_.empty() && !ho_stop_ && ho_spin_us_ > 0) {  // brief spin before sleeping (see pump_loop)
        lk.unlock();
        SpinPermit permit;
        const auto until = clk::now() + std::chrono::microseconds(ho_spin_us_);
        for (unsigned n = 1; permit.ok && !ho_pending_.load(std::memory_order_acquire); ++n) {
          _mm_pause();
          if ((n & 31) == 0 && clk::now() >= until) break;
        }
        lk.lock();
      }
      if (ho_q_.empty()) {
        if (ho_stop_) break;
        ho_sleeping_ = true;
        ho_cv_.wait(lk, [&] { return ho_stop_ || !ho_q_.empty(); });
        ho_sleeping_ = false;
        if (ho_q_.empty()) break;  // stopping with nothing left
      }
      batch.swap(ho_q_);
      ho_pending_.store(false, std::memory_order_relaxed);
    }
    for (auto& h : batch) {
      if (h.fence) {
        ++fences;
        continue;
      }
      h.unit->post_responses(h, spare);
    }
    if (fences) {
      {
        std::lock_guard<std::mutex> g(ho_mu_);
        ho_fences_done_ += fences;
      }
      ho_fence_cv_.notify_all();
    }
  }
  for (auto* p : spare) delete p;
}

}  // namespace sca::gpu
