// DeviceDriver: the thread pair that runs every micro-batched unit on one GPU.
//
// A graph spreads its nodes over units (an A/B test: router + two model
// units; a bandit: router + N replicas; a pipeline: one unit per stage).
// With a device thread and a hand-off thread per unit, an A/B graph folded on
// one GPU ran 4 spinning service threads next to the front end's 10 on a
// 16-CPU share, and the OS time-slicing them set the tail: p99 1.7-2.0 ms at
// p50 0.16 ms, while the same graph with 8 front-end threads had p99 0.49 ms
// (profiles/r04b_multiunit).  Here ONE pump thread per GPU round-robins
// every unit placed on it (take queued requests -> launch into free slots ->
// reap finished batches, BatchedUnit::pump) and ONE hand-off thread posts
// every unit's completed batches to the front-end executors -- the same two
// cores whatever the graph, which is also how the hardware is organised:
// one command-processor front end per device.
//
// CPU-batching units (device -1) get a private driver: their launch() may run
// a model inline on the pump thread.
#pragma once

#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "batcher.h"

namespace sca::gpu {

// Driver key of the shared pump for asynchronous CPU-batching units.
constexpr int kAsyncCpuDriver = -2;

class DeviceDriver {
 public:
  // The shared driver of `device` (created on first use, gone with its last
  // unit); `shared` false gives a private one.  SCA_DRIVER_PER_UNIT=1 makes
  // every driver private (the pre-r04 thread layout, for A/B runs).
  static std::shared_ptr<DeviceDriver> acquire(int device, bool shared);
  explicit DeviceDriver(int device);
  ~DeviceDriver();
  DeviceDriver(const DeviceDriver&) = delete;
  DeviceDriver& operator=(const DeviceDriver&) = delete;

  void add(BatchedUnit* u);
  // Launches what `u` has taken, completes its batches in flight, posts all
  // its responses; `u` is not touched once this returns.
  void remove(BatchedUnit* u);
  // A unit queued work: wake the pump thread if it sleeps.
  void notify() {
    if (sleeping_.load(std::memory_order_seq_cst)) wake();
  }
  // Completed batches of a unit, in completion order, to the hand-off thread.
  void push_handoff(BatchedUnit::Handoff&& h);
  BatchedUnit::Handoff take_free_handoff();  // recycled buffers (or a fresh one)
  int units() const;

 private:
  void wake();
  void pump_loop();
  void handoff_loop();
  void retire(const std::vector<BatchedUnit*>& gone);  // pump thread: finish + fence, then release
  bool any_queued(const std::vector<BatchedUnit*>& us) const;

  int device_;
  mutable std::mutex mu_;
  std::condition_variable cv_;          // pump thread sleep / wake
  std::condition_variable cv_removed_;  // remove() waits for the pump thread
  std::vector<BatchedUnit*> units_;     // guarded by mu_
  std::vector<BatchedUnit*> removing_;  // guarded by mu_
  std::atomic<uint64_t> version_{0};    // bumped when units_ / removing_ change
  std::atomic<bool> sleeping_{false};
  bool stop_ = false;                   // guarded by mu_
  int idle_spin_us_ = 50;               // SCA_IDLE_SPIN_US
  int ho_spin_us_ = 50;                 // SCA_HANDOFF_SPIN_US (default: the idle spin)
  // hand-off queue
  std::mutex ho_mu_;
  std::condition_variable ho_cv_;
  std::condition_variable ho_fence_cv_;
  std::vector<BatchedUnit::Handoff> ho_q_;     // guarded by ho_mu_
  std::vector<BatchedUnit::Handoff> ho_free_;  // guarded by ho_mu_
  bool ho_sleeping_ = false;                   // guarded by ho_mu_
  bool ho_stop_ = false;                       // guarded by ho_mu_
  uint64_t ho_fences_pushed_ = 0, ho_fences_done_ = 0;  // guarded by ho_mu_
  std::atomic<bool> ho_pending_{false};
  // The shared pump of asynchronous CPU units (mesh programs) posts their
  // responses itself: their batches complete in the pump's done() poll with
  // no device work to overlap, and a second thread would add a wake-up per
  // batch (fences still go through the hand-off thread).
  bool inline_handoff_ = false;
  std::vector<BatchedUnit::Parcel*> inline_spare_;  // pump thread only
  std::thread pump_th_, ho_th_;
};

}  // namespace sca::gpu
