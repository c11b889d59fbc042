// Dynamic micro-batching GPU unit.
//
// Replaces the reference's one-HTTP-hop-per-request model call
// (engine/.../InternalPredictionService.java:248-296 -> python wrapper ->
// sklearn/xgboost on the CPU) with an in-process queue feeding a GPU.
//
//   request threads --(rows)--> queue --submit thread--> slot k: pack rows into
//   pinned memory, launch kernel(s) on slot stream, record event
//   --completion thread--> wait event, scatter rows back into responses, resume
//   each request's graph continuation.
//
// Batching is "greedy continuous": when the device is idle a lone request is
// launched immediately (latency = one launch); while `slots` batches are in
// flight new requests accumulate and the next batch takes all of them (up to
// max_batch rows), so throughput scales with load without a fixed timeout.
// Small batches run zero-copy (the kernel reads/writes fine-grained pinned host
// memory over PCIe: one launch, no DMA); large ones use async H2D/D2H copies.
#pragma once

#include <atomic>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../core/engine.h"
#include "models.h"

namespace sca::gpu {

struct BatcherOptions {
  int device = 0;            // -1 = run on the CPU (reference path)
  int max_batch = 1024;      // rows per launch
  int max_wait_us = 0;       // extra wait for a fuller batch (0 = greedy)
  int slots = 4;             // batches in flight
  bool zero_copy = true;
  size_t zero_copy_max_bytes = 256 << 10;
  bool spin_wait = true;     // completion thread spins on the event (lowest latency)
};

struct BatcherStats {
  uint64_t batches = 0;
  uint64_t rows = 0;
  uint64_t requests = 0;
  uint64_t max_rows = 0;
  double gpu_busy_s = 0;
};

class BatchedUnit : public Unit {
 public:
  BatchedUnit(RowModelPtr model, BatcherOptions opts);
  ~BatchedUnit() override;

  void transform_input(const CallCtx& c, MsgPtr in, Done k) override;
  void transform_output(const CallCtx& c, MsgPtr in, Done k) override { transform_input(c, std::move(in), std::move(k)); }
  std::string kind() const override { return "gpu:" + model_->name(); }
  bool ready() const override { return running_.load(); }

  BatcherStats stats() const;
  void reset_stats();
  const BatcherOptions& options() const { return opts_; }
  // Rows queued or on the device (replica load balancing).
  int64_t inflight_rows() const { return inflight_rows_.load(std::memory_order_relaxed); }
  RowModelPtr model() const { return model_; }

  // Synchronous dense call (tests / python ops): X [rows, cols] -> out.
  std::vector<double> run_dense(const std::vector<double>& X, int rows, int cols);

  void stop();

 private:
  struct Item {
    MsgPtr req;
    std::vector<double> x;
    int rows = 0;
    int cols = 0;
    Done k;
  };
  struct Slot {
    PinnedBuffer h_in, h_out;
    DeviceBuffer d_in, d_out, ws;
    PinnedBuffer h_seg;  // request row offsets (segmented models)
    Stream stream;
    Event ev;
    size_t cap_rows = 0;
    std::vector<Item> items;
    int rows = 0;
    int cols = 0;
    int out_cols = 0;
    bool busy = false;      // guarded by BatchedUnit::mu_
    bool launched = false;  // guarded by BatchedUnit::mu_
    std::condition_variable cv;
    std::thread th;         // per-slot completion thread
  };

  void ensure_capacity(Slot& s, int rows, int cols);
  void submit_loop();
  void complete_loop(Slot* s);
  void finish_items(std::vector<Item>& items, const double* out, int out_cols);
  MsgPtr make_response(const Item& it, const double* out, int out_cols) const;

  RowModelPtr model_;
  BatcherOptions opts_;
  std::vector<std::unique_ptr<Slot>> slots_;
  std::mutex mu_;
  std::condition_variable cv_submit_;
  std::deque<Item> queue_;
  size_t queued_rows_ = 0;
  std::atomic<bool> running_{false};
  std::atomic<int64_t> inflight_rows_{0};
  bool device_io_ = false;  // model needs device-memory I/O (no zero-copy)
  bool zc_input_ = true;
  bool segmented_ = false;    // model reads X once per element (zero-copy input is cheaper than a DMA)
  std::thread submit_th_;
  std::vector<std::string> default_names_;
  mutable std::mutex stats_mu_;
  BatcherStats stats_;
};

}  // namespace sca::gpu
