// Dynamic micro-batching GPU unit.
//
// Replaces the reference's one-HTTP-hop-per-request model call
// (engine/.../InternalPredictionService.java:248-296 -> python wrapper ->
// sklearn/xgboost on the CPU) with an in-process queue feeding a GPU.
//
//   front-end threads --(rows)--> queue --> device thread: pack rows into a
//   slot's pinned buffer, launch on the slot's stream, record its event ...
//   poll the in-flight events; a finished batch is split per request and each
//   request's continuation is posted back to the front-end thread that owns
//   it (Executor), which builds the response and walks on through the graph.
//
// One device thread per GPU (DeviceDriver, driver.h) does all launching and
// completion polling for every unit placed on that GPU, and one hand-off
// thread per GPU posts their responses, so a GPU costs two cores while busy
// and none while idle however many graph nodes it serves; the per-request
// work (response construction, meta merge, serialisation) runs on the
// front-end threads.  Batching is "greedy continuous": when the device is
// idle a lone request is launched immediately (latency = one launch); while
// `slots` batches are in flight new requests accumulate and the next batch
// takes all of them (up to max_batch rows), so batch size tracks load without
// a fixed timeout.  Small batches run zero-copy (kernels read/write
// fine-grained pinned host memory: one launch, no DMA); large ones, or models
// that re-read their input from many workgroups, go through HBM.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../core/engine.h"
#include "models.h"

namespace sca::gpu {

class DeviceDriver;

struct BatcherOptions {
  int device = 0;            // -1 = run on the CPU (reference path)
  int max_batch = 1024;      // rows per launch
  int max_wait_us = 0;       // extra wait for a fuller batch when the device is idle (0 = greedy)
  int slots = 4;             // batches in flight
  bool zero_copy = true;
  size_t zero_copy_max_bytes = 256 << 10;
  bool spin_wait = true;     // poll events (lowest latency); false = block on the oldest batch
  // device -1 only: run the CPU reference path through the same queue /
  // device-thread / executor machinery instead of inline (tests, CPU serving
  // of heavier models).
  bool cpu_batching = false;
  // Failure detection (the reference relies on k8s probes,
  // seldondeployment_controller.go:518,521, and the engine's TCP readiness
  // checker, SeldonGraphReadyChecker.java:45-118).  A unit whose batches fail
  // `fail_threshold` times in a row, or whose oldest in-flight batch is older
  // than `hang_timeout_ms` (the watchdog: its requests are answered with 210
  // at once, the slot is parked until the device lets it go), is unhealthy for
  // `cooldown_ms`: ready() is false and replica sets route around it.  After
  // the cooldown it takes traffic again (half-open); one more failure re-trips.
  int fail_threshold = 3;
  int cooldown_ms = 2000;
  int hang_timeout_ms = 10000;  // 0 = no watchdog
};

// Fault injection for tests and drills (SURVEY §5.3 "fault-injection hook").
// Set per unit (inject_fault) or from the environment at construction:
//   SCA_FAULT="gpu:1:fail_after=100,fail_count=5;cpu:*:hang_ms=50"
// entries `<gpu|cpu>:<device|*>:key=value,...`.  Injected failures never
// touch the device: the batch is failed before launch (fail_*), or its
// completion is held on the host (hang_ms), so a drill cannot wedge a GPU.
struct FaultSpec {
  int64_t fail_after = -1;  // batches that run normally before injected failures begin (-1 = off)
  int64_t fail_count = -1;  // injected failures before the unit recovers (-1 = forever)
  int hang_ms = 0;          // hold each batch's completion this long (slow / hung device)
};
FaultSpec fault_from_env(int device);

struct UnitHealth {
  bool healthy = true;
  int consecutive_failures = 0;
  uint64_t failed_batches = 0;
  uint64_t hangs = 0;
  uint64_t trips = 0;
  uint64_t injected = 0;
};

struct BatcherStats {
  uint64_t batches = 0;
  uint64_t rows = 0;
  uint64_t requests = 0;
  uint64_t max_rows = 0;
  double gpu_busy_s = 0;     // sum over batches of launch -> completion observed
  double launch_cpu_s = 0;   // device thread: staging + kernel launch + event record
  double complete_cpu_s = 0; // device thread: response hand-off to the front-end threads
};

class BatchedUnit : public Unit {
 public:
  BatchedUnit(RowModelPtr model, BatcherOptions opts);
  ~BatchedUnit() override;

  void transform_input(const CallCtx& c, MsgPtr in, Done k) override;
  void transform_output(const CallCtx& c, MsgPtr in, Done k) override { transform_input(c, std::move(in), std::move(k)); }
  std::string kind() const override { return "gpu:" + model_->name(); }
  bool ready() const override { return running_.load() && healthy(); }
  // Circuit state (see BatcherOptions): false while a trip's cooldown runs.
  bool healthy() const;
  UnitHealth health() const;
  void inject_fault(const FaultSpec& f);

  BatcherStats stats() const;
  void reset_stats();
  void collect_metrics(MetricsRegistry& m, const Labels& labels) const override;
  const BatcherOptions& options() const { return opts_; }
  RowModelPtr model() const { return model_; }
  // Rows queued or on the device (replica load balancing).
  int64_t inflight_rows() const { return inflight_rows_.load(std::memory_order_relaxed); }

  // Synchronous dense call (tests / python ops): X [rows, cols] -> out.
  std::vector<double> run_dense(const std::vector<double>& X, int rows, int cols);
  // Same, reading the rows straight from caller memory (kept alive by the
  // caller until the call returns): no copy before the GPU staging / DMA.
  std::vector<double> run_ptr(const double* X, int rows, int cols, int64_t* seq = nullptr);

  void stop();

  friend class DeviceDriver;
  // Response construction shared with posted continuations (outlives no unit
  // state it does not own).
  struct RespInfo {
    RowModelPtr model;
    std::vector<std::string> names;  // client_class_names: explicit, else t:0..t:C-1
  };

 private:
  struct Item {
    MsgPtr req;
    std::vector<double> x;     // decoded rows, when the message holds no flat fp64 array
    const double* xp = nullptr;  // the rows: into req's tensor values, `x`, or caller memory (run_ptr)
    int rows = 0;
    int cols = 0;
    Done k;
    ExecPtr exec;
    bool caller_mem = false;  // xp is the run_ptr caller's buffer (freed once the caller is answered)
    int64_t* seq_out = nullptr;  // run_ptr callers: where the model applied this request's first row
  };
  struct Slot {
    PinnedBuffer h_in, h_out, h_seg;
    BarBuffer v_in;  // SCA_BATCH_INPUT=bar: zero-copy batch rows in HBM, written by the CPU
    std::vector<double> cpu_out;  // device -1 (cpu_batching)
    std::vector<double> fin;      // host-finished outputs (RowModel::finish_host)
    int raw_cols = 0;             // > 0: the kernel wrote raw_cols values per row into h_out
    std::vector<double> cpu_in;   // device -1, asynchronous models: the batch's rows back to back
    CpuCallPtr call;              // device -1: the batch's outstanding start_cpu() call
    DeviceBuffer d_in, d_out, ws;
    Stream stream;
    Event ev;
    size_t cap_rows = 0;
    std::vector<Item> items;
    int rows = 0;
    int cols = 0;
    int out_cols = 0;
    bool abandoned = false;  // watchdog answered its requests; waiting for the device to finish
    // Direct path (one message-owned request >= kDirectH2DBytes DMA'd from
    // its own memory): a watchdog-abandoned batch keeps the request alive
    // here until the slot's event completes, since that copy may still be
    // reading it.  (run_ptr callers' buffers never take this path.)
    bool direct = false;
    std::vector<Item> parked;
    uint64_t roctx = 0;      // marker range of the batch (SCA_ROCTX=1)
    std::chrono::steady_clock::time_point t_launch;
  };

  // One completed batch on its way to the front-end threads: the requests and
  // one copy of the slot's output rows (the slot is reused at once).
  struct Handoff {
    BatchedUnit* unit = nullptr;
    bool fence = false;        // marker: every earlier hand-off of `unit` has been posted
    std::vector<Item> items;
    std::vector<size_t> offs;  // each item's first output value in `out`
    std::vector<double> out;
    int out_cols = 0;
  };

  // One batch's requests bound for one front-end executor, with their output
  // rows.  Parcels are recycled: the worker that ran one returns it to the
  // pool, the hand-off thread refills it, so in steady state no buffer is
  // allocated on one thread and freed on another (cross-thread frees took the
  // allocator's arena locks in the r02i CPU profiles).  The Items themselves
  // were created by the worker that finally destroys them.
  struct Parcel;
  struct ParcelPool {
    std::atomic<Parcel*> head{nullptr};
    ~ParcelPool();
    void put(Parcel* p);  // lock-free push (any thread)
    Parcel* take_all() { return head.exchange(nullptr, std::memory_order_acquire); }  // single consumer
  };
  struct Parcel {
    std::shared_ptr<ParcelPool> pool;  // set while out of the pool
    std::shared_ptr<const RespInfo> info;
    std::vector<Item> items;
    std::vector<double> y;  // the items' output rows, back to back
    int oc = 0;
    Parcel* next = nullptr;
    void run();  // on the executor: respond to every item, then go back to the pool
  };

  void ensure_capacity(Slot& s, int rows, int cols);
  // Driven by the DeviceDriver thread of this unit's GPU (one thread per GPU
  // pumps every unit placed there): one round of take queued requests ->
  // launch into free slots -> reap finished batches.  Returns whether it made
  // progress; `busy` = batches in flight or requests taken but not launched.
  bool pump(bool watch, bool& busy);
  void finish_all();            // stop(): launch what was taken, complete everything in flight
  bool block_on_oldest();       // low-CPU mode: wait for the oldest batch (false: cannot here)
  bool has_queued() const { return queued_n_.load(std::memory_order_acquire) > 0; }
  bool spin_wait() const { return opts_.spin_wait && !cpu_; }
  void post_responses(Handoff& h, std::vector<Parcel*>& spare);
  bool launch(Slot* s);
  void complete(Slot* s, hipError_t st);
  void abandon(Slot* s);
  bool take_injected_failure();
  void note_failure();
  void note_success();
  static ErrPtr device_error(ApiError kind, std::string info);
  static MsgPtr make_response(const RespInfo& info, const Item& it, const double* out, int out_cols);
  void submit_item(Item it);

  RowModelPtr model_;
  BatcherOptions opts_;
  Histogram batch_hist_;  // device time per batch (launch -> completion event), exported at scrape time
  Histogram rows_hist_;   // rows per batch (observed as "seconds" = rows * 1e-6 for the shared bucket grid)
  std::shared_ptr<const RespInfo> resp_;
  std::vector<std::unique_ptr<Slot>> slots_;
  // Submission shards: a front-end thread pushes into the shard of its thread
  // index under that shard's own lock, so producers do not contend with each
  // other (one queue mutex cost 5-15% of the front end's CPU in futex waits at
  // 600-900k req/s, profiles/r02i_frontend); the device thread drains every
  // non-empty shard into its private backlog.
  struct alignas(64) Shard {
    std::mutex mu;
    std::deque<Item> q;
    std::atomic<int> n{0};
  };
  static constexpr int kShards = 16;
  Shard shards_[kShards];
  void drain_shards(std::deque<Item>& into);
  std::atomic<int64_t> queued_rows_{0};
  std::atomic<int> queued_n_{0};        // items in the shards (the device thread's "work waiting" test)
  std::atomic<bool> running_{false};
  std::atomic<int64_t> inflight_rows_{0};
  bool device_io_ = false;  // model needs device-memory I/O (no zero-copy)
  bool bar_input_ = false;  // SCA_BATCH_INPUT=bar on a large-BAR device
  // HDP_MEM_COHERENCY_FLUSH_CNTL of the device (BAR staging): CPU stores into
  // HBM pass the GPU's host data path, whose write buffer is flushed before
  // the kernel that reads them is launched (SCA_HDP_FLUSH=0 skips it)
  volatile uint32_t* hdp_flush_ = nullptr;
  bool zc_input_ = true;    // model reads X once per element (zero-copy input is cheaper than a DMA)
  bool segmented_ = false;
  bool cpu_ = false;        // device -1 with cpu_batching
  // Device-thread state (touched only by the driver's pump thread)
  struct PumpState {
    std::vector<Slot*> free_list, inflight;
    std::deque<Item> pending;  // taken from the shards, not yet in a slot
    std::chrono::steady_clock::time_point hold_start{};
    bool holding = false;      // max_wait_us: waiting for a fuller first batch
  };
  PumpState ps_;
  std::shared_ptr<DeviceDriver> driver_;  // the thread pair that pumps this unit and posts its responses
  std::shared_ptr<ParcelPool> parcels_ = std::make_shared<ParcelPool>();
  mutable std::mutex stats_mu_;
  BatcherStats stats_;
  // device-thread CPU time (single writer: the device thread; relaxed reads)
  std::atomic<double> launch_cpu_s_{0.0}, complete_cpu_s_{0.0};
  // health / fault injection
  std::atomic<int> consec_fail_{0};
  std::atomic<int64_t> open_until_ns_{0};  // steady_clock ns; unhealthy before this
  std::atomic<uint64_t> failed_batches_{0}, hangs_{0}, trips_{0};
  std::atomic<int> hang_ms_{0};             // injected completion delay (read by the device thread)
  std::atomic<bool> fault_armed_{false};
  std::atomic<int> abandoned_slots_{0};    // all of them = device wedged: fail fast
  mutable std::mutex fault_mu_;
  FaultSpec fault_;
  int64_t fault_launches_ = 0, fault_injected_ = 0;
};

}  // namespace sca::gpu
