// Device-resident Mahalanobis outlier detector (reference
// components/outlier-detection/mahalanobis/CoreMahalanobis.py:68-151).
//
// The running mean / covariance / clip bounds live in HBM (MahaState).  The
// detector is a segmented RowModel served by the GPU micro-batcher: a batch of
// concurrent requests is ONE single-workgroup launch that steps the state
// through each request in order (csrc/kernels/mahalanobis.hip:
// maha_step_segments), completion is observed by the batcher's device thread,
// and consecutive batches -- which the batcher puts on different slot streams
// -- are chained on the state's own event, so the state advances in
// submission order with no host synchronisation between requests.
//
// Two views share one state: scores (the Python component computes its
// prediction / metrics from them) and predictions (`score > threshold`, the
// reference's predict() output; bound as a native graph node).
#pragma once

#include <memory>
#include <mutex>
#include <vector>

#include "../kernels/kernels.h"
#include "batcher.h"
#include "hip_util.h"
#include "models.h"

namespace sca::gpu {

// State + serialisation shared by every view of one detector.
struct MahaState {
  kern::MahaParams prm;
  int device = -1;                 // -1: host state (CPU reference path)
  DeviceBuffer d_state;
  DeviceBuffer d_eig;              // device diagnostics (step count, phase timers; not state)
  std::vector<double> h_state;     // device -1
  Event chain;                     // completes after the last launched step
  bool chained = false;
  // launch ordering across views / batchers; recursive so the Python
  // component can hold it across a pull -> host step -> push section
  // (MahalanobisDevice::lock_state) while state() / set_state() re-take it
  std::recursive_mutex mu;
  // rows launched so far, every view (under mu): the application order the
  // chained launches give the device state
  int64_t seq = 0;
};

class MahalanobisModel : public RowModel {
 public:
  MahalanobisModel(int p, int k, double n_stdev, double start_clip, double max_n, double eps, int out_mode,
                   double threshold);
  // Another view (output mode / threshold) over the same state.
  MahalanobisModel(std::shared_ptr<MahaState> st, int out_mode, double threshold);
  std::string name() const override { return "mahalanobis"; }
  int in_cols() const override { return st_->prm.p; }
  int out_cols(int) const override { return 1; }
  void to_device(int device) override;
  bool segmented() const override { return true; }
  int64_t last_sequence_base() const override { return seq_base_; }
  // launch_segments() takes the state mutex, which the Python component holds
  // across its pull -> host step -> push section: a pump thread of
  // its own, so that wait never stalls the other units on this GPU
  bool exclusive_driver() const override { return true; }
  bool zero_copy_input() const override { return false; }
  bool zero_copy_input_for(int rows, int cols) const override { return size_t(rows) * cols <= 4096; }
  size_t workspace_bytes(int max_rows, int cols) const override;
  void launch(const double* X, int rows, int cols, double* out, void* ws, hipStream_t s) override;
  void launch_segments(const double* X, int rows, int cols, double* out, void* ws, const int32_t* seg, int nseg,
                       hipStream_t s) override;
  // One request on the host state (device -1; the batcher calls it per request).
  void run_cpu(const double* X, int rows, int cols, double* out) const override;

  std::vector<double> state() const;  // mean[p] | C[p*p] | lo[p] | hi[p] | n | c_zero | has_clip
  void set_state(const std::vector<double>& s);
  std::shared_ptr<MahaState> shared_state() const { return st_; }
  // Device diagnostics: {0, steps, 0, phase us x 10} (GPU state only).
  std::vector<double> solver_stats() const;
  int p() const { return st_->prm.p; }
  int k() const { return st_->prm.k; }
  int device() const { return st_->device; }
  std::recursive_mutex& state_mutex() const { return st_->mu; }

 private:
  void init_state(int device);
  std::shared_ptr<MahaState> st_;
  kern::MahaParams view_;  // prm with this view's out_mode / threshold
  mutable int64_t seq_base_ = -1;  // this view's last launch (one batcher, one pump thread)
};

// Synchronous scores for the Python component: one batcher over a scores view.
// step() submits through the batcher (run_ptr) and returns when the device
// thread has seen the batch's completion event -- the caller never blocks in
// hipStreamSynchronize, and concurrent callers share launches.
class MahalanobisDevice {
 public:
  MahalanobisDevice(int p, int k, double n_stdev, double start_clip, double max_n, double eps, int device);
  ~MahalanobisDevice();
  std::vector<double> step(const double* X, int nb, int64_t* seq = nullptr);
  std::vector<double> state() const { return model_->state(); }
  void set_state(const std::vector<double>& s) { model_->set_state(s); }
  // Predictions view over the same state (for a native graph node).
  std::shared_ptr<MahalanobisModel> predict_view(double threshold) const;
  BatcherStats stats() const { return unit_->stats(); }
  std::vector<double> solver_stats() const { return model_->solver_stats(); }
  // Exclusive section over the shared state (same thread locks and unlocks):
  // native steps of the graph node wait until it ends.
  void lock_state() { model_->state_mutex().lock(); }
  void unlock_state() { model_->state_mutex().unlock(); }
  int p() const { return model_->p(); }
  int k() const { return model_->k(); }
  int device() const { return model_->device(); }

 private:
  std::shared_ptr<MahalanobisModel> model_;
  std::unique_ptr<BatchedUnit> unit_;
};

}  // namespace sca::gpu
