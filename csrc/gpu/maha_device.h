// Device-resident Mahalanobis outlier detector state (reference
// components/outlier-detection/mahalanobis/CoreMahalanobis.py:68-151).  The
// running mean / covariance / clip bounds live in HBM; each request batch is
// one single-workgroup kernel launch (csrc/kernels/mahalanobis.hip:
// maha_step) that reads the rows from pinned host memory and writes the
// scores back to it -- no per-request host linear algebra, no DMA.
#pragma once

#include <mutex>
#include <vector>

#include "../kernels/kernels.h"
#include "hip_util.h"

namespace sca::gpu {

class MahalanobisDevice {
 public:
  MahalanobisDevice(int p, int k, double n_stdev, double start_clip, double max_n, double eps, int device);
  // Scores of one request batch X [nb, p]; advances the state.
  std::vector<double> step(const double* X, int nb);
  // Flat state: mean[p] | C[p*p] | clip_lo[p] | clip_hi[p] | n | c_zero | has_clip
  std::vector<double> state() const;
  void set_state(const std::vector<double>& s);
  int p() const { return prm_.p; }
  int k() const { return prm_.k; }
  int device() const { return device_; }

 private:
  kern::MahaParams prm_;
  int device_;
  Stream stream_;
  DeviceBuffer state_, ws_;
  PinnedBuffer io_;  // X rows in, scores out
  size_t ws_rows_ = 0, io_rows_ = 0;
  mutable std::mutex mu_;
};

}  // namespace sca::gpu
