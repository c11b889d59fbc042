#include "maha_device.h"

#include <algorithm>
#include <stdexcept>

namespace sca::gpu {

MahalanobisDevice::MahalanobisDevice(int p, int k, double n_stdev, double start_clip, double max_n, double eps,
                                     int device)
    : device_(device) {
  if (p < 1 || p > kern::kMahaMaxP) throw std::runtime_error("MahalanobisDevice: 1 <= p <= 64 features");
  k = std::min(k, p);
  if (k < 1 || k > kern::kMahaMaxK) throw std::runtime_error("MahalanobisDevice: 1 <= n_components <= 16");
  prm_.p = p;
  prm_.k = k;
  prm_.n_stdev = n_stdev;
  prm_.start_clip = start_clip;
  prm_.max_n = max_n;
  prm_.eps = eps;
  stream_.create(device);
  state_.alloc(kern::maha_state_doubles(p) * sizeof(double), device);
  std::vector<double> init(kern::maha_state_doubles(p), 0.0);
  init[init.size() - 2] = 1.0;  // c_zero: the reference starts from C = 0 (int)
  state_.upload(init.data(), init.size() * sizeof(double));
}

std::vector<double> MahalanobisDevice::step(const double* X, int nb) {
  std::lock_guard<std::mutex> g(mu_);
  if (nb <= 0) return {};
  DeviceGuard dg(device_);
  const int p = prm_.p;
  if (size_t(nb) > ws_rows_) {
    ws_rows_ = std::max<size_t>(size_t(nb), ws_rows_ * 2);
    ws_.alloc(kern::maha_ws_doubles(int(ws_rows_), p, prm_.k) * sizeof(double), device_);
  }
  if (size_t(nb) > io_rows_) {
    io_rows_ = std::max<size_t>(size_t(nb), io_rows_ * 2);
    io_.alloc(io_rows_ * size_t(p + 1) * sizeof(double));
  }
  double* xin = io_.host<double>();
  std::copy(X, X + size_t(nb) * p, xin);
  double* dx = io_.dev<double>();
  double* dscore = dx + io_rows_ * size_t(p);
  kern::maha_step(dx, nb, prm_, state_.as<double>(), ws_.as<double>(), dscore, stream_.get());
  SCA_HIP_CHECK(hipGetLastError());
  SCA_HIP_CHECK(hipStreamSynchronize(stream_.get()));
  const double* hs = io_.host<double>() + io_rows_ * size_t(p);
  return std::vector<double>(hs, hs + nb);
}

std::vector<double> MahalanobisDevice::state() const {
  std::lock_guard<std::mutex> g(mu_);
  DeviceGuard dg(device_);
  std::vector<double> s(kern::maha_state_doubles(prm_.p));
  SCA_HIP_CHECK(hipMemcpy(s.data(), state_.get(), s.size() * sizeof(double), hipMemcpyDeviceToHost));
  return s;
}

void MahalanobisDevice::set_state(const std::vector<double>& s) {
  std::lock_guard<std::mutex> g(mu_);
  if (s.size() != kern::maha_state_doubles(prm_.p)) throw std::runtime_error("MahalanobisDevice: bad state size");
  DeviceGuard dg(device_);
  state_.upload(s.data(), s.size() * sizeof(double));
}

}  // namespace sca::gpu
