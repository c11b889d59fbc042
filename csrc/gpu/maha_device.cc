#include "maha_device.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <stdexcept>

namespace sca::gpu {

namespace {

kern::MahaParams make_params(int p, int k, double n_stdev, double start_clip, double max_n, double eps) {
  if (p < 1 || p > kern::kMahaMaxP) throw std::runtime_error("Mahalanobis: 1 <= p <= 64 features");
  k = std::min(k, p);
  if (k < 1 || k > kern::kMahaMaxK) throw std::runtime_error("Mahalanobis: 1 <= n_components <= 16");
  kern::MahaParams prm;
  prm.p = p;
  prm.k = k;
  prm.n_stdev = n_stdev;
  prm.start_clip = start_clip;
  prm.max_n = max_n;
  prm.eps = eps;
  if (const char* v = std::getenv("SCA_MAHA_MW_MIN_P")) prm.mw_min_p = std::atoi(v);
  if (const char* v = std::getenv("SCA_MAHA_JACOBI_MAX_P"))
    prm.jacobi_max_p = std::min(kern::kMahaMaxP, std::max(0, std::atoi(v)));
  if (const char* v = std::getenv("SCA_MAHA_RANK1_MAX_P"))
    prm.rank1_max_p = std::min(kern::kMahaMaxP, std::max(0, std::atoi(v)));
  return prm;
}

// Gauss-Jordan with partial pivoting; returns det(A) (0 if singular).
double invert_host(std::vector<double> M, std::vector<double>& inv, int k) {
  inv.assign(size_t(k) * k, 0.0);
  for (int i = 0; i < k; ++i) inv[size_t(i) * k + i] = 1.0;
  double det = 1.0;
  for (int c = 0; c < k; ++c) {
    int piv = c;
    for (int r = c + 1; r < k; ++r)
      if (std::fabs(M[size_t(r) * k + c]) > std::fabs(M[size_t(piv) * k + c])) piv = r;
    if (M[size_t(piv) * k + c] == 0.0) return 0.0;
    if (piv != c) {
      for (int j = 0; j < k; ++j) {
        std::swap(M[size_t(c) * k + j], M[size_t(piv) * k + j]);
        std::swap(inv[size_t(c) * k + j], inv[size_t(piv) * k + j]);
      }
      det = -det;
    }
    const double d = M[size_t(c) * k + c];
    det *= d;
    for (int j = 0; j < k; ++j) {
      M[size_t(c) * k + j] /= d;
      inv[size_t(c) * k + j] /= d;
    }
    for (int r = 0; r < k; ++r) {
      if (r == c) continue;
      const double f = M[size_t(r) * k + c];
      if (f == 0.0) continue;
      for (int j = 0; j < k; ++j) {
        M[size_t(r) * k + j] -= f * M[size_t(c) * k + j];
        inv[size_t(r) * k + j] -= f * inv[size_t(c) * k + j];
      }
    }
  }
  return det;
}

// Host reference of one detector step (the kernel's maha_one, serial): used
// for device -1 placement and as the oracle of the segmented launch.
void maha_step_host(const double* X, int nb, const kern::MahaParams& prm, double* state, double* out) {
  const int p = prm.p, k = prm.k;
  double* s_mean = state;
  double* s_C = state + p;
  double* s_lo = s_C + size_t(p) * p;
  double* s_hi = s_lo + p;
  double* s_tail = s_hi + p;
  const double n_state = s_tail[0];
  const bool c_zero = s_tail[1] != 0.0;
  const bool do_clip = n_state > prm.start_clip && s_tail[2] != 0.0;
  const double n = prm.max_n > 0 ? std::min(n_state, prm.max_n) : n_state;
  std::vector<double> Cold(size_t(p) * p), XC(size_t(nb) * p), MO(size_t(nb) * p), D(size_t(nb) * p);
  for (size_t e = 0; e < Cold.size(); ++e) Cold[e] = c_zero ? 0.0 : s_C[e];
  for (int j = 0; j < p; ++j) {
    const double m0 = s_mean[j];
    double cum = 0.0, prev = m0;
    for (int i = 0; i < nb; ++i) {
      double x = X[size_t(i) * p + j];
      if (do_clip) x = std::min(std::max(x, s_lo[j]), s_hi[j]);
      cum += x;
      const double roll = cum / double(i + 1);
      const double nm = m0 + (double(i + 1) / (double(i) + n + 1.0)) * (roll - m0);
      XC[size_t(i) * p + j] = x;
      MO[size_t(i) * p + j] = prev;
      D[size_t(i) * p + j] = x - prev;
      prev = nm;
    }
    s_mean[j] = prev;
  }
  const double den = n + std::max(1.0, double(nb) - 1.0);
  std::vector<double> A(size_t(p) * p);
  for (int a = 0; a < p; ++a)
    for (int b = 0; b < p; ++b) {
      double acc = 0.0;
      for (int i = 0; i < nb; ++i) acc += ((n + i) / (n + i + 1.0)) * (D[size_t(i) * p + a] * D[size_t(i) * p + b]);
      const double cov = (n - 1.0) / den * Cold[size_t(a) * p + b] + 1.0 / den * acc;
      A[size_t(a) * p + b] = cov;
      s_C[size_t(a) * p + b] = cov;
    }
  // cyclic Jacobi eigenvectors (V columns)
  std::vector<double> V(size_t(p) * p, 0.0);
  for (int i = 0; i < p; ++i) V[size_t(i) * p + i] = 1.0;
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0.0, all = 0.0;
    for (int a = 0; a < p; ++a)
      for (int b = 0; b < p; ++b) {
        const double v = A[size_t(a) * p + b];
        all += v * v;
        if (a != b) off += v * v;
      }
    if (off <= 1e-30 * all || off == 0.0) break;
    for (int pp = 0; pp < p - 1; ++pp)
      for (int qq = pp + 1; qq < p; ++qq) {
        const double app = A[size_t(pp) * p + pp], aqq = A[size_t(qq) * p + qq], apq = A[size_t(pp) * p + qq];
        if (apq == 0.0 || std::fabs(apq) <= 1e-18 * (std::fabs(app) + std::fabs(aqq))) continue;
        const double th = (aqq - app) / (2.0 * apq);
        const double t = (th >= 0.0 ? 1.0 : -1.0) / (std::fabs(th) + std::sqrt(th * th + 1.0));
        const double c = 1.0 / std::sqrt(t * t + 1.0), sn = t * c;
        for (int r = 0; r < p; ++r) {
          const double ap = A[size_t(r) * p + pp], aq = A[size_t(r) * p + qq];
          A[size_t(r) * p + pp] = c * ap - sn * aq;
          A[size_t(r) * p + qq] = sn * ap + c * aq;
          const double vp = V[size_t(r) * p + pp], vq = V[size_t(r) * p + qq];
          V[size_t(r) * p + pp] = c * vp - sn * vq;
          V[size_t(r) * p + qq] = sn * vp + c * vq;
        }
        for (int col = 0; col < p; ++col) {
          const double ap = A[size_t(pp) * p + col], aq = A[size_t(qq) * p + col];
          A[size_t(pp) * p + col] = c * ap - sn * aq;
          A[size_t(qq) * p + col] = sn * ap + c * aq;
        }
      }
  }
  std::vector<int> sel;
  for (int a = 0; a < k; ++a) {
    int best = -1;
    for (int j = 0; j < p; ++j) {
      if (std::find(sel.begin(), sel.end(), j) != sel.end()) continue;
      if (best < 0 || A[size_t(j) * p + j] > A[size_t(best) * p + best]) best = j;
    }
    sel.push_back(best);
  }
  const size_t kk = size_t(k) * k;
  std::vector<double> P(kk, 0.0), DPC(size_t(nb) * k), XD(size_t(nb) * k);
  if (!c_zero)
    for (int a = 0; a < k; ++a)
      for (int b = 0; b < k; ++b) {
        double acc = 0.0;
        for (int r = 0; r < p; ++r) {
          double t = 0.0;
          for (int c = 0; c < p; ++c) t += Cold[size_t(r) * p + c] * V[size_t(c) * p + sel[b]];
          acc += V[size_t(r) * p + sel[a]] * t;
        }
        P[size_t(a) * k + b] = acc;
      }
  for (int i = 0; i < nb; ++i)
    for (int a = 0; a < k; ++a) {
      double px = 0.0, pxc = 0.0, pm = 0.0;
      for (int j = 0; j < p; ++j) {
        const double w = V[size_t(j) * p + sel[a]];
        px += X[size_t(i) * p + j] * w;
        pxc += XC[size_t(i) * p + j] * w;
        pm += MO[size_t(i) * p + j] * w;
      }
      DPC[size_t(i) * k + a] = pxc - pm;
      XD[size_t(i) * k + a] = px - pm;
    }
  auto emit = [&](int i, double score) {
    out[i] = prm.out_mode == 1 ? (score > prm.threshold ? 1.0 : 0.0) : score;
  };
  bool valid = false;
  std::vector<double> Cp(kk), T1(kk), T2(kk), inv;
  for (int i = 0; i < nb; ++i) {
    if (!valid) {
      if (std::fabs(invert_host(P, inv, k)) > prm.eps) {
        Cp = inv;
        valid = true;
      } else {
        if (n + i != 0.0) {
          const double a = (n + i - 1.0) / (n + i), cb = 1.0 / (n + i + 1.0);
          const double* dp = DPC.data() + size_t(i) * k;
          for (size_t e = 0; e < kk; ++e) P[e] = a * P[e] + cb * dp[e / k] * dp[e % k];
        }
        emit(i, 0.0);
        continue;
      }
    } else {
      const double a = (n + i - 1.0) / (n + i - 2.0), cb = 1.0 / (n + i);
      const double* dp = DPC.data() + size_t(i - 1) * k;
      for (size_t e = 0; e < kk; ++e) T1[e] = a * Cp[e];
      double tr = 0.0;
      for (int r = 0; r < k; ++r)
        for (int c = 0; c < k; ++c) {
          double s = 0.0;
          for (int j = 0; j < k; ++j) s += (cb * dp[r] * dp[j]) * T1[size_t(j) * k + c];
          T2[size_t(r) * k + c] = s;
          if (r == c) tr += s;
        }
      const double scal = 1.0 / (1.0 + tr);
      for (int r = 0; r < k; ++r)
        for (int c = 0; c < k; ++c) {
          double s = 0.0;
          for (int j = 0; j < k; ++j) s += T1[size_t(r) * k + j] * T2[size_t(j) * k + c];
          Cp[size_t(r) * k + c] = T1[size_t(r) * k + c] - scal * s;
        }
    }
    const double* d = XD.data() + size_t(i) * k;
    double part = 0.0;
    for (size_t e = 0; e < kk; ++e) part += d[e / k] * Cp[e] * d[e % k];
    emit(i, part);
  }
  const double n_new = n_state + nb;
  if (n_new > prm.start_clip)
    for (int j = 0; j < p; ++j) {
      const double sd = std::sqrt(s_C[size_t(j) * p + j]);
      s_lo[j] = s_mean[j] - prm.n_stdev * sd;
      s_hi[j] = s_mean[j] + prm.n_stdev * sd;
    }
  s_tail[0] = n_new;
  s_tail[1] = 0.0;
  if (n_new > prm.start_clip) s_tail[2] = 1.0;
}

}  // namespace

// ------------------------------------------------------------ MahalanobisModel
MahalanobisModel::MahalanobisModel(int p, int k, double n_stdev, double start_clip, double max_n, double eps,
                                   int out_mode, double threshold)
    : st_(std::make_shared<MahaState>()) {
  st_->prm = make_params(p, k, n_stdev, start_clip, max_n, eps);
  view_ = st_->prm;
  view_.out_mode = out_mode;
  view_.threshold = threshold;
  set_flat_output(out_mode == 1);  // predict() returns a 1-D prediction array
  init_state(-1);
}

MahalanobisModel::MahalanobisModel(std::shared_ptr<MahaState> st, int out_mode, double threshold)
    : st_(std::move(st)) {
  view_ = st_->prm;
  view_.out_mode = out_mode;
  view_.threshold = threshold;
  set_flat_output(out_mode == 1);
}

void MahalanobisModel::init_state(int device) {
  std::vector<double> init(kern::maha_state_doubles(st_->prm.p), 0.0);
  init[init.size() - 2] = 1.0;  // c_zero: the reference starts from C = 0 (int)
  st_->h_state = init;
  st_->device = device;
}

void MahalanobisModel::to_device(int device) {
  std::lock_guard<std::recursive_mutex> g(st_->mu);
  if (st_->device == device) return;
  if (st_->device >= 0) throw std::runtime_error("Mahalanobis state already lives on GPU " + std::to_string(st_->device));
  DeviceGuard dg(device);
  st_->d_state.alloc(st_->h_state.size() * sizeof(double), device);
  st_->d_state.upload(st_->h_state.data(), st_->h_state.size() * sizeof(double));
  st_->d_eig.alloc(kern::kMahaEigDoubles * sizeof(double), device);  // zeroed: cold start
  st_->chain.create(device);
  st_->device = device;
}

size_t MahalanobisModel::workspace_bytes(int max_rows, int) const {
  return kern::maha_ws_doubles(std::max(1, max_rows), st_->prm.p, st_->prm.k) * sizeof(double);
}

void MahalanobisModel::launch(const double* X, int rows, int cols, double* out, void* ws, hipStream_t s) {
  // a whole batch as one request (direct callers); the batcher uses launch_segments
  launch_segments(X, rows, cols, out, ws, nullptr, 0, s);
}

void MahalanobisModel::launch_segments(const double* X, int rows, int cols, double* out, void* ws,
                                       const int32_t* seg, int nseg, hipStream_t s) {
  if (cols != st_->prm.p) throw std::runtime_error("Mahalanobis: expected " + std::to_string(st_->prm.p) + " features");
  std::lock_guard<std::recursive_mutex> g(st_->mu);
  seq_base_ = st_->seq;
  st_->seq += rows;
  // after the previous step on whatever stream it ran
  if (st_->chained) SCA_HIP_CHECK(hipStreamWaitEvent(s, st_->chain.get(), 0));
  double* eig = st_->d_eig.as<double>();
  if (seg)
    kern::maha_step_segments(X, seg, nseg, view_, st_->d_state.as<double>(), eig, static_cast<double*>(ws), out, s);
  else
    kern::maha_step(X, rows, view_, st_->d_state.as<double>(), eig, static_cast<double*>(ws), out, s);
  SCA_HIP_CHECK(hipGetLastError());
  SCA_HIP_CHECK(hipEventRecord(st_->chain.get(), s));
  st_->chained = true;
}

void MahalanobisModel::run_cpu(const double* X, int rows, int cols, double* out) const {
  if (cols != st_->prm.p) throw std::runtime_error("Mahalanobis: expected " + std::to_string(st_->prm.p) + " features");
  std::lock_guard<std::recursive_mutex> g(st_->mu);
  if (st_->device >= 0) throw std::runtime_error("Mahalanobis: state lives on the GPU (no CPU step)");
  seq_base_ = st_->seq;
  st_->seq += rows;
  maha_step_host(X, rows, view_, st_->h_state.data(), out);
}

std::vector<double> MahalanobisModel::state() const {
  std::lock_guard<std::recursive_mutex> g(st_->mu);
  if (st_->device < 0) return st_->h_state;
  DeviceGuard dg(st_->device);
  if (st_->chained) SCA_HIP_CHECK(hipEventSynchronize(st_->chain.get()));
  std::vector<double> s(kern::maha_state_doubles(st_->prm.p));
  SCA_HIP_CHECK(hipMemcpy(s.data(), st_->d_state.get(), s.size() * sizeof(double), hipMemcpyDeviceToHost));
  return s;
}

std::vector<double> MahalanobisModel::solver_stats() const {
  std::lock_guard<std::recursive_mutex> g(st_->mu);
  if (st_->device < 0) return {};
  DeviceGuard dg(st_->device);
  if (st_->chained) SCA_HIP_CHECK(hipEventSynchronize(st_->chain.get()));
  std::vector<double> t(17);
  SCA_HIP_CHECK(hipMemcpy(t.data(), st_->d_eig.as<double>() + kern::kMahaEigTail + 2, 13 * sizeof(double),
                          hipMemcpyDeviceToHost));
  SCA_HIP_CHECK(hipMemcpy(t.data() + 13, st_->d_eig.as<double>() + kern::kMahaEigMeta + 1, 4 * sizeof(double),
                          hipMemcpyDeviceToHost));
  return t;
}

void MahalanobisModel::set_state(const std::vector<double>& s) {
  std::lock_guard<std::recursive_mutex> g(st_->mu);
  if (s.size() != kern::maha_state_doubles(st_->prm.p)) throw std::runtime_error("Mahalanobis: bad state size");
  if (st_->device < 0) {
    st_->h_state = s;
    return;
  }
  DeviceGuard dg(st_->device);
  if (st_->chained) SCA_HIP_CHECK(hipEventSynchronize(st_->chain.get()));
  st_->d_state.upload(s.data(), s.size() * sizeof(double));
  // the cached eigendecomposition describes the old covariance: the next
  // step re-solves (a NaN never equals the state's n)
  const double nan = std::nan("");
  SCA_HIP_CHECK(hipMemcpy(st_->d_eig.as<double>() + kern::kMahaEigMeta, &nan, sizeof nan, hipMemcpyHostToDevice));
}

// ----------------------------------------------------------- MahalanobisDevice
MahalanobisDevice::MahalanobisDevice(int p, int k, double n_stdev, double start_clip, double max_n, double eps,
                                     int device)
    : model_(std::make_shared<MahalanobisModel>(p, k, n_stdev, start_clip, max_n, eps, 0, 0.0)) {
  BatcherOptions o;
  o.device = device;
  o.max_batch = 4096;
  o.slots = 2;
  unit_ = std::make_unique<BatchedUnit>(model_, o);
}

MahalanobisDevice::~MahalanobisDevice() {
  if (unit_) unit_->stop();
}

std::vector<double> MahalanobisDevice::step(const double* X, int nb, int64_t* seq) {
  if (nb <= 0) return {};
  return unit_->run_ptr(X, nb, model_->p(), seq);
}

std::shared_ptr<MahalanobisModel> MahalanobisDevice::predict_view(double threshold) const {
  return std::make_shared<MahalanobisModel>(model_->shared_state(), 1, threshold);
}

}  // namespace sca::gpu
