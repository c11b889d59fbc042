// Mahalanobis outlier score recurrence (reference
// components/outlier-detection/mahalanobis/CoreMahalanobis.py:118-146).
//
// Per request batch of nb rows in the k-dim principal subspace: the inverse
// covariance is carried row to row by Sherman-Morrison rank-1 updates
//   C_i = a C_{i-1} - (a C_{i-1} B_{i-1} a C_{i-1}) / (1 + tr(B_{i-1} a C_{i-1})),
//   a = (n+i-1)/(n+i-2),  score_i = d_i^T C_i d_i
// (until the projected covariance first becomes invertible it is accumulated
// instead and the score is 0).  The recurrence is sequential in i and k is
// small (n_components, <= 16), so one wave owns the whole batch: the k x k
// state lives in LDS, each lane owns <= 4 matrix elements, and the row loop
// costs a few LDS round trips instead of the reference's ~5 numpy calls per
// row.  fp64 throughout (parity with the numpy reference to rounding).
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace sca::kern {
namespace {

constexpr int kMaxK = 16;

// Gauss-Jordan with partial pivoting on a k x k copy; returns det.
__device__ double invert(const double* A, double* inv, int k) {
  double M[kMaxK * kMaxK];
  for (int e = 0; e < k * k; ++e) {
    M[e] = A[e];
    inv[e] = (e / k == e % k) ? 1.0 : 0.0;
  }
  double det = 1.0;
  for (int c = 0; c < k; ++c) {
    int piv = c;
    for (int r = c + 1; r < k; ++r)
      if (fabs(M[r * k + c]) > fabs(M[piv * k + c])) piv = r;
    if (M[piv * k + c] == 0.0) return 0.0;
    if (piv != c) {
      for (int j = 0; j < k; ++j) {
        double t = M[c * k + j]; M[c * k + j] = M[piv * k + j]; M[piv * k + j] = t;
        t = inv[c * k + j]; inv[c * k + j] = inv[piv * k + j]; inv[piv * k + j] = t;
      }
      det = -det;
    }
    const double d = M[c * k + c];
    det *= d;
    const double id = 1.0 / d;
    for (int j = 0; j < k; ++j) { M[c * k + j] *= id; inv[c * k + j] *= id; }
    for (int r = 0; r < k; ++r) {
      if (r == c) continue;
      const double f = M[r * k + c];
      if (f == 0.0) continue;
      for (int j = 0; j < k; ++j) { M[r * k + j] -= f * M[c * k + j]; inv[r * k + j] -= f * inv[c * k + j]; }
    }
  }
  return det;
}

__global__ __launch_bounds__(64) void maha_sm_kernel(const double* __restrict__ B, const double* __restrict__ cov0,
                                                     const double* __restrict__ xd, int nb, int k, double n,
                                                     double eps, double* __restrict__ out) {
  __shared__ double P[kMaxK * kMaxK], Cp[kMaxK * kMaxK], T1[kMaxK * kMaxK], T2[kMaxK * kMaxK];
  __shared__ int valid, inverted;
  __shared__ double scal;
  const int lane = threadIdx.x;
  const int kk = k * k;
  for (int e = lane; e < kk; e += 64) P[e] = cov0[e];
  if (lane == 0) valid = 0;
  __syncthreads();
  for (int i = 0; i < nb; ++i) {
    const double* d = xd + size_t(i) * k;
    if (!valid) {
      if (lane == 0) {
        inverted = 0;
        double inv[kMaxK * kMaxK];
        const double det = invert(P, inv, k);
        if (fabs(det) > eps) {
          for (int e = 0; e < kk; ++e) Cp[e] = inv[e];
          inverted = 1;
          valid = 1;
        }
      }
      __syncthreads();
      if (!inverted) {
        if (n + i != 0.0) {
          const double a = (n + i - 1.0) / (n + i);
          const double* b = B + size_t(i) * kk;
          for (int e = lane; e < kk; e += 64) P[e] = a * P[e] + b[e];
        }
        if (lane == 0) out[i] = 0.0;
        __syncthreads();
        continue;
      }
    } else {
      const double a = (n + i - 1.0) / (n + i - 2.0);
      const double* bp = B + size_t(i - 1) * kk;
      for (int e = lane; e < kk; e += 64) T1[e] = a * Cp[e];  // c_inv
      __syncthreads();
      for (int e = lane; e < kk; e += 64) {  // BC1 = B_{i-1} c_inv
        const int r = e / k, c = e - r * k;
        double s = 0.0;
        for (int j = 0; j < k; ++j) s += bp[r * k + j] * T1[j * k + c];
        T2[e] = s;
      }
      __syncthreads();
      if (lane == 0) {
        double tr = 0.0;
        for (int j = 0; j < k; ++j) tr += T2[j * k + j];
        scal = 1.0 / (1.0 + tr);
      }
      __syncthreads();
      for (int e = lane; e < kk; e += 64) {  // C_i = c_inv - scal * c_inv BC1
        const int r = e / k, c = e - r * k;
        double s = 0.0;
        for (int j = 0; j < k; ++j) s += T1[r * k + j] * T2[j * k + c];
        Cp[e] = T1[e] - scal * s;
      }
      __syncthreads();
    }
    // score_i = d^T C_i d
    double part = 0.0;
    for (int e = lane; e < kk; e += 64) {
      const int r = e / k, c = e - r * k;
      part += d[r] * Cp[e] * d[c];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
    if (lane == 0) out[i] = part;
    __syncthreads();
  }
}

}  // namespace

bool mahalanobis_sm_scores(const double* B, const double* cov0, const double* xd, int nb, int k, double n,
                           double* out, hipStream_t s) {
  if (k < 1 || k > kMaxK) return false;
  if (nb <= 0) return true;
  hipLaunchKernelGGL(maha_sm_kernel, dim3(1), dim3(64), 0, s, B, cov0, xd, nb, k, n, 1e-8, out);
  return true;
}

}  // namespace sca::kern
