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


// ------------------------------------------------------------ full detector step
// One workgroup runs CoreMahalanobis._get_preds (:68-151) for one request
// batch against the device-resident state: NT = 64 threads (one wave: every
// barrier is nearly free) for p <= 16, 256 otherwise.  p <= 64 features,
// k <= 16 components; p x p matrices live in LDS (row stride kLd = 65).
//
// Eigenvectors: parallel cyclic Jacobi, warm-started from the previous step's
// eigenvectors (kept in `eig`, a hint outside the checkpointed state): V is
// re-orthonormalised by one Newton-Schulz step (V <- 1.5 V - 0.5 V V^T V), A =
// V^T C V is then nearly diagonal and converges in 1-3 sweeps instead of
// ~8-10 from the identity.  A round applies every pair's rotation to both
// sides at once (2 x 2 block B_ij <- J_i^T B_ij J_j), two barriers per round.
// Converged to the same 1e-15 relative off-diagonal norm as a cold start, so
// the scores do not depend on the hint (eigenvector signs / order cancel).
constexpr int kLd = kMahaMaxP + 1;
constexpr int kMaxSweeps = 40;

template <int NT> __device__ double block_sum(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if constexpr (NT == 64) {
    return v;
  } else {
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) t += red[w];
    return t;
  }
}

// C = op(A) . B for m x m LDS matrices (stride kLd), 4 x 4 register tiles;
// op = transpose when TA.  Rows / columns past m read whatever the 64 x 65
// buffers hold but only feed outputs that are not written.
template <int NT, bool TA>
__device__ void mm(const double* A, const double* B, double* C, int m) {
  const int tm = (m + 3) >> 2;
  for (int t = threadIdx.x; t < tm * tm; t += NT) {
    const int ti = t / tm;
    const int i0 = ti * 4, j0 = (t - ti * tm) * 4;
    double acc[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[r][c] = 0.0;
    for (int kx = 0; kx < m; ++kx) {
      double a[4], b[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) a[r] = TA ? A[kx * kLd + i0 + r] : A[(i0 + r) * kLd + kx];
#pragma unroll
      for (int c = 0; c < 4; ++c) b[c] = B[kx * kLd + j0 + c];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[r][c] += a[r] * b[c];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (i0 + r < m && j0 + c < m) C[(i0 + r) * kLd + j0 + c] = acc[r][c];
  }
}

// Gauss-Jordan with partial pivoting; M and inv are caller-provided (LDS)
// k x k buffers, so nothing spills to scratch.  Returns det(A).
__device__ double invert_into(const double* A, double* M, double* inv, int k) {
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

// 64-bit DPP move (both halves) and a whole-wave sum: quad_perm / row
// mirrors inside each 16-lane row (VALU, no LDS crossbar), then the four row
// sums through v_readlane -- every lane gets the total.
template <int CTRL> __device__ __forceinline__ double dpp64(double v) {
  const int2 h = __builtin_bit_cast(int2, v);
  int2 o;
  o.x = __builtin_amdgcn_update_dpp(0, h.x, CTRL, 0xF, 0xF, false);
  o.y = __builtin_amdgcn_update_dpp(0, h.y, CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, o);
}
__device__ __forceinline__ double readlane64(double v, int l) {
  const int2 h = __builtin_bit_cast(int2, v);
  int2 o;
  o.x = __builtin_amdgcn_readlane(h.x, l);
  o.y = __builtin_amdgcn_readlane(h.y, l);
  return __builtin_bit_cast(double, o);
}
__device__ __forceinline__ double wave_sum(double v) {  // requires all 64 lanes active
  v += dpp64<0xB1>(v);   // lane ^ 1
  v += dpp64<0x4E>(v);   // lane ^ 2
  v += dpp64<0x141>(v);  // row_half_mirror: the other quad of the 8
  v += dpp64<0x140>(v);  // row_mirror: the other 8 of the 16
  return (readlane64(v, 0) + readlane64(v, 16)) + (readlane64(v, 32) + readlane64(v, 48));
}
__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

// Top-k eigenpairs of the symmetric p x p matrix in A (LDS, stride kLd;
// destroyed) for p > 16, the way LAPACK's syevr computes a subset (which is
// what the reference's scipy eigh(eigvals=(p-k, p-1)) runs):
//  1. Householder tridiagonalisation: per column one wave forms the
//     reflector v (kept in W row j) and w = 2 A22 v - 2 (v.A22 v) v, then all
//     threads apply A22 -= v w^T + w v^T (two barriers per column);
//  2. the k largest eigenvalues by 64-way multisection on Sturm counts, one
//     wave per eigenvalue (ballot picks the subinterval, no barriers);
//  3. their tridiagonal eigenvectors by inverse iteration (LU with partial
//     pivoting on one lane, 3 iterations), re-orthogonalised within clusters;
//  4. back-transformation through the reflectors, one wave per vector.
// Output: eigenvectors in V[:, 0..k-1], sel[a] = a.  Replaces ~3.5 warm
// Jacobi sweeps (63 two-barrier rounds each at p = 64, ~485 us) with ~2p
// barriers.
template <int NT>
__device__ void topk_tridiag(double* A, double* V, const double* W_, double* dg, double* eo, double* e2, double* wv,
                             double* lam, int* sel, int p, int k, uint64_t* sub) {
  double* W = const_cast<double*>(W_);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint64_t t_prev = __builtin_amdgcn_s_memrealtime();
  auto mark = [&](int i) {  // sub-phase timer (thread 0)
    if (tid == 0) {
      const uint64_t t = __builtin_amdgcn_s_memrealtime();
      sub[i] += t - t_prev;
      t_prev = t;
    }
  };
  constexpr int NW = NT / 64;
  // ---- 1. tridiagonalisation
  for (int j = 0; j + 2 < p; ++j) {
    const int m = p - j - 1;
    if (wave == 0) {
      const double x = lane < m ? A[(j + 1 + lane) * kLd + j] : 0.0;
      const double s2 = wave_sum(x * x);
      const double x0 = __shfl(x, 0, 64);
      double alpha = 0.0, v = 0.0;
      if (s2 > 0.0) {
        alpha = x0 >= 0.0 ? -sqrt(s2) : sqrt(s2);
        v = lane == 0 ? x - alpha : x;
        const double vn2 = s2 - x0 * x0 + (x0 - alpha) * (x0 - alpha);  // > 0: x0 and alpha have opposite signs
        v *= 1.0 / sqrt(vn2);
      }
      if (lane < m) W[j * kLd + lane] = v;
      if (lane == 0) eo[j] = alpha;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // W row j visible to the wave's other lanes
      double pv = 0.0;
      if (lane < m) {  // 4 independent chains, 16 loads in flight per unrolled block
        const double* __restrict__ arow = A + (j + 1 + lane) * kLd + (j + 1);
        const double* __restrict__ vr = W + j * kLd;
        double s0 = 0.0, s1 = 0.0, s2v = 0.0, s3 = 0.0;
        int c = 0;
        for (; c + 8 <= m; c += 8) {
          s0 += arow[c] * vr[c] + arow[c + 4] * vr[c + 4];
          s1 += arow[c + 1] * vr[c + 1] + arow[c + 5] * vr[c + 5];
          s2v += arow[c + 2] * vr[c + 2] + arow[c + 6] * vr[c + 6];
          s3 += arow[c + 3] * vr[c + 3] + arow[c + 7] * vr[c + 7];
        }
        for (; c < m; ++c) s0 += arow[c] * vr[c];
        pv = (s0 + s1) + (s2v + s3);
      }
      const double K = wave_sum(lane < m ? v * pv : 0.0);
      if (lane < m) wv[lane] = 2.0 * pv - 2.0 * K * v;
    }
    __syncthreads();
    if (lane < m) {  // A22 -= v w^T + w v^T: lane = column, wave w = rows w, w + NW, ...
      const double* __restrict__ vr = W + j * kLd;
      const double* __restrict__ wr = wv;
      const double vc = vr[lane], wc = wr[lane];
      double* __restrict__ acol = A + (j + 1) * kLd + (j + 1) + lane;
#pragma unroll 4
      for (int r = wave; r < m; r += NW) acol[r * kLd] -= vr[r] * wc + wr[r] * vc;
    }
    __syncthreads();
  }
  for (int i = tid; i < p; i += NT) dg[i] = A[i * kLd + i];
  if (tid == 0 && p >= 2) eo[p - 2] = A[(p - 1) * kLd + (p - 2)];
  __syncthreads();
  for (int i = tid; i + 1 < p; i += NT) e2[i] = eo[i] * eo[i];
  __syncthreads();
  mark(0);
  // ---- 2. k largest eigenvalues: Gershgorin bracket, 64-way multisection per wave
  const double di = lane < p ? dg[lane] : 0.0;
  const double ei = lane + 1 < p ? fabs(eo[lane]) : 0.0, em = lane >= 1 && lane < p ? fabs(eo[lane - 1]) : 0.0;
  const double lo0 = wave_min(lane < p ? di - ei - em : 1e300), hi0 = wave_max(lane < p ? di + ei + em : -1e300);
  const double tnorm = fmax(fabs(lo0), fabs(hi0));
  const double pivmin = fmax(tnorm, 1e-300) * 2.3e-16;
  const double lo = lo0 - 1e-10 * tnorm - 1e-300, hi = hi0 + 1e-10 * tnorm + 1e-300;
  for (int a = wave; a < k; a += NW) {
    const int idx = p - 1 - a;  // ascending index of the a-th largest eigenvalue
    double l = lo, u = hi;
    for (int it = 0; it < 64; ++it) {
      const double x = l + (u - l) * (double(lane + 1) * (1.0 / 65.0));
      // Sturm count: eigenvalues < x.  Only signs are counted, so 1/q is a
      // v_rcp_f64 estimate refined by one Newton step instead of an IEEE
      // division (a ~10-instruction dependent chain per element)
      double qv = dg[0] - x;
      int cnt = qv < 0.0;
#pragma unroll 4
      for (int i = 1; i < p; ++i) {
        if (fabs(qv) < pivmin) qv = -pivmin;
        double r = __builtin_amdgcn_rcp(qv);
        r = r * (2.0 - qv * r);
        qv = (dg[i] - x) - e2[i - 1] * r;
        cnt += qv < 0.0;
      }
      const unsigned long long mask = __ballot(cnt > idx);
      double nl, nu;
      if (mask) {
        const int f = __ffsll(static_cast<long long>(mask)) - 1;
        nu = __shfl(x, f, 64);
        nl = f > 0 ? __shfl(x, f - 1, 64) : l;
      } else {
        nl = __shfl(x, 63, 64);
        nu = u;
      }
      l = nl;
      u = nu;
      if (u - l <= 2.3e-16 * fmax(fabs(l), fabs(u)) + 1e-18 * tnorm + 1e-300) break;
    }
    if (lane == 0) lam[a] = 0.5 * (l + u);
  }
  __syncthreads();
  mark(1);
  // ---- 3. inverse iteration on T - lam I: wave 0, lane a for eigenvalue a;
  // LU factors in LDS (scratch in A, now free), the iterate y in registers
  // (fully unrolled over kMahaMaxP rows), reciprocal pivots (no division in
  // the solves); 2 iterations from a fixed start vector
  if (wave == 0 && lane < k) {
    const int a = lane;
    double* u0 = A + a * 4 * kMahaMaxP;  // holds 1 / pivot; 16 x 4 x 64 <= 64 x kLd doubles
    double* u1 = u0 + kMahaMaxP;
    double* u2 = u1 + kMahaMaxP;
    double* lm = u2 + kMahaMaxP;
    unsigned long long swm = 0;  // row i + 1 was the pivot of step i
    const double L = lam[a];
    double cd = dg[0] - L, cu1 = p > 1 ? eo[0] : 0.0;
    for (int i = 0; i + 1 < p; ++i) {
      const double b = eo[i], an = dg[i + 1] - L, bn = i + 2 < p ? eo[i + 1] : 0.0;
      if (fabs(b) > fabs(cd)) {  // pivot on row i + 1
        u0[i] = 1.0 / b;
        u1[i] = an;
        u2[i] = bn;
        const double mult = cd / b;
        lm[i] = mult;
        swm |= 1ull << i;
        cd = cu1 - mult * an;
        cu1 = -mult * bn;
      } else {
        if (fabs(cd) < pivmin) cd = pivmin;
        u0[i] = 1.0 / cd;
        u1[i] = cu1;
        u2[i] = 0.0;
        const double mult = b / cd;
        lm[i] = mult;
        cd = an - mult * cu1;
        cu1 = bn;
      }
    }
    if (fabs(cd) < pivmin) cd = pivmin;
    u0[p - 1] = 1.0 / cd;
    double y[kMahaMaxP];
#pragma unroll
    for (int i = 0; i < kMahaMaxP; ++i) y[i] = 1.0 + 0.1 * sin(1.7 * double(i + 1) + double(a));
    for (int itr = 0; itr < 2; ++itr) {
#pragma unroll
      for (int i = 0; i + 1 < kMahaMaxP; ++i) {
        if (i + 1 < p) {
          if ((swm >> i) & 1ull) {
            const double t0 = y[i];
            y[i] = y[i + 1];
            y[i + 1] = t0;
          }
          y[i + 1] -= lm[i] * y[i];
        }
      }
      double nrm = 0.0;
#pragma unroll
      for (int i = kMahaMaxP - 1; i >= 0; --i) {
        if (i < p) {
          double t0 = y[i];
          if (i + 1 < p) t0 -= u1[i] * y[i + 1];
          if (i + 2 < p) t0 -= u2[i] * y[i + 2];
          t0 *= u0[i];
          y[i] = t0;
          nrm = fmax(nrm, fabs(t0));
        }
      }
      const double sc = nrm > 0.0 ? 1.0 / nrm : 1.0;
#pragma unroll
      for (int i = 0; i < kMahaMaxP; ++i) y[i] *= sc;
    }
#pragma unroll
    for (int i = 0; i < kMahaMaxP; ++i)
      if (i < p) V[i * kLd + a] = y[i];
  }
  __syncthreads();
  if (wave == 0) {  // normalise; re-orthogonalise within clusters (|lam_a - lam_b| < 1e-3 ||T||, as dstein)
    for (int a = 0; a < k; ++a) {
      double y = lane < p ? V[lane * kLd + a] : 0.0;
      for (int b = 0; b < a; ++b) {
        if (fabs(lam[a] - lam[b]) < 1e-3 * tnorm) {
          const double yb = lane < p ? V[lane * kLd + b] : 0.0;
          y -= wave_sum(y * yb) * yb;
        }
      }
      y *= 1.0 / sqrt(fmax(wave_sum(y * y), 1e-300));
      if (lane < p) V[lane * kLd + a] = y;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    if (lane < k) sel[lane] = lane;
  }
  __syncthreads();
  // ---- 4. back-transformation x = H_0 ... H_{p-3} y, one wave per vector
  for (int a = wave; a < k; a += NW) {
    double x = lane < p ? V[lane * kLd + a] : 0.0;
    for (int j = p - 3; j >= 0; --j) {
      const double vt = lane > j && lane < p ? W[j * kLd + (lane - j - 1)] : 0.0;
      x -= 2.0 * wave_sum(vt * x) * vt;
    }
    if (lane < p) V[lane * kLd + a] = x;
  }
  __syncthreads();
  mark(2);
}

// One request's step (CoreMahalanobis._get_preds for X [nb][p]) against the
// state in HBM; called once per segment by maha_step_kernel.  Callers
// __syncthreads() between calls: the next segment reads the state this one
// wrote (same workgroup, same CU: its L1 is coherent at workgroup scope).
template <int NT>
__device__ void maha_one(const double* __restrict__ X, int nb, const MahaParams& prm, double* __restrict__ state,
                         double* __restrict__ eig, double* __restrict__ ws, double* __restrict__ scores) {
  __shared__ double A[kMahaMaxP * kLd], V[kMahaMaxP * kLd], W[kMahaMaxP * kLd], Tm[kMahaMaxP * kLd];
  __shared__ double mean0[kMahaMaxP];
  __shared__ double rc[kMahaMaxP / 2], rs[kMahaMaxP / 2];
  __shared__ int rp[kMahaMaxP / 2], rq[kMahaMaxP / 2];
  __shared__ double red[NT / 64];
  __shared__ int sel[kMahaMaxK];
  __shared__ double P[kMahaMaxK * kMahaMaxK], Cp[kMahaMaxK * kMahaMaxK], T1[kMahaMaxK * kMahaMaxK],
      T2[kMahaMaxK * kMahaMaxK];
  __shared__ int valid, inverted;
  __shared__ double scal;
  __shared__ double tdg[kMahaMaxP], teo[kMahaMaxP], te2[kMahaMaxP], twv[kMahaMaxP], tlam[kMahaMaxK];
  const int tid = threadIdx.x;
  const int p = prm.p, k = prm.k, kk = k * k;
  double* s_mean = state;
  double* s_C = state + p;
  double* s_lo = s_C + p * p;
  double* s_hi = s_lo + p;
  double* s_tail = s_hi + p;  // n, c_zero, has_clip
  const double n_state = s_tail[0];
  const bool c_zero = s_tail[1] != 0.0;
  const bool do_clip = n_state > prm.start_clip && s_tail[2] != 0.0;
  const double n = prm.max_n > 0 ? fmin(n_state, prm.max_n) : n_state;
  double* XC = ws;                          // [nb][p] clipped rows
  double* MO = XC + size_t(nb) * p;         // [nb][p] means_offset
  double* D = MO + size_t(nb) * p;          // [nb][p] Xc - means_offset
  double* XR = D + size_t(nb) * p;          // [nb][p] raw rows (X may be host memory: read it once)
  double* DPC = XR + size_t(nb) * p;        // [nb][k] projected (Xc - m)
  double* XD = DPC + size_t(nb) * k;        // [nb][k] projected (X - m)

  uint64_t t_prev = __builtin_amdgcn_s_memrealtime(), ph[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  auto stamp = [&](int i) {  // phase timer (100 MHz), thread 0; accumulated into eig's tail
    if (tid == 0) {
      const uint64_t t = __builtin_amdgcn_s_memrealtime();
      ph[i] += t - t_prev;
      t_prev = t;
    }
  };
  for (int j = tid; j < p; j += NT) mean0[j] = s_mean[j];
  __syncthreads();

  // ---- clip + running means (sequential in rows, parallel in features)
  for (int j = tid; j < p; j += NT) {
    const double m0 = mean0[j];
    double cum = 0.0, prev = m0;
    const double lo = do_clip ? s_lo[j] : 0.0, hi = do_clip ? s_hi[j] : 0.0;
    for (int i = 0; i < nb; ++i) {
      double x = X[size_t(i) * p + j];
      XR[size_t(i) * p + j] = x;
      if (do_clip) x = fmin(fmax(x, lo), hi);
      cum += x;
      const double roll = cum / double(i + 1);
      const double nm = m0 + (double(i + 1) / (double(i) + n + 1.0)) * (roll - m0);
      XC[size_t(i) * p + j] = x;
      MO[size_t(i) * p + j] = prev;
      D[size_t(i) * p + j] = x - prev;
      prev = nm;
    }
    s_mean[j] = prev;  // new_means[-1] (mean0 keeps the old value for this step)
  }
  __syncthreads();
  stamp(0);

  // ---- covariance update: cov = (n-1)/(n+max(1,nb-1)) C + 1/(n+max(1,nb-1)) sum_i coef_i d_i d_i^T
  // (the old C is read from the state in HBM; the new one is written back
  // after the projections, which still need the old one)
  const double den = n + fmax(1.0, double(nb) - 1.0);
  const int m = p + (p & 1);
  for (int e = tid; e < m * m; e += NT) {
    const int a = e / m, b = e - a * m;
    double cov = 0.0;
    if (a < p && b < p) {  // dummy index of an odd p stays 0
      double acc = 0.0;
      for (int i = 0; i < nb; ++i)
        acc += ((n + i) / (n + i + 1.0)) * (D[size_t(i) * p + a] * D[size_t(i) * p + b]);
      cov = (n - 1.0) / den * (c_zero ? 0.0 : s_C[a * p + b]) + 1.0 / den * acc;
    }
    A[a * kLd + b] = cov;
    Tm[a * kLd + b] = cov;  // kept: written to the state after the projections
  }
  if constexpr (NT == 256) {  // p > 16: top-k via tridiagonalisation (topk_tridiag)
    __syncthreads();
    stamp(1);
    stamp(2);
    topk_tridiag<NT>(A, V, W, tdg, teo, te2, twv, tlam, sel, p, k, ph + 7);
    stamp(3);
    if (tid == 0) eig[kMahaMaxP * kMahaMaxP + 3] += 1.0;
  } else {
  // ---- eigenvectors: warm-started parallel cyclic Jacobi (m = p rounded up to even)
  const bool warm = eig[kMahaMaxP * kMahaMaxP] != 0.0 && int(eig[kMahaMaxP * kMahaMaxP + 1]) == m;
  for (int e = tid; e < m * m; e += NT) {
    const int a = e / m, b = e - a * m;
    V[a * kLd + b] = warm ? eig[e] : (a == b ? 1.0 : 0.0);
  }
  __syncthreads();
  stamp(1);
  if (warm) {
    // Newton-Schulz re-orthonormalisation every 16 steps: the rotations lose
    // ~1e-16 of orthogonality per sweep, the step squares the error away
    if ((int(eig[kMahaMaxP * kMahaMaxP + 3]) & 15) == 0) {
      mm<NT, true>(V, V, W, m);  // G = V^T V
      __syncthreads();
      mm<NT, false>(V, W, A, m);  // V G (A is rebuilt below from Tm)
      __syncthreads();
      for (int e = tid; e < m * m; e += NT) {
        const int a = e / m, b = e - a * m;
        V[a * kLd + b] = 1.5 * V[a * kLd + b] - 0.5 * A[a * kLd + b];
      }
      __syncthreads();
    }
    mm<NT, false>(Tm, V, W, m);  // C V
    __syncthreads();
    mm<NT, true>(V, W, A, m);    // V^T C V
    __syncthreads();
  }
  stamp(2);
  const int half = m / 2;
  // striping: thread -> (pair my_i, first column pair / row my_j0, stride jstep)
  const int jstep = NT / max(half, 1);
  const int my_i = tid % max(half, 1), my_j0 = tid / max(half, 1);
  int sweeps = 0;
  for (int sweep = 0; sweep < kMaxSweeps && m > 1; ++sweep, ++sweeps) {
    double off = 0.0, all = 0.0;
    for (int e = tid; e < m * m; e += NT) {
      const int a = e / m, b = e - a * m;
      const double v = A[a * kLd + b];
      all += v * v;
      if (a != b) off += v * v;
    }
    off = block_sum<NT>(off, red);
    all = block_sum<NT>(all, red);
    if (off <= 1e-30 * all || off == 0.0) break;
    // round-robin pairs: lane i < half keeps its two positions mod (m - 1)
    // (no integer division in the round loop); block / V work is striped so
    // a thread's pair rows are fixed for the whole sweep
    int ua = tid == 0 ? -1 : tid % (m - 1), ub = tid == 0 ? 0 : (m - 1 - tid) % (m - 1);
    for (int r = 0; r < m - 1; ++r) {
      if (tid < half) {
        const int a = tid == 0 ? 0 : 1 + ua, b = 1 + ub;
        const int pp = min(a, b), qq = max(a, b);
        const double app = A[pp * kLd + pp], aqq = A[qq * kLd + qq], apq = A[pp * kLd + qq];
        double c = 1.0, sn = 0.0;
        if (apq != 0.0 && fabs(apq) > 1e-18 * (fabs(app) + fabs(aqq))) {
          const double th = (aqq - app) / (2.0 * apq);
          const double t = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
          c = 1.0 / sqrt(t * t + 1.0);
          sn = t * c;
        }
        rc[tid] = c;
        rs[tid] = sn;
        rp[tid] = pp;
        rq[tid] = qq;
        if (tid != 0 && ++ua == m - 1) ua = 0;
        if (++ub == m - 1) ub = 0;
      }
      __syncthreads();
      // A <- J^T A J as 2 x 2 blocks (pair rows bi x pair columns bj); V <- V J
      if (my_i < half) {
        const int pi = rp[my_i], qi = rq[my_i];
        const double ci = rc[my_i], si = rs[my_i];
        for (int bj = my_j0; bj < half; bj += jstep) {
          const int pj = rp[bj], qj = rq[bj];
          const double cj = rc[bj], sj = rs[bj];
          const double x00 = A[pi * kLd + pj], x01 = A[pi * kLd + qj], x10 = A[qi * kLd + pj], x11 = A[qi * kLd + qj];
          const double y00 = cj * x00 - sj * x01, y01 = sj * x00 + cj * x01;
          const double y10 = cj * x10 - sj * x11, y11 = sj * x10 + cj * x11;
          A[pi * kLd + pj] = ci * y00 - si * y10;
          A[pi * kLd + qj] = ci * y01 - si * y11;
          A[qi * kLd + pj] = si * y00 + ci * y10;
          A[qi * kLd + qj] = si * y01 + ci * y11;
        }
        for (int row = my_j0; row < m; row += jstep) {
          const double vp = V[row * kLd + pi], vq = V[row * kLd + qi];
          V[row * kLd + pi] = ci * vp - si * vq;
          V[row * kLd + qi] = si * vp + ci * vq;
        }
      }
      __syncthreads();
    }
  }
  stamp(3);
  // the eigenvectors seed the next step
  for (int e = tid; e < m * m; e += NT) {
    const int a = e / m, b = e - a * m;
    eig[e] = V[a * kLd + b];
  }
  if (tid == 0) {
    double* tail = eig + kMahaMaxP * kMahaMaxP;
    tail[0] = 1.0;
    tail[1] = double(m);
    tail[2] = double(sweeps);
    tail[3] += 1.0;
    tail[4] += double(sweeps);
  }
  // ---- top-k eigenpairs (any order: the scores are invariant to it)
  if (tid == 0) {
    for (int a = 0; a < k; ++a) {
      int best = -1;
      for (int j = 0; j < p; ++j) {
        bool taken = false;
        for (int b = 0; b < a; ++b) taken |= sel[b] == j;
        if (!taken && (best < 0 || A[j * kLd + j] > A[best * kLd + best])) best = j;
      }
      sel[a] = best;
    }
  }
  }  // Jacobi (p <= 16)
  // ---- projections; proj_cov = V^T C_old V over the selected columns:
  // C_old (still in HBM) -> W, U = C_old V_sel -> A (free after the
  // selection), P = V_sel^T U
  for (int e = tid; e < p * p; e += NT) W[(e / p) * kLd + e % p] = c_zero ? 0.0 : s_C[e];
  __syncthreads();
  for (int e = tid; e < p * k; e += NT) {
    const int r = e / k, b = e - r * k;
    const double* vb = V + sel[b];
    double t = 0.0;
    for (int c = 0; c < p; ++c) t += W[r * kLd + c] * vb[c * kLd];
    A[r * kLd + b] = t;
  }
  // row projections: one wave per (row, component), lanes over the features
  // (coalesced, independent loads; a 6-step shuffle sum instead of a
  // p-long dependent chain in one thread)
  {
    const int lane = tid & 63, wave = tid >> 6;
    for (int e = wave; e < nb * k; e += NT / 64) {
      const int i = e / k, a = e - i * k;
      double px = 0.0, pxc = 0.0, pm = 0.0;
      if (lane < p) {
        const double w = V[lane * kLd + sel[a]];
        px = XR[size_t(i) * p + lane] * w;
        pxc = XC[size_t(i) * p + lane] * w;
        pm = MO[size_t(i) * p + lane] * w;
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        px += __shfl_xor(px, o, 64);
        pxc += __shfl_xor(pxc, o, 64);
        pm += __shfl_xor(pm, o, 64);
      }
      if (lane == 0) {
        DPC[e] = pxc - pm;
        XD[e] = px - pm;
      }
    }
  }
  __syncthreads();
  for (int e = tid; e < kk; e += NT) {
    const int a = e / k, b = e - a * k;
    const double* va = V + sel[a];
    double acc = 0.0;
    for (int r = 0; r < p; ++r) acc += va[r * kLd] * A[r * kLd + b];
    P[e] = acc;
  }
  if (tid == 0) valid = 0;
  __syncthreads();
  stamp(4);
  // new covariance into the state (the projections above read the old one)
  for (int e = tid; e < p * p; e += NT) s_C[e] = Tm[(e / p) * kLd + e % p];
  // ---- Sherman-Morrison scores (sequential in rows)
  for (int i = 0; i < nb; ++i) {
    const double* d = XD + size_t(i) * k;
    if (!valid) {
      if (tid == 0) {  // Gauss-Jordan in LDS (T1 = working copy of P, T2 = inverse)
        inverted = 0;
        const double det = invert_into(P, T1, T2, k);
        if (fabs(det) > prm.eps) {
          for (int e = 0; e < kk; ++e) Cp[e] = T2[e];
          inverted = 1;
          valid = 1;
        }
      }
      __syncthreads();
      if (!inverted) {
        if (n + i != 0.0) {
          const double a = (n + i - 1.0) / (n + i), cb = 1.0 / (n + i + 1.0);
          const double* dp = DPC + size_t(i) * k;
          for (int e = tid; e < kk; e += NT) P[e] = a * P[e] + cb * dp[e / k] * dp[e % k];
        }
        if (tid == 0) scores[i] = prm.out_mode == 1 ? (0.0 > prm.threshold ? 1.0 : 0.0) : 0.0;
        __syncthreads();
        continue;
      }
    } else {
      const double a = (n + i - 1.0) / (n + i - 2.0), cb = 1.0 / (n + i);  // B_{i-1} = dpc dpc^T / (n + i)
      const double* dp = DPC + size_t(i - 1) * k;
      for (int e = tid; e < kk; e += NT) T1[e] = a * Cp[e];
      __syncthreads();
      for (int e = tid; e < kk; e += NT) {  // BC1 = B_{i-1} c_inv
        const int r = e / k, c = e - r * k;
        double sacc = 0.0;
        for (int j = 0; j < k; ++j) sacc += (cb * dp[r] * dp[j]) * T1[j * k + c];
        T2[e] = sacc;
      }
      __syncthreads();
      if (tid == 0) {
        double tr = 0.0;
        for (int j = 0; j < k; ++j) tr += T2[j * k + j];
        scal = 1.0 / (1.0 + tr);
      }
      __syncthreads();
      for (int e = tid; e < kk; e += NT) {
        const int r = e / k, c = e - r * k;
        double sacc = 0.0;
        for (int j = 0; j < k; ++j) sacc += T1[r * k + j] * T2[j * k + c];
        Cp[e] = T1[e] - scal * sacc;
      }
      __syncthreads();
    }
    double part = 0.0;
    for (int e = tid; e < kk; e += NT) part += d[e / k] * Cp[e] * d[e % k];
    part = block_sum<NT>(part, red);
    if (tid == 0) scores[i] = prm.out_mode == 1 ? (part > prm.threshold ? 1.0 : 0.0) : part;
    __syncthreads();
  }
  stamp(5);
  // ---- state update: n, clip bounds from the new covariance diagonal
  const double n_new = n_state + nb;
  for (int j = tid; j < p; j += NT) {
    if (n_new > prm.start_clip) {
      const double sd = sqrt(Tm[j * kLd + j]);
      s_lo[j] = s_mean[j] - prm.n_stdev * sd;
      s_hi[j] = s_mean[j] + prm.n_stdev * sd;
    }
  }
  if (tid == 0) {
    s_tail[0] = n_new;
    s_tail[1] = 0.0;
    if (n_new > prm.start_clip) s_tail[2] = 1.0;
  }
  stamp(6);
  if (tid == 0) {
    double* acc = eig + kMahaMaxP * kMahaMaxP + 5;
    for (int i = 0; i < 10; ++i) acc[i] += double(ph[i]) * 0.01;  // microseconds
  }
}

template <int NT>
__global__ __launch_bounds__(NT) void maha_step_kernel(const double* __restrict__ X, const int32_t* __restrict__ seg,
                                                       int nseg, int nb, MahaParams prm, double* __restrict__ state,
                                                       double* __restrict__ eig, double* __restrict__ ws,
                                                       double* __restrict__ out) {
  if (seg == nullptr) {
    maha_one<NT>(X, nb, prm, state, eig, ws, out);
    return;
  }
  for (int r = 0; r < nseg; ++r) {
    const int b = seg[r], e = seg[r + 1];
    if (e > b) maha_one<NT>(X + size_t(b) * prm.p, e - b, prm, state, eig, ws, out + b);
    __syncthreads();
  }
}

void launch_step(const double* X, const int32_t* seg, int nseg, int nb, const MahaParams& prm, double* state,
                 double* eig, double* ws, double* out, hipStream_t s) {
  if (prm.p <= 16)
    hipLaunchKernelGGL(maha_step_kernel<64>, dim3(1), dim3(64), 0, s, X, seg, nseg, nb, prm, state, eig, ws, out);
  else
    hipLaunchKernelGGL(maha_step_kernel<256>, dim3(1), dim3(256), 0, s, X, seg, nseg, nb, prm, state, eig, ws, out);
}

}  // namespace

bool mahalanobis_sm_scores(const double* B, const double* cov0, const double* xd, int nb, int k, double n,
                           double* out, hipStream_t s) {
  if (k < 1 || k > kMaxK) return false;
  if (nb <= 0) return true;
  hipLaunchKernelGGL(maha_sm_kernel, dim3(1), dim3(64), 0, s, B, cov0, xd, nb, k, n, 1e-8, out);
  return true;
}

void maha_step(const double* X, int nb, const MahaParams& prm, double* state, double* eig, double* ws,
               double* scores, hipStream_t s) {
  if (nb <= 0) return;
  launch_step(X, nullptr, 0, nb, prm, state, eig, ws, scores, s);
}

void maha_step_segments(const double* X, const int32_t* seg, int nseg, const MahaParams& prm, double* state,
                        double* eig, double* ws, double* out, hipStream_t s) {
  if (nseg <= 0) return;
  launch_step(X, seg, nseg, 0, prm, state, eig, ws, out, s);
}

}  // namespace sca::kern
