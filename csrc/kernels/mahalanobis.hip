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

__device__ double invert_into(const double* A, double* M, double* inv, int k);

__global__ __launch_bounds__(64) void maha_sm_kernel(const double* __restrict__ B, const double* __restrict__ cov0,
                                                     const double* __restrict__ xd, int nb, int k, double n,
                                                     double eps, double* __restrict__ out) {
  __shared__ double P[kMaxK * kMaxK], Cp[kMaxK * kMaxK], T1[kMaxK * kMaxK], T2[kMaxK * kMaxK], Mw[kMaxK * kMaxK];
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
        const double det = invert_into(P, Mw, T1, k);  // T1 is free here
        if (fabs(det) > eps) {
          for (int e = 0; e < kk; ++e) Cp[e] = T1[e];
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
// batch against the device-resident state: NT = 64 threads (one wave) for
// p <= 16, 256 otherwise.  p <= 64 features, k <= 16 components; p x p
// matrices live in LDS (row stride kLd = 65, conflict-free row-per-lane
// access).  The top-k eigenpairs are computed by ONE wave (topk_wave): a
// latency chain of ~p dependent steps, where extra waves would only add
// barriers.
constexpr int kLd = kMahaMaxP + 1;
// A (the matrix the eigen-solver streams) has 8 private padding columns per
// row, so 8-wide blocks may run past p without guards (73: still odd, rows
// on distinct banks)
constexpr int kLdA = kMahaMaxP + 9;

__device__ __forceinline__ double wave_sum(double v);
template <int NT> __device__ double block_sum(double v, double* red) {
  v = wave_sum(v);
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
template <int CTRL> __device__ __forceinline__ double mdpp64(double v) {  // DPP move, no old-value operand
  const int2 h = __builtin_bit_cast(int2, v);
  int2 o;
  o.x = __builtin_amdgcn_mov_dpp(h.x, CTRL, 0xF, 0xF, true);
  o.y = __builtin_amdgcn_mov_dpp(h.y, CTRL, 0xF, 0xF, true);
  return __builtin_bit_cast(double, o);
}
// v + (v of the partner lane) for v_permlane16_swap (lane ^ 16) or
// v_permlane32_swap (lane ^ 32): a half exchange of vdst with src, here both v
template <bool P32> __device__ __forceinline__ double swap_add64(double v) {
  const int2 h = __builtin_bit_cast(int2, v);
  const auto a = P32 ? __builtin_amdgcn_permlane32_swap(h.x, h.x, false, false)
                     : __builtin_amdgcn_permlane16_swap(h.x, h.x, false, false);
  const auto b = P32 ? __builtin_amdgcn_permlane32_swap(h.y, h.y, false, false)
                     : __builtin_amdgcn_permlane16_swap(h.y, h.y, false, false);
  return __builtin_bit_cast(double, make_int2(int(a[0]), int(b[0]))) +
         __builtin_bit_cast(double, make_int2(int(a[1]), int(b[1])));
}
// whole-wave double sum, every lane gets the total: 4 DPP stages inside
// each 16-lane row, then the two cross-row exchanges (VALU only, no SGPR
// hop; 172 vs 192 clocks for DPP + v_readlane, 492 for __shfl_xor on
// MI355X, tools/micro/wave_latency.hip).  Requires all 64 lanes active.
__device__ __forceinline__ double wave_sum(double v) {
  v += mdpp64<0xB1>(v);   // lane ^ 1
  v += mdpp64<0x4E>(v);   // lane ^ 2
  v += mdpp64<0x141>(v);  // row_half_mirror: the other quad of the 8
  v += mdpp64<0x140>(v);  // row_mirror: the other 8 of the 16
  v = swap_add64<false>(v);
  return swap_add64<true>(v);
}
template <bool P32> __device__ __forceinline__ double swap_partner64(double v) {  // v of lane ^ 16 / ^ 32
  const int2 h = __builtin_bit_cast(int2, v);
  const auto a = P32 ? __builtin_amdgcn_permlane32_swap(h.x, h.x, false, false)
                     : __builtin_amdgcn_permlane16_swap(h.x, h.x, false, false);
  const auto b = P32 ? __builtin_amdgcn_permlane32_swap(h.y, h.y, false, false)
                     : __builtin_amdgcn_permlane16_swap(h.y, h.y, false, false);
  return __builtin_bit_cast(double, make_int2(int(a[0]), int(b[0])));  // own or partner value
}
template <bool P32> __device__ __forceinline__ double swap_other64(double v) {
  const int2 h = __builtin_bit_cast(int2, v);
  const auto a = P32 ? __builtin_amdgcn_permlane32_swap(h.x, h.x, false, false)
                     : __builtin_amdgcn_permlane16_swap(h.x, h.x, false, false);
  const auto b = P32 ? __builtin_amdgcn_permlane32_swap(h.y, h.y, false, false)
                     : __builtin_amdgcn_permlane16_swap(h.y, h.y, false, false);
  return __builtin_bit_cast(double, make_int2(int(a[1]), int(b[1])));  // the other one
}
__device__ __forceinline__ double wave_min(double v) {
  v = fmin(v, mdpp64<0xB1>(v));
  v = fmin(v, mdpp64<0x4E>(v));
  v = fmin(v, mdpp64<0x141>(v));
  v = fmin(v, mdpp64<0x140>(v));
  // one of the two swap results is the lane's own value: min over both
  v = fmin(v, fmin(swap_partner64<false>(v), swap_other64<false>(v)));
  return fmin(v, fmin(swap_partner64<true>(v), swap_other64<true>(v)));
}
__device__ __forceinline__ double wave_max(double v) {
  v = fmax(v, mdpp64<0xB1>(v));
  v = fmax(v, mdpp64<0x4E>(v));
  v = fmax(v, mdpp64<0x141>(v));
  v = fmax(v, mdpp64<0x140>(v));
  v = fmax(v, fmax(swap_partner64<false>(v), swap_other64<false>(v)));
  return fmax(v, fmax(swap_partner64<true>(v), swap_other64<true>(v)));
}
// 1 / x from v_rcp_f64 plus two Newton steps (full double precision; no
// IEEE division sequence in the dependent chains below)
__device__ __forceinline__ double rcp_nr(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = r * fma(-x, r, 2.0);
  return r * fma(-x, r, 2.0);
}
// LDS ordering point for one wave: the lanes' stores above are visible to
// the wave's loads below (LDS executes one wave's accesses in order; this
// keeps the compiler from moving them across).
__device__ __forceinline__ void wave_lds_sync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

// 1 / sqrt(x) from v_rsq_f64 plus two Newton steps
__device__ __forceinline__ double rsq_nr(double x) {
  double r = __builtin_amdgcn_rsq(x);
  r = r * fma(-0.5 * x * r, r, 1.5);
  return r * fma(-0.5 * x * r, r, 1.5);
}

// x = H_0 ... H_{p-3} x for the KB vectors in V columns a0..a0+KB-1 (lane =
// row): per reflector, KB independent wave sums (their latencies overlap)
template <int KB>
__device__ void back_transform(double* __restrict__ V, const double* __restrict__ Wr, int p, int a0) {
  const int lane = threadIdx.x & 63;
  const bool inp = lane < p;
  double xa[KB];
#pragma unroll
  for (int a = 0; a < KB; ++a) xa[a] = inp ? V[lane * kLd + a0 + a] : 0.0;
  double vt = p >= 3 && lane > p - 3 && inp ? Wr[(p - 3) * kLd + lane] : 0.0;
  for (int j = p - 3; j >= 0; --j) {
    const double vnext = j >= 1 && lane > j - 1 && inp ? Wr[(j - 1) * kLd + lane] : 0.0;  // read ahead
    double sa[KB];
#pragma unroll
    for (int a = 0; a < KB; ++a) sa[a] = wave_sum(vt * xa[a]);
#pragma unroll
    for (int a = 0; a < KB; ++a) xa[a] -= 2.0 * sa[a] * vt;
    vt = vnext;
  }
#pragma unroll
  for (int a = 0; a < KB; ++a)
    if (inp) V[lane * kLd + a0 + a] = xa[a];
}

// LDS scratch of the eigen-solver (padded by 8 so blocked loops may read
// past p without leaving the arrays)
struct EigScratch {
  double2 rv[kMahaMaxP + 8];  // (v_c, w_c) of the reflector being applied
  double rn[kMahaMaxP + 8];   // the next reflector
  double dg[kMahaMaxP + 8], eo[kMahaMaxP + 8];   // tridiagonal T
  double sd[kMahaMaxP + 16], se2[kMahaMaxP + 16];  // T / 2^E, squared off-diagonal / 2^2E (Sturm counts; a block read ahead)
  double lam[kMahaMaxK];
  double part[3][64];  // multi-wave tridiagonalisation: waves 1-3's partial (A v)_g
};

// Top-k eigenpairs of the symmetric p x p matrix in A (LDS, stride kLd;
// destroyed), the way LAPACK's syevr computes a subset (what the reference's
// scipy eigh(eigvals=(p-k, p-1)) runs), by the 64 lanes of ONE wave -- lane g
// owns matrix row g, so no step needs a workgroup barrier.  Every loop that
// streams LDS is blocked by 8 with the block's loads issued before its
// arithmetic, so one LDS latency covers 8 elements of a dependent chain.
//  1. Householder tridiagonalisation, one pass over the active rows per
//     column: the pass applies column j's rank-2 update A -= v w^T + w v^T
//     and, in the same sweep, the matrix-vector product of column j + 1's
//     reflector (column j + 1 is updated in registers first -- its entries
//     were kept from the previous pass -- so the reflector exists before the
//     pass);
//  2. the k largest eigenvalues by multisection on Sturm counts, the wave
//     split into k lane groups (64 / k points per group and round, the
//     subinterval picked by ballot; every lane recomputes the same section
//     points, no shuffles).  Counts are sign changes of the leading minors
//     P_{i+1} = (d_i - x) P_i - e_{i-1}^2 P_{i-1} on T scaled by 2^-E ~
//     1 / ||T|| (renormalised every 8 steps): 2 dependent flops per element
//     instead of a reciprocal chain;
//  3. their tridiagonal eigenvectors by inverse iteration, lane a for
//     eigenvalue a (LU with partial pivoting, 2 iterations), normalised and
//     re-orthogonalised within clusters (as dstein);
//  4. back-transformation through the reflectors, all k vectors per step.
// Wr: reflectors (row j = reflector j, indexed by global row).  Output:
// eigenvectors in V[:, 0..k-1], sel[a] = a.
//
// nw = 4 (the 256-thread kernel, p >= MahaParams::mw_min_p): every thread
// calls this; waves 1-3 take part only in step 1's per-column sweep (a share
// of the 8-column blocks of every row, partial products through LDS, two
// workgroup barriers per column) and return before step 2.
__device__ void topk_wave(double* __restrict__ A, double* __restrict__ V, double* __restrict__ Wr, EigScratch& es,
                          int* sel, int p, int k, uint64_t* ph, int nw) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool inp = lane < p;
  uint64_t t_prev = __builtin_amdgcn_s_memrealtime();
  auto col_sync = [&] {  // the sweep's data (rn, rv, other waves' columns) visible to every participating wave
    if (nw > 1) __syncthreads();
    else wave_lds_sync();
  };
  auto mark = [&](int i) {  // sub-phase timer (thread 0): ph[i] of the caller's phase array
    if (threadIdx.x == 0) {
      const uint64_t t = __builtin_amdgcn_s_memrealtime();
      ph[i] += t - t_prev;
      t_prev = t;
    }
  };
  double* __restrict__ arow = A + lane * kLdA;
  double* __restrict__ dg = es.dg;
  double* __restrict__ eo = es.eo;
  // ---- 1. tridiagonalisation
  // reflector j from x (column j, rows j+1..p-1 on their lanes, 0 elsewhere):
  // v (unit norm) -> Wr row j and rn; alpha -> eo[j]
  auto reflect = [&](int j, double x) -> double {
    const double s2 = wave_sum(x * x);
    const double x0 = readlane64(x, j + 1);
    double v = 0.0, alpha = 0.0;
    if (s2 > 0.0) {
      const double nrm = s2 * rsq_nr(s2);
      alpha = x0 >= 0.0 ? -nrm : nrm;
      // |v_raw|^2 = s2 - x0^2 + (x0 - alpha)^2 = 2 (s2 + |x0| nrm)
      v = (lane == j + 1 ? x - alpha : x) * rsq_nr(2.0 * fma(fabs(x0), nrm, s2));
    }
    if (lane == 0) eo[j] = alpha;
    if (lane > j && inp) {
      Wr[j * kLd + lane] = v;
      es.rn[lane] = v;
    }
    return v;
  };
  // zero padding: columns p..p+7 of every active row, reflector slots past p;
  // Sturm pads (d = 4 > any scaled shift, e^2 = 0) add no sign change
  if (wv == 0) {
  if (inp)
    for (int c = p; c < kMahaMaxP + 8; ++c) arow[c] = 0.0;
  for (int c = p + lane; c < kMahaMaxP + 8; c += 64) {
    es.rv[c] = make_double2(0.0, 0.0);
    es.rn[c] = 0.0;
  }
  for (int c = p + lane; c < kMahaMaxP + 16; c += 64) es.sd[c] = 4.0;
  for (int c = p - 1 + lane; c < kMahaMaxP + 16; c += 64)
    if (c >= 0) es.se2[c] = 0.0;
  if (lane == 0) dg[0] = A[0];
  if (p == 2 && lane == 0) {
    dg[1] = A[kLdA + 1];
    eo[0] = A[kLdA];
  }
  }  // wv == 0
  if (p >= 3) {
    double vg = 0.0, col = 0.0, pv = 0.0, K = 0.0, wg = 0.0;
    if (wv == 0) {
    vg = reflect(0, lane >= 1 && inp ? arow[0] : 0.0);
    col = lane >= 1 && inp ? arow[1] : 0.0;  // this row's entry of the next column
    wave_lds_sync();
    if (lane >= 1 && inp) {
      double s[4] = {0.0, 0.0, 0.0, 0.0};
      for (int cb = 1; cb < p; cb += 8) {
        double av[8], nv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          av[u] = arow[cb + u];
          nv[u] = es.rn[cb + u];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) s[u & 3] += av[u] * nv[u];
      }
      pv = (s[0] + s[1]) + (s[2] + s[3]);
    }
    K = wave_sum(vg * pv);
    wg = 2.0 * pv - 2.0 * K * vg;
    if (inp) es.rv[lane] = make_double2(vg, wg);
    wave_lds_sync();
    }  // wv == 0
    for (int j = 0; j + 2 < p; ++j) {
      // column j + 1 after update j (lane j + 1: the new diagonal entry)
      double x = 0.0, vn = 0.0;
      if (wv == 0) {
        const double vj1 = readlane64(vg, j + 1), wj1 = readlane64(wg, j + 1);
        x = lane > j && inp ? col - (vg * wj1 + wg * vj1) : 0.0;
        if (lane == j + 1) dg[j + 1] = x;
        if (j + 3 < p) vn = reflect(j + 1, lane > j + 1 ? x : 0.0);
      }
      if (j + 3 < p) {
        col_sync();
        // fused pass over columns j+2..p-1 of rows j+2..p-1: update j, then
        // (A v_{j+1}) with the updated entries; wave wv takes 8-column blocks
        // [ceil(wv nb / nw), ceil((wv + 1) nb / nw)), so wave 0 always owns
        // column j + 2 (the next x)
        const int c0 = j + 2, nb = (p - c0 + 7) >> 3;
        const int cb0 = c0 + 8 * ((wv * nb + nw - 1) / nw), cb1 = c0 + 8 * (((wv + 1) * nb + nw - 1) / nw);
        double rvg = vg, rwg = wg;
        if (wv != 0) {
          const double2 r = es.rv[lane];
          rvg = r.x;
          rwg = r.y;
        }
        pv = 0.0;
        if (lane > j + 1 && inp) {
          double s[4] = {0.0, 0.0, 0.0, 0.0};
          // (a single wave is VALU-issue bound here, ~3 f64 ops per entry:
          // reading the next block ahead measured slower, not faster)
          for (int cb = cb0; cb < cb1; cb += 8) {
            double av[8], nv[8];
            double2 rw[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              av[u] = arow[cb + u];
              rw[u] = es.rv[cb + u];
              nv[u] = es.rn[cb + u];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {  // past p: 0 - 0 written back to the row's own padding
              const double a = fma(-rwg, rw[u].x, fma(-rvg, rw[u].y, av[u]));
              arow[cb + u] = a;
              s[u & 3] = fma(a, nv[u], s[u & 3]);
            }
            if (cb == c0) col = fma(-rwg, rw[0].x, fma(-rvg, rw[0].y, av[0]));
          }
          pv = (s[0] + s[1]) + (s[2] + s[3]);
        }
        if (nw > 1) {
          if (wv != 0) es.part[wv - 1][lane] = pv;
          __syncthreads();
          if (wv == 0) pv += (es.part[0][lane] + es.part[1][lane]) + es.part[2][lane];
        }
        if (wv == 0) {
          K = wave_sum(vn * pv);
          vg = vn;
          wg = 2.0 * pv - 2.0 * K * vn;
          wave_lds_sync();
          if (inp) es.rv[lane] = make_double2(vg, wg);
          wave_lds_sync();
        }
      } else if (wv == 0 && lane == p - 1) {  // j = p - 3: the trailing 2 x 2 block
        eo[p - 2] = x;
        dg[p - 1] = arow[p - 1] - 2.0 * vg * wg;
      }
    }
  }
  if (wv != 0) return;  // steps 2-4 are wave 0's
  wave_lds_sync();
  // ---- 2. k largest eigenvalues: Gershgorin bracket, multisection in k lane groups
  const double di = inp ? dg[lane] : 0.0;
  const double ei = lane + 1 < p ? fabs(eo[lane]) : 0.0, em = lane >= 1 && inp ? fabs(eo[lane - 1]) : 0.0;
  const double lo0 = wave_min(inp ? di - ei - em : 1e300), hi0 = wave_max(inp ? di + ei + em : -1e300);
  const double tnorm = fmax(fabs(lo0), fabs(hi0));
  const double pivmin = fmax(tnorm * 2.3e-16, 1e-280);  // the floor keeps 1 / pivmin finite (all-zero C)
  // scale T by 2^-E (exact) so |d - x| and e^2 are O(1) in the minors' recurrence
  const int E = tnorm > 0.0 ? __builtin_amdgcn_frexp_exp(tnorm) : 0;
  if (inp) {
    es.sd[lane] = ldexp(di, -E);
    if (lane + 1 < p) {
      const double es_ = ldexp(eo[lane], -E);
      es.se2[lane] = es_ * es_;
    }
  }
  wave_lds_sync();
  mark(7);  // tridiagonalisation
  {
    const int s = 64 / k;  // points per group
    const int grp = min(lane / s, k - 1), gi = lane - grp * s;
    const bool gact = lane < k * s;
    const int idx = p - 1 - grp;  // ascending index of the grp-th largest eigenvalue
    const double inv_s1 = 1.0 / double(s + 1);
    const unsigned long long gmask = s == 64 ? ~0ull : ((1ull << s) - 1ull);
    double l = lo0 - 1e-10 * tnorm - 1e-300, u = hi0 + 1e-10 * tnorm + 1e-300;
    for (int it = 0; it < 128; ++it) {
      const bool done = u - l <= 2.3e-16 * fmax(fabs(l), fabs(u)) + 1e-18 * tnorm + 1e-300;
      if (__ballot(gact && !done) == 0) break;
      const double x = l + (u - l) * (double(gi + 1) * inv_s1);
      const double xs = ldexp(x, -E);
      // eigenvalues < x = sign changes of P_0 = 1, P_1, ..., P_p (a zero counts as +)
      // (sign changes from the sign bits of consecutive minors; padding
      // steps past p keep the sign)
      double pm = 1.0, pc = es.sd[0] - xs;
      unsigned cnt = unsigned(__double2hiint(pc)) >> 31;
      for (int ib = 1; ib < p; ib += 8) {
        double dd[8], ee[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          dd[q] = es.sd[ib + q] - xs;
          ee[q] = es.se2[ib + q - 1];
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const double pn = fma(-ee[q], pm, dd[q] * pc);
          cnt += unsigned(__double2hiint(pn) ^ __double2hiint(pc)) >> 31;
          pm = pc;
          pc = pn;
        }
        const int ex = __builtin_amdgcn_frexp_exp(pc);  // renormalise (pc == 0: exponent 0)
        pc = ldexp(pc, -ex);
        pm = ldexp(pm, -ex);
      }
      const unsigned long long bal = __ballot(gact && int(cnt) > idx);
      const unsigned long long gm = (bal >> (grp * s)) & gmask;
      const int f = gm ? __ffsll(static_cast<long long>(gm)) - 1 : s;  // eigenvalue in (x_{f-1}, x_f]
      if (!done) {
        const double nl = f > 0 ? l + (u - l) * (double(f) * inv_s1) : l;
        const double nu = f < s ? l + (u - l) * (double(f + 1) * inv_s1) : u;
        l = nl;
        u = nu;
      }
    }
    if (gact && gi == 0) es.lam[grp] = 0.5 * (l + u);
  }
  wave_lds_sync();
  mark(8);  // eigenvalues
  // ---- 3. eigenvectors of T by twisted factorisation (the MRRR kernel,
  // LAPACK dlar1v), lane a for eigenvalue a: T - lam I = L+ D+ L+^T
  // (top-down) = U- D- U-^T (bottom-up), both stationary qd recurrences run
  // interleaved; twist index r = argmin |gamma_r|, gamma_r = d+_r + d-_r -
  // (t_rr - lam); z_r = 1 and z follows by one product recurrence each way.
  // No iteration, no pivoting; scratch in A (free now) as [row][kMahaMaxK].
  if (lane < k) {
    const int a = lane;
    double* LP = A;                             // l+_i = e_i / d+_i
    double* UM = LP + kMahaMaxP * kMahaMaxK;    // u-_i = e_i / d-_{i+1}
    double* DP = UM + kMahaMaxP * kMahaMaxK;    // d+_i
    double* DM = DP + kMahaMaxP * kMahaMaxK;    // d-_i
    const double L = es.lam[a];
    double dp = dg[0] - L, dm = dg[p - 1] - L;
    DP[a] = dp;
    DM[(p - 1) * kMahaMaxK + a] = dm;
#pragma unroll 4
    for (int t = 0; t + 1 < p; ++t) {
      const int i = t, ib = p - 2 - t;
      const double bf = eo[i], bb = eo[ib];
      if (fabs(dp) < pivmin) dp = -pivmin;
      if (fabs(dm) < pivmin) dm = -pivmin;
      const double lp = bf * rcp_nr(dp), um = bb * rcp_nr(dm);
      LP[i * kMahaMaxK + a] = lp;
      UM[ib * kMahaMaxK + a] = um;
      dp = (dg[i + 1] - L) - lp * bf;
      dm = (dg[ib] - L) - um * bb;
      DP[(i + 1) * kMahaMaxK + a] = dp;
      DM[ib * kMahaMaxK + a] = dm;
    }
    int r = 0;
    double gbest = 1e308;
#pragma unroll 4
    for (int i = 0; i < p; ++i) {
      const double g = fabs(DP[i * kMahaMaxK + a] + DM[i * kMahaMaxK + a] - (dg[i] - L));
      if (g < gbest) {
        gbest = g;
        r = i;
      }
    }
    double z = 1.0;
    V[r * kLd + a] = 1.0;
    for (int i = r - 1; i >= 0; --i) {
      z = -LP[i * kMahaMaxK + a] * z;
      V[i * kLd + a] = z;
    }
    z = 1.0;
    for (int i = r; i + 1 < p; ++i) {
      z = -UM[i * kMahaMaxK + a] * z;
      V[(i + 1) * kLd + a] = z;
    }
  }
  wave_lds_sync();
  // normalise; re-orthogonalise within clusters (|lam_a - lam_b| < 1e-3 ||T||, as dstein)
  for (int a = 0; a < k; ++a) {
    double y = inp ? V[lane * kLd + a] : 0.0;
    for (int b = 0; b < a; ++b) {
      if (fabs(es.lam[a] - es.lam[b]) < 1e-3 * tnorm) {
        const double yb = inp ? V[lane * kLd + b] : 0.0;
        y -= wave_sum(y * yb) * yb;
      }
    }
    y *= rsq_nr(fmax(wave_sum(y * y), 1e-300));
    if (inp) V[lane * kLd + a] = y;
    wave_lds_sync();
  }
  if (lane < k) sel[lane] = lane;
  mark(2);  // eigenvectors (twisted factorisation, normalisation)
  // ---- 4. back-transformation x = H_0 ... H_{p-3} y, all k vectors per
  // reflector (their k wave sums overlap); vectors a0.. in groups of 4
  for (int a0 = 0; a0 < k; a0 += 4) {
    switch (min(k - a0, 4)) {
      case 1: back_transform<1>(V, Wr, p, a0); break;
      case 2: back_transform<2>(V, Wr, p, a0); break;
      case 3: back_transform<3>(V, Wr, p, a0); break;
      default: back_transform<4>(V, Wr, p, a0); break;
    }
  }
  wave_lds_sync();
  mark(9);  // back-transformation
}

// Full eigendecomposition by cyclic Jacobi (one wave), WARM-STARTED from
// the previous step's eigenvectors (kept in eig[0 .. p*p)).  The covariance
// changes by a rank-nb update of weight ~1/n per request, so
// B = V0^T C V0 is diagonal but for O(1/n) off-diagonals and two or three
// threshold-Jacobi sweeps (quadratic convergence) diagonalise it.  Cold
// starts (no cache, the first step, every `refresh`-th step to bound the
// drift of V0's orthogonality) start from V0 = I.  The score depends only on
// the top-k SUBSPACE (projections, proj_cov and the Sherman-Morrison
// recurrence all change by the same k x k rotation), so any orthonormal basis
// of it gives the reference's scores.
//
// Thread (r, c) owns row r of B and of V^T (the eigenvectors are kept
// transposed during the sweeps), columns of chunk c = its wave: the whole
// workgroup (1 or 4 waves) sweeps, 3 barriers per round.  A round rotates m/2 disjoint pairs
// (round-robin tournament, m = p rounded up to even; pairs with the dummy
// index p are skipped); every lane needs only ITS pair's (c, s) and partner:
//   U = R^T B      row mix:          U[r][:]  = a_r B[r][:] + b_r B[pi_r][:]
//   B' = U R       by symmetry:      B'[r][q] = a_r U[q][r] + b_r U[q][pi_r]
//                  (column reads of U, conflict-free across the wave)
//   V'^T = R^T V^T row mix in place (a column's loads precede its stores)
// A pair rotates only
// while |b_ij| > tol * sqrt(|b_ii b_jj|) (tol = 1e-14; the rotated element is
// set to exactly 0): the sweep with no rotation ends the solve.  On exit the eigenpairs are sorted by
// descending eigenvalue into V (columns; sel = 0..k-1) and cached with their
// eigenvalues for the eigen-tracking path (rank1_eigen).
constexpr int kJacobiRefresh = 256;   // Jacobi-only mode: cold solve period
constexpr int kTrackRefresh = 1024;   // eigen-tracking mode: Newton-Schulz re-orthogonalisation period
constexpr int kTrackMaxRows = 16;     // requests with more rows re-solve by Jacobi
constexpr bool kMahaMfmaGemm = true;  // eigen-tracking V Q on v_mfma_f64_16x16x4

template <int NT>
__device__ __forceinline__ void jacobi_solve(double* __restrict__ A, double* __restrict__ V, double* __restrict__ W,
                                             int* sel, int p, int k, double* __restrict__ cache,
                                             double* __restrict__ tail, double* __restrict__ lamv,
                                             double* __restrict__ lam_cache, bool warm, double* __restrict__ stats) {
  // thread (r, c): row r of B / V^T, column chunk c (= its wave) of width cw
  constexpr int kWaves = NT / 64;
  const int tid = threadIdx.x, r = tid & 63, c = tid >> 6;
  const int m = p + (p & 1);
  const int cw = (p + kWaves - 1) / kWaves;
  const int q_lo = min(p, c * cw), q_hi = min(p, q_lo + cw);
  const bool row = r < p;
  if (warm) {
    for (int e = tid; e < p * p; e += NT) V[(e / p) * kLd + e % p] = cache[e];
    __syncthreads();
    // T = C V0 -> W, then B = V0^T T -> A (each thread its row's chunk)
    if (row)
      for (int q = q_lo; q < q_hi; ++q) {
        double t = 0.0;
        for (int j = 0; j < p; ++j) t += A[r * kLdA + j] * V[j * kLd + q];
        W[r * kLd + q] = t;
      }
    __syncthreads();
    if (row)
      for (int q = q_lo; q < q_hi; ++q) {
        double b = 0.0;
        for (int j = 0; j < p; ++j) b += V[j * kLd + r] * W[j * kLd + q];
        A[r * kLdA + q] = b;
      }
    __syncthreads();
    if (row)
      for (int q = q_lo; q < q_hi; ++q) V[r * kLd + q] = cache[q * p + r];  // V^T = V0^T
  } else if (row) {
    for (int q = q_lo; q < q_hi; ++q) V[r * kLd + q] = r == q ? 1.0 : 0.0;
  }
  __syncthreads();
  // symmetric working copy: B[r][q] for q < r taken from the upper triangle
  if (row)
    for (int q = q_lo; q < min(q_hi, r); ++q) A[r * kLdA + q] = A[q * kLdA + r];
  __syncthreads();
  constexpr double tol = 1e-14;
  int sweeps = 40;
  for (int sweep = 0; sweep < 40; ++sweep) {
    int rotated = 0;
    for (int rnd = 0; rnd < m - 1; ++rnd) {
      // tournament position of player r, and its partner
      int pr = r;
      if (r < m) {
        const int pos = r == 0 ? 0 : ((r - 1 - rnd) % (m - 1) + (m - 1)) % (m - 1) + 1;
        const int opp = m - 1 - pos;
        pr = opp == 0 ? 0 : 1 + (opp - 1 + rnd) % (m - 1);
      }
      double al = 1.0, be = 0.0;
      int pl = r;
      if (row && pr < p) {
        const int i = min(r, pr), j = max(r, pr);
        const double aii = A[i * kLdA + i], ajj = A[j * kLdA + j], aij = A[i * kLdA + j];
        if (aij != 0.0 && fabs(aij) > tol * sqrt(fabs(aii * ajj))) {
          const double th = (aii - ajj) / (2.0 * aij);
          const double t = -copysign(1.0, th) / (fabs(th) + sqrt(1.0 + th * th));
          const double cs = 1.0 / sqrt(1.0 + t * t), sn = t * cs;
          al = cs;
          be = r == i ? -sn : sn;
          pl = pr;
          rotated = 1;
        }
      }
      __syncthreads();  // every thread has read this round's B entries
      if (row)  // U = R^T B -> W (rows)
        for (int q = q_lo; q < q_hi; ++q) W[r * kLd + q] = al * A[r * kLdA + q] + be * A[pl * kLdA + q];
      __syncthreads();
      if (row) {
        // B' = U R -> A, through the symmetry: B'[r][q] = a_r U[q][r] + b_r U[q][pi_r];
        // the annihilated pair exactly 0
        for (int q = q_lo; q < q_hi; ++q)
          A[r * kLdA + q] = (q == pl && pl != r) ? 0.0 : al * W[q * kLd + r] + be * W[q * kLd + pl];
        // V^T <- R^T V^T in place: partner rows share this thread's chunk, so
        // its wave; each column's loads are issued before its stores
        for (int q0 = q_lo; q0 < q_hi; q0 += 8) {
          double x[8], y[8];
#pragma unroll
          for (int b = 0; b < 8; ++b) {
            const int q = min(q0 + b, q_hi - 1);
            x[b] = V[r * kLd + q];
            y[b] = V[pl * kLd + q];
          }
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
          for (int b = 0; b < 8; ++b)
            if (q0 + b < q_hi) V[r * kLd + q0 + b] = al * x[b] + be * y[b];
        }
      }
      __syncthreads();
    }
    if (!__syncthreads_or(rotated)) {
      sweeps = sweep + 1;
      break;
    }
  }
  if (tid == 0) {  // solver statistics (kMahaEigMeta + 3 / + 4)
    stats[0] += double(sweeps);
    stats[1] += 1.0;
  }
  // eigenvalues (the diagonal) in descending order: row r's rank; the
  // eigenvectors (rows of V^T) land sorted in the COLUMNS of V through W
  if (row && c == 0) lamv[r] = A[r * kLdA + r];
  __syncthreads();
  if (row) {
    const double lam = lamv[r];
    int pos = 0;
    for (int j = 0; j < p; ++j) {
      const double lj = lamv[j];
      pos += (lj > lam || (lj == lam && j < r)) ? 1 : 0;
    }
    if (c == 0) lam_cache[pos] = lam;
    for (int q = q_lo; q < q_hi; ++q) W[q * kLd + pos] = V[r * kLd + q];
  }
  if (tid < k) sel[tid] = tid;
  __syncthreads();
  for (int e = tid; e < p * p; e += NT) {
    const double v = W[(e / p) * kLd + e % p];
    V[(e / p) * kLd + e % p] = v;
    cache[e] = v;  // the basis for the next step's warm start / eigen-tracking
  }
  if (tid == 0) {
    tail[0] = double(p);
    tail[1] = warm ? tail[1] + 1.0 : 0.0;
  }
  __syncthreads();
}

// Eigen-tracking update for one row of a request (CoreMahalanobis.py:92-103;
// a request of nb <= kTrackMaxRows rows is nb of these in turn, the residual
// checked after the last): C_new = alpha C_old + rho d d^T, and the cache holds C_old =
// V diag(lam) V^T (lam descending).  In that basis C_new = V (D + rho z z^T)
// V^T with D = alpha diag(lam), z = V^T d: a diagonal-plus-rank-1 problem
// whose eigenvalues are the roots of the secular equation
//   f(x) = 1 + rho' sum_j zh_j^2 / (D_j - x) = 0,   zh = z / |z|, rho' = rho |z|^2,
// one root in each interval (D_i, D_{i-1}) (and (D_0, D_0 + rho')).  Lane i
// finds root i from the pole nearer to it (x = D_K + tau, the differences
// D_j - x kept as (D_j - D_K) - tau), starting from the one-pole estimate,
// by a bracketed two-pole rational model (Bunch-Nielsen-Sorensen: 2-3
// iterations typical, 10 worst in 10^5 roots of the prototype).  The
// eigenvectors use the Gu-Eisenstat recomputed zt (numerically orthogonal
// even when roots crowd a pole), and V_new = V Q is one p^3 product in 4x4
// register blocks (all NT threads).  Returns false -- the caller re-solves by
// Jacobi -- on deflation (a tiny |zh_j| or a near-double eigenvalue), a root
// that did not converge, or a residual |C_new v - lam v| above 1e-11 lam_max
// on any of the top-k pairs (which also catches a stale cache).  A numpy
// prototype over 1,000 steps stayed within 6e-15 of eigh's eigenvalues and
// 1e-13 of its top-k subspace at p = 9, 32, 64.
// Z[M x N] = op(X) Y on the f64 matrix cores (v_mfma_f64_16x16x4: lane l
// holds X[l&15][k = l>>4] and Y[k = l>>4][l&15], result rows (l>>4) + 4i of
// column l&15), 16x16 tiles over the workgroup's waves; op(X) = X^T when
// TRANS.  Operands live in LDS with row strides ldx / ldy; k past K is fed
// as zeros, rows / columns past M / N read in-bounds LDS whose results are
// not stored.
template <int NT, bool TRANS>
__device__ void mfma_gemm_lds(const double* __restrict__ X, int ldx, const double* __restrict__ Y, int ldy,
                              double* __restrict__ Z, int ldz, int M, int N, int K) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, lk = lane >> 4;
  const int tr = (M + 15) >> 4, tc = (N + 15) >> 4;
  typedef double d4 __attribute__((ext_vector_type(4)));
  for (int t = wave; t < tr * tc; t += NT / 64) {
    const int r0 = (t / tc) * 16, c0 = (t - (t / tc) * tc) * 16;
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    for (int k0 = 0; k0 < K; k0 += 4) {
      const int kk = k0 + lk;
      const double a = kk < K ? (TRANS ? X[kk * ldx + r0 + li] : X[(r0 + li) * ldx + kk]) : 0.0;
      const double b = kk < K ? Y[kk * ldy + c0 + li] : 0.0;
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    }
    const int col = c0 + li;
    if (col < N)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = r0 + lk + 4 * i;
        if (row < M) Z[row * ldz + col] = acc[i];
      }
  }
}

template <int NT>
__device__ bool rank1_eigen(const double* __restrict__ dvec, double alpha, double rho, int p, int k,
                            const double* __restrict__ Cn, double* __restrict__ A, double* __restrict__ V,
                            double* __restrict__ W, EigScratch& es, int* sel, double* __restrict__ cache,
                            double* __restrict__ tail, double* __restrict__ lam_cache, double* red, int* flag,
                            bool first, bool last, uint64_t* ph) {
  // first: the basis / eigenvalues come from the cache (else from the
  // previous update of this request: V and lam_sorted in LDS); last: check
  // the residual against C_new and write the cache
  const int tid = threadIdx.x, lane = tid & 63;
  double* dd = es.dg;                                      // [orig] D = alpha lam
  double* zhp = es.eo;                                     // [orig] z / |z| after the cluster reflections
  double* uvec = reinterpret_cast<double*>(es.rv);         // [orig] cluster reflector
  double* ztA = reinterpret_cast<double*>(es.rv) + 72;     // [active] Gu-Eisenstat z
  double* ddA = es.sd;                                     // [active] D of the secular problem
  double* zzA = es.se2;                                    // [active] zh^2
  double* taus = es.part[0];                               // [active] root offsets from their pole
  double* lam_sorted = es.part[1];                         // [sorted] eigenvalues (also inv_norm [active] before)
  double* inv_norm = es.part[1];
  double* vals = es.part[2];                               // [entry] eigenvalue of entry e (active roots, then the rest)
  int* Ks = reinterpret_cast<int*>(es.rn);                 // [active] root poles; later [entry] sorted position
  int* perm = reinterpret_cast<int*>(es.rn) + 64;          // [entry] original index (active first)
  int* npc = reinterpret_cast<int*>(es.rn) + 128;          // [0] active count
  double* rsc = es.lam;                                    // [0] rho'
  const double* lam_src = first ? lam_cache : lam_sorted;
  // sub-phase timers (thread 0; the Householder path's slots, unused here):
  // 7 = z, deflation, 8 = secular roots + zt, 2 = Q + norms, 9 = V Q + sort + residual + cache
  uint64_t t_prev = __builtin_amdgcn_s_memrealtime();
  auto mark = [&](int i) {
    if (tid == 0) {
      const uint64_t t = __builtin_amdgcn_s_memrealtime();
      ph[i] += t - t_prev;
      t_prev = t;
    }
  };
  if (first)
    for (int e = tid; e < p * p; e += NT) V[(e / p) * kLd + e % p] = cache[e];
  if (tid == 0) *flag = 1;
  __syncthreads();
  // ---- z = V^T d; deflation (wave 0, lane j = index j): clusters of
  // eigenvalues closer than tol get one reflection within their columns of V
  // that puts all of the cluster's z on its first index (any basis of a
  // double eigenvalue's space is an eigenbasis); then every index with a
  // negligible z keeps its eigenpair, the rest form the secular problem
  if (tid < 64) {
    const bool own = lane < p;
    double z = 0.0;
    if (own) {
#pragma unroll 8
      for (int r = 0; r < p; ++r) z += V[r * kLd + lane] * dvec[r];
    }
    const double nz2 = wave_sum(z * z);
    const double rho2 = rho * nz2;
    double zh = nz2 > 0.0 ? z * rsq_nr(nz2) : 0.0;
    const double dl = own ? alpha * lam_src[lane] : 0.0;
    wave_lds_sync();  // (lam_src may be lam_sorted: every lane has read it)
    dd[lane] = dl;
    const double tol = 8.0 * __DBL_EPSILON__ * fmax(wave_max(fabs(dl)), rho2);
    if (lane == 0) rsc[0] = rho2;
    wave_lds_sync();
    // cluster heads: a gap above tol to the previous eigenvalue
    const unsigned long long heads = __ballot(own && (lane == 0 || dd[lane - 1] - dl > tol));
    zhp[lane] = zh;
    wave_lds_sync();
    // visit only the clusters with more than one member (usually none): each
    // holds a non-head index; the cluster runs from the last head at or below
    // it to the next head
    unsigned long long nonheads = __ballot(own) & ~heads;
    while (nonheads) {
      const int j0 = int(__builtin_ctzll(nonheads));
      const int s0 = 63 - int(__builtin_clzll(heads & ((2ull << j0) - 1ull)));
      const unsigned long long rest = heads >> j0;  // (bit j0 of heads is clear)
      const int e0 = rest ? min(p, j0 + int(__builtin_ctzll(rest))) : p;
      nonheads &= e0 >= 64 ? 0ull : (~0ull << e0);
      {
        double nrm2 = 0.0;
        for (int c = s0; c < e0; ++c) nrm2 += zhp[c] * zhp[c];
        if (nrm2 > 0.0) {
          const double nrm = nrm2 * rsq_nr(nrm2), z0 = zhp[s0];
          const double sg = z0 >= 0.0 ? 1.0 : -1.0;
          const double beta = 1.0 / (nrm * (nrm + fabs(z0)));
          if (lane >= s0 && lane < e0) uvec[lane] = lane == s0 ? z0 + sg * nrm : zhp[lane];
          wave_lds_sync();
          if (own) {  // V[r][cluster] <- V[r][cluster] (I - beta u u^T)
            double t = 0.0;
            for (int c = s0; c < e0; ++c) t += V[lane * kLd + c] * uvec[c];
            t *= beta;
            for (int c = s0; c < e0; ++c) V[lane * kLd + c] -= t * uvec[c];
          }
          if (lane >= s0 && lane < e0) zhp[lane] = lane == s0 ? -sg * nrm : 0.0;
          wave_lds_sync();
        }
      }
    }
    zh = zhp[lane];
    // active set: compaction by ballot (active indices first, in order)
    const bool act = own && rho2 > 0.0 && rho2 * fabs(zh) > tol;
    const unsigned long long am = __ballot(act), im = __ballot(own && !act);
    const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;
    const int pc = __popcll(am);
    if (act) {
      const int a = __popcll(am & below);
      perm[a] = lane;
      ddA[a] = dl;
      zzA[a] = zh * zh;
    } else if (own) {
      const int e = pc + __popcll(im & below);
      perm[e] = lane;
      vals[e] = dl;  // a kept eigenvalue
    }
    if (lane == 0) *npc = pc;
  }
  __syncthreads();
  mark(7);
  const int pc = *npc;
  const double rho2 = rsc[0];
  // ---- secular roots of the active set: 4 threads per root, each summing
  // every 4th term.  64-thread kernel (p <= 16): lanes 4i..4i+3 (shuffle
  // sums); 256-thread kernel: thread i of each wave (partials through LDS, W
  // is free here).  All 4 hold identical sums (fixed combine order), hence
  // identical iterates.
  constexpr int kSub = 4;
  const int root = NT == 64 ? lane >> 2 : lane;
  const int sub = NT == 64 ? lane & 3 : tid >> 6;
  const bool own = root < pc;
  auto combine = [&](double (&v)[4], int nq) {
    if constexpr (NT == 64) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (q < nq) {
          v[q] += __shfl_xor(v[q], 1, 64);
          v[q] += __shfl_xor(v[q], 2, 64);
        }
    } else {
      for (int q = 0; q < nq; ++q) W[(sub * 4 + q) * 64 + lane] = v[q];
      __syncthreads();
      for (int q = 0; q < nq; ++q)
        v[q] = (W[(0 * 4 + q) * 64 + lane] + W[(1 * 4 + q) * 64 + lane]) +
               (W[(2 * 4 + q) * 64 + lane] + W[(3 * 4 + q) * 64 + lane]);
      __syncthreads();
    }
  };
  int K = 0;
  double tau = 0.0, lo = 0.0, hi = rho2, dK = 0.0, Dp = 0.0;
  bool conv = !own;
  {
    // which pole is nearer: the sign of f at the interval's midpoint
    double v[4] = {0.0, 0.0, 0.0, 0.0};
    const double dr = own ? ddA[root] : 0.0;
    const double mid = root > 0 && own ? 0.5 * (dr + ddA[root - 1]) : 0.0;
    if (own && root > 0)
#pragma unroll 4
      for (int j = sub; j < pc; j += kSub) v[0] += zzA[j] * rcp_nr(ddA[j] - mid);
    combine(v, 1);
    if (own && root > 0) {
      if (1.0 + rho2 * v[0] > 0.0) {  // f increases: the root lies below mid, nearer pole D_i
        K = root;
        hi = mid - dr;
      } else {
        K = root - 1;
        lo = mid - ddA[root - 1];
        hi = 0.0;
      }
    }
    dK = own ? ddA[K] : 0.0;
    Dp = own && root > 0 ? ddA[root - 1] - dK : 0.0;
    // start from the one-pole estimate
    v[0] = 0.0;
    if (own)
#pragma unroll 4
      for (int j = sub; j < pc; j += kSub)
        if (j != K) v[0] += zzA[j] * rcp_nr(ddA[j] - dK);
    combine(v, 1);
    if (own) {
      const double t0 = rho2 * zzA[K] / (1.0 + rho2 * v[0]);
      tau = (t0 > lo && t0 < hi) ? t0 : 0.5 * (lo + hi);
    }
  }
  for (int it = 0; it < 48; ++it) {
    double v[4] = {0.0, 0.0, 0.0, 0.0};  // psi, psi', phi, phi'
    if (own && !conv)
#pragma unroll 4
      for (int j = sub; j < pc; j += kSub) {
        const double r = rcp_nr((ddA[j] - dK) - tau);
        const double t = zzA[j] * r;
        if (j >= root) {
          v[0] += t;
          v[1] += t * r;
        } else {
          v[2] += t;
          v[3] += t * r;
        }
      }
    combine(v, 4);
    if (own && !conv) {
      const double psi = rho2 * v[0], dpsi = rho2 * v[1], phi = rho2 * v[2], dphi = rho2 * v[3];
      const double f = 1.0 + psi + phi;
      if (f < 0.0) lo = tau;
      else hi = tau;
      if (fabs(f) <= 32.0 * __DBL_EPSILON__ * (1.0 + fabs(psi) + fabs(phi)) ||
          hi - lo <= 4.0 * __DBL_EPSILON__ * fmax(fabs(lo), fabs(hi))) {
        conv = true;
      } else {
        // psi ~ P / (Q - t) (poles at and below the interval), phi ~ R + S / (Dp - t)
        // (the model only proposes the next iterate -- the bracket and the
        // test on f above decide convergence -- so Newton reciprocals do)
        const double idp = rcp_nr(dpsi);
        const double qm = tau + psi * idp, pp = psi * psi * idp;
        double nt = 0.5 * (lo + hi);
        if (root == 0) {
          nt = qm + pp;
        } else {
          const double dt = Dp - tau;
          const double S = dphi * dt * dt, R = phi - S * rcp_nr(dt);
          const double a = 1.0 + R, b = -(a * (qm + Dp) + pp + S), c = a * qm * Dp + pp * Dp + S * qm;
          const double disc = b * b - 4.0 * a * c;
          if (a != 0.0 && disc > 0.0) {
            const double r1 = (-b - copysign(disc * rsq_nr(disc), b)) * rcp_nr(2.0 * a);
            const double r2 = r1 != 0.0 ? c * rcp_nr(a * r1) : r1;
            if (r1 > lo && r1 < hi) nt = r1;
            else if (r2 > lo && r2 < hi) nt = r2;
          }
        }
        tau = (nt > lo && nt < hi) ? nt : 0.5 * (lo + hi);
      }
    }
    if (!__syncthreads_or(!conv)) break;
  }
  if (own && sub == 0) {
    Ks[root] = K;
    taus[root] = tau;
    vals[root] = dK + tau;
  }
  if (!__syncthreads_or(!conv)) {
    // zt_a^2 = prod_k (lam_k - D_a) / prod_{k != a} (D_k - D_a) / rho'  (wave 0, lane a)
    if (tid < 64) {
      bool bad = false;
      if (lane < pc) {
        const double da = ddA[lane];
        double prod = ((ddA[Ks[lane]] - da) + taus[lane]) / rho2;
#pragma unroll 8
        for (int q = 0; q < pc; ++q)
          if (q != lane) prod *= ((ddA[Ks[q]] - da) + taus[q]) * rcp_nr(ddA[q] - da);
        bad = !(prod > 0.0) || !isfinite(prod);
        ztA[lane] = copysign(sqrt(fmax(prod, 0.0)), zhp[perm[lane]]);
      }
      if (__any(bad) && lane == 0) *flag = 0;
    }
  } else if (tid == 0) {
    *flag = 0;  // a root did not converge
  }
  __syncthreads();
  mark(8);
  if (!*flag) return false;
  // ---- Q (active block, columns unnormalised) -> W: Q[a][b] = zt_a / (D_a - lam_b)
  for (int e = tid; e < pc * pc; e += NT) {
    const int a = e / pc, b = e - a * pc;
    W[a * kLd + b] = ztA[a] / ((ddA[a] - ddA[Ks[b]]) - taus[b]);
  }
  __syncthreads();
  if (tid < pc) {
    double sq = 0.0;
#pragma unroll 8
    for (int a = 0; a < pc; ++a) {
      const double q = W[a * kLd + tid];
      sq += q * q;
    }
    inv_norm[tid] = rsq_nr(sq);
  }
  __syncthreads();
  mark(2);
  // ---- entries -> A's columns: e < pc the new vectors V[:, act] Q[:, e],
  // e >= pc the kept columns of V.  The product on the f64 matrix cores
  // (v_mfma_f64_16x16x4: lane l holds A[l&15][k = l>>4] and B[k = l>>4][l&15],
  // result rows (l>>4) + 4i of column l&15): 16x16 tiles over the waves, k
  // past pc fed as zeros; rows / columns past the ends read in-bounds LDS
  // garbage that reaches only results that are not stored.  (The 4x4
  // register-block VALU loop below is the kMahaMfmaGemm = false variant.)
  if (kMahaMfmaGemm) {
    const int tr = (p + 15) >> 4, tc = (pc + 15) >> 4;
    const int wave = tid >> 6, li = lane & 15, lk = lane >> 4;
    for (int t = wave; t < tr * tc; t += NT / 64) {
      const int r0 = (t / tc) * 16, c0 = (t - (t / tc) * tc) * 16;
      typedef double d4 __attribute__((ext_vector_type(4)));
      d4 acc = {0.0, 0.0, 0.0, 0.0}, acc2 = {0.0, 0.0, 0.0, 0.0};
      // 16 k per round: the operand loads first (independent), then four
      // MFMAs on two accumulators
      for (int k0 = 0; k0 < pc; k0 += 16) {
        double a[4], b[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int kk = k0 + 4 * u + lk;
          const int src = perm[min(kk, pc - 1)];
          a[u] = kk < pc ? V[(r0 + li) * kLd + src] : 0.0;
          b[u] = kk < pc ? W[kk * kLd + c0 + li] : 0.0;
        }
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[0], b[0], acc, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[1], b[1], acc2, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[2], b[2], acc, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[3], b[3], acc2, 0, 0, 0);
      }
      acc += acc2;
      const int col = c0 + li;
      if (col < pc) {
        const double sc = inv_norm[col];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = r0 + lk + 4 * i;
          if (row < p) A[row * kLdA + col] = acc[i] * sc;
        }
      }
    }
  }
  const int nr4 = (p + 3) >> 2, nc4 = kMahaMfmaGemm ? 0 : (pc + 3) >> 2;
  for (int e = tid; e < nr4 * nc4; e += NT) {
    const int r0 = (e / nc4) * 4, c0 = (e - (e / nc4) * nc4) * 4;
    double acc[4][4] = {};
#pragma unroll 2
    for (int q = 0; q < pc; ++q) {
      const int src = perm[q];
      double v[4], w[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) v[a] = V[(r0 + a) * kLd + src];
#pragma unroll
      for (int b = 0; b < 4; ++b) w[b] = W[q * kLd + c0 + b];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] += v[a] * w[b];
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b)
        if (r0 + a < p && c0 + b < pc) A[(r0 + a) * kLdA + c0 + b] = acc[a][b] * inv_norm[c0 + b];
  }
  for (int e = tid; e < p * (p - pc); e += NT) {
    const int r = e / (p - pc), c = pc + (e - r * (p - pc));
    A[r * kLdA + c] = V[r * kLd + perm[c]];
  }
  __syncthreads();
  // ---- descending order: the active roots (entries < pc) and the kept
  // eigenvalues (entries >= pc) are each already descending, so an entry's
  // rank is its place in its own list plus a binary search in the other
  // (ties: active first); eigenvalues and vectors land sorted (Ks is free
  // again: it holds the ranks)
  int* rank_of = Ks;
  if (tid < p) {
    const double ve = vals[tid];
    const bool is_act = tid < pc;
    // count of the other list's entries ranked above: active values >= ve
    // (for a kept entry) or kept values > ve (for an active one)
    int lo_i = is_act ? pc : 0, hi_i = is_act ? p : pc;  // search range [lo_i, hi_i)
    const int base = lo_i;
    while (lo_i < hi_i) {
      const int mid = (lo_i + hi_i) >> 1;
      const double vm = vals[mid];
      if (is_act ? vm > ve : vm >= ve) lo_i = mid + 1;
      else hi_i = mid;
    }
    rank_of[tid] = (is_act ? tid : tid - pc) + (lo_i - base);
  }
  __syncthreads();
  if (tid < p) lam_sorted[rank_of[tid]] = vals[tid];  // (inv_norm is done with)
  for (int e = tid; e < p * p; e += NT) {
    const int r = e / p, c = e - r * p;
    const double v = A[r * kLdA + c];
    V[r * kLd + rank_of[c]] = v;
    if (last) cache[r * p + rank_of[c]] = v;  // (invalidated below if the check fails)
  }
  __syncthreads();
  if (!last) return true;  // the next row's update starts from this basis
  // ---- every kTrackRefresh-th tracked step: one Newton-Schulz step
  // V <- V (3I - V^T V) / 2, which takes V's orthogonality error e to O(e^2)
  // (products of Gu-Eisenstat Q's drift by ~eps per step).  It replaces the
  // periodic cold Jacobi re-solve (2 ms at p = 64, 25x a tracked step:
  // profiles/r04c_maha) at the cost of two p^3 MFMA products; the residual
  // check below then validates the refreshed basis, and a failure still
  // falls back to Jacobi.
  const bool refresh = tail[1] + 1.0 >= double(kTrackRefresh);  // (uniform: every thread reads the same word)
  if (refresh) {
    mfma_gemm_lds<NT, true>(V, kLd, V, kLd, W, kLd, p, p, p);  // G = V^T V
    __syncthreads();
    for (int e = tid; e < p * p; e += NT) {
      const int r = e / p, c = e - r * p;
      W[r * kLd + c] = (r == c ? 1.5 : 0.0) - 0.5 * W[r * kLd + c];
    }
    __syncthreads();
    mfma_gemm_lds<NT, false>(V, kLd, W, kLd, A, kLdA, p, p, p);  // V (3I - G) / 2
    __syncthreads();
    for (int e = tid; e < p * p; e += NT) {
      const int r = e / p, c = e - r * p;
      const double v = A[r * kLdA + c];
      V[r * kLd + c] = v;
      cache[r * p + c] = v;
    }
    __syncthreads();
  }
  // ---- residual of the top-k pairs against the new covariance, R = C_new
  // V[:, 0:16] on the f64 matrix cores (one 16-row tile per wave; columns
  // past k and rows past p are computed but not summed)
  double res = 0.0;
  {
    const int wave = tid >> 6, li = lane & 15, lk = lane >> 4;
    for (int r0 = wave * 16; r0 < p; r0 += (NT / 64) * 16) {
      typedef double d4 __attribute__((ext_vector_type(4)));
      d4 acc = {0.0, 0.0, 0.0, 0.0};
      for (int k0 = 0; k0 < p; k0 += 4) {
        const int kk = k0 + lk;
        const double a = kk < p ? Cn[(r0 + li) * kLd + kk] : 0.0;
        const double b = kk < p ? V[kk * kLd + li] : 0.0;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
      }
      if (li < k)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = r0 + lk + 4 * i;
          if (row < p) {
            const double d = acc[i] - lam_sorted[li] * V[row * kLd + li];
            res += d * d;
          }
        }
    }
  }
  res = block_sum<NT>(res, red);
  const double lim = 1e-11 * fabs(lam_sorted[0]);
  if (!(res <= lim * lim)) {  // (uniform: every thread holds the block sum)
    if (tid == 0) tail[0] = -1.0;  // the cache already holds this basis: the re-solve starts cold
    __syncthreads();
    return false;
  }
  if (tid < p) lam_cache[tid] = lam_sorted[tid];
  if (tid < k) sel[tid] = tid;
  if (tid == 0) tail[1] = refresh ? 0.0 : tail[1] + 1.0;  // steps since the last refresh (tail[0] = p already)
  __syncthreads();
  mark(9);
  return true;
}

// Sherman-Morrison scores for k <= 4 on one lane (CoreMahalanobis.py:118-146,
// the same recurrence as the LDS path below): P, C^-1 and the per-row
// updates live in registers as padded 4 x 4 matrices (identity block past
// k, so determinants and inverses of the k x k block are unchanged).  The
// LDS path costs ~60 dependent LDS round trips (60-90 clocks each) per
// inversion plus a barrier per step.
__device__ void sm_scores_small(const double* __restrict__ Pin, const double* __restrict__ XD,
                                const double* __restrict__ DPC, int nb, int k, double n, const MahaParams& prm,
                                double* __restrict__ scores) {
  double P[4][4], C[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      P[r][c] = r < k && c < k ? Pin[r * k + c] : (r == c ? 1.0 : 0.0);
      C[r][c] = 0.0;
    }
  bool valid = false;
  for (int i = 0; i < nb; ++i) {
    double d[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) d[r] = r < k ? XD[size_t(i) * k + r] : 0.0;
    if (!valid) {
      // Gauss-Jordan, first maximal pivot per column (as invert_into)
      double M[4][4], I[4][4];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          M[r][c] = P[r][c];
          I[r][c] = r == c ? 1.0 : 0.0;
        }
      double det = 1.0;
      bool sing = false;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        int piv = c;
        double best = fabs(M[c][c]);
#pragma unroll
        for (int r = c + 1; r < 4; ++r)
          if (fabs(M[r][c]) > best) {
            best = fabs(M[r][c]);
            piv = r;
          }
        sing |= best == 0.0;
#pragma unroll
        for (int r = c + 1; r < 4; ++r)
          if (piv == r) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              double t = M[c][j];
              M[c][j] = M[r][j];
              M[r][j] = t;
              t = I[c][j];
              I[c][j] = I[r][j];
              I[r][j] = t;
            }
            det = -det;
          }
        const double dd = M[c][c];
        det *= dd;
        const double id = sing ? 0.0 : 1.0 / dd;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          M[c][j] *= id;
          I[c][j] *= id;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (r == c) continue;
          const double f = M[r][c];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            M[r][j] -= f * M[c][j];
            I[r][j] -= f * I[c][j];
          }
        }
      }
      if (!sing && fabs(det) > prm.eps) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int c = 0; c < 4; ++c) C[r][c] = I[r][c];
        valid = true;
      } else {
        if (n + i != 0.0) {
          const double a = (n + i - 1.0) / (n + i), cb = 1.0 / (n + i + 1.0);
          double dp[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) dp[r] = r < k ? DPC[size_t(i) * k + r] : 0.0;
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c)
              if (r < k && c < k) P[r][c] = a * P[r][c] + cb * dp[r] * dp[c];
        }
        scores[i] = prm.out_mode == 1 ? (0.0 > prm.threshold ? 1.0 : 0.0) : 0.0;
        continue;
      }
    } else {
      const double a = (n + i - 1.0) / (n + i - 2.0), cb = 1.0 / (n + i);  // B_{i-1} = dpc dpc^T / (n + i)
      double dp[4], T2[4][4];
#pragma unroll
      for (int r = 0; r < 4; ++r) dp[r] = r < k ? DPC[size_t(i - 1) * k + r] : 0.0;
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) C[r][c] *= a;  // c_inv = a C (in place)
      double tr = 0.0;
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          double s = 0.0;
#pragma unroll
          for (int j = 0; j < 4; ++j) s += (cb * dp[r] * dp[j]) * C[j][c];
          T2[r][c] = s;
          if (r == c) tr += s;
        }
      const double scal = 1.0 / (1.0 + tr);
#pragma unroll
      for (int r = 0; r < 4; ++r) {  // row r of c_inv - scal c_inv BC1 needs only row r of c_inv
        double row[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          double s = 0.0;
#pragma unroll
          for (int j = 0; j < 4; ++j) s += C[r][j] * T2[j][c];
          row[c] = C[r][c] - scal * s;
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) C[r][c] = row[c];
      }
    }
    double part = 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) part += d[r] * C[r][c] * d[c];
    scores[i] = prm.out_mode == 1 ? (part > prm.threshold ? 1.0 : 0.0) : part;
  }
}

// One request's step (CoreMahalanobis._get_preds for X [nb][p]) against the
// state in HBM; called once per segment by maha_step_kernel.  Callers
// __syncthreads() between calls: the next segment reads the state this one
// wrote (same workgroup, same CU: its L1 is coherent at workgroup scope).
template <int NT>
__device__ void maha_one(const double* __restrict__ X, int nb, const MahaParams& prm, double* __restrict__ state,
                         double* __restrict__ eig, double* __restrict__ ws, double* __restrict__ scores) {
  __shared__ double A[kMahaMaxP * kLdA], V[kMahaMaxP * kLd], W[kMahaMaxP * kLd], Tm[kMahaMaxP * kLd];
  __shared__ double mean0[kMahaMaxP];
  __shared__ EigScratch es;
  __shared__ double red[NT / 64];
  __shared__ int sel[kMahaMaxK];
  __shared__ double P[kMahaMaxK * kMahaMaxK], Cp[kMahaMaxK * kMahaMaxK], T1[kMahaMaxK * kMahaMaxK],
      T2[kMahaMaxK * kMahaMaxK];
  __shared__ int valid, inverted, r1flag, track;
  __shared__ double scal;
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
  // (unrolled: several of the state's HBM loads in flight per thread)
#pragma unroll 4
  for (int e = tid; e < m * m; e += NT) {
    const int a = e / m, b = e - a * m;
    double cov = 0.0;
    if (a < p && b < p) {  // dummy index of an odd p stays 0
      double acc = 0.0;
      for (int i = 0; i < nb; ++i)
        acc += ((n + i) / (n + i + 1.0)) * (D[size_t(i) * p + a] * D[size_t(i) * p + b]);
      cov = (n - 1.0) / den * (c_zero ? 0.0 : s_C[a * p + b]) + 1.0 / den * acc;
    }
    A[a * kLdA + b] = cov;
    Tm[a * kLd + b] = cov;  // kept: written to the state after the projections
  }
  __syncthreads();
  stamp(1);
  const uint64_t c_eig0 = __builtin_amdgcn_s_memtime(), r_eig0 = __builtin_amdgcn_s_memrealtime();
  const bool tracked = p <= prm.rank1_max_p || p <= prm.jacobi_max_p;
  if (tracked) {
    double* tail = eig + kMahaEigTail;
    bool done = false;
    // The branch below has barriers: decided by ONE thread from the cache
    // words (global memory) and broadcast, so every wave takes it or none.
    if (tid == 0)
      track = p <= prm.rank1_max_p && nb <= kTrackMaxRows && !c_zero && tail[0] == double(p) &&
               eig[kMahaEigMeta] == n_state;  // (the periodic refresh happens inside the tracked step)
    __syncthreads();
    if (track) {
      // C_new = alpha C_old + sum_i c_i / den d_i d_i^T: one rank-1 update per row
      done = true;
      for (int i = 0; i < nb && done; ++i)
        done = rank1_eigen<NT>(D + size_t(i) * p, i == 0 ? (n - 1.0) / den : 1.0, ((n + i) / (n + i + 1.0)) / den, p,
                               k, Tm, A, V, W, es, sel, eig, tail, eig + kMahaEigLam, red, &r1flag, i == 0,
                               i == nb - 1, ph);
      if (tid == 0) eig[kMahaEigMeta + (done ? 1 : 2)] += 1.0;
      if (!done) {  // A held V_new: the new covariance back for the re-solve
        for (int e = tid; e < m * m; e += NT) A[(e / m) * kLdA + e % m] = Tm[(e / m) * kLd + e % m];
        __syncthreads();
      }
    }
    if (!done) {
      // warm or cold: decided by one thread from the cache words (the solve has barriers)
      if (tid == 0)
        track = tail[0] == double(p) && tail[1] < double(p <= prm.rank1_max_p ? kTrackRefresh : kJacobiRefresh);
      __syncthreads();
      jacobi_solve<NT>(A, V, W, sel, p, k, eig, tail, es.dg, eig + kMahaEigLam, track != 0, eig + kMahaEigMeta + 3);
    }
  } else if (NT >= 256 && p >= prm.mw_min_p) {
    topk_wave(A, V, W, es, sel, p, k, ph, 4);
  } else if (tid < 64) {
    topk_wave(A, V, W, es, sel, p, k, ph, 1);
  }
  __syncthreads();
  stamp(3);
  if (tid == 0) {  // shader-clock cycles and 100 MHz ticks of the eigen phase (effective clock)
    double* tail = eig + kMahaEigTail;
    tail[2] += double(__builtin_amdgcn_s_memtime() - c_eig0);
    tail[4] += double(__builtin_amdgcn_s_memrealtime() - r_eig0);
    tail[3] += 1.0;
  }
  // ---- projections; proj_cov = V^T C_old V over the selected columns:
  // C_old (still in HBM) -> W, U = C_old V_sel -> A (free after the
  // selection), P = V_sel^T U
#pragma unroll 4
  for (int e = tid; e < p * p; e += NT) W[(e / p) * kLd + e % p] = c_zero ? 0.0 : s_C[e];
  __syncthreads();
  for (int e = tid; e < p * k; e += NT) {
    const int r = e / k, b = e - r * k;
    const double* vb = V + sel[b];
    double t = 0.0;
    for (int c = 0; c < p; ++c) t += W[r * kLd + c] * vb[c * kLd];
    A[r * kLdA + b] = t;
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
    for (int r = 0; r < p; ++r) acc += va[r * kLd] * A[r * kLdA + b];
    P[e] = acc;
  }
  if (tid == 0) valid = 0;
  __syncthreads();
  stamp(4);
  // new covariance into the state (the projections above read the old one)
  for (int e = tid; e < p * p; e += NT) s_C[e] = Tm[(e / p) * kLd + e % p];
  // ---- Sherman-Morrison scores (sequential in rows)
  if (k <= 4) {
    if (tid == 0) sm_scores_small(P, XD, DPC, nb, k, n, prm, scores);
    __syncthreads();
  }
  for (int i = 0; i < (k <= 4 ? 0 : nb); ++i) {
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
    // the cached eigendecomposition now describes the state's new covariance
    eig[kMahaEigMeta] = (p <= prm.rank1_max_p || p <= prm.jacobi_max_p) ? n_new : -1.0;
    double* acc = eig + kMahaEigTail + 5;
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
