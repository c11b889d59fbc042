// Linear / logistic-regression predict (reference
// servers/sklearnserver/sklearnserver/SKLearnServer.py:32-42 which calls
// sklearn's predict_proba on the CPU for every request).
//
// Three CDNA4 mappings, chosen by shape on the host:
//  * thread-per-row: tiny K*C (iris: K=4, C=3).  W, b and the per-thread
//    logits live in LDS; a 64-wide wave covers 64 requests of a micro-batch.
//  * wave-per-row: larger K, small batches.  Lanes stride K (coalesced row
//    reads), each class logit is a 64-lane shuffle reduction.
//  * MFMA: large batches / wide models (rows*K*C >= 2^20, C <= 1024): the
//    logits GEMM on v_mfma_f64_16x16x4 with the activation fused.
// fp64 throughout so results match sklearn bit-for-bit up to summation order.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "kernels.h"

namespace sca::kern {
namespace {

constexpr int kBlock = 256;
constexpr int kMaxThreadC = 16;
constexpr int kMaxLdsDoubles = 6144;  // 48 KiB for W + b in the thread path

__device__ inline double sigmoid(double z) { return 1.0 / (1.0 + exp(-z)); }

template <int ACT>
__device__ inline void finish_row(double* logit, int C, double* out_row) {
  if constexpr (ACT == kActIdentity) {
    for (int c = 0; c < C; ++c) out_row[c] = logit[c];
  } else if constexpr (ACT == kActSoftmax) {
    double m = logit[0];
    for (int c = 1; c < C; ++c) m = fmax(m, logit[c]);
    double s = 0.0;
    for (int c = 0; c < C; ++c) { logit[c] = exp(logit[c] - m); s += logit[c]; }
    const double inv = 1.0 / s;
    for (int c = 0; c < C; ++c) out_row[c] = logit[c] * inv;
  } else if constexpr (ACT == kActBinaryLogistic) {
    const double p = sigmoid(logit[0]);
    out_row[0] = 1.0 - p;
    out_row[1] = p;
  } else if constexpr (ACT == kActOvr) {
    double s = 0.0;
    for (int c = 0; c < C; ++c) { logit[c] = sigmoid(logit[c]); s += logit[c]; }
    const double inv = 1.0 / s;
    for (int c = 0; c < C; ++c) out_row[c] = logit[c] * inv;
  } else {
    for (int c = 0; c < C; ++c) out_row[c] = sigmoid(logit[c]);
  }
}

template <int ACT>
__global__ __launch_bounds__(kBlock) void linear_thread_rows(const double* __restrict__ X, int rows, int K,
                                                             const double* __restrict__ W,
                                                             const double* __restrict__ b, int C,
                                                             double* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  double* sW = lds;                          // [C*K]
  double* sb = sW + C * K;                   // [C]
  double* sLogit = sb + C;                   // [kBlock * C]
  for (int i = threadIdx.x; i < C * K; i += kBlock) sW[i] = W[i];
  for (int i = threadIdx.x; i < C; i += kBlock) sb[i] = b ? b[i] : 0.0;
  __syncthreads();
  const int r = blockIdx.x * kBlock + threadIdx.x;
  if (r >= rows) return;
  const double* x = X + size_t(r) * K;
  double* logit = sLogit + threadIdx.x * C;
  for (int c = 0; c < C; ++c) logit[c] = sb[c];
  for (int k = 0; k < K; ++k) {
    const double xv = x[k];
    for (int c = 0; c < C; ++c) logit[c] = fma(xv, sW[c * K + k], logit[c]);
  }
  const int out_cols = ACT == kActBinaryLogistic ? 2 : C;
  finish_row<ACT>(logit, C, out + size_t(r) * out_cols);
}

__device__ inline double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

template <int ACT>
__global__ __launch_bounds__(kBlock) void linear_wave_rows(const double* __restrict__ X, int rows, int K,
                                                           const double* __restrict__ W,
                                                           const double* __restrict__ b, int C,
                                                           double* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double* logit = lds + wave * C;
  const int r = blockIdx.x * (kBlock / 64) + wave;
  if (r >= rows) return;
  const double* x = X + size_t(r) * K;
  for (int c = 0; c < C; ++c) {
    const double* w = W + size_t(c) * K;
    double acc = 0.0;
    for (int k = lane; k < K; k += 64) acc = fma(x[k], w[k], acc);
    acc = wave_sum(acc);
    if (lane == 0) logit[c] = acc + (b ? b[c] : 0.0);
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  if (lane == 0) {
    const int out_cols = ACT == kActBinaryLogistic ? 2 : C;
    finish_row<ACT>(logit, C, out + size_t(r) * out_cols);
  }
}

// ---------------------------------------------------------------- MFMA path
// Large batches and wide models (rows * K * C >= 2^20, C <= 1024): the
// logits tile is a GEMM on the fp64 matrix cores, v_mfma_f64_16x16x4 --
// A = 16 rows of X x 4 k, B = 4 k x 16 classes of W^T, result lane l holds
// rows (l>>4) + 4i of column l&15 -- with bias + softmax / sigmoid fused into
// the epilogue, so logits never reach HBM.
//
// One workgroup (4 waves) owns 16 rows and EVERY class, so the row
// normaliser needs no second pass: the waves split the classes (CW waves x
// NCT 16-column tiles each) and the rest of the factor 4 splits K (KS = 4 /
// CW slices, partial logits summed through LDS).  Operands come straight
// from global memory as 32-byte vectors: lane group g = l>>4 reads k = 4g..4g+3
// of its row / class for a 16-k chunk and feeds them to the chunk's 4 MFMAs
// as k-step s = 0..3 -- the k order inside a chunk is permuted identically in
// A and B, so the dot products are exact sums of the same terms.  K past the
// end (and classes past C) are fed as zeros.
using f64x4 = __attribute__((ext_vector_type(4))) double;

// NCT 16-column tiles x RT 16-row tiles per wave; CW waves split the classes
// and KS waves split K (KS > 1 only with CW == 1); a workgroup owns 16 RT rows
// and every class.
template <int ACT, int NCT, int CW, int KS, int RT, int G>
__global__ __launch_bounds__(64 * CW * KS) void linear_mfma_rows(const double* __restrict__ X, int rows, int K,
                                                                 const double* __restrict__ W,
                                                                 const double* __restrict__ b, int C,
                                                                 double* __restrict__ out) {
  static_assert(KS == 1 || CW == 1, "split K or split classes");
  constexpr int R = 16 * RT;                 // rows per workgroup
  __shared__ double red[KS > 1 ? (KS - 1) * NCT * RT * 4 * 64 : 1];  // partial logits of slices 1..KS-1
  __shared__ double rowst[CW][R];            // per-wave row max / sum
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int cw = wave % CW, ks = wave / CW;
  const int li = lane & 15, g = lane >> 4;
  const int r0 = blockIdx.x * R;
  const int col0 = cw * NCT * 16;            // first class of this wave
  const int chunks = (K + 15) >> 4;          // K in 16-k chunks, split over the KS slices
  const int per = (chunks + KS - 1) / KS;
  const int c_begin = ks * per, c_end = min(chunks, c_begin + per);
  // P accumulator sets: a 1-2 tile wave alternates two sets by k-step so
  // consecutive MFMAs are independent (a dependent MFMA waits out the whole
  // latency of the one before)
  constexpr int P = NCT * RT <= 2 ? 2 : 1;
  f64x4 acc[RT][NCT], acc2[P > 1 ? RT : 1][P > 1 ? NCT : 1];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int t = 0; t < NCT; ++t) acc[rt][t] = f64x4{0.0, 0.0, 0.0, 0.0};
  if constexpr (P > 1)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int t = 0; t < NCT; ++t) acc2[rt][t] = f64x4{0.0, 0.0, 0.0, 0.0};
  const bool vec = (K & 3) == 0;             // rows 32-byte aligned: vector loads
  auto load4 = [&](const double* p, bool ok, int k, double* v) {
    if (ok && vec && k + 3 < K) {
      const double2 lo = *reinterpret_cast<const double2*>(p + k);
      const double2 hi = *reinterpret_cast<const double2*>(p + k + 2);
      v[0] = lo.x; v[1] = lo.y; v[2] = hi.x; v[3] = hi.y;
    } else {
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) v[s2] = (ok && k + s2 < K) ? p[k + s2] : 0.0;
    }
  };
  // Chunks go in groups of G: the group's loads are issued together, then its
  // MFMAs -- narrow tiles (the memory-bound shapes) keep several chunks' loads
  // in flight per wave instead of one 2 KB round trip at a time.
  for (int c0 = c_begin; c0 < c_end; c0 += G) {
    double a[G][RT][4], w[G][NCT][4];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const int c = c0 + u;
      const bool live = c < c_end;
      const int k = (c << 4) + (g << 2);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const int row = r0 + rt * 16 + li;   // the A row this lane reads
        load4(X + size_t(row < rows ? row : 0) * K, live && row < rows, k, a[u][rt]);
      }
#pragma unroll
      for (int t = 0; t < NCT; ++t) {
        const int j = col0 + t * 16 + li;    // the B column (class) this lane reads
        load4(W + size_t(j < C ? j : 0) * K, live && j < C, k, w[u][t]);
      }
    }
    // (class tile, k-step, row tile): a W fragment feeds its RT MFMAs back to
    // back (k-step outermost measured the same at 8192 x 256 -> 1000: 139.7
    // vs 136-140 us, profiles/r06m_linear_split)
#pragma unroll
    for (int u = 0; u < G; ++u)
#pragma unroll
      for (int t = 0; t < NCT; ++t)
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
          for (int rt = 0; rt < RT; ++rt) {
            if constexpr (P > 1) {
              if (s2 & 1) {
                acc2[rt][t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u][rt][s2], w[u][t][s2], acc2[rt][t], 0, 0, 0);
                continue;
              }
            }
            acc[rt][t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u][rt][s2], w[u][t][s2], acc[rt][t], 0, 0, 0);
          }
  }
  if constexpr (P > 1)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int t = 0; t < NCT; ++t) acc[rt][t] += acc2[rt][t];
  if constexpr (KS > 1) {  // slices 1.. hand their partial logits to slice 0
    if (ks > 0) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int t = 0; t < NCT; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            red[((((size_t(ks - 1) * RT + rt) * NCT + t) * 4) + i) * 64 + lane] = acc[rt][t][i];
    }
    __syncthreads();
    if (ks > 0) return;
#pragma unroll
    for (int q = 0; q < KS - 1; ++q)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int t = 0; t < NCT; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[rt][t][i] += red[((((size_t(q) * RT + rt) * NCT + t) * 4) + i) * 64 + lane];
  }
  // ---- epilogue: lane holds rows 16 rt + g + 4i of columns col0 + 16t + li
#pragma unroll
  for (int t = 0; t < NCT; ++t) {
    const int j = col0 + t * 16 + li;
    const double bj = (b && j < C) ? b[j] : 0.0;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[rt][t][i] += bj;
  }
  const int out_cols = ACT == kActBinaryLogistic ? 2 : C;
  if constexpr (ACT == kActSoftmax || ACT == kActOvr) {
    // row normaliser over every class: lanes (16 per row group), then waves
    double m[RT][4], ssum[RT][4];
    if constexpr (ACT == kActSoftmax) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          double v = -__builtin_inf();
#pragma unroll
          for (int t = 0; t < NCT; ++t) v = (col0 + t * 16 + li) < C ? fmax(v, acc[rt][t][i]) : v;
#pragma unroll
          for (int off = 1; off < 16; off <<= 1) v = fmax(v, __shfl_xor(v, off, 64));
          m[rt][i] = v;
        }
      if constexpr (CW > 1) {
        if (li == 0)
#pragma unroll
          for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int i = 0; i < 4; ++i) rowst[cw][rt * 16 + g + 4 * i] = m[rt][i];
        __syncthreads();
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            double v = rowst[0][rt * 16 + g + 4 * i];
#pragma unroll
            for (int q = 1; q < CW; ++q) v = fmax(v, rowst[q][rt * 16 + g + 4 * i]);
            m[rt][i] = v;
          }
        __syncthreads();
      }
    }
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        double v = 0.0;
#pragma unroll
        for (int t = 0; t < NCT; ++t) {
          const int j = col0 + t * 16 + li;
          const double e = ACT == kActSoftmax ? exp(acc[rt][t][i] - m[rt][i]) : sigmoid(acc[rt][t][i]);
          acc[rt][t][i] = e;
          v += j < C ? e : 0.0;
        }
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) v += __shfl_xor(v, off, 64);
        ssum[rt][i] = v;
      }
    if constexpr (CW > 1) {
      if (li == 0)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int i = 0; i < 4; ++i) rowst[cw][rt * 16 + g + 4 * i] = ssum[rt][i];
      __syncthreads();
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          double v = 0.0;
#pragma unroll
          for (int q = 0; q < CW; ++q) v += rowst[q][rt * 16 + g + 4 * i];
          ssum[rt][i] = v;
        }
    }
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = r0 + rt * 16 + g + 4 * i;
        if (r >= rows) continue;
        const double inv = 1.0 / ssum[rt][i];
#pragma unroll
        for (int t = 0; t < NCT; ++t) {
          const int j = col0 + t * 16 + li;
          if (j < C) out[size_t(r) * out_cols + j] = acc[rt][t][i] * inv;
        }
      }
  } else {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = r0 + rt * 16 + g + 4 * i;
        if (r >= rows) continue;
#pragma unroll
        for (int t = 0; t < NCT; ++t) {
          const int j = col0 + t * 16 + li;
          if (j >= C) continue;
          const double z = acc[rt][t][i];
          if constexpr (ACT == kActIdentity) {
            out[size_t(r) * out_cols + j] = z;
          } else if constexpr (ACT == kActBinaryLogistic) {
            const double p = sigmoid(z);
            out[size_t(r) * 2] = 1.0 - p;
            out[size_t(r) * 2 + 1] = p;
          } else {
            out[size_t(r) * out_cols + j] = sigmoid(z);
          }
        }
      }
  }
}

// Shape rule of the MFMA path (also exported for the host's choice / tests).
bool mfma_eligible(int rows, int K, int C) {
  if (const char* e = std::getenv("SCA_LINEAR_MFMA")) {
    if (std::atoi(e) == 0) return false;
    if (std::atoi(e) == 2) return C <= 1024;  // forced on (tests, A/B)
  }
  return C <= 1024 && double(rows) * K * C >= double(1 << 20);
}

template <int ACT, int NCT, int CW, int KS, int RT, int G = (NCT * RT <= 2 ? 4 : 1)>
void launch_mfma_t(const double* X, int rows, int K, const double* W, const double* b, int C, double* out,
                   hipStream_t s, hipEvent_t stop);

// `stop` (optional) is completed by the kernel's own dispatch packet
// (hipExtLaunchKernelGGL): one HIP call per batch instead of launch +
// hipEventRecord (2.1 + 2.6 us of host time, tools/micro/launch_cost.hip).
template <class... Args, class... P>
void launch_maybe_ext(void (*k)(Args...), dim3 grid, dim3 block, size_t lds, hipStream_t s, hipEvent_t stop,
                      P... args) {
  if (stop) hipExtLaunchKernelGGL(k, grid, block, uint32_t(lds), s, nullptr, stop, 0, args...);
  else hipLaunchKernelGGL(k, grid, block, lds, s, args...);
}

template <int ACT, int NCT, int CW, int KS, int RT, int G>
void launch_mfma_t(const double* X, int rows, int K, const double* W, const double* b, int C, double* out,
                   hipStream_t s, hipEvent_t stop) {
  constexpr int R = 16 * RT;
  launch_maybe_ext(linear_mfma_rows<ACT, NCT, CW, KS, RT, G>, dim3((rows + R - 1) / R), dim3(64 * CW * KS), 0, s, stop,
                   X, rows, K, W, b, C, out);
}

// ---------------------------------------------------------- wide softmax
// Wide softmax models (C > 256 classes) at large batches.  linear_mfma_rows
// keeps every class of a row in one workgroup's registers, which caps a
// workgroup at 32 rows: each W fragment then feeds only 32 rows, and W is
// re-read from L2 rows / 32 times (8192 x 256 -> 1000: 512 MB for a 2 MB W).
// Here a workgroup owns a 64-row x 128-class tile (2 x 2 waves, each 32 rows
// x 64 classes: 8 independent MFMA chains, next chunk's operands prefetched),
// so W is re-read rows / 64 times and X C / 128 times, and the grid has
// (rows / 64) x (C / 128) workgroups instead of rows / 32.  The softmax is
// split: a tile writes exp(z - m_tile) and its rows' (m_tile, s_tile); then
// either a second launch rescales every row by exp(m_tile - M) / S (variant
// 2), or -- variant 1 -- the tiles store with write-through (agent-scope)
// stores and the last of a row tile's class-group workgroups (one arrival
// counter per row tile) folds and rescales the row tile in place with
// coherent loads, the tree kernels' last-arriver protocol.
constexpr int kWideRows = 64, kWideCols = 128;

__device__ __forceinline__ void wide_store(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double wide_load(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool FOLD>
__global__ __launch_bounds__(256) void linear_mfma_wide_softmax(const double* __restrict__ X, int rows, int K,
                                                                const double* __restrict__ W,
                                                                const double* __restrict__ b, int C,
                                                                double* __restrict__ out, double* __restrict__ ms,
                                                                int* __restrict__ counter) {
  constexpr int RT = 2, NCT = 4;
  __shared__ double s_red[2][kWideRows];               // per class-wave row max / sum
  __shared__ double s_fac[kWideRows][8];               // fixup: per row, per class group factor
  __shared__ int s_last;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wave >> 1, wc = wave & 1;
  const int li = lane & 15, g = lane >> 4;
  const int tile_r0 = blockIdx.x * kWideRows;
  const int r0 = tile_r0 + wr * 32;
  const int grp = blockIdx.y, groups = gridDim.y;
  const int col0 = grp * kWideCols + wc * 64;
  f64x4 acc[RT][NCT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int t = 0; t < NCT; ++t) acc[rt][t] = f64x4{0.0, 0.0, 0.0, 0.0};
  const bool vec = (K & 3) == 0;
  auto load4 = [&](const double* p, bool ok, int k, double* v) {
    if (ok && vec && k + 3 < K) {
      const double2 lo = *reinterpret_cast<const double2*>(p + k);
      const double2 hi = *reinterpret_cast<const double2*>(p + k + 2);
      v[0] = lo.x; v[1] = lo.y; v[2] = hi.x; v[3] = hi.y;
    } else {
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) v[s2] = (ok && k + s2 < K) ? p[k + s2] : 0.0;
    }
  };
  const int chunks = (K + 15) >> 4;
  constexpr int G = 2;  // chunks whose loads are in flight together
  for (int c0 = 0; c0 < chunks; c0 += G) {
    double a[G][RT][4], w[G][NCT][4];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const bool live = c0 + u < chunks;
      const int k = ((c0 + u) << 4) + (g << 2);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const int row = r0 + rt * 16 + li;
        load4(X + size_t(row < rows ? row : 0) * K, live && row < rows, k, a[u][rt]);
      }
#pragma unroll
      for (int t = 0; t < NCT; ++t) {
        const int j = col0 + t * 16 + li;
        load4(W + size_t(j < C ? j : 0) * K, live && j < C, k, w[u][t]);
      }
    }
#pragma unroll
    for (int u = 0; u < G; ++u)
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
        for (int t = 0; t < NCT; ++t)
#pragma unroll
          for (int rt = 0; rt < RT; ++rt)
            acc[rt][t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u][rt][s2], w[u][t][s2], acc[rt][t], 0, 0, 0);
  }
  // ---- tile softmax: lane holds rows 16 rt + g + 4i (of the wave's 32) of
  // classes col0 + 16 t + li
#pragma unroll
  for (int t = 0; t < NCT; ++t) {
    const int j = col0 + t * 16 + li;
    const double bj = (b && j < C) ? b[j] : 0.0;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[rt][t][i] += bj;
  }
  double m[RT][4], ssum[RT][4];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      double v = -__builtin_inf();
#pragma unroll
      for (int t = 0; t < NCT; ++t) v = (col0 + t * 16 + li) < C ? fmax(v, acc[rt][t][i]) : v;
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) v = fmax(v, __shfl_xor(v, off, 64));
      m[rt][i] = v;
    }
  if (li == 0)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) s_red[wc][wr * 32 + rt * 16 + g + 4 * i] = m[rt][i];
  __syncthreads();
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int lr = wr * 32 + rt * 16 + g + 4 * i;
      m[rt][i] = fmax(s_red[0][lr], s_red[1][lr]);
    }
  __syncthreads();
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      double v = 0.0;
#pragma unroll
      for (int t = 0; t < NCT; ++t) {
        const bool in = (col0 + t * 16 + li) < C;
        const double e = in ? exp(acc[rt][t][i] - m[rt][i]) : 0.0;
        acc[rt][t][i] = e;
        v += e;
      }
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) v += __shfl_xor(v, off, 64);
      ssum[rt][i] = v;
    }
  if (li == 0)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) s_red[wc][wr * 32 + rt * 16 + g + 4 * i] = ssum[rt][i];
  __syncthreads();
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int lr = wr * 32 + rt * 16 + g + 4 * i;
      const int r = tile_r0 + lr;
      if (r >= rows) continue;
#pragma unroll
      for (int t = 0; t < NCT; ++t) {
        const int j = col0 + t * 16 + li;
        if (j < C) {
          if constexpr (FOLD) wide_store(out + size_t(r) * C + j, acc[rt][t][i]);
          else out[size_t(r) * C + j] = acc[rt][t][i];
        }
      }
      if (wc == 0 && li == 0) {  // the tile's (max, sum) of this row
        if constexpr (FOLD) {
          wide_store(ms + (size_t(r) * groups + grp) * 2, m[rt][i]);
          wide_store(ms + (size_t(r) * groups + grp) * 2 + 1, s_red[0][lr] + s_red[1][lr]);
        } else {
          ms[(size_t(r) * groups + grp) * 2] = m[rt][i];
          ms[(size_t(r) * groups + grp) * 2 + 1] = s_red[0][lr] + s_red[1][lr];
        }
      }
    }
  if constexpr (!FOLD) return;  // linear_wide_softmax_fix rescales after this launch
  // ---- last of the row tile's class groups: fold and rescale
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // stores acknowledged at the coherence point
  __syncthreads();
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(counter + blockIdx.x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             groups - 1;
  __syncthreads();
  if (!s_last) return;
  if (threadIdx.x < kWideRows) {
    const int r = tile_r0 + threadIdx.x;
    if (r < rows) {
      double M = -__builtin_inf();
      for (int q = 0; q < groups; ++q) M = fmax(M, wide_load(ms + (size_t(r) * groups + q) * 2));
      double S = 0.0;
      for (int q = 0; q < groups; ++q)
        S += wide_load(ms + (size_t(r) * groups + q) * 2 + 1) * exp(wide_load(ms + (size_t(r) * groups + q) * 2) - M);
      for (int q = 0; q < groups; ++q) s_fac[threadIdx.x][q] = exp(wide_load(ms + (size_t(r) * groups + q) * 2) - M) / S;
    }
  }
  __syncthreads();
  const int nr = min(kWideRows, rows - tile_r0);
  for (int lr = 0; lr < nr; ++lr) {
    double* o = out + size_t(tile_r0 + lr) * C;
    for (int j = threadIdx.x; j < C; j += 256) o[j] = wide_load(o + j) * s_fac[lr][j / kWideCols];
  }
  if (threadIdx.x == 0) __hip_atomic_store(counter + blockIdx.x, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Second pass of the two-launch variant: one workgroup per row rescales the
// row's tiles by exp(m_tile - M) / S (plain loads: the kernel boundary orders
// them after the first launch's stores).
__global__ __launch_bounds__(256) void linear_wide_softmax_fix(double* __restrict__ out, const double* __restrict__ ms,
                                                               int rows, int C, int groups) {
  const int r = blockIdx.x;
  if (r >= rows) return;
  const double* p = ms + size_t(r) * groups * 2;
  double M = -__builtin_inf();
  for (int q = 0; q < groups; ++q) M = fmax(M, p[2 * q]);
  double S = 0.0;
  for (int q = 0; q < groups; ++q) S += p[2 * q + 1] * exp(p[2 * q] - M);
  double* o = out + size_t(r) * C;
  for (int j = threadIdx.x; j < C; j += 256) o[j] *= exp(p[2 * (j / kWideCols)] - M) / S;
}

// Variant: 0 = off (linear_mfma_rows), 1 = one launch with the last-arriver
// fold, 2 = two launches.  Measured (profiles/r06s_linear_wide, us per call):
// the fold's write-through stores cost ~70 us of a 200 us launch, so the
// two-launch form is the one used.  It wins where linear_mfma_rows underfills
// the chip -- fewer than 8192 rows is fewer than 256 of its 32-row
// workgroups: 4096 x 512 -> 1000 132 vs 239 us, 2048 x 1024 -> 1000 138 vs
// 450 -- and for deep, wide rows (8192 x 784 -> 1000: 333 vs 358); from 8192
// rows at K < 512 or C < 512 the old kernel stays ahead (8192 x 256 -> 1000:
// 135 vs 157; 16384 x 384 -> 300: 160 vs 178).  SCA_LINEAR_WIDE=v forces one.
int wide_softmax_variant(int rows, int K, int C) {
  if (C <= 256 || C > 8 * kWideCols || rows < 256) return 0;
  if (const char* e = std::getenv("SCA_LINEAR_WIDE")) return std::atoi(e);
  return (rows < 8192 || (K >= 512 && C >= 512)) ? 2 : 0;
}

// Scratch (per-row per-group (max, sum) pairs + one counter per row tile) is
// stream-ordered: allocated, zeroed, used and freed on the launch's stream, so
// concurrent launches on other streams never share it.
void launch_wide_softmax(const double* X, int rows, int K, const double* W, const double* b, int C, double* out,
                         hipStream_t s, hipEvent_t stop, int variant) {
  const int tiles = (rows + kWideRows - 1) / kWideRows, groups = (C + kWideCols - 1) / kWideCols;
  const size_t ms_bytes = size_t(rows) * groups * 2 * sizeof(double);
  const size_t bytes = ms_bytes + size_t(tiles) * sizeof(int);
  void* buf = nullptr;
  if (hipMallocAsync(&buf, bytes, s) != hipSuccess) {
    (void)hipGetLastError();  // no pool memory: the one-workgroup-per-row-tile kernel instead
    launch_mfma_t<kActSoftmax, 8, 8, 1, 2>(X, rows, K, W, b, C, out, s, stop);
    return;
  }
  int* counter = reinterpret_cast<int*>(static_cast<char*>(buf) + ms_bytes);
  if (variant == 2) {  // two launches: plain stores, separate rescale pass
    hipLaunchKernelGGL(linear_mfma_wide_softmax<false>, dim3(tiles, groups), dim3(256), 0, s, X, rows, K, W, b, C,
                       out, static_cast<double*>(buf), counter);
    launch_maybe_ext(linear_wide_softmax_fix, dim3(rows), dim3(256), 0, s, stop, out,
                     static_cast<const double*>(buf), rows, C, groups);
  } else {
    (void)hipMemsetAsync(counter, 0, size_t(tiles) * sizeof(int), s);
    launch_maybe_ext(linear_mfma_wide_softmax<true>, dim3(tiles, groups), dim3(256), 0, s, stop, X, rows, K, W, b,
                     C, out, static_cast<double*>(buf), counter);
  }
  (void)hipFreeAsync(buf, s);
}

// Narrow models (<= 2 class tiles) are memory bound on X: what matters is
// how many bytes each CU keeps in flight.  Variant v = (K slices KS, chunk
// group G): 0 (4, 4), 1 (4, 8), 2 (8, 4), 3 (16, 4), 4 (16, 2), 5 (8, 8).
// Measured (profiles/r06m_linear_split): deep rows (K >= 512) in batches of
// fewer than 16384 rows want more K slices -- 4096 x 784 -> 10 8.8 us on
// (16, 2) vs 11.3 on (4, 4), 4096 x 3072 22.7 on (8, 4) vs 29.7 -- while
// shallow rows and very large batches already fill the chip with (4, 4)
// (16384 x 64: 6.4 vs 7.4-15 us; 32768 x 784: 45 vs 48-62).
// SCA_LINEAR_MFMA_SPLIT=v+1 forces one (A/B).
template <int ACT, int NCT>
void launch_mfma_narrow(const double* X, int rows, int K, const double* W, const double* b, int C, double* out,
                        hipStream_t s, hipEvent_t stop) {
  int v = -1;
  if (const char* e = std::getenv("SCA_LINEAR_MFMA_SPLIT")) v = std::atoi(e) - 1;
  if (v < 0 || v > 5) v = (rows < 16384 && K >= 512) ? (K <= 1024 ? 4 : 2) : 0;
  switch (v) {
    case 1: launch_mfma_t<ACT, NCT, 1, 4, 1, 8>(X, rows, K, W, b, C, out, s, stop); break;
    case 2: launch_mfma_t<ACT, NCT, 1, 8, 1, 4>(X, rows, K, W, b, C, out, s, stop); break;
    case 3: launch_mfma_t<ACT, NCT, 1, 16, 1, 4>(X, rows, K, W, b, C, out, s, stop); break;
    case 4: launch_mfma_t<ACT, NCT, 1, 16, 1, 2>(X, rows, K, W, b, C, out, s, stop); break;
    case 5: launch_mfma_t<ACT, NCT, 1, 8, 1, 8>(X, rows, K, W, b, C, out, s, stop); break;
    default: launch_mfma_t<ACT, NCT, 1, 4, 1, 4>(X, rows, K, W, b, C, out, s, stop); break;
  }
}

// Tiling by C (16-column tiles T): up to 4 tiles in one wave with K split over
// 4 waves; up to 16 tiles over 4 class-waves; beyond, 8 class-waves with two
// 16-row tiles each (every W fragment feeds two MFMAs: half the L2 traffic
// per MFMA), <= 1024 classes.
template <int ACT>
void launch_mfma(const double* X, int rows, int K, const double* W, const double* b, int C, double* out,
                 hipStream_t s, hipEvent_t stop) {
  const int tiles = (C + 15) / 16;
  if (ACT == kActSoftmax) {
    const int v = wide_softmax_variant(rows, K, C);
    if (v == 1 || v == 2) {
      launch_wide_softmax(X, rows, K, W, b, C, out, s, stop, v);
      return;
    }
  }
  if (tiles <= 1) launch_mfma_narrow<ACT, 1>(X, rows, K, W, b, C, out, s, stop);
  else if (tiles <= 2) launch_mfma_narrow<ACT, 2>(X, rows, K, W, b, C, out, s, stop);
  else if (tiles <= 4) launch_mfma_t<ACT, 4, 1, 4, 1>(X, rows, K, W, b, C, out, s, stop);
  else if (tiles <= 8) launch_mfma_t<ACT, 2, 4, 1, 1>(X, rows, K, W, b, C, out, s, stop);
  else if (tiles <= 16) launch_mfma_t<ACT, 4, 4, 1, 1>(X, rows, K, W, b, C, out, s, stop);
  else if (tiles <= 32) launch_mfma_t<ACT, 4, 8, 1, 2>(X, rows, K, W, b, C, out, s, stop);
  else launch_mfma_t<ACT, 8, 8, 1, 2>(X, rows, K, W, b, C, out, s, stop);
}

template <int ACT>
void launch_linear(const double* X, int rows, int K, const double* W, const double* b, int C, double* out,
                   hipStream_t s, hipEvent_t stop) {
  if (rows <= 0) return;
  if (mfma_eligible(rows, K, C) && (ACT != kActBinaryLogistic || C == 1)) {
    launch_mfma<ACT>(X, rows, K, W, b, C, out, s, stop);
  } else if (C <= kMaxThreadC && C * K + C <= kMaxLdsDoubles) {
    const size_t lds = size_t(C * K + C + kBlock * C) * sizeof(double);
    launch_maybe_ext(linear_thread_rows<ACT>, dim3((rows + kBlock - 1) / kBlock), dim3(kBlock), lds, s, stop, X, rows,
                     K, W, b, C, out);
  } else {
    const int rows_per_block = kBlock / 64;
    const size_t lds = size_t(rows_per_block * C) * sizeof(double);
    launch_maybe_ext(linear_wave_rows<ACT>, dim3((rows + rows_per_block - 1) / rows_per_block), dim3(kBlock), lds, s,
                     stop, X, rows, K, W, b, C, out);
  }
}

}  // namespace

bool linear_uses_mfma(int rows, int K, int C) { return mfma_eligible(rows, K, C); }

void linear_f64(const double* X, int rows, int K, const double* W, const double* b, int C, int act, double* out,
                hipStream_t s, hipEvent_t stop) {
  switch (act) {
    case kActIdentity: launch_linear<kActIdentity>(X, rows, K, W, b, C, out, s, stop); break;
    case kActSoftmax: launch_linear<kActSoftmax>(X, rows, K, W, b, C, out, s, stop); break;
    case kActBinaryLogistic: launch_linear<kActBinaryLogistic>(X, rows, K, W, b, C, out, s, stop); break;
    case kActOvr: launch_linear<kActOvr>(X, rows, K, W, b, C, out, s, stop); break;
    default: launch_linear<kActSigmoid>(X, rows, K, W, b, C, out, s, stop); break;
  }
}

}  // namespace sca::kern
