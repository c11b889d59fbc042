// Linear / logistic-regression predict (reference
// servers/sklearnserver/sklearnserver/SKLearnServer.py:32-42 which calls
// sklearn's predict_proba on the CPU for every request).
//
// Two CDNA4 mappings, chosen by shape on the host:
//  * thread-per-row: tiny K*C (iris: K=4, C=3).  W, b and the per-thread
//    logits live in LDS; a 64-wide wave covers 64 requests of a micro-batch.
//  * wave-per-row: larger K.  Lanes stride K (coalesced row reads), each
//    class logit is a 64-lane shuffle reduction; logits staged in LDS.
// fp64 throughout so results match sklearn bit-for-bit up to summation order.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

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

// `stop` (optional) is completed by the kernel's own dispatch packet
// (hipExtLaunchKernelGGL): one HIP call per batch instead of launch +
// hipEventRecord (2.1 + 2.6 us of host time, tools/micro/launch_cost.hip).
template <class... Args, class... P>
void launch_maybe_ext(void (*k)(Args...), dim3 grid, dim3 block, size_t lds, hipStream_t s, hipEvent_t stop,
                      P... args) {
  if (stop) hipExtLaunchKernelGGL(k, grid, block, uint32_t(lds), s, nullptr, stop, 0, args...);
  else hipLaunchKernelGGL(k, grid, block, lds, s, args...);
}

template <int ACT>
void launch_linear(const double* X, int rows, int K, const double* W, const double* b, int C, double* out,
                   hipStream_t s, hipEvent_t stop) {
  if (rows <= 0) return;
  if (C <= kMaxThreadC && C * K + C <= kMaxLdsDoubles) {
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
