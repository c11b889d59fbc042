// Fused device graph of small linear stages (SURVEY K3,
// K1, X3).  The reference walks such a graph -- TRANSFORMER -> COMBINER over
// N sklearn MODELs -- as one HTTP hop per node
// (engine/.../PredictiveUnitBean.java:128-138,170-192); the batched device
// graph (csrc/gpu/graph.cc) made it one micro-batch but still one kernel per
// stage, and the pump thread pays ~2 us of launch per kernel.  When every
// stage is a small linear model (K, C <= 16: scalers, logistic regressions)
// or an AVERAGE_COMBINER, the whole graph is ONE kernel: a thread per row
// carries the row through every stage in LDS (activations never leave the
// CU), with every stage's W / b staged once per workgroup.
//
// Stage table (LinearGraphStage, kernels.h) in topological order; stage
// inputs are -1 (the request row) or earlier stages.  Activations live in a
// [slot][thread] LDS array (column per thread: consecutive threads hit
// consecutive banks).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace sca::kern {
namespace {

constexpr int kLgThreads = 128;

__device__ inline double lg_sigmoid(double z) { return 1.0 / (1.0 + exp(-z)); }

__global__ __launch_bounds__(kLgThreads) void linear_graph_rows(const double* __restrict__ X, int rows, int cols,
                                                                const LinearGraphStage* __restrict__ stages,
                                                                int n_stages, const double* __restrict__ params,
                                                                int n_params, int act_slots,
                                                                double* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  double* sP = lds;                                  // [n_params]
  double* sA = sP + ((n_params + 1) & ~1);           // [act_slots][kLgThreads]
  __shared__ __attribute__((aligned(16))) char sS_raw[sizeof(LinearGraphStage) * kLinearGraphMaxStages];
  LinearGraphStage* sS = reinterpret_cast<LinearGraphStage*>(sS_raw);
  for (int i = threadIdx.x; i < n_params; i += kLgThreads) sP[i] = params[i];
  if (threadIdx.x < n_stages) sS[threadIdx.x] = stages[threadIdx.x];
  __syncthreads();
  const int r = blockIdx.x * kLgThreads + threadIdx.x;
  if (r >= rows) return;
  const double* x = X + size_t(r) * cols;
  const int t = threadIdx.x;
  for (int si = 0; si < n_stages; ++si) {
    const LinearGraphStage& S = sS[si];
    double* o = sA + size_t(S.out_off) * kLgThreads + t;
    if (S.kind == 1) {  // mean of n_in equal-width inputs
      const double inv = 1.0 / double(S.n_in);
      for (int c = 0; c < S.C; ++c) {
        double v = 0.0;
        for (int q = 0; q < S.n_in; ++q) {
          const int j = S.in[q];
          v += j < 0 ? x[c] : sA[size_t(sS[j].out_off + c) * kLgThreads + t];
        }
        o[size_t(c) * kLgThreads] = v * inv;
      }
      continue;
    }
    const int j = S.in[0];
    const double* W = sP + S.w_off;
    double z[kLinearGraphMaxWidth];
#pragma unroll
    for (int c = 0; c < kLinearGraphMaxWidth; ++c) z[c] = 0.0;
    for (int c = 0; c < S.C; ++c) z[c] = S.b_off >= 0 ? sP[S.b_off + c] : 0.0;
    for (int k = 0; k < S.K; ++k) {
      const double xv = j < 0 ? x[k] : sA[size_t(sS[j].out_off + k) * kLgThreads + t];
      for (int c = 0; c < S.C; ++c) z[c] = fma(xv, W[c * S.K + k], z[c]);
    }
    if (S.act == kActSoftmax) {
      double m = z[0];
      for (int c = 1; c < S.C; ++c) m = fmax(m, z[c]);
      double s = 0.0;
      for (int c = 0; c < S.C; ++c) { z[c] = exp(z[c] - m); s += z[c]; }
      const double inv = 1.0 / s;
      for (int c = 0; c < S.C; ++c) o[size_t(c) * kLgThreads] = z[c] * inv;
    } else if (S.act == kActBinaryLogistic) {
      const double p = lg_sigmoid(z[0]);
      o[0] = 1.0 - p;
      o[kLgThreads] = p;
    } else if (S.act == kActOvr) {
      double s = 0.0;
      for (int c = 0; c < S.C; ++c) { z[c] = lg_sigmoid(z[c]); s += z[c]; }
      const double inv = 1.0 / s;
      for (int c = 0; c < S.C; ++c) o[size_t(c) * kLgThreads] = z[c] * inv;
    } else if (S.act == kActSigmoid) {
      for (int c = 0; c < S.C; ++c) o[size_t(c) * kLgThreads] = lg_sigmoid(z[c]);
    } else {
      for (int c = 0; c < S.C; ++c) o[size_t(c) * kLgThreads] = z[c];
    }
  }
  const LinearGraphStage& L = sS[n_stages - 1];
  const int oc = L.out_cols;
  const double* src = sA + size_t(L.out_off) * kLgThreads + t;
  for (int c = 0; c < oc; ++c) out[size_t(r) * oc + c] = src[size_t(c) * kLgThreads];
}

}  // namespace

size_t linear_graph_lds_bytes(int n_params, int act_slots) {
  return (size_t((n_params + 1) & ~1) + size_t(act_slots) * kLgThreads) * sizeof(double);
}

void linear_graph_f64(const double* X, int rows, int cols, const LinearGraphStage* stages, int n_stages,
                      const double* params, int n_params, int act_slots, double* out, hipStream_t s,
                      hipEvent_t stop) {
  if (rows <= 0) return;
  const dim3 grid((rows + kLgThreads - 1) / kLgThreads), block(kLgThreads);
  const uint32_t lds = uint32_t(linear_graph_lds_bytes(n_params, act_slots));
  if (stop)
    hipExtLaunchKernelGGL(linear_graph_rows, grid, block, lds, s, nullptr, stop, 0, X, rows, cols, stages, n_stages,
                          params, n_params, act_slots, out);
  else
    hipLaunchKernelGGL(linear_graph_rows, grid, block, lds, s, X, rows, cols, stages, n_stages, params, n_params,
                       act_slots, out);
}

}  // namespace sca::kern
