// Device-side multi-armed-bandit routers (reference
// components/routers/epsilon-greedy/EpsilonGreedy.py:87-106 and
// components/routers/thompson-sampling/ThompsonSampling.py:78-91, which draw
// numpy random numbers on the CPU for every request).
//
// A micro-batch of n routing decisions is one launch: thread i owns request i
// and a counter-based Philox4x32-10 stream (seed, offset + i), so decisions are
// reproducible and independent of how requests were grouped into batches.
// Router state (best branch / Beta parameters) is read straight from
// fine-grained pinned host memory that feedback updates, so no copy precedes
// a launch.  Decisions are written as fp64 (the batcher's output format).
#include <hip/hip_runtime.h>

#include "kernels.h"
#include "philox.h"

namespace sca::kern {
namespace {


// EpsilonGreedy.route: x > eps -> best branch, else uniform over the others.
__global__ void eg_route_kernel(const int32_t* __restrict__ best, int nb, float eps, uint64_t seed, uint64_t offset,
                                int n, double* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Philox rng(seed, offset + uint64_t(i));
  const int b = best[0];
  int pick = b;
  if (nb > 1 && rng.uniform() <= eps) {
    int other = int(rng.next() % uint32_t(nb - 1));
    if (other >= b) ++other;
    pick = other;
  }
  out[i] = double(pick);
}

// ThompsonSampling.route: sample Beta(a_i, b_i) per branch, argmax.
__global__ void ts_route_kernel(const float* __restrict__ alpha, const float* __restrict__ beta, int nb, uint64_t seed,
                                uint64_t offset, int n, double* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Philox rng(seed, offset + uint64_t(i));
  float best = -1.0f;
  int pick = 0;
  for (int b = 0; b < nb; ++b) {
    const float x = rng.gamma(alpha[b]);
    const float y = rng.gamma(beta[b]);
    const float s = x / (x + y);
    if (s > best) { best = s; pick = b; }
  }
  out[i] = double(pick);
}

}  // namespace

void eg_route(const int32_t* best_branch, int n_branches, float epsilon, uint64_t seed, uint64_t offset, int n,
              double* branch_out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(eg_route_kernel, dim3((n + 255) / 256), dim3(256), 0, s, best_branch, n_branches, epsilon, seed,
                     offset, n, branch_out);
}

void ts_route(const float* alpha, const float* beta, int n_branches, uint64_t seed, uint64_t offset, int n,
              double* branch_out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(ts_route_kernel, dim3((n + 255) / 256), dim3(256), 0, s, alpha, beta, n_branches, seed, offset,
                     n, branch_out);
}

}  // namespace sca::kern
