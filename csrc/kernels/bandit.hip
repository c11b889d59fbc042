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

namespace sca::kern {
namespace {

struct Philox {
  uint32_t c[4];
  uint32_t k[2];
  uint32_t out[4];
  int used = 4;

  __device__ Philox(uint64_t seed, uint64_t subseq) {
    k[0] = uint32_t(seed);
    k[1] = uint32_t(seed >> 32);
    c[0] = uint32_t(subseq);
    c[1] = uint32_t(subseq >> 32);
    c[2] = 0;
    c[3] = 0;
  }
  __device__ void round() {
    uint32_t kk0 = k[0], kk1 = k[1];
    uint32_t x0 = c[0], x1 = c[1], x2 = c[2], x3 = c[3];
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      const uint64_t p0 = uint64_t(0xD2511F53u) * x0;
      const uint64_t p1 = uint64_t(0xCD9E8D57u) * x2;
      const uint32_t y0 = uint32_t(p1 >> 32) ^ x1 ^ kk0;
      const uint32_t y1 = uint32_t(p1);
      const uint32_t y2 = uint32_t(p0 >> 32) ^ x3 ^ kk1;
      const uint32_t y3 = uint32_t(p0);
      x0 = y0; x1 = y1; x2 = y2; x3 = y3;
      kk0 += 0x9E3779B9u;
      kk1 += 0xBB67AE85u;
    }
    out[0] = x0; out[1] = x1; out[2] = x2; out[3] = x3;
    if (++c[2] == 0) ++c[3];
    used = 0;
  }
  __device__ uint32_t next() {
    if (used == 4) round();
    return out[used++];
  }
  // (0, 1]
  __device__ float uniform() { return (float(next() >> 8) + 1.0f) * (1.0f / 16777216.0f); }
  __device__ float normal() {
    const float u1 = uniform(), u2 = uniform();
    return sqrtf(-2.0f * logf(u1)) * cospif(2.0f * u2);
  }
  // Marsaglia-Tsang gamma(alpha, 1); alpha < 1 boosted by U^(1/alpha).
  __device__ float gamma(float alpha) {
    float boost = 1.0f;
    if (alpha < 1.0f) {
      boost = powf(uniform(), 1.0f / alpha);
      alpha += 1.0f;
    }
    const float d = alpha - 1.0f / 3.0f, c = rsqrtf(9.0f * d);
    for (int it = 0; it < 64; ++it) {  // bounded: acceptance rate > 95%
      float x, v;
      int tries = 0;
      do {
        x = normal();
        v = 1.0f + c * x;
      } while (v <= 0.0f && ++tries < 64);
      v = v * v * v;
      const float u = uniform();
      if (u < 1.0f - 0.0331f * x * x * x * x) return d * v * boost;
      if (logf(u) < 0.5f * x * x + d * (1.0f - v + logf(v))) return d * v * boost;
    }
    return d * boost;
  }
};

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
