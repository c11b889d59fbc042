// Counter-based Philox4x32-10 generator shared by the device-side samplers
// (bandit routers, VAE reparameterisation): stream = (seed, subsequence), so
// draws are reproducible and independent of launch geometry / batching.
// The integer stream and uniform() also compile for the host (bit-identical:
// integer arithmetic and one exact int->float conversion), so the host
// epsilon-greedy path (csrc/gpu/router.cc) makes the same decisions.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace sca::kern {

struct Philox {
  uint32_t c[4];
  uint32_t k[2];
  uint32_t out[4];
  int used = 4;

  __host__ __device__ Philox(uint64_t seed, uint64_t subseq) {
    k[0] = uint32_t(seed);
    k[1] = uint32_t(seed >> 32);
    c[0] = uint32_t(subseq);
    c[1] = uint32_t(subseq >> 32);
    c[2] = 0;
    c[3] = 0;
  }
  __host__ __device__ void round() {
    uint32_t kk0 = k[0], kk1 = k[1];
    uint32_t x0 = c[0], x1 = c[1], x2 = c[2], x3 = c[3];
    for (int i = 0; i < 10; ++i) {  // (fully unrolled by the compiler: constant trip count)
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
  __host__ __device__ uint32_t next() {
    if (used == 4) round();
    return out[used++];
  }
  // (0, 1]
  __host__ __device__ float uniform() { return (float(next() >> 8) + 1.0f) * (1.0f / 16777216.0f); }
#ifdef __HIPCC__  // device-only samplers (host translation units, e.g. router.cc, use the integer stream)
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
#endif
};

}  // namespace sca::kern
