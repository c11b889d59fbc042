// Fused MLP / VAE-reconstruction kernel (SURVEY K10 + dense models served by
// SKLearnServer / MLFlowServer).  Reference: components/outlier-detection/vae/
// CoreVAE.py:106-141 (10 Keras predict passes, row MSE) and vae/model.py:23-91
// (Dense relu encoder, z_mean / z_log_var heads, reparameterisation,
// Dense relu decoder, sigmoid output).
//
// Layout (one 256-thread workgroup = 4 waves per 16-row tile):
//   LDS buffers hold [16][ld] fp32 activations (ld odd -> the 16 rows of an
//   A fragment hit 16 different banks); buffer 0 keeps the input tile for the
//   reconstruction error.  Dense layer: each wave owns 16-column output tiles;
//   per tile two independent f32x4 accumulators alternate over K (the
//   16x16x4 f32 MFMA has a 40-cycle dependent latency vs a 32-cycle issue),
//   A fragments come from LDS, B fragments (transposed weights) from L2 --
//   the whole model is a few hundred KB and stays L2-resident across tiles.
//   The epilogue adds the bias, applies the activation and writes the next
//   buffer, or (DenseMse) reduces (act(y) - x)^2 across the tile's 16 lanes
//   and accumulates per-row sums in LDS.  The MC loop re-runs only the
//   decoder ops: the encoder is deterministic, so computing it once is
//   identical to the reference's 10 full predict() calls.
#include <hip/hip_runtime.h>

#include "kernels.h"
#include "philox.h"

namespace sca::kern {
namespace {

using f32x4 = __attribute__((ext_vector_type(4))) float;

__device__ __forceinline__ float act_f(float v, int a) {
  switch (a) {
    case kMlpRelu: return fmaxf(v, 0.f);
    case kMlpSigmoid: return 1.f / (1.f + expf(-v));
    case kMlpTanh: return tanhf(v);
    default: return v;
  }
}

__device__ void dense(const MlpOp& op, const MlpProgram& p, float* lds, const float* __restrict__ params,
                      float* mse) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
  const float* A = lds + p.buf_off[op.in_buf];
  const int lda = p.buf_ld[op.in_buf];
  const float* W = params + op.w_off;
  const float* B = params + op.b_off;
  const float* x0 = lds + p.buf_off[0];
  const int ld0 = p.buf_ld[0];
  float* O = lds + p.buf_off[op.out_buf];
  const int ldo = p.buf_ld[op.out_buf];
  const float* a_ptr = A + r16 * lda + kq;
  for (int t = wave; t < op.Np / 16; t += 4) {
    const int n0 = t * 16;
    const float* w_ptr = W + size_t(kq) * op.Np + n0 + r16;
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    int k0 = 0;
    for (; k0 + 8 <= op.Kp; k0 += 8) {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a_ptr[k0], w_ptr[size_t(k0) * op.Np], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a_ptr[k0 + 4], w_ptr[size_t(k0 + 4) * op.Np], acc1, 0, 0, 0);
    }
    if (k0 < op.Kp) acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a_ptr[k0], w_ptr[size_t(k0) * op.Np], acc0, 0, 0, 0);
    const f32x4 acc = acc0 + acc1;
    const int col = n0 + r16;  // C/D map: col = lane & 15, row = (lane >> 4) * 4 + i
    const float bias = B[col];
    const bool live = col < op.N;
    if (op.type == kMlpDense) {
#pragma unroll
      for (int i = 0; i < 4; ++i) O[(kq * 4 + i) * ldo + col] = live ? act_f(acc[i] + bias, op.act) : 0.f;
    } else {  // kMlpDenseMse: reconstruction error against the input tile
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = kq * 4 + i;
        float d = live ? act_f(acc[i] + bias, op.act) - x0[row * ld0 + col] : 0.f;
        d *= d;
        d += __shfl_xor(d, 1, 64);
        d += __shfl_xor(d, 2, 64);
        d += __shfl_xor(d, 4, 64);
        d += __shfl_xor(d, 8, 64);
        if (r16 == 0) atomicAdd(&mse[row], d);
      }
    }
  }
}

__device__ void reparam(const MlpOp& op, const MlpProgram& p, float* lds, int row0, int sample, uint64_t key) {
  const float* A = lds + p.buf_off[op.in_buf];
  const int lda = p.buf_ld[op.in_buf];
  float* O = lds + p.buf_off[op.out_buf];
  const int ldo = p.buf_ld[op.out_buf];
  for (int i = threadIdx.x; i < kMlpRows * op.Np; i += blockDim.x) {
    const int r = i / op.Np, j = i - r * op.Np;
    float z = 0.f;
    if (j < op.N) {
      // eps ~ N(0, 1), one Philox stream per (row, MC sample, latent unit)
      Philox rng(key, (uint64_t(row0 + r) << 24) ^ (uint64_t(sample) << 14) ^ uint64_t(j));
      const float eps = rng.normal();
      z = A[r * lda + j] + expf(0.5f * A[r * lda + op.N + j]) * eps;
    }
    O[r * ldo + j] = z;
  }
}

__global__ __launch_bounds__(256) void mlp_kernel(const double* __restrict__ X, int rows, const MlpProgram p,
                                                  const float* __restrict__ params, uint64_t key,
                                                  double* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* mse = lds + p.lds_floats;  // [16] per-row reconstruction-error sums
  const int row0 = blockIdx.x * kMlpRows;
  {  // stage the fp64 request rows as fp32 (the precision Keras / torch consume)
    float* x0 = lds + p.buf_off[0];
    const int ld0 = p.buf_ld[0];
    for (int i = threadIdx.x; i < kMlpRows * p.Fp; i += blockDim.x) {
      const int r = i / p.Fp, c = i - r * p.Fp;
      x0[r * ld0 + c] = (row0 + r < rows && c < p.F) ? float(X[size_t(row0 + r) * p.F + c]) : 0.f;
    }
    if (threadIdx.x < kMlpRows) mse[threadIdx.x] = 0.f;
  }
  __syncthreads();
  for (int o = 0; o < p.n_pre; ++o) {
    const MlpOp& op = p.ops[o];
    if (op.type == kMlpReparam) reparam(op, p, lds, row0, 0, key);
    else dense(op, p, lds, params, mse);
    __syncthreads();
  }
  for (int s = 0; s < p.loops; ++s)
    for (int o = p.n_pre; o < p.n_pre + p.n_loop; ++o) {
      const MlpOp& op = p.ops[o];
      if (op.type == kMlpReparam) reparam(op, p, lds, row0, s, key);
      else dense(op, p, lds, params, mse);
      __syncthreads();
    }
  if (p.mse_mode) {
    const int r = threadIdx.x;
    if (r < kMlpRows && row0 + r < rows) out[row0 + r] = double(mse[r]) / (double(p.mse_dim) * double(p.loops));
    return;
  }
  const float* O = lds + p.buf_off[p.out_buf];
  const int ldo = p.buf_ld[p.out_buf];
  if (p.out_softmax == 2) {  // binary logistic head (sigmoid unit) -> [1 - p, p]
    for (int r = threadIdx.x; r < kMlpRows; r += blockDim.x)
      if (row0 + r < rows) {
        const double q = double(O[r * ldo]);
        out[size_t(row0 + r) * 2] = 1.0 - q;
        out[size_t(row0 + r) * 2 + 1] = q;
      }
    return;
  }
  if (!p.out_softmax) {
    for (int i = threadIdx.x; i < kMlpRows * p.out_dim; i += blockDim.x) {
      const int r = i / p.out_dim, c = i - r * p.out_dim;
      if (row0 + r < rows) out[size_t(row0 + r) * p.out_dim + c] = double(O[r * ldo + c]);
    }
    return;
  }
  // softmax over the output row: one wave per row
  const int lane = threadIdx.x & 63;
  for (int r = threadIdx.x >> 6; r < kMlpRows; r += blockDim.x >> 6) {
    if (row0 + r >= rows) break;
    float m = -3.4e38f;
    for (int c = lane; c < p.out_dim; c += 64) m = fmaxf(m, O[r * ldo + c]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    float sum = 0.f;
    for (int c = lane; c < p.out_dim; c += 64) sum += expf(O[r * ldo + c] - m);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
    for (int c = lane; c < p.out_dim; c += 64)
      out[size_t(row0 + r) * p.out_dim + c] = double(expf(O[r * ldo + c] - m) / sum);
  }
}

}  // namespace

void mlp_forward(const double* X, int rows, const MlpProgram& prog, const float* params, uint64_t seed,
                 uint64_t offset, double* out, hipStream_t s) {
  if (rows <= 0) return;
  const size_t lds = (size_t(prog.lds_floats) + kMlpRows) * sizeof(float);
  if (lds > 65536)  // > 64 KiB of dynamic LDS needs the opt-in (160 KiB per CU on gfx950)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&mlp_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                              int(lds));
  const uint64_t key = seed ^ (offset * 0x9E3779B97F4A7C15ULL);
  hipLaunchKernelGGL(mlp_kernel, dim3((rows + kMlpRows - 1) / kMlpRows), dim3(256), lds, s, X, rows, prog, params, key,
                     out);
}

}  // namespace sca::kern
