// Fused MLP / VAE-reconstruction kernel (SURVEY K10 + dense models served by
// SKLearnServer / MLFlowServer).  Reference: components/outlier-detection/vae/
// CoreVAE.py:106-141 (10 Keras predict passes, row MSE) and vae/model.py:23-91
// (Dense relu encoder, z_mean / z_log_var heads, reparameterisation,
// Dense relu decoder, sigmoid output).
//
// Layout (one workgroup of 4 or 8 waves per 16-row tile):
//   LDS buffers hold [16][ld] fp32 activations, ld = 8 (mod 64) floats, so
//   the ds_read_b128 A-fragment reads of the 16 rows are bank-conflict free
//   in all four lane groups of that instruction; buffer 0 keeps the input
//   tile for the reconstruction error.  Dense layer: each wave owns 16-column
//   output tiles.  K runs in blocks of 16: a block is four 16x16x4 f32 MFMAs
//   whose k-index for lane (kq = lane / 16) and MFMA j is 16 kb + 4 kq + j --
//   a permutation of the block's 16 k's, applied to A and B alike -- so one
//   ds_read_b128 gives a lane its A values of all four MFMAs and one 16-byte
//   global load its B values: the host packs the transposed weights
//   fragment-major ([Np/16][Kp/16][64 lanes][4]), one coalesced 1 KiB load
//   per wave per block.  B blocks are prefetched four ahead (the whole
//   model is a few MB and stays L2-resident, so the loop is L2-latency
//   bound without it) and four accumulators rotate to cover the MFMA's
//   dependent latency.  The epilogue adds the bias, applies the activation
//   and writes the next buffer, or (DenseMse) reduces (act(y) - x)^2 across
//   the tile's 16 lanes and accumulates per-row sums in LDS.  The MC loop
//   re-runs only the decoder ops: the encoder is deterministic, so computing
//   it once is identical to the reference's 10 full predict() calls.
#include <hip/hip_runtime.h>

#include <algorithm>

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
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
  const float* A = lds + p.buf_off[op.in_buf];
  const int lda = p.buf_ld[op.in_buf];
  const f32x4* __restrict__ Wf = reinterpret_cast<const f32x4*>(params + op.w_off);
  const float* B = params + op.b_off;
  const float* x0 = lds + p.buf_off[0];
  const int ld0 = p.buf_ld[0];
  float* O = lds + p.buf_off[op.out_buf];
  const int ldo = p.buf_ld[op.out_buf];
  const float* a_row = A + r16 * lda + kq * 4;
  const int KB = op.Kp >> 4;
  for (int t = wave; t < op.Np / 16; t += nwaves) {
    const int n0 = t * 16;
    // Four blocks (16 MFMAs) per step with the next four blocks' B loads in
    // flight: a prefetch distance of ~16 MFMAs covers the L2 latency.  The
    // look-ahead past the tile's last block reads the next tile (or the zero
    // pad after the blob); those values are never used.  sched_barrier keeps
    // the compiler from sinking the loads back next to their use.
    const f32x4* wt = Wf + size_t(t) * KB * 64 + lane;
    f32x4 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) b[u] = wt[u * 64];
    int kb = 0;
    for (; kb + 4 <= KB; kb += 4) {
      f32x4 nb[4], a[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) nb[u] = wt[size_t(kb + 4 + u) * 64];
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] = *reinterpret_cast<const f32x4*>(a_row + (kb + u) * 16);
      __builtin_amdgcn_sched_barrier(0);
      // MFMA j of every block accumulates into acc[j]: consecutive MFMAs are
      // independent and each accumulator is reused 4 MFMAs (128 cycles) later,
      // past the 16x16x4 f32 dependent latency.  The barriers pin this order
      // (the scheduler otherwise groups each accumulator's chain).
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][j], b[u][j], acc[j], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
      for (int u = 0; u < 4; ++u) b[u] = nb[u];
    }
#pragma unroll
    for (int u = 0; u < 3; ++u)  // KB % 4 tail blocks, already loaded
      if (kb + u < KB) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(a_row + (kb + u) * 16);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[u][j], acc[j], 0, 0, 0);
      }
    const f32x4 accs = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    const int col = n0 + r16;  // C/D map: col = lane & 15, row = (lane >> 4) * 4 + i
    const float bias = B[col];
    const bool live = col < op.N;
    if (op.type == kMlpDense) {
#pragma unroll
      for (int i = 0; i < 4; ++i) O[(kq * 4 + i) * ldo + col] = live ? act_f(accs[i] + bias, op.act) : 0.f;
    } else {  // kMlpDenseMse: reconstruction error against the input tile
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = kq * 4 + i;
        float d = live ? act_f(accs[i] + bias, op.act) - x0[row * ld0 + col] : 0.f;
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

__global__ __launch_bounds__(512) void mlp_kernel(const double* __restrict__ X, int rows, const MlpProgram p,
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


// ------------------------------------------------------------ layer-wise
// One wave = one 16x16 output tile of one layer; 4 waves per workgroup take
// consecutive column tiles of the same 16-row tile (A fragments shared in L1).
// Branch-free A loads (row clamped to the last live row: rows past rows_eff
// only feed output rows that are never stored; reparameterised k past the
// latent width selects 0), so the
// look-ahead loads stay in flight across the loop -- a branch around a load
// makes the waitcnt pass drain the queue and serialises every block on its
// memory latency.
template <int AMODE>  // 0: fp32 activations, 2: VAE reparameterisation
__device__ __forceinline__ f32x4 layer_a(const MlpLayerArgs& a, int row, int k0) {
  row = min(row, a.rows_eff - 1);
  f32x4 v;
  if constexpr (AMODE == 0) {
    // k0 may run up to 4 blocks past the row (look-ahead): the workspace has slack
    v = *reinterpret_cast<const f32x4*>(a.A + size_t(row) * a.lda + k0);
  } else {
    const int r = row % a.rows, smp = row / a.rows;
    const float* h = a.H + size_t(r) * a.ldh;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = min(k0 + j, a.latent - 1);  // same stream as reparam() of the fused kernel
      Philox rng(a.key, (uint64_t(r) << 24) ^ (uint64_t(smp) << 14) ^ uint64_t(k));
      const float z = h[k] + expf(0.5f * h[a.latent + k]) * rng.normal();
      v[j] = k0 + j < a.latent ? z : 0.f;
    }
  }
  return v;
}

// SPLITK = 1: the 4 waves of a workgroup own 4 consecutive column tiles.
// SPLITK = 4: they share one tile, each running a quarter of the K blocks,
// and fold their accumulators through LDS -- 4x the waves (and loads) in
// flight for long-K layers on batches too small to fill the chip.
template <int AMODE, int SPLITK>
__global__ __launch_bounds__(256) void mlp_layer_kernel(const MlpLayerArgs a) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int t = SPLITK == 1 ? blockIdx.x * 4 + wave : blockIdx.x;
  if (SPLITK == 1 && t >= a.Np / 16) return;  // whole wave; no barriers when SPLITK == 1
  const int r16 = lane & 15, kq = lane >> 4;
  const int row0 = blockIdx.y * kMlpRows;
  const int arow = row0 + r16;
  const int KB = a.Kp >> 4;
  const int kb0 = SPLITK == 1 ? 0 : (KB * wave) / SPLITK, kb1 = SPLITK == 1 ? KB : (KB * (wave + 1)) / SPLITK;
  const f32x4* wt = reinterpret_cast<const f32x4*>(a.W) + size_t(t) * KB * 64 + lane;
  f32x4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // A and B of the next four blocks are loaded while the current four run
  // (the B look-ahead past the last block reads the next range / tile or the pad).
  f32x4 b[4], av[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    b[u] = wt[size_t(kb0 + u) * 64];
    av[u] = layer_a<AMODE>(a, arow, (kb0 + u) * 16 + kq * 4);
  }
  int kb = kb0;
  for (; kb + 4 <= kb1; kb += 4) {
    f32x4 nb[4], na[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      nb[u] = wt[size_t(kb + 4 + u) * 64];
      na[u] = layer_a<AMODE>(a, arow, (kb + 4 + u) * 16 + kq * 4);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u][j], b[u][j], acc[j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      b[u] = nb[u];
      av[u] = na[u];
    }
  }
#pragma unroll
  for (int u = 0; u < 3; ++u)
    if (kb + u < kb1) {
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u][j], b[u][j], acc[j], 0, 0, 0);
    }
  if constexpr (SPLITK > 1) {
    __shared__ f32x4 part[SPLITK - 1][64];
    if (wave > 0) part[wave - 1][lane] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    __syncthreads();
    if (wave > 0) return;
#pragma unroll
    for (int w = 0; w < SPLITK - 1; ++w) acc[w & 3] += part[w][lane];
  }
  const f32x4 accs = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  const int col = t * 16 + r16;
  const bool live = col < a.N;
  const float bias = a.bias[col];
  if (!a.mse) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = row0 + kq * 4 + i;
      if (row < a.rows_eff) a.O[size_t(row) * a.ldo + col] = live ? act_f(accs[i] + bias, a.act) : 0.f;
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = row0 + kq * 4 + i;
    const bool ok = live && row < a.rows_eff;
    const int r = row % a.rows;
    float d = ok ? act_f(accs[i] + bias, a.act) - a.xref[size_t(r) * a.ldx + col] : 0.f;
    d *= d;
    d += __shfl_xor(d, 1, 64);
    d += __shfl_xor(d, 2, 64);
    d += __shfl_xor(d, 4, 64);
    d += __shfl_xor(d, 8, 64);
    if (r16 == 0 && row < a.rows_eff) atomicAdd(&a.mse[r], d);
  }
}

__global__ __launch_bounds__(256) void mlp_finish_kernel(const float* __restrict__ L, int ld, int rows, int n, int mode,
                                                          double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float* l = L + size_t(r) * ld;
  if (mode == 2) {
    if (lane == 0) {
      const double q = double(l[0]);
      out[size_t(r) * 2] = 1.0 - q;
      out[size_t(r) * 2 + 1] = q;
    }
    return;
  }
  if (mode == 0) {
    for (int c = lane; c < n; c += 64) out[size_t(r) * n + c] = double(l[c]);
    return;
  }
  float m = -3.4e38f;
  for (int c = lane; c < n; c += 64) m = fmaxf(m, l[c]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  float sum = 0.f;
  for (int c = lane; c < n; c += 64) sum += expf(l[c] - m);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
  for (int c = lane; c < n; c += 64) out[size_t(r) * n + c] = double(expf(l[c] - m) / sum);
}

// fp64 request rows -> fp32 [rows][ld], columns >= F zeroed (the layer-wise
// path's first A operand; the fused kernel does the same while staging to LDS)
__global__ void mlp_convert_kernel(const double* __restrict__ X, int rows, int F, int ld, float* __restrict__ out) {
  const size_t n = size_t(rows) * ld;
  for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
    const int r = int(i / ld), c = int(i - size_t(r) * ld);
    out[i] = c < F ? float(X[size_t(r) * F + c]) : 0.f;
  }
}

__global__ void mlp_mse_finish_kernel(const float* __restrict__ mse, int rows, double scale, double* __restrict__ out) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < rows) out[r] = double(mse[r]) * scale;
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
  hipLaunchKernelGGL(mlp_kernel, dim3((rows + kMlpRows - 1) / kMlpRows), dim3(64 * prog.waves), lds, s, X, rows, prog, params, key,
                     out);
}

void mlp_layer(const MlpLayerArgs& a, hipStream_t s) {
  if (a.rows_eff <= 0) return;
  const int row_tiles = (a.rows_eff + kMlpRows - 1) / kMlpRows, col_tiles = a.Np / 16;
  // split K over the workgroup's waves when the tiles alone leave most of the
  // chip's 1024 SIMDs idle and each wave would still get >= 4 blocks
  const bool split = row_tiles * col_tiles < 512 && a.Kp / 16 >= 16;
  const dim3 grid(split ? col_tiles : (col_tiles + 3) / 4, row_tiles);
#define SCA_MLP_LAYER(M)                                                               \
  if (split) hipLaunchKernelGGL((mlp_layer_kernel<M, 4>), grid, dim3(256), 0, s, a); \
  else hipLaunchKernelGGL((mlp_layer_kernel<M, 1>), grid, dim3(256), 0, s, a);
  if (a.H) {
    SCA_MLP_LAYER(2)
  } else {
    SCA_MLP_LAYER(0)
  }
#undef SCA_MLP_LAYER
}

void mlp_finish(const float* logits, int ld, int rows, int n, int mode, double* out, hipStream_t s) {
  if (rows <= 0) return;
  hipLaunchKernelGGL(mlp_finish_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, logits, ld, rows, n, mode, out);
}

void mlp_convert(const double* X, int rows, int F, int ld, float* out, hipStream_t s) {
  if (rows <= 0) return;
  const size_t n = size_t(rows) * ld;
  const int blocks = int(std::min<size_t>((n + 255) / 256, 2048));
  hipLaunchKernelGGL(mlp_convert_kernel, dim3(blocks), dim3(256), 0, s, X, rows, F, ld, out);
}

void mlp_mse_finish(const float* mse, int rows, double scale, double* out, hipStream_t s) {
  if (rows <= 0) return;
  hipLaunchKernelGGL(mlp_mse_finish_kernel, dim3((rows + 255) / 256), dim3(256), 0, s, mse, rows, scale, out);
}

}  // namespace sca::kern
