// Large-batch Dense layer GEMM with fused epilogue (SURVEY K10 / dense models;
// reference: the Keras / sklearn dense layers of vae/model.py:23-91 and the
// MLP servers).  See DenseGemmArgs in kernels.h for the layouts.
//
// One wave per workgroup owns a 64-row x 16*TN-column output tile: 4 x TN
// independent 16x16 accumulators.  Operands come straight from global memory
// in MFMA fragment order (A rows are contiguous along K, W is pre-packed), so
// there is no LDS staging and no barrier; the next K block's fragments are
// loaded before the current block's MFMAs issue (register double buffering),
// and with 4 x TN accumulators consecutive MFMAs never depend on each other.
// Per 16-B B fragment the wave issues 4 MFMAs (one per row tile) and per A
// fragment TN -- the layer kernel with 16x16 per wave issued 1 per B load.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "kernels.h"
#include "philox.h"

namespace sca::kern {
namespace {

using f32x4 = __attribute__((ext_vector_type(4))) float;
using f32x16 = __attribute__((ext_vector_type(16))) float;
using f64x2 = __attribute__((ext_vector_type(2))) double;
using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;
constexpr int kTM = 4;  // row tiles (of 16) per wave

__device__ __forceinline__ float act_f(float v, int a) {
  switch (a) {
    case kMlpRelu: return fmaxf(v, 0.f);
    case kMlpSigmoid: return 1.f / (1.f + expf(-v));
    case kMlpTanh: return tanhf(v);
    default: return v;
  }
}

// Calls f(integral_constant<int, ACT>, integral_constant<bool, OF32>) for the
// runtime activation / output type: epilogues branch once, not per element.
template <class F>
__device__ __forceinline__ void act_dispatch(int act, bool of32, F&& f) {
  using std::integral_constant;
  switch (act * 2 + (of32 ? 1 : 0)) {
    case kMlpRelu * 2 + 1: f(integral_constant<int, kMlpRelu>{}, integral_constant<bool, true>{}); break;
    case kMlpRelu * 2: f(integral_constant<int, kMlpRelu>{}, integral_constant<bool, false>{}); break;
    case kMlpSigmoid * 2 + 1: f(integral_constant<int, kMlpSigmoid>{}, integral_constant<bool, true>{}); break;
    case kMlpSigmoid * 2: f(integral_constant<int, kMlpSigmoid>{}, integral_constant<bool, false>{}); break;
    case kMlpTanh * 2 + 1: f(integral_constant<int, kMlpTanh>{}, integral_constant<bool, true>{}); break;
    case kMlpTanh * 2: f(integral_constant<int, kMlpTanh>{}, integral_constant<bool, false>{}); break;
    case kMlpIdentity * 2 + 1: f(integral_constant<int, kMlpIdentity>{}, integral_constant<bool, true>{}); break;
    default: f(integral_constant<int, kMlpIdentity>{}, integral_constant<bool, false>{}); break;
  }
}

// VAE reparameterised input value z[row][k] (same Philox streams as the fused
// kernel's reparam() and mlp_layer's AMODE 2)
__device__ __forceinline__ float reparam_z(const DenseGemmArgs& a, int row, int k) {
  const int r = row % a.rows, smp = row / a.rows;
  const int kk = min(k, a.latent - 1);
  const float* h = a.H + size_t(r) * a.ldh;
  Philox rng(a.key, (uint64_t(r) << 24) ^ (uint64_t(smp) << 14) ^ uint64_t(kk));
  const float z = h[kk] + expf(0.5f * h[a.latent + kk]) * rng.normal();
  return k < a.latent ? z : 0.f;
}

// ---- operand fragments
template <int BF16> struct Frag;
template <> struct Frag<0> {  // fp32: one 16-k block = 4 MFMAs (16x16x4), 4 floats per lane
  using T = f32x4;
  static constexpr int kK = 16;
};
template <> struct Frag<1> {  // bf16: one 32-k block = 1 MFMA (16x16x32), 8 bf16 per lane
  using T = bf16x8;
  static constexpr int kK = 32;
};

template <int BF16, int AMODE>
__device__ __forceinline__ typename Frag<BF16>::T load_a(const DenseGemmArgs& a, int row, int kb, int kq) {
  row = min(row, a.rows_eff - 1);
  if constexpr (AMODE == 0) {
    if constexpr (BF16) {
      return *reinterpret_cast<const bf16x8*>(static_cast<const __bf16*>(a.A) + size_t(row) * a.lda + kb * 32 + kq * 8);
    } else {
      return *reinterpret_cast<const f32x4*>(static_cast<const float*>(a.A) + size_t(row) * a.lda + kb * 16 + kq * 4);
    }
  } else {
    typename Frag<BF16>::T v;
    constexpr int n = BF16 ? 8 : 4;
    const int k0 = kb * Frag<BF16>::kK + kq * n;
#pragma unroll
    for (int j = 0; j < n; ++j) {
      if constexpr (BF16) v[j] = __bf16(reparam_z(a, row, k0 + j));
      else v[j] = reparam_z(a, row, k0 + j);
    }
    return v;
  }
}

template <int BF16>
__device__ __forceinline__ f32x4 mma(const typename Frag<BF16>::T& x, const typename Frag<BF16>::T& y, f32x4 acc,
                                     int j) {
  if constexpr (BF16) {
    (void)j;
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, y, acc, 0, 0, 0);
  } else {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(x[j], y[j], acc, 0, 0, 0);
  }
}

template <int BF16, int AMODE, int TN>
__global__ __launch_bounds__(64) void dense_gemm_kernel(const DenseGemmArgs a) {
  using T = typename Frag<BF16>::T;
  const int lane = threadIdx.x, r16 = lane & 15, kq = lane >> 4;
  const int m0 = blockIdx.y * (16 * kTM);
  const int t0 = blockIdx.x * TN;  // first column tile
  const int ntiles = a.Np >> 4;
  const int KB = a.Kp / Frag<BF16>::kK;
  const T* W = static_cast<const T*>(a.W);
  const T* wt[TN];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) wt[tn] = W + size_t(min(t0 + tn, ntiles - 1)) * KB * 64 + lane;
  f32x4 acc[kTM][TN];
#pragma unroll
  for (int tm = 0; tm < kTM; ++tm)
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = f32x4{0.f, 0.f, 0.f, 0.f};
  T av[kTM], bv[TN];
#pragma unroll
  for (int tm = 0; tm < kTM; ++tm) av[tm] = load_a<BF16, AMODE>(a, m0 + 16 * tm + r16, 0, kq);
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) bv[tn] = wt[tn][0];
  for (int kb = 0; kb < KB; ++kb) {
    T an[kTM], bn[TN];
    const int kn = min(kb + 1, KB - 1);  // the last block reloads itself (never used)
#pragma unroll
    for (int tm = 0; tm < kTM; ++tm) an[tm] = load_a<BF16, AMODE>(a, m0 + 16 * tm + r16, kn, kq);
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) bn[tn] = wt[tn][size_t(kn) * 64];
    __builtin_amdgcn_sched_barrier(0);
    constexpr int J = BF16 ? 1 : 4;
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
      for (int tm = 0; tm < kTM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = mma<BF16>(av[tm], bv[tn], acc[tm][tn], j);
#pragma unroll
    for (int tm = 0; tm < kTM; ++tm) av[tm] = an[tm];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) bv[tn] = bn[tn];
  }
  // ---- epilogue (C/D map: col = lane & 15, row = (lane >> 4) * 4 + i)
  if (!a.mse) {
    act_dispatch(a.act, a.o_f32, [&](auto actc, auto of32c) {
      constexpr int ACT = decltype(actc)::value;
      constexpr bool OF32 = decltype(of32c)::value;
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int t = t0 + tn;
        if (t >= ntiles) break;
        const int col = t * 16 + r16;
        const bool live = col < a.N;
        const float bias = live ? a.bias[col] : 0.f;
#pragma unroll
        for (int tm = 0; tm < kTM; ++tm) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int row = m0 + 16 * tm + kq * 4 + i;
            if (row < a.rows_eff) {
              const float v = live ? act_f(acc[tm][tn][i] + bias, ACT) : 0.f;
              if constexpr (OF32) static_cast<float*>(a.O)[size_t(row) * a.ldo + col] = v;
              else static_cast<__bf16*>(a.O)[size_t(row) * a.ldo + col] = __bf16(v);
            }
          }
        }
      }
    });
    return;
  }
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) {
    const int t = t0 + tn;
    if (t >= ntiles) break;
    const int col = t * 16 + r16;
    const bool live = col < a.N;
    const float bias = live ? a.bias[col] : 0.f;
#pragma unroll
    for (int tm = 0; tm < kTM; ++tm) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m0 + 16 * tm + kq * 4 + i;
        {
          const bool ok = live && row < a.rows_eff;
          const int r = row % a.rows;
          float d = ok ? act_f(acc[tm][tn][i] + bias, a.act) - a.xref[size_t(r) * a.ldx + col] : 0.f;
          d *= d;
          d += __shfl_xor(d, 1, 64);
          d += __shfl_xor(d, 2, 64);
          d += __shfl_xor(d, 4, 64);
          d += __shfl_xor(d, 8, 64);
          if (r16 == 0 && row < a.rows_eff) atomicAdd(&a.mse[r], d);
        }
      }
    }
  }
}

// ---- LDS-tiled GEMM (bf16 or exact fp32).  A 256-thread workgroup (2 x 2
// waves) owns a BM x BN output tile (BM = 128 or 32, BN = 64).  Per K stage the
// A and W panels (128 B per row) are staged in LDS with full-line 16-B loads;
// each wave reads its BM/32 + BN/32 fragments with ds_read_b128 and issues
// (BM/32) * (BN/32) MFMAs per fragment step.  The LDS rows are XOR-swizzled
// (gemm_lds_kernel's sw()): fragment reads and staging stores are both
// bank-conflict-free.  Global loads run two stages ahead (two register sets)
// into two LDS buffers: the L2 / HBM round trip of stage k+2 overlaps the
// MFMAs of stages k and k+1.
//
// Grid: 1-D, remapped XCD-aware.  Workgroups are dealt round-robin over the 8
// XCDs (each with its own L2), so with a 2-D (N, M) grid the N tiles that share
// one A panel landed on 8 different XCDs and every A panel came from HBM 8
// times (r02d: 27 us for 8192 x 784 x 512 at ~6 TB/s of mostly redundant
// traffic).  The remap gives each XCD a contiguous run of tiles in (m, n)
// order, n fastest: an A panel is fetched from HBM once and then hit in that
// XCD's L2 by its other N tiles; W (<= 1 MB) stays L2-resident everywhere.
//
// Measured on MI355X (profiles/r02h_gemm): MLP 784-512-256-10 @ 8192 rows,
// layer 1 26.9 -> 23.7 us, layer 2 15.7 -> 14.6 us with the remap
// (SCA_GEMM_REMAP=0 restores the plain order for A/B runs); the 10-wide head
// 9.4 -> 6.0 us on 32 x 64 tiles.  Converting the fp64 batch while staging
// layer 1 (instead of the separate convert pass) measured 71-79 us vs 24 + 19:
// 4x the staging loads per chunk serialise the two-stage register pipeline.
//
// AMODE 0: A is bf16 [rows][lda]; 2: VAE reparameterised z from H.
// W is row-major [Npb][Kpb] bf16 (Kpb, Npb multiples of 64, zero padded).
using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;  // one 16-B staging chunk

template <int AMODE>
__device__ __forceinline__ bf16x8 stage_a(const DenseGemmArgs& a, int row, int k) {
  row = min(row, a.rows_eff - 1);
  if constexpr (AMODE == 0) {
    return *reinterpret_cast<const bf16x8*>(static_cast<const __bf16*>(a.A) + size_t(row) * a.lda + k);
  } else {
    bf16x8 v;
    if (k >= a.latent) {  // K padding past the latent width: no draws
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = __bf16(0.f);
      return v;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = __bf16(reparam_z(a, row, k + j));
    return v;
  }
}

using f64x4 = __attribute__((ext_vector_type(4))) double;

// AMODE 3: four fp64 request values (row `row`, [k, k + 4)) for one fp32
// staging chunk, kept raw in the register ring and converted at the LDS store
// (converting here would make the load wait at issue and drain the ring);
// elements past K (the Kp padding) are zero.  Two 16-B loads when in range
// and 16-B aligned (K even), else masked scalar loads.
__device__ __forceinline__ f64x4 stage_a64(const DenseGemmArgs& a, int row, int k) {
  row = min(row, a.rows_eff - 1);
  const double* x = static_cast<const double*>(a.A) + size_t(row) * a.lda + k;
  if (k + 3 < a.K && (a.lda & 1) == 0) {
    const f64x2 lo = *reinterpret_cast<const f64x2*>(x), hi = *reinterpret_cast<const f64x2*>(x + 2);
    return f64x4{lo[0], lo[1], hi[0], hi[1]};
  }
  f64x4 v;
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = k + j < a.K ? x[j] : 0.0;
  return v;
}

// One 16-B chunk of the A panel (row `row`, elements [k, k + 16 / sizeof(T))).
template <typename T, int AMODE>
__device__ __forceinline__ u32x4 stage_a_chunk(const DenseGemmArgs& a, int row, int k) {
  if constexpr (AMODE == 0) {
    row = min(row, a.rows_eff - 1);
    return *reinterpret_cast<const u32x4*>(static_cast<const T*>(a.A) + size_t(row) * a.lda + k);
  } else {
    static_assert(sizeof(T) == 2, "reparameterised A is staged as bf16");
    return __builtin_bit_cast(u32x4, stage_a<AMODE>(a, row, k));
  }
}

// bijective XCD-aware tile index for workgroup `L` of `nwg` (cdna guide §5)
__device__ __forceinline__ int xcd_tile(int L, int nwg) {
  const int xcd = L & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (L >> 3);
}

// Tile t (XCD-contiguous, from xcd_tile) -> (tile row, tile column) in
// groups of gm tile rows, column-major inside a group: the ~32 tiles an XCD
// runs at once cover gm A panels x 32/gm B panels instead of 1 x 32, so the
// XCD's 4 MB L2 serves each K slice to gm (A) and 32/gm (B) tiles.  At
// 8192^3 (256^2 tiles, row-major) the L2 hit rate was 44% and the fetch 2.3 GB
// per GEMM against hipBLASLt's 80% / 0.8 GB (profiles/r03i_gemm_l2).
__device__ __forceinline__ void grouped_tile(int t, int nM, int nN, int gm, int& mi, int& ni) {
  if (gm <= 1) {
    mi = t / nN;
    ni = t - mi * nN;
    return;
  }
  const int per = gm * nN, g = t / per, first = g * gm, gs = min(nM - first, gm), r = t - g * per;
  mi = first + r % gs;
  ni = r / gs;
}

// T = __bf16: v_mfma_f32_16x16x32_bf16, 64-deep K stages; T = float: exact
// fp32 products on v_mfma_f32_16x16x4_f32 (four per 16-B fragment), 32-deep
// stages.  The LDS image is the same in bytes either way: 128-B rows of eight
// 16-B chunks, XOR-swizzled per row pair.
template <typename T, int AMODE, int BM, int BN, int NT, int NS = 2, bool M32 = false>
__global__ __launch_bounds__(NT) void gemm_lds_kernel(const DenseGemmArgs a) {
  // M32 (fp32 only): v_mfma_f32_32x32x2_f32 on 32 x 32 tiles -- a wave's
  // BM/2 x 32 block is BM/64 accumulators of 16 registers; per 32-deep stage
  // lane (i, h) reads k in [16h, 16h + 16) of its A row / W row (4 x
  // ds_read_b128, same swizzled image) and the 16 MFMA steps pair k = s with
  // k = 16 + s.  Half the MFMA instructions of the 16x16x4 form for the same
  // FLOPs, and its 64-cycle dependent latency equals its issue interval, so
  // each accumulator chain issues back to back (cdna guide §3).
  static_assert(!M32 || sizeof(T) == 4, "M32 is the fp32 MFMA form");
  constexpr int kEl = 16 / int(sizeof(T));    // elements per 16-B chunk
  constexpr int kBKe = 8 * kEl;               // K elements per stage (128 B per row)
  constexpr int kLdr = kBKe;                  // LDS row = the 128-B panel row, XOR-swizzled (see sw())
  constexpr int WN = NT / 128;                // waves along N (2 along M); each wave owns BM/2 x 32
  constexpr int TM = BM / 32;                 // 16-row tiles per wave
  constexpr int TN = 2;                       // 16-col tiles per wave
  static_assert(M32 ? BN % (32 * WN) == 0 : BN == 32 * WN, "BN must be 32 x waves along N (a multiple for M32)");
  constexpr int CA = BM * 8 / NT;             // A staging chunks per thread (BM rows x 8 chunks)
  constexpr int CW = BN * 8 / NT;             // W staging chunks per thread
  constexpr int kBuf = (BM + BN) * kLdr;      // one LDS buffer: A panel then W panel
  static_assert(CA >= 1 && CW >= 1, "tile too small for the stagers");
  // Element offset of 16-B chunk `ch` (0..7) of panel row `r`: chunk ch ^ ((r >> 1) & 7).
  // A ds_read_b128 lane group (16 rows, one chunk) then hits 16 distinct
  // 16-B slots of the 256-B bank row, and a staging store group (2 rows x 8
  // chunks) fills the two halves -- both conflict-free (the 144-B padded rows
  // this replaces left the stores 2-way conflicted: 33% of LDS-active cycles,
  // profiles/r02h_gemm/pmc_summary.md).
  auto sw = [](int r, int ch) { return r * kLdr + ((ch ^ ((r >> 1) & 7)) * kEl); };
  __shared__ __attribute__((aligned(16))) T smem[2 * kBuf];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wr = wave / WN, wc = wave % WN, r16 = lane & 15, kq = lane >> 4;
  const int nN = (a.Np + BN - 1) / BN;
  const int t = a.xcd_remap ? xcd_tile(blockIdx.x, gridDim.x) : int(blockIdx.x);
  const int m0 = (t / nN) * BM, n0 = (t % nN) * BN;
  const T* W = static_cast<const T*>(a.W);
  const int KS = a.Kp / kBKe;
  // NS sets of staging registers; every set index below is a compile-time
  // constant (the K loop is unrolled by NS), so they stay in VGPRs
  using RA = std::conditional_t<AMODE == 3, f64x4, u32x4>;  // A ring element (raw fp64 for AMODE 3)
  RA ra[NS][CA];
  u32x4 rw[NS][CW];
  auto gload = [&](int ks, bool live, RA* ra, u32x4* rw) {
    // A computed on the fly (AMODE 2: reparameterised draws, no memory loads)
    // is skipped for the clamped stages past the end; loaded operands are not
    // (see the unconditional ring below)
    if (AMODE != 2 || live) {
#pragma unroll
      for (int j = 0; j < CA; ++j) {
        const int c = tid + NT * j;
        if constexpr (AMODE == 3) ra[j] = stage_a64(a, m0 + (c >> 3), ks * kBKe + (c & 7) * kEl);
        else ra[j] = stage_a_chunk<T, AMODE>(a, m0 + (c >> 3), ks * kBKe + (c & 7) * kEl);
      }
    }
#pragma unroll
    for (int j = 0; j < CW; ++j) {
      const int c = tid + NT * j;
      rw[j] = *reinterpret_cast<const u32x4*>(W + size_t(min(n0 + (c >> 3), a.Np - 1)) * a.Kp + ks * kBKe +
                                              (c & 7) * kEl);
    }
  };
  auto lstore = [&](int buf, const RA* ra, const u32x4* rw) {
    T* As = smem + buf * kBuf;
    T* Ws = As + BM * kLdr;
#pragma unroll
    for (int j = 0; j < CA; ++j) {
      const int c = tid + NT * j;
      if constexpr (AMODE == 3)
        *reinterpret_cast<f32x4*>(As + sw(c >> 3, c & 7)) =
            f32x4{float(ra[j][0]), float(ra[j][1]), float(ra[j][2]), float(ra[j][3])};
      else
        *reinterpret_cast<u32x4*>(As + sw(c >> 3, c & 7)) = ra[j];
    }
#pragma unroll
    for (int j = 0; j < CW; ++j) {
      const int c = tid + NT * j;
      *reinterpret_cast<u32x4*>(Ws + sw(c >> 3, c & 7)) = rw[j];
    }
  };
  f32x4 acc[TM][TN];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm)
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int TM32 = M32 ? BM / 64 : 1, TN32 = M32 ? BN / (32 * WN) : 1;
  constexpr int WCOLS = BN / WN;  // columns per wave
  f32x16 acc32[TM32][TN32];
#pragma unroll
  for (int t = 0; t < TM32; ++t)
#pragma unroll
    for (int u = 0; u < TN32; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc32[t][u][i] = 0.f;
  auto compute = [&](int buf) {
    const T* As = smem + buf * kBuf;
    const T* Ws = As + BM * kLdr;
    if constexpr (M32) {
      const int i32 = lane & 31, h = lane >> 5;
      f32x4 bq[TN32][4], aq[TM32][4];
#pragma unroll
      for (int u = 0; u < TN32; ++u)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          bq[u][c] = *reinterpret_cast<const f32x4*>(Ws + sw(wc * WCOLS + u * 32 + i32, 4 * h + c));
#pragma unroll
      for (int t = 0; t < TM32; ++t)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          aq[t][c] = *reinterpret_cast<const f32x4*>(As + sw(wr * (BM / 2) + t * 32 + i32, 4 * h + c));
#pragma unroll
      for (int s = 0; s < 16; ++s)
#pragma unroll
        for (int t = 0; t < TM32; ++t)
#pragma unroll
          for (int u = 0; u < TN32; ++u)
            acc32[t][u] = __builtin_amdgcn_mfma_f32_32x32x2f32(aq[t][s >> 2][s & 3], bq[u][s >> 2][s & 3], acc32[t][u],
                                                               0, 0, 0);
      return;
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {  // two 16-B fragments per row per stage (bytes kk * 64 + kq * 16)
      u32x4 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *reinterpret_cast<const u32x4*>(As + sw(wr * (BM / 2) + i * 16 + r16, kk * 4 + kq));
#pragma unroll
      for (int i = 0; i < TN; ++i)
        bf[i] = *reinterpret_cast<const u32x4*>(Ws + sw(wc * 32 + i * 16 + r16, kk * 4 + kq));
      if constexpr (sizeof(T) == 2) {
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
          for (int tn = 0; tn < TN; ++tn)
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[tm]),
                                                                  __builtin_bit_cast(bf16x8, bf[tn]), acc[tm][tn], 0, 0, 0);
      } else {
        // lane (r16, kq) holds k = kk * 16 + 4 kq + j of MFMA j: every k once
        // per stage.  j outermost: consecutive MFMAs go to the TM x TN
        // independent accumulators, so the 16x16x4 f32 MFMA's 40-cycle
        // dependent latency (32-cycle issue) is never exposed; each
        // accumulator still sees j = 0..3 in order (bit-identical sums).
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int tm = 0; tm < TM; ++tm)
#pragma unroll
            for (int tn = 0; tn < TN; ++tn)
              acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x4f32(__builtin_bit_cast(f32x4, af[tm])[j],
                                                                 __builtin_bit_cast(f32x4, bf[tn])[j], acc[tm][tn], 0,
                                                                 0, 0);
      }
    }
  };
  // NS register sets: the global loads of stage ks + NS are issued as stage ks
  // starts (its set was stored to LDS one stage earlier), so NS stages of
  // L2 / HBM latency are in flight behind the MFMAs; LDS is double-buffered.
  // Loads and LDS stores are issued unconditionally (stage indices clamped to
  // the last stage, the K loop padded to a multiple of NS with the compute
  // skipped): a load inside a branch makes the compiler's vmcnt bookkeeping
  // wait for every outstanding load at the join, which drains the ring.
#pragma unroll
  for (int st = 0; st < NS; ++st) gload(min(st, KS - 1), st < KS, ra[st], rw[st]);
  lstore(0, ra[0], rw[0]);
  __syncthreads();
  const int KSr = (KS + NS - 1) / NS * NS;
  for (int ks0 = 0; ks0 < KSr; ks0 += NS) {
#pragma unroll
    for (int st = 0; st < NS; ++st) {
      const int ks = ks0 + st;
      gload(min(ks + NS, KS - 1), ks + NS < KS, ra[st], rw[st]);
      if (ks < KS) compute(ks & 1);
      lstore((ks + 1) & 1, ra[(st + 1) % NS], rw[(st + 1) % NS]);  // past the last stage: never read
      __syncthreads();
    }
  }
  // ---- epilogue (C/D map: col = lane & 15, row = (lane >> 4) * 4 + i)
  if (a.out64) {  // N <= 16: wave wc = 0, tile tn = 0 holds a row's every column (16 lanes of one kq)
    if (wc != 0 || n0 != 0) return;
    const bool live = r16 < a.N;
    const float bias = live ? a.bias[r16] : 0.f;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m0 + wr * (BM / 2) + tm * 16 + kq * 4 + i;
        const float v = act_f(acc[tm][0][i] + bias, a.act);
        if (a.out_mode == 1) {  // softmax over the row's N lanes
          float m = live ? v : -3.4e38f;
          m = fmaxf(m, __shfl_xor(m, 1, 64));
          m = fmaxf(m, __shfl_xor(m, 2, 64));
          m = fmaxf(m, __shfl_xor(m, 4, 64));
          m = fmaxf(m, __shfl_xor(m, 8, 64));
          const float e = live ? expf(v - m) : 0.f;
          float sum = e;
          sum += __shfl_xor(sum, 1, 64);
          sum += __shfl_xor(sum, 2, 64);
          sum += __shfl_xor(sum, 4, 64);
          sum += __shfl_xor(sum, 8, 64);
          if (live && row < a.rows_eff) a.out64[size_t(row) * a.N + r16] = double(e / sum);
        } else if (a.out_mode == 2) {
          if (r16 == 0 && row < a.rows_eff) {
            a.out64[size_t(row) * 2] = 1.0 - double(v);
            a.out64[size_t(row) * 2 + 1] = double(v);
          }
        } else if (live && row < a.rows_eff) {
          a.out64[size_t(row) * a.N + r16] = double(v);
        }
      }
    }
    return;
  }
  const int n_store = a.n_store > 0 ? a.n_store : a.Np;
  if constexpr (M32) {  // C/D map of 32x32: col = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)
    if (!a.mse) {
      act_dispatch(a.act, a.o_f32, [&](auto actc, auto of32c) {
        constexpr int ACT = decltype(actc)::value;
        constexpr bool OF32 = decltype(of32c)::value;
#pragma unroll
        for (int u = 0; u < TN32; ++u) {
          const int col = n0 + wc * WCOLS + u * 32 + (lane & 31);
          const bool live = col < a.N, store = col < n_store;
          const float bias = live ? a.bias[col] : 0.f;
#pragma unroll
          for (int t = 0; t < TM32; ++t) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int row = m0 + wr * (BM / 2) + t * 32 + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
              const float v = live ? act_f(acc32[t][u][i] + bias, ACT) : 0.f;
              if (store && row < a.rows_eff) {
                if constexpr (OF32) static_cast<float*>(a.O)[size_t(row) * a.ldo + col] = v;
                else static_cast<__bf16*>(a.O)[size_t(row) * a.ldo + col] = __bf16(v);
              }
            }
          }
        }
      });
      return;
    }
#pragma unroll
    for (int u = 0; u < TN32; ++u) {
      const int col = n0 + wc * WCOLS + u * 32 + (lane & 31);
      const bool live = col < a.N, store = col < n_store;
      const float bias = live ? a.bias[col] : 0.f;
#pragma unroll
      for (int t = 0; t < TM32; ++t) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int row = m0 + wr * (BM / 2) + t * 32 + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
          const float v = live ? act_f(acc32[t][u][i] + bias, a.act) : 0.f;
          {  // the 32 lanes of a half hold one row's 32 columns: sum them, one atomic per row
            const bool ok = live && store && row < a.rows_eff;
            const int r = row % a.rows;
            float d = ok ? v - a.xref[size_t(r) * a.ldx + col] : 0.f;
            d *= d;
#pragma unroll
            for (int o = 1; o < 32; o <<= 1) d += __shfl_xor(d, o, 64);
            if ((lane & 31) == 0 && row < a.rows_eff) atomicAdd(&a.mse[r], d);
          }
        }
      }
    }
    return;
  }
  if (!a.mse) {
    act_dispatch(a.act, a.o_f32, [&](auto actc, auto of32c) {
      constexpr int ACT = decltype(actc)::value;
      constexpr bool OF32 = decltype(of32c)::value;
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int col = n0 + wc * 32 + tn * 16 + r16;
        if (col >= n_store) continue;
        const bool live = col < a.N;
        const float bias = live ? a.bias[col] : 0.f;
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int row = m0 + wr * (BM / 2) + tm * 16 + kq * 4 + i;
            if (row < a.rows_eff) {
              const float v = live ? act_f(acc[tm][tn][i] + bias, ACT) : 0.f;
              if constexpr (OF32) static_cast<float*>(a.O)[size_t(row) * a.ldo + col] = v;
              else static_cast<__bf16*>(a.O)[size_t(row) * a.ldo + col] = __bf16(v);
            }
          }
        }
      }
    });
    return;
  }
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) {
    const int col = n0 + wc * 32 + tn * 16 + r16;
    if (col >= n_store) continue;
    const bool live = col < a.N;
    const float bias = live ? a.bias[col] : 0.f;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m0 + wr * (BM / 2) + tm * 16 + kq * 4 + i;
        {
          const bool ok = live && row < a.rows_eff;
          const int r = row % a.rows;
          float d = ok ? act_f(acc[tm][tn][i] + bias, a.act) - a.xref[size_t(r) * a.ldx + col] : 0.f;
          d *= d;
          d += __shfl_xor(d, 1, 64);
          d += __shfl_xor(d, 2, 64);
          d += __shfl_xor(d, 4, 64);
          d += __shfl_xor(d, 8, 64);
          if (r16 == 0 && row < a.rows_eff) atomicAdd(&a.mse[r], d);
        }
      }
    }
  }
}

// ---- bf16 GEMM with a global_load_lds ring (S stages in flight)
// For layers whose 128 x 128 tiles fill the chip (e.g. the MLP's 784 -> 512
// layer at 8192 rows: 256 tiles).  The register-staged kernel above keeps two
// 64-deep stages in flight per workgroup and is latency bound there (MFMA busy
// 9%, profiles/r02h_gemm): each CU streams ~400 KB of A and W per tile, so at
// ~1.5-2 us of L2 / HBM latency it needs >100 KB in flight.  Here the loads are
// LDS-DMA (global_load_lds_dwordx4: no staging VGPRs, no ds_write pass) into an
// S-deep ring of 32 KB stages (S = 4: 128 KB, one workgroup per CU), waited
// with counted `s_waitcnt vmcnt` and raw `s_barrier` so the younger stages stay
// in flight across the barrier (cdna guide §5 "Pipelining across barriers").
//
// The LDS image is lane-linear per glds instruction (base + lane * 16 B), so
// the row XOR swizzle of the register-staged kernel (chunk ^ ((row >> 1) & 7):
// conflict-free ds_read_b128 fragment reads) is applied to the per-lane GLOBAL
// source address instead, and the same involution on the read (guide rule 21).
// 4 waves (2 x 2), each a 64 x 64 quadrant = 4 x 4 16x16x32 accumulators.
template <int S>
__global__ __launch_bounds__(256) void gemm_glds_kernel(const DenseGemmArgs a) {
  constexpr int BM = 128, BN = 128, BK = 64;
  constexpr int kStageA = BM * BK, kStage = (BM + BN) * BK;  // elements
  extern __shared__ __attribute__((aligned(16))) __bf16 ring[];  // S x [A 128 x 64 | B 128 x 64], one array
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wr = wave >> 1, wc = wave & 1, r16 = lane & 15, kq = lane >> 4;
  const int nN = (a.Np + BN - 1) / BN;
  int mi, ni;
  grouped_tile(xcd_tile(blockIdx.x, gridDim.x), (a.rows_eff + BM - 1) / BM, nN, a.group_m, mi, ni);
  const int m0 = mi * BM, n0 = ni * BN;
  const int KS = a.Kp / BK;
  const __bf16* A = static_cast<const __bf16*>(a.A);
  const __bf16* W = static_cast<const __bf16*>(a.W);
  // this thread's 4 + 4 source rows / swizzled chunks (fixed across stages)
  const __bf16* srcA[4];
  const __bf16* srcB[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int L = (j * 4 + wave) * 64 + lane;  // LDS chunk of instruction j: lane-linear 1 KB per wave
    const int r = L >> 3, c = (L & 7) ^ ((r >> 1) & 7);
    srcA[j] = A + size_t(min(m0 + r, a.rows_eff - 1)) * a.lda + c * 8;
    srcB[j] = W + size_t(min(n0 + r, a.Np - 1)) * a.Kp + c * 8;
  }
  auto issue = [&](int ks) {
    __bf16* st = ring + (ks % S) * kStage;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_global_load_lds(
          (const void __attribute__((address_space(1)))*)(srcA[j] + ks * BK),
          (void __attribute__((address_space(3)))*)(st + (j * 4 + wave) * 512), 16, 0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_global_load_lds(
          (const void __attribute__((address_space(1)))*)(srcB[j] + ks * BK),
          (void __attribute__((address_space(3)))*)(st + kStageA + (j * 4 + wave) * 512), 16, 0, 0);
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int st = 0; st < S - 1; ++st)
    if (st < KS) issue(st);
  for (int ks = 0; ks < KS; ++ks) {
    // stage ks complete: the younger issued stages (<= S - 2, 8 glds each) may stay in flight
    const int younger = min(ks + S - 2, KS - 1) - ks;
    if (younger >= 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's DMA of stage ks landed; everyone is done reading ks - 1
    __builtin_amdgcn_sched_barrier(0);
    if (ks + S - 1 < KS) issue(ks + S - 1);  // into the slot of stage ks - 1
    const __bf16* As = ring + (ks % S) * kStage;
    const __bf16* Bs = As + kStageA;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int c = kk * 4 + kq;
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ra = wr * 64 + i * 16 + r16, rb = wc * 64 + i * 16 + r16;
        af[i] = *reinterpret_cast<const bf16x8*>(As + ra * BK + ((c ^ ((ra >> 1) & 7)) << 3));
        bfr[i] = *reinterpret_cast<const bf16x8*>(Bs + rb * BK + ((c ^ ((rb >> 1) & 7)) << 3));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  // ---- epilogue (C/D map: col = lane & 15, row = (lane >> 4) * 4 + i)
  const int n_store = a.n_store > 0 ? a.n_store : a.Np;
#pragma unroll
  for (int tn = 0; tn < 4; ++tn) {
    const int col = n0 + wc * 64 + tn * 16 + r16;
    const bool live = col < a.N;
    const float bias = live ? a.bias[col] : 0.f;
#pragma unroll
    for (int tm = 0; tm < 4; ++tm) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m0 + wr * 64 + tm * 16 + kq * 4 + i;
        if (!a.mse) {
          if (row < a.rows_eff && col < n_store) {
            const float v = live ? act_f(acc[tm][tn][i] + bias, a.act) : 0.f;
            if (a.o_f32) static_cast<float*>(a.O)[size_t(row) * a.ldo + col] = v;
            else static_cast<__bf16*>(a.O)[size_t(row) * a.ldo + col] = __bf16(v);
          }
        } else {
          const bool ok = live && row < a.rows_eff && col < n_store;
          const int r = row % a.rows;
          float d = ok ? act_f(acc[tm][tn][i] + bias, a.act) - a.xref[size_t(r) * a.ldx + col] : 0.f;
          d *= d;
          d += __shfl_xor(d, 1, 64);
          d += __shfl_xor(d, 2, 64);
          d += __shfl_xor(d, 4, 64);
          d += __shfl_xor(d, 8, 64);
          if (r16 == 0 && row < a.rows_eff) atomicAdd(&a.mse[r], d);
        }
      }
    }
  }
}

// Epilogue of the 256 x 256 kernels: a wave's 128 x (16 TN) block of fp32
// accumulators (acc[tm][tn], C/D map col = lane & 15, row = (lane >> 4) * 4 +
// i) plus bias and a compile-time activation, stored as fp32 or bf16.
template <int ACT, bool OF32, int TN>
__device__ __forceinline__ void epi_256(const DenseGemmArgs& a, const f32x4 (&acc)[8][TN], int m0, int n0, int wr,
                                        int wc, int r16, int kq) {
  const int n_store = a.n_store > 0 ? a.n_store : a.Np;
  if (m0 + 256 <= a.rows_eff && n0 + 256 <= min(n_store, a.N)) {
    // interior tile (every tile of a large GEMM): no per-element predicates,
    // one row pointer per (tm, i) and the column tiles as immediate offsets
    const int col0 = n0 + wc * (16 * TN) + r16;
    float bias[TN];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) bias[tn] = a.bias[col0 + tn * 16];
#pragma unroll
    for (int tm = 0; tm < 8; ++tm) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const size_t off = size_t(m0 + wr * 128 + tm * 16 + kq * 4 + i) * a.ldo + col0;
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
          const float v = act_f(acc[tm][tn][i] + bias[tn], ACT);
          if constexpr (OF32) static_cast<float*>(a.O)[off + tn * 16] = v;
          else static_cast<__bf16*>(a.O)[off + tn * 16] = __bf16(v);
        }
      }
    }
    return;
  }
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) {
    const int col = n0 + wc * (16 * TN) + tn * 16 + r16;
    const bool live = col < a.N;
    const bool keep = col < n_store;
    const float bias = live ? a.bias[col] : 0.f;
#pragma unroll
    for (int tm = 0; tm < 8; ++tm) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m0 + wr * 128 + tm * 16 + kq * 4 + i;
        const float v = live ? act_f(acc[tm][tn][i] + bias, ACT) : 0.f;
        if (keep && row < a.rows_eff) {
          if constexpr (OF32) static_cast<float*>(a.O)[size_t(row) * a.ldo + col] = v;
          else static_cast<__bf16*>(a.O)[size_t(row) * a.ldo + col] = __bf16(v);
        }
      }
    }
  }
}
// reconstruction-error form: per-row sum of squared differences against xref
template <int TN>
__device__ __forceinline__ void epi_256_mse(const DenseGemmArgs& a, const f32x4 (&acc)[8][TN], int m0, int n0,
                                            int wr, int wc, int r16, int kq) {
  const int n_store = a.n_store > 0 ? a.n_store : a.Np;
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) {
    const int col = n0 + wc * (16 * TN) + tn * 16 + r16;
    const bool live = col < a.N;
    const float bias = live ? a.bias[col] : 0.f;
#pragma unroll
    for (int tm = 0; tm < 8; ++tm) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m0 + wr * 128 + tm * 16 + kq * 4 + i;
        const bool ok = live && row < a.rows_eff && col < n_store;
        const int r = row % a.rows;
        float d = ok ? act_f(acc[tm][tn][i] + bias, a.act) - a.xref[size_t(r) * a.ldx + col] : 0.f;
        d *= d;
        d += __shfl_xor(d, 1, 64);
        d += __shfl_xor(d, 2, 64);
        d += __shfl_xor(d, 4, 64);
        d += __shfl_xor(d, 8, 64);
        if (r16 == 0 && row < a.rows_eff) atomicAdd(&a.mse[r], d);
      }
    }
  }
}

// one uniform dispatch on (mse, act, output type), outside the element loops
template <int TN>
__device__ __forceinline__ void epi_256_store(const DenseGemmArgs& a, const f32x4 (&acc)[8][TN], int m0, int n0,
                                              int wr, int wc, int r16, int kq) {
  switch (a.mse ? -1 : a.act * 2 + (a.o_f32 ? 1 : 0)) {
    case kMlpIdentity * 2 + 1: epi_256<kMlpIdentity, true, TN>(a, acc, m0, n0, wr, wc, r16, kq); break;
    case kMlpIdentity * 2: epi_256<kMlpIdentity, false, TN>(a, acc, m0, n0, wr, wc, r16, kq); break;
    case kMlpRelu * 2 + 1: epi_256<kMlpRelu, true, TN>(a, acc, m0, n0, wr, wc, r16, kq); break;
    case kMlpRelu * 2: epi_256<kMlpRelu, false, TN>(a, acc, m0, n0, wr, wc, r16, kq); break;
    case kMlpSigmoid * 2 + 1: epi_256<kMlpSigmoid, true, TN>(a, acc, m0, n0, wr, wc, r16, kq); break;
    case kMlpSigmoid * 2: epi_256<kMlpSigmoid, false, TN>(a, acc, m0, n0, wr, wc, r16, kq); break;
    case kMlpTanh * 2 + 1: epi_256<kMlpTanh, true, TN>(a, acc, m0, n0, wr, wc, r16, kq); break;
    case kMlpTanh * 2: epi_256<kMlpTanh, false, TN>(a, acc, m0, n0, wr, wc, r16, kq); break;
    default: epi_256_mse<TN>(a, acc, m0, n0, wr, wc, r16, kq); break;
  }
}

// ---- bf16 GEMM, 256 x 256 tiles, 4 waves of 128 x 128 (one wave per SIMD)
// The 8-wave kernels read each A / B fragment from LDS 4x / 2x (a wave's
// 128 x 64 block): 192 KB of ds_read per 64-deep K tile per CU, ~75% of the
// MFMA time (LDS-bound phases).  Here a wave owns 128 x 128 (8 x 8 16x16
// accumulators = 256 registers, in AGPRs at one wave per SIMD): 128 KB of
// ds_read per K tile, 25% of the MFMA time, and the next k-step's 16
// fragments are read while the current 64 MFMAs issue (two register sets).
// LDS-DMA double buffer, one vmcnt(0) + barrier per K tile (the next tile
// had the whole K tile of MFMAs, ~1 us, to land).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_w4_kernel(
    const DenseGemmArgs a) {
  constexpr int BM = 256, BN = 256, BK = 64;
  constexpr int kStageA = BM * BK, kStage = (BM + BN) * BK;
  extern __shared__ __attribute__((aligned(16))) __bf16 ring[];  // 2 x [A 256 x 64 | B 256 x 64]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wr = wave >> 1, wc = wave & 1, r16 = lane & 15, kq = lane >> 4;
  const int nN = (a.Np + BN - 1) / BN;
  int mi, ni;
  grouped_tile(xcd_tile(blockIdx.x, gridDim.x), (a.rows_eff + BM - 1) / BM, nN, a.group_m, mi, ni);
  const int m0 = mi * BM, n0 = ni * BN;
  const int KS = a.Kp / BK;
  const __bf16* A = static_cast<const __bf16*>(a.A);
  const __bf16* W = static_cast<const __bf16*>(a.W);
  const __bf16* srcA[8];
  const __bf16* srcB[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int L = (j * 4 + wave) * 64 + lane;  // LDS chunk of instruction j (1 KB per wave-instruction)
    const int r = L >> 3, c = (L & 7) ^ ((r >> 1) & 7);
    srcA[j] = A + size_t(min(m0 + r, a.rows_eff - 1)) * a.lda + c * 8;
    srcB[j] = W + size_t(min(n0 + r, a.Np - 1)) * a.Kp + c * 8;
  }
  auto issue = [&](int ks) {
    __bf16* st = ring + (ks & 1) * kStage;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      __builtin_amdgcn_global_load_lds(
          (const void __attribute__((address_space(1)))*)(srcA[j] + ks * BK),
          (void __attribute__((address_space(3)))*)(st + (j * 4 + wave) * 512), 16, 0, 0);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      __builtin_amdgcn_global_load_lds(
          (const void __attribute__((address_space(1)))*)(srcB[j] + ks * BK),
          (void __attribute__((address_space(3)))*)(st + kStageA + (j * 4 + wave) * 512), 16, 0, 0);
  };
  auto frag = [&](const __bf16* b, int row, int kk) {
    const int c = kk * 4 + kq;
    return *reinterpret_cast<const bf16x8*>(b + row * BK + ((c ^ ((row >> 1) & 7)) << 3));
  };
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // Per K tile ks (buffer ks & 1):
  //   reads of k-step 1 fly under k-step 0's 64 MFMAs (k-step 0's fragments
  //   were read under the previous tile's k-step 1); then lgkmcnt(0) +
  //   vmcnt(0) (tile ks + 1 landed) + barrier; then tile ks + 2 is issued into
  //   this tile's buffer (every wave's reads of it retired before the barrier)
  //   and tile ks + 1's k-step-0 fragments are read under k-step 1's MFMAs.
  bf16x8 a0[8], b0[8], a1[8], b1[8];
  issue(0);
  if (KS > 1) {
    issue(1);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // tile 0 (16 glds per thread per tile)
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a0[i] = frag(ring, wr * 128 + i * 16 + r16, 0);
    b0[i] = frag(ring + kStageA, wc * 128 + i * 16 + r16, 0);
  }
  for (int ks = 0; ks < KS; ++ks) {
    const __bf16* As = ring + (ks & 1) * kStage;
    const __bf16* Bs = As + kStageA;
    // k-step 0's fragments (read under the previous MFMAs) retired, as a
    // builtin so hipcc's wait tracking sees it: the 16 reads below then need
    // no wait before the MFMAs (lgkmcnt cannot express 16 younger reads)
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0), vmcnt / expcnt untouched
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      a1[i] = frag(As, wr * 128 + i * 16 + r16, 1);
      b1[i] = frag(Bs, wc * 128 + i * 16 + r16, 1);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[i], b0[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0), as a builtin (hipcc's tracker sees it)
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (ks + 2 < KS) issue(ks + 2);
    if (ks + 1 < KS) {
      const __bf16* An = ring + ((ks + 1) & 1) * kStage;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        a0[i] = frag(An, wr * 128 + i * 16 + r16, 0);
        b0[i] = frag(An + kStageA, wc * 128 + i * 16 + r16, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[i], b1[j], acc[i][j], 0, 0, 0);
  }
  epi_256_store(a, acc, m0, n0, wr, wc, r16, kq);  // (C/D map: col = lane & 15, row = (lane >> 4) * 4 + i)
}

// ---- bf16 GEMM, 256 x 256 tiles, 8-phase ping-pong schedule
// Same tile and wave layout as gemm_glds256_kernel, but each 64-deep K tile is
// four phases, one per 64 x 32 quadrant of a wave's 128 x 64 block (16
// MFMAs), and the two wave groups (wr = 0 / 1) run one barrier apart, so one
// group's ds_reads overlap the other's MFMAs on every SIMD (cdna guide §5
// "The 256^2 8-phase template", T3 + T4 + T5).  LDS: 8 half-tile buffers
// (K-tile parity x A/B x rows 0-127 / 128-255) of 128 x 64 bf16; one half
// tile (2 glds per thread) is issued per phase:
//   q0: read all B + A rows 0-63; issue A1 of tile t+1;       | MFMA (mh0, nh0)
//       retire the B reads before the barrier (B0 is restaged in q1)
//   q1: read A rows 64-127; issue B0 of tile t+2              | MFMA (mh0, nh1)
//   q2: issue B1 of tile t+2                                  | MFMA (mh1, nh0)
//   q3: issue A0 of tile t+2; vmcnt(6) = tile t+1 landed      | MFMA (mh1, nh1)
//       (3 younger half tiles in flight), placed before the first barrier:
//       the other group reads it one barrier later (the stagger's margin)
// so a buffer is restaged >= 2 phases after its last read (B0: 1 phase, with
// the reads retired first), the last half tile of a K tile is issued 3 phases
// before its wait, and data is read only after a barrier that follows the
// vmcnt of every issuing wave.  Loads are counted by hand (raw s_barrier,
// explicit s_waitcnt): __syncthreads() would drain the DMA queue.
//
// SPREAD (path 6): the fragment reads spread over the phases as 12 / 4 / 8 /
// 0 (q0: B cols 0-31 + A rows 0-63, q1: B cols 32-63, q2: A rows 64-127)
// instead of 16 / 8 / 0 / 0, so no phase asks the LDS for more than ~75% of
// the other group's MFMA time (16 ds_read_b128 per wave x 4 waves is 256
// LDS clocks = 16 MFMAs).  Restaging moves with the reads: B0 / B1 of tile
// t + 2 in q2 / q3 (the q1 B reads retired before q1's barrier), A0 of tile
// t + 2 in q3 (the q2 A reads retired before q2's barrier), A1 of tile t + 1
// in q0 as before; vmcnt(6) in q3 as before.
// ABL (ablation, paths 7 / 8, timing only -- results are garbage): 1 drops
// the MFMAs (the fragments are kept live), 2 drops the fragment ds_reads.
// RING (path 9, SPREAD only): the 8 parity buffers become a ring of 10 half
// tiles (160 KB, all of the CU's LDS), so every half tile is issued >= 5
// phases before its wait instead of 3 (the no-MFMA ablation showed the
// loads latency bound, profiles/r03i_gemm_l2).  Half tile p = 4 t + {B0, B1,
// A0, A1} lives in slot p mod 10, so A of tile t + 2 reuses the B slots of
// tile t (free after q1) and is issued in q2, B of tile t + 3 reuses A's
// (free after q2) in q3; the q3 wait leaves the 6 younger half tiles in
// flight (vmcnt(12)).
template <bool SPREAD, int ABL = 0, bool RING = false>
__global__ __launch_bounds__(512) void gemm_8ph_kernel(const DenseGemmArgs a) {
  constexpr int BM = 256, BN = 256, BK = 64, HT = 128 * BK;  // half tile (elements)
  extern __shared__ __attribute__((aligned(16))) __bf16 ring[];  // [parity][A/B][half] x HT
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wr = wave >> 2, wc = wave & 3, r16 = lane & 15, kq = lane >> 4;
  const int nN = (a.Np + BN - 1) / BN;
  int mi, ni;
  grouped_tile(xcd_tile(blockIdx.x, gridDim.x), (a.rows_eff + BM - 1) / BM, nN, a.group_m, mi, ni);
  const int m0 = mi * BM, n0 = ni * BN;
  const int KT = a.Kp / BK;
  const __bf16* A = static_cast<const __bf16*>(a.A);
  const __bf16* W = static_cast<const __bf16*>(a.W);
  // this thread's two chunks of any half tile (rows r, swizzled chunk c)
  const __bf16* srcA[2][2];  // [half][j]
  const __bf16* srcB[2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int L = (j * 8 + wave) * 64 + lane;
    const int r = L >> 3, c = (L & 7) ^ ((r >> 1) & 7);
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      srcA[hf][j] = A + size_t(min(m0 + hf * 128 + r, a.rows_eff - 1)) * a.lda + c * 8;
      srcB[hf][j] = W + size_t(min(n0 + hf * 128 + r, a.Np - 1)) * a.Kp + c * 8;
    }
  }
  auto buf = [&](int kt, int op, int hf) -> __bf16* {
    if constexpr (RING) {
      const int s0 = (4 * (kt % 5)) % 10;  // slot of B0; B1 follows, A0 / A1 after that mod 10
      return ring + ((op == 1 ? s0 : (s0 + 2) % 10) + hf) * HT;
    } else {
      return ring + (((kt & 1) * 2 + op) * 2 + hf) * HT;
    }
  };
  auto issue = [&](int kt, int op, int hf) {  // half tile (op 0 = A, 1 = B) of K tile kt
    __bf16* dst = buf(kt, op, hf);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_global_load_lds(
          (const void __attribute__((address_space(1)))*)((op == 0 ? srcA[hf][j] : srcB[hf][j]) + kt * BK),
          (void __attribute__((address_space(3)))*)(dst + (j * 8 + wave) * 512), 16, 0, 0);
  };
  auto frag = [&](const __bf16* b, int row, int kk) {
    const int c = kk * 4 + kq;
    return *reinterpret_cast<const bf16x8*>(b + row * BK + ((c ^ ((row >> 1) & 7)) << 3));
  };
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 am0[4][2], am1[4][2], bq[4][2];
  auto mfma_q = [&](bf16x8 (&af)[4][2], int mh, int nh) {
    if constexpr (ABL == 1) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(af[i][kk]), "v"(bq[nh * 2 + (i & 1)][kk]));
      return;
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[mh * 4 + i][nh * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][kk], bq[nh * 2 + j][kk], acc[mh * 4 + i][nh * 2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // prologue: tile 0 whole, then B0 / B1 / A0 of tile 1 (3 half tiles may fly);
  // RING: tiles 0 and 1 whole and B of tile 2 (6 may fly)
  issue(0, 1, 0);
  issue(0, 1, 1);
  issue(0, 0, 0);
  issue(0, 0, 1);
  if constexpr (RING) {
    if (KT > 1) {
      issue(1, 1, 0);
      issue(1, 1, 1);
      issue(1, 0, 0);
      issue(1, 0, 1);
    }
    if (KT > 2) {
      issue(2, 1, 0);
      issue(2, 1, 1);
      asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    } else if (KT > 1) {
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  } else if (KT > 1) {
    issue(1, 1, 0);
    issue(1, 1, 1);
    issue(1, 0, 0);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();  // stagger: group 1 runs one barrier behind
  const int bh = wc >> 1, bo = (wc & 1) * 64;
  for (int kt = 0; kt < KT && SPREAD; ++kt) {
    const __bf16* As = buf(kt, 0, wr);
    const __bf16* Bs = buf(kt, 1, bh);
    // ---- q0: B cols 0-31, then A rows 0-63; A1 of tile kt + 1 (RING: nothing)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 2; ++j) bq[j][kk] = ABL == 2 ? bq[j][kk] : frag(Bs, bo + j * 16 + r16, kk);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) am0[i][kk] = ABL == 2 ? am0[i][kk] : frag(As, i * 16 + r16, kk);
    if (!RING && kt + 1 < KT) issue(kt + 1, 0, 1);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_sched_barrier(0);
    mfma_q(am0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    // ---- q1: B cols 32-63 (retired before the barrier: B is restaged from q2)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 2; j < 4; ++j) bq[j][kk] = ABL == 2 ? bq[j][kk] : frag(Bs, bo + j * 16 + r16, kk);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    mfma_q(am0, 0, 1);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    // ---- q2: A rows 64-127 (retired before the barrier: A0 is restaged in q3); B0 of tile kt + 2
    //      (RING: A0 / A1 of tile kt + 2 into this tile's B slots)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) am1[i][kk] = ABL == 2 ? am0[i][kk] : frag(As, 64 + i * 16 + r16, kk);
    if (RING && kt + 2 < KT) {
      issue(kt + 2, 0, 0);
      issue(kt + 2, 0, 1);
    } else if (!RING && kt + 2 < KT) {
      issue(kt + 2, 1, 0);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    mfma_q(am1, 1, 0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    // ---- q3: B1 and A0 of tile kt + 2; tile kt + 1 landed (3 younger half tiles may fly)
    //      (RING: B0 / B1 of tile kt + 3 into this tile's A slots; 6 younger may fly)
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (RING) {
      if (kt + 3 < KT) {
        issue(kt + 3, 1, 0);
        issue(kt + 3, 1, 1);
        asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      } else if (kt + 2 < KT) {
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    } else if (kt + 2 < KT) {
      issue(kt + 2, 1, 1);
      issue(kt + 2, 0, 0);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    mfma_q(am1, 1, 1);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
  }
  for (int kt = 0; kt < KT && !SPREAD; ++kt) {
    const __bf16* As = buf(kt, 0, wr);
    const __bf16* Bs = buf(kt, 1, bh);
    // ---- q0: all of this wave's B fragments, then A rows 0-63; A1 of tile kt + 1
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 4; ++j) bq[j][kk] = frag(Bs, bo + j * 16 + r16, kk);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) am0[i][kk] = frag(As, i * 16 + r16, kk);
    if (kt + 1 < KT) issue(kt + 1, 0, 1);
    asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");  // the 8 B reads retired: B0 is restaged in q1
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    mfma_q(am0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    // ---- q1: A rows 64-127; B0 of tile kt + 2
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) am1[i][kk] = frag(As, 64 + i * 16 + r16, kk);
    if (kt + 2 < KT) issue(kt + 2, 1, 0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    mfma_q(am0, 0, 1);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    // ---- q2: B1 of tile kt + 2
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 2 < KT) issue(kt + 2, 1, 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // am1 (q1's reads)
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    mfma_q(am1, 1, 0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    // ---- q3: A0 of tile kt + 2; tile kt + 1 landed (3 younger half tiles may fly)
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 2 < KT) {
      issue(kt + 2, 0, 0);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    mfma_q(am1, 1, 1);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();  // balance the stagger
  // ---- epilogue (C/D map: col = lane & 15, row = (lane >> 4) * 4 + i).  The
  // activation and output type are dispatched once, outside the element
  // loops: with a per-element switch the tanh / sigmoid code raised register
  // pressure past the 128 live accumulators and the whole tile went through
  // 528 B per lane of scratch (2x the output's bytes written per GEMM).
  epi_256_store(a, acc, m0, n0, wr, wc, r16, kq);
}

// ---- bf16 GEMM, 256 x 256 tiles, 8 waves, glds double buffer ("2-phase")
// For GEMMs with enough 256-square tiles to fill the chip (>= 256, e.g.
// 4096^3): per 64-deep K step a wave owns a 128 x 64 quadrant (8 x 4
// accumulators, 64 MFMAs) and reads 12 fragments per 32-k half step, so the
// operand traffic per FLOP is a quarter of the 128 x 128 kernel's (which is
// L2->CU bound at ~50% MFMA).  Schedule (cdna guide §5.5 T3+T4 minimum form):
// issue the next K tile's LDS-DMA, read + MFMA the current one, then one
// vmcnt(0) + barrier per K tile; 2 x 64 KB buffers, one workgroup per CU
// (two waves per SIMD interleave MFMA and ds_read), XCD-aware tile order,
// source-side XOR swizzle as in gemm_glds_kernel.
__global__ __launch_bounds__(512) void gemm_glds256_kernel(const DenseGemmArgs a) {
  constexpr int BM = 256, BN = 256, BK = 64;
  constexpr int kStageA = BM * BK, kStage = (BM + BN) * BK;  // elements
  extern __shared__ __attribute__((aligned(16))) __bf16 ring[];  // 2 x [A 256 x 64 | B 256 x 64]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wr = wave >> 2, wc = wave & 3, r16 = lane & 15, kq = lane >> 4;
  const int nN = (a.Np + BN - 1) / BN;
  int mi, ni;
  grouped_tile(xcd_tile(blockIdx.x, gridDim.x), (a.rows_eff + BM - 1) / BM, nN, a.group_m, mi, ni);
  const int m0 = mi * BM, n0 = ni * BN;
  const int KS = a.Kp / BK;
  const __bf16* A = static_cast<const __bf16*>(a.A);
  const __bf16* W = static_cast<const __bf16*>(a.W);
  const __bf16* srcA[4];
  const __bf16* srcB[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int L = (j * 8 + wave) * 64 + lane;  // LDS chunk of instruction j (1 KB per wave-instruction)
    const int r = L >> 3, c = (L & 7) ^ ((r >> 1) & 7);
    srcA[j] = A + size_t(min(m0 + r, a.rows_eff - 1)) * a.lda + c * 8;
    srcB[j] = W + size_t(min(n0 + r, a.Np - 1)) * a.Kp + c * 8;
  }
  auto issue = [&](int ks) {
    __bf16* st = ring + (ks & 1) * kStage;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_global_load_lds(
          (const void __attribute__((address_space(1)))*)(srcA[j] + ks * BK),
          (void __attribute__((address_space(3)))*)(st + (j * 8 + wave) * 512), 16, 0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_global_load_lds(
          (const void __attribute__((address_space(1)))*)(srcB[j] + ks * BK),
          (void __attribute__((address_space(3)))*)(st + kStageA + (j * 8 + wave) * 512), 16, 0, 0);
  };
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  issue(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int ks = 0; ks < KS; ++ks) {
    __builtin_amdgcn_sched_barrier(0);
    if (ks + 1 < KS) issue(ks + 1);  // the other buffer: everyone passed the barrier after reading it
    const __bf16* As = ring + (ks & 1) * kStage;
    const __bf16* Bs = As + kStageA;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int c = kk * 4 + kq;
      bf16x8 af[8], bfr[4];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int ra = wr * 128 + i * 16 + r16;
        af[i] = *reinterpret_cast<const bf16x8*>(As + ra * BK + ((c ^ ((ra >> 1) & 7)) << 3));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rb = wc * 64 + i * 16 + r16;
        bfr[i] = *reinterpret_cast<const bf16x8*>(Bs + rb * BK + ((c ^ ((rb >> 1) & 7)) << 3));
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  epi_256_store(a, acc, m0, n0, wr, wc, r16, kq);  // (C/D map: col = lane & 15, row = (lane >> 4) * 4 + i)
}

template <typename T, int AMODE>
void launch_lds(DenseGemmArgs a, hipStream_t s) {  // by value: the dispatch fills defaults in
  // 128 x 64 tiles (two resident workgroups per CU) when they fill the chip,
  // 32 x 64 otherwise (narrow layers such as a 10-class head: 4x the
  // workgroups, so the A stream is spread over every CU).  The VAE decoder's
  // first layer (AMODE 2) recomputes its reparameterised A panel per N tile,
  // so it takes 128 x 128 tiles on 8 waves: half the draws, 71.5 -> 44 us at
  // 40960 x 128 (profiles/r02h_gemm); for plain A the 128 x 128 variant and
  // a global_load_lds 3-stage ring at one workgroup per CU measured slower,
  // and so did 128 x 128 tiles for fp32 (layer 784->512: 74.6 vs 71.4 us,
  // profiles/r02r_gemm_fp32).
  const int nN = (a.Np + 63) / 64;
  const int big = nN * ((a.rows_eff + 127) / 128);
  const int wide = ((a.Np + 127) / 128) * ((a.rows_eff + 127) / 128);
  if constexpr (AMODE == 2) {
    if (wide >= 256) {
      hipLaunchKernelGGL((gemm_lds_kernel<T, AMODE, 128, 128, 512>), dim3(wide), dim3(512), 0, s, a);
      return;
    }
  }
  if constexpr (AMODE == 0 && sizeof(T) == 2) {
    static const int gm_env = [] { const char* v = getenv("SCA_GEMM_GROUP_M"); return v ? atoi(v) : 4; }();
    if (a.group_m <= 0) a.group_m = gm_env;
    // glds ring kernel: 128 x 128 tiles that fill the chip, N wide enough not
    // to waste the tile, no fused N <= 16 head (SCA_GEMM_GLDS=0 disables)
    static const int glds = [] { const char* v = getenv("SCA_GEMM_GLDS"); return v ? atoi(v) : 1; }();
    const int tiles128 = ((a.Np + 127) / 128) * ((a.rows_eff + 127) / 128);
    const bool fits = !a.out64 && a.Kp % 64 == 0 && (a.lda & 7) == 0;
    const int tiles256 = ((a.Np + 255) / 256) * ((a.rows_eff + 255) / 256);
    if (fits && a.path == 5) {
      const size_t lds = size_t(2) * (256 + 256) * 64 * sizeof(__bf16);
      hipLaunchKernelGGL(gemm_w4_kernel, dim3(tiles256), dim3(256), lds, s, a);
      return;
    }
    // default for chip-filling 256^2 grids: the 8-phase kernel with the reads
    // spread 12 / 4 / 8 / 0 over the phases (no scratch; the 16 / 8 / 0 / 0
    // form spills 528 B per lane) -- 1055 TF at 8192^3 with 4-row tile groups
    if (fits && (a.path == 7 || a.path == 8)) {  // ablations (timing only)
      const size_t lds = size_t(8) * 128 * 64 * sizeof(__bf16);
      if (a.path == 7) hipLaunchKernelGGL((gemm_8ph_kernel<true, 1>), dim3(tiles256), dim3(512), lds, s, a);
      else hipLaunchKernelGGL((gemm_8ph_kernel<true, 2>), dim3(tiles256), dim3(512), lds, s, a);
      return;
    }
    if (fits && (a.path == 6 || (a.path == 0 && glds && a.Np >= 256 && tiles256 >= 256))) {
      const size_t lds = size_t(8) * 128 * 64 * sizeof(__bf16);
      hipLaunchKernelGGL(gemm_8ph_kernel<true>, dim3(tiles256), dim3(512), lds, s, a);
      return;
    }
    if (fits && a.path == 9) {  // 10-half-tile ring (160 KB)
      const size_t lds = size_t(10) * 128 * 64 * sizeof(__bf16);
      hipLaunchKernelGGL((gemm_8ph_kernel<true, 0, true>), dim3(tiles256), dim3(512), lds, s, a);
      return;
    }
    if (fits && a.path == 4) {
      const size_t lds = size_t(8) * 128 * 64 * sizeof(__bf16);
      hipLaunchKernelGGL(gemm_8ph_kernel<false>, dim3(tiles256), dim3(512), lds, s, a);
      return;
    }
    if (fits && a.path == 3) {
      const size_t lds = size_t(2) * (256 + 256) * 64 * sizeof(__bf16);
      hipLaunchKernelGGL(gemm_glds256_kernel, dim3(tiles256), dim3(512), lds, s, a);
      return;
    }
    if (fits && (a.path == 2 || (a.path == 0 && glds && a.Np >= 128 && tiles128 >= 192 && false))) {
      constexpr int S = 4;
      const size_t lds = size_t(S) * (128 + 128) * 64 * sizeof(__bf16);
      hipLaunchKernelGGL((gemm_glds_kernel<S>), dim3(tiles128), dim3(256), lds, s, a);
      return;
    }
  }
  if constexpr (sizeof(T) == 4) {
    static const int m32 = [] { const char* v = getenv("SCA_GEMM_F32_M32"); return v ? atoi(v) : 1; }();
    // (128 x 128 tiles with 2 x 2 32x32 accumulators per wave -- one workgroup
    // per CU -- measured 9-90% slower on every MLP / VAE layer, r03d)
    // 64 x 64 tiles (4x the workgroups of 128 x 64, several resident per CU
    // to hide the LDS / MFMA latencies) for fp32 A panels: MLP 512->256
    // 32.7 -> 27.1 us, VAE decoder layers 53.2 -> 34.8 and 49.2 -> 43.8 us;
    // not for fp64 rows staged by the GEMM (AMODE 3: 88.9 vs 91.8 us) --
    // profiles/r03h_frontend_fp32.  SCA_GEMM_F32_T64: 0 never, 1 auto, 2 always.
    static const int t64 = [] { const char* v = getenv("SCA_GEMM_F32_T64"); return v ? atoi(v) : 1; }();
    const int tiles64 = nN * ((a.rows_eff + 63) / 64);
    if (m32 && !a.out64 && tiles64 >= 256 && ((t64 == 1 && AMODE != 3) || t64 == 2)) {
      hipLaunchKernelGGL((gemm_lds_kernel<T, AMODE, 64, 64, 256, 2, true>), dim3(tiles64), dim3(256), 0, s, a);
      return;
    }
    if (m32 && !a.out64 && big >= 256) {
      hipLaunchKernelGGL((gemm_lds_kernel<T, AMODE, 128, 64, 256, 2, true>), dim3(big), dim3(256), 0, s, a);
      return;
    }
  }
  if (big >= 256) {
    hipLaunchKernelGGL((gemm_lds_kernel<T, AMODE, 128, 64, 256>), dim3(big), dim3(256), 0, s, a);
  } else {
    const int small = nN * ((a.rows_eff + 31) / 32);
    hipLaunchKernelGGL((gemm_lds_kernel<T, AMODE, 32, 64, 256>), dim3(small), dim3(256), 0, s, a);
  }
}

// fp64 [rows][F] -> bf16 [rows][ld] (zero-padded).  Each lane converts one
// pair of adjacent columns per step: the wave's 16-B loads and 4-B stores are
// lane-contiguous.
__global__ void convert_bf16_kernel(const double* __restrict__ X, int rows, int F, int ld, __bf16* __restrict__ out) {
  const int half = ld >> 1;  // ld is even (a multiple of 64)
  const size_t n = size_t(rows) * half;

  using bf16x2 = __attribute__((ext_vector_type(2))) __bf16;
  const bool vec = (F & 1) == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0;
  for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
    const int r = int(i / half), c = int(i - size_t(r) * half) * 2;
    const double* x = X + size_t(r) * F + c;
    bf16x2 v;
    if (c + 2 <= F && vec) {
      const f64x2 d = *reinterpret_cast<const f64x2*>(x);
      v[0] = __bf16(float(d[0]));
      v[1] = __bf16(float(d[1]));
    } else {
      v[0] = __bf16(c < F ? float(x[0]) : 0.f);
      v[1] = __bf16(c + 1 < F ? float(x[1]) : 0.f);
    }
    reinterpret_cast<bf16x2*>(out)[i] = v;
  }
}

template <int BF16, int AMODE>
void launch_tn(const DenseGemmArgs& a, hipStream_t s) {
  const int ntiles = a.Np >> 4;
  const int row_blocks = (a.rows_eff + 16 * kTM - 1) / (16 * kTM);
  // TN: as wide as the layer allows, narrower when that leaves the chip's
  // 1024 SIMDs short of waves
  int tn = ntiles >= 4 ? 4 : ntiles >= 2 ? 2 : 1;
  while (tn > 1 && row_blocks * ((ntiles + tn - 1) / tn) < 1024) tn >>= 1;
  const dim3 grid((ntiles + tn - 1) / tn, row_blocks);
  if (tn == 4) hipLaunchKernelGGL((dense_gemm_kernel<BF16, AMODE, 4>), grid, dim3(64), 0, s, a);
  else if (tn == 2) hipLaunchKernelGGL((dense_gemm_kernel<BF16, AMODE, 2>), grid, dim3(64), 0, s, a);
  else hipLaunchKernelGGL((dense_gemm_kernel<BF16, AMODE, 1>), grid, dim3(64), 0, s, a);
}

}  // namespace

void dense_gemm(const DenseGemmArgs& a, hipStream_t s) {
  if (a.rows_eff <= 0) return;
  if (a.bf16) {
    static const int remap = [] { const char* v = getenv("SCA_GEMM_REMAP"); return v ? atoi(v) : 1; }();
    DenseGemmArgs b = a;
    b.xcd_remap = remap;
    // (the 128 x 128 variant needs 230 VGPRs -> one workgroup per CU, and
    // measured 2.5x slower on the VAE decoder)
    if (b.H) launch_lds<__bf16, 2>(b, s);
    else launch_lds<__bf16, 0>(b, s);
  } else if (a.lds_f32 && !a.H) {  // large fp32 layer: LDS-tiled exact-fp32 MFMA GEMM
    DenseGemmArgs b = a;
    b.xcd_remap = 1;
    if (b.a_f64) launch_lds<float, 3>(b, s);
    else launch_lds<float, 0>(b, s);
  } else {
    if (a.H) launch_tn<0, 2>(a, s);
    else launch_tn<0, 0>(a, s);
  }
}

void convert_bf16(const double* X, int rows, int F, int ld, void* out, hipStream_t s) {
  if (rows <= 0) return;
  const size_t n = size_t(rows) * (ld / 2);
  const int bs = 256;
  const int blocks = int((n + bs - 1) / bs < 8192 ? (n + bs - 1) / bs : 8192);
  hipLaunchKernelGGL(convert_bf16_kernel, dim3(blocks), dim3(bs), 0, s, X, rows, F, ld, static_cast<__bf16*>(out));
}

}  // namespace sca::kern
