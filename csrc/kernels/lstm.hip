// Seq2seq LSTM reconstruction error on MFMA (reference
// components/outlier-detection/seq2seq-lstm/CoreSeq2SeqLSTM.py:107-174 runs the
// Keras encoder once and the decoder model T-1 times per observation, one
// observation at a time, on the CPU).
//
// One persistent kernel per batch.  A 256-thread workgroup owns a tile of 16
// sequences (the M dimension of v_mfma_f32_16x16x4_f32) and runs the whole
// model for them:
//   encoder layer l (bidirectional): waves 0-1 run the forward direction and
//   waves 2-3 the backward one concurrently, T steps each;
//   decoder: T-1 greedy steps through every decoder layer (all four waves),
//   then the Dense output, whose result is the next step's input, and the
//   squared error against the input sequence.
// A step of one LSTM is  gates[16 x 4H] = [x_t | h_{t-1}] (16 x K) . W^T (K x 4H)
// on MFMA -- A rows in LDS (row stride == 2 mod 32: the 16x2 lane pattern of an
// A fragment hits 32 distinct banks), W pre-packed on the host in fragment
// order ([tile][k-step][lane]) so a B fragment is one conflict-free dword per
// lane -- followed by the fused cell update (sigmoid/tanh, c and h in LDS)
// that also writes h into the next step's A row and stages the next x.  Two
// barriers per LSTM step; the weights of the running phase sit in LDS when
// they fit (the reference's 20/40-unit models: ~36 KiB), else they are read
// from global memory (L2-resident).  fp32 throughout (matches torch / Keras
// fp32 LSTMs to ~1e-6).
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace sca::kern {
namespace {

constexpr int kThreads = 256;
typedef float f32x4 __attribute__((ext_vector_type(4)));

// v_exp_f32 + v_rcp_f32 (1 ulp): no IEEE division sequence on the step's
// critical path (the kernel is instruction-issue bound, profiles/r02c_lstm).
__device__ __forceinline__ float sigm(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float tanh_f(float x) { return 2.f * __builtin_amdgcn_rcpf(1.f + __expf(-2.f * x)) - 1.f; }

// Walks the (row, column) pairs p = start, start + step, ... of a [rows x n]
// index space without an integer division per pair (one at the start).
struct PairIter {
  int s, u, ds, du, n;
  __device__ __forceinline__ PairIter(int start, int step, int n_) : n(n_) {
    s = start / n_;
    u = start - s * n_;
    ds = step / n_;
    du = step - ds * n_;
  }
  __device__ __forceinline__ void next() {
    s += ds;
    u += du;
    if (u >= n) {
      u -= n;
      ++s;
    }
  }
};
__device__ __forceinline__ float act_out(float x, int a) {
  switch (a) {
    case 1: return sigm(x);
    case 2: return tanh_f(x);
    case 3: return x > 0.f ? x : 0.f;
    default: return x;
  }
}

// C[16][Np] (LDS, stride ldc) = A[16][Kp] (LDS, stride lda) . W^T with W
// packed in fragment order ([tile][k-step][lane]).  This wave's column tiles
// are tile = gwave, gwave + nwaves, ...; two tiles per pass give two
// independent accumulator chains, and the A / B fragments of up to 16 k-steps
// are loaded into registers before the MFMAs that use them (clamped
// addresses, no branches between the loads), so a k-block costs one LDS
// round trip instead of one per MFMA.
__device__ __forceinline__ void gemm16(const float* A, int lda, const float* __restrict__ W, int Kp, int Np, float* C,
                                       int ldc, int gwave, int nwaves, int lane) {
  constexpr int kKB = 16;
  const int ntiles = Np >> 4, ksteps = Kp >> 2;
  const float* arow = A + (lane & 15) * lda + (lane >> 4);
  for (int t0 = gwave; t0 < ntiles; t0 += 2 * nwaves) {
    const int t1 = t0 + nwaves;
    const bool two = t1 < ntiles;
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    const float* w0 = W + size_t(t0) * ksteps * 64 + lane;
    const float* w1 = W + size_t(two ? t1 : t0) * ksteps * 64 + lane;
    for (int kb = 0; kb < ksteps; kb += kKB) {
      float a[kKB], b0[kKB], b1[kKB];
#pragma unroll
      for (int j = 0; j < kKB; ++j) {
        const int ks = min(kb + j, ksteps - 1);
        a[j] = arow[ks * 4];
        b0[j] = w0[ks * 64];
        b1[j] = w1[ks * 64];
      }
#pragma unroll
      for (int j = 0; j < kKB; ++j) {
        if (kb + j < ksteps) {
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b0[j], acc0, 0, 0, 0);
          if (two) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b1[j], acc1, 0, 0, 0);
        }
      }
    }
    const int col = lane & 15, rbase = (lane >> 4) * 4;
#pragma unroll
    for (int r = 0; r < 4; ++r) C[(rbase + r) * ldc + t0 * 16 + col] = acc0[r];
    if (two) {
#pragma unroll
      for (int r = 0; r < 4; ++r) C[(rbase + r) * ldc + t1 * 16 + col] = acc1[r];
    }
  }
}

__device__ __forceinline__ void gate_gemm(const LstmCell& c, const float* __restrict__ wbase, float* lds, int gwave,
                                          int nwaves, int lane) {
  gemm16(lds + c.a_off, c.lda, wbase + c.w_off, c.Kp, c.Np, lds + c.g_off, c.ldg, gwave, nwaves, lane);
}

// Fused cell update for (sequence, unit) pairs p = gtid, gtid + gsize, ...
// Gate order i, f, g(=c~), o (torch / Keras).  h goes to this LSTM's own A row
// (recurrent input of the next step) and, if given, to `h_next` (the next
// layer's input row, stride ld_next) and `seq_out` (return_sequences).
__device__ __forceinline__ void cell_update(const LstmCell& c, const float* __restrict__ bias, float* lds, int gtid,
                                            int gsize, float* h_next, int ld_next, float* seq_out, int seq_stride,
                                            int seq_col) {
  const float* G = lds + c.g_off;
  float* A = lds + c.a_off;
  float* C = lds + c.c_off;
  const int H = c.H;
  PairIter it(gtid, gsize, H);
  for (int p = gtid; p < kLstmRows * H; p += gsize, it.next()) {
    const int s = it.s, u = it.u;
    const float* g = G + s * c.ldg;
    const float i = sigm(g[u] + bias[u]);
    const float f = sigm(g[H + u] + bias[H + u]);
    const float gg = tanh_f(g[2 * H + u] + bias[2 * H + u]);
    const float o = sigm(g[3 * H + u] + bias[3 * H + u]);
    const float cs = f * C[s * H + u] + i * gg;
    C[s * H + u] = cs;
    const float h = o * tanh_f(cs);
    A[s * c.lda + c.in + u] = h;
    if (h_next) h_next[s * ld_next + u] = h;
    if (seq_out) seq_out[size_t(s) * seq_stride + seq_col + u] = h;
  }
}

// Copy `n` floats global -> LDS (16-B granules when the source is aligned;
// the host pads every phase blob to a multiple of 4 floats).
__device__ __forceinline__ void load_phase(float* dst, const float* __restrict__ src, int n) {
  if ((reinterpret_cast<uintptr_t>(src) & 15) == 0) {
    const float4* s4 = reinterpret_cast<const float4*>(src);
    float4* d4 = reinterpret_cast<float4*>(dst);
    for (int i = threadIdx.x; i < (n >> 2); i += kThreads) d4[i] = s4[i];
    for (int i = (n & ~3) + threadIdx.x; i < n; i += kThreads) dst[i] = src[i];
  } else {
    for (int i = threadIdx.x; i < n; i += kThreads) dst[i] = src[i];
  }
}

template <bool WLDS>
__global__ __launch_bounds__(kThreads) void lstm_seq2seq_kernel(const double* __restrict__ X, int rows,
                                                                const LstmProgram p, const float* __restrict__ P,
                                                                float* __restrict__ ws, double* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int row0 = blockIdx.x * kLstmRows;
  const int T = p.T, F = p.F;
  const int nvalid = min(kLstmRows, rows - row0);
  float* wlds = lds;  // weights of the running phase (WLDS)
  float* wsb = ws + size_t(blockIdx.x) * size_t(p.seq_ws_floats);
  const size_t seq_buf = size_t(kLstmRows) * T * p.Hmax2;

  // The input tile is read at every encoder step and again for the decoder's
  // error: stage it in LDS once (fp32) so no step waits on an HBM round trip.
  float* xs = lds + p.x_off;
  if (p.x_lds) {
    const int n = kLstmRows * T * F;
    for (int i = tid; i < n; i += kThreads) {
      const int s = i / (T * F);
      xs[i] = s < nvalid ? float(X[size_t(row0) * T * F + i]) : 0.f;
    }
    __syncthreads();
  }
  // x_t of the input sequence of encoder layer l, row s, feature f
  auto x_in = [&](int l, int s, int t, int f, int in) -> float {
    if (l == 0) {
      if (p.x_lds) return xs[(s * T + t) * F + f];
      return s < nvalid ? float(X[(size_t(row0 + s) * T + t) * F + f]) : 0.f;
    }
    return wsb[((l - 1) & 1) * seq_buf + (size_t(s) * T + t) * p.Hmax2 + f];
  };

  // ------------------------------------------------------------ encoder
  for (int l = 0; l < p.n_enc; ++l) {
    const float* wb = WLDS ? wlds : P + p.enc_phase[l];
    if (WLDS) load_phase(wlds, P + p.enc_phase[l], p.enc_phase_floats[l]);
    const int dir = wave >> 1, gwave = wave & 1, gtid = tid & 127;
    const LstmCell& c = p.enc[l][dir];
    float* A = lds + c.a_off;
    float* Cs = lds + c.c_off;
    for (int i = gtid; i < kLstmRows * c.H; i += 128) {
      const int s = i / c.H, u = i - s * c.H;
      A[s * c.lda + c.in + u] = 0.f;
      Cs[i] = 0.f;
    }
    for (int i = gtid; i < kLstmRows * c.lda; i += 128) {  // zero the K padding columns too
      const int s = i / c.lda, k = i - s * c.lda;
      if (k < c.in) A[i] = x_in(l, s, dir == 0 ? 0 : T - 1, k, c.in);
      else if (k >= c.in + c.H) A[i] = 0.f;
    }
    __syncthreads();
    const bool last = l + 1 == p.n_enc;
    float* seq_out = last ? nullptr : wsb + (l & 1) * seq_buf;
    const float* bias = wb + c.b_off;
    for (int step = 0; step < T; ++step) {
      const int t = dir == 0 ? step : T - 1 - step;
      gate_gemm(c, wb, lds, gwave, 2, lane);
      __syncthreads();
      // next step's x: loads issued before the cell update so their latency
      // hides behind it (global inputs), written into A after it
      constexpr int kPre = 4;
      float xv[kPre];
      const int tn = dir == 0 ? step + 1 : T - 2 - step;
      const bool more = step + 1 < T;
      PairIter xi(gtid, 128, c.in);
      if (more) {
        PairIter q = xi;
#pragma unroll
        for (int j = 0; j < kPre; ++j, q.next()) {
          const int i = gtid + j * 128;
          xv[j] = i < kLstmRows * c.in ? x_in(l, q.s, tn, q.u, c.in) : 0.f;
        }
      }
      cell_update(c, bias, lds, gtid, 128, nullptr, 0, seq_out ? seq_out + size_t(t) * p.Hmax2 : nullptr,
                  T * p.Hmax2, dir * c.H);
      if (more) {
#pragma unroll
        for (int j = 0; j < kPre; ++j, xi.next()) {
          const int i = gtid + j * 128;
          if (i < kLstmRows * c.in) A[xi.s * c.lda + xi.u] = xv[j];
        }
        for (int i = gtid + kPre * 128; i < kLstmRows * c.in; i += 128, xi.next())
          A[xi.s * c.lda + xi.u] = x_in(l, xi.s, tn, xi.u, c.in);
      }
      __syncthreads();
    }
  }

  // ------------------------------------------------------------ decoder
  const float* wb = WLDS ? wlds : P + p.dec_phase;
  if (WLDS) load_phase(wlds, P + p.dec_phase, p.dec_phase_floats);
  const LstmCell& f0 = p.enc[p.n_enc - 1][0];
  const LstmCell& b0 = p.enc[p.n_enc - 1][1];
  float* mse = lds + p.mse_off;
  for (int l = 0; l < p.n_dec; ++l) {
    const LstmCell& c = p.dec[l];
    float* A = lds + c.a_off;
    float* Cs = lds + c.c_off;
    // initial state = [forward | backward] final encoder states
    for (int i = tid; i < kLstmRows * c.H; i += kThreads) {
      const int s = i / c.H, u = i - s * c.H;
      const bool fw = u < f0.H;
      const LstmCell& e = fw ? f0 : b0;
      const int ue = fw ? u : u - f0.H;
      A[s * c.lda + c.in + u] = lds[e.a_off + s * e.lda + e.in + ue];
      Cs[i] = lds[e.c_off + s * e.H + ue];
    }
    for (int i = tid; i < kLstmRows * c.lda; i += kThreads) {
      const int s = i / c.lda, k = i - s * c.lda;
      if (k < c.in) A[i] = l == 0 ? x_in(0, s, 0, k, F) : 0.f;  // target = x[:, 0]
      else if (k >= c.in + c.H) A[i] = 0.f;
    }
  }
  if (tid < kLstmRows) mse[tid] = 0.f;
  __syncthreads();
  const LstmCell& top = p.dec[p.n_dec - 1];
  const float* Wd = wb + p.dense_w;
  const float* bd = wb + p.dense_b;
  float* A0 = lds + p.dec[0].a_off;
  const int lda0 = p.dec[0].lda;
  for (int t = 1; t < T; ++t) {
    for (int l = 0; l < p.n_dec; ++l) {
      const LstmCell& c = p.dec[l];
      gate_gemm(c, wb, lds, wave, 4, lane);
      __syncthreads();
      const bool has_next = l + 1 < p.n_dec;
      cell_update(c, wb + c.b_off, lds, tid, kThreads, has_next ? lds + p.dec[l + 1].a_off : nullptr,
                  has_next ? p.dec[l + 1].lda : 0, nullptr, 0, 0);
      __syncthreads();
    }
    // Dense output on MFMA ([16 x D] . Wd^T) -> next target and squared error
    // vs the input sequence
    gemm16(lds + top.a_off + top.in, top.lda, Wd, p.dense_kp, p.dense_np, lds + p.y_off, p.dense_np + 4, wave, 4,
           lane);
    __syncthreads();
    float err = 0.f;
    int s_err = -1;
    PairIter yi(tid, kThreads, F);
    for (int i = tid; i < kLstmRows * F; i += kThreads, yi.next()) {
      const int s = yi.s, f = yi.u;
      const float y = act_out(lds[p.y_off + s * (p.dense_np + 4) + f] + bd[f], p.out_act);
      A0[s * lda0 + f] = y;
      const float d = x_in(0, s, t, f, F) - y;
      if (s_err != s && s_err >= 0) {
        atomicAdd(&mse[s_err], err);
        err = 0.f;
      }
      s_err = s;
      err += d * d;
    }
    if (s_err >= 0) atomicAdd(&mse[s_err], err);
    __syncthreads();
  }
  if (tid < nvalid) out[row0 + tid] = double(mse[tid]) / double(T * F);
}

}  // namespace

void lstm_seq2seq_mse(const double* X, int rows, const LstmProgram& prog, const float* params, float* ws, double* out,
                      hipStream_t s) {
  if (rows <= 0) return;
  const dim3 grid((rows + kLstmRows - 1) / kLstmRows);
  const size_t lds = size_t(prog.lds_floats) * sizeof(float);
  if (prog.w_lds)
    hipLaunchKernelGGL(lstm_seq2seq_kernel<true>, grid, dim3(kThreads), lds, s, X, rows, prog, params, ws, out);
  else
    hipLaunchKernelGGL(lstm_seq2seq_kernel<false>, grid, dim3(kThreads), lds, s, X, rows, prog, params, ws, out);
}

}  // namespace sca::kern
