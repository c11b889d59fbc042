// Seq2seq LSTM reconstruction error, small-batch form (reference
// components/outlier-detection/seq2seq-lstm/CoreSeq2SeqLSTM.py:107-174).
//
// The MFMA kernel (lstm.hip) runs 16 sequences per workgroup: a 1-sequence
// request pays the full 16-row tile and each step is a chain of dependent
// MFMAs on 2-4 waves (~3.6 us per step, profiles/r02c_lstm).  Here one
// workgroup owns R <= 4 sequences and every gate row lives in VGPRs:
//
//   unit u of a cell is Q consecutive lanes; lane (u, q) holds the 4 gate rows
//   of u over k in [q*KPL, q*KPL + KPL) of v = [h_{t-1} | x_t | 0 pad]
//   (4*KPL weights, loaded once per phase), so a step is KPL/4 ds_read_b128 of
//   v + 4*KPL FMAs + a DPP butterfly over the Q lanes (quad_perm /
//   row_half_mirror / row_mirror, no LDS), after which every lane of the
//   group holds all four gate sums and updates the cell state in registers.
//   Lane q == 0 writes h into the NEXT step's v row (double-buffered), so an
//   encoder step has one barrier; a decoder step has one per layer plus one
//   for the Dense feedback y_t (the next step's x).
//
// Cells start on 64-lane boundaries, so Q (and every branch on the lane's
// role) is wave-uniform.  All of LDS is zeroed first: pad columns of v read
// as 0 against zero weights.  fp32, gate order i, f, g, o (torch / Keras).
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace sca::kern {
namespace {

__device__ __forceinline__ float sigm(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float tanh_f(float x) { return 2.f * __builtin_amdgcn_rcpf(1.f + __expf(-2.f * x)) - 1.f; }
__device__ __forceinline__ float act_out(float x, int a) {
  switch (a) {
    case 1: return sigm(x);
    case 2: return tanh_f(x);
    case 3: return x > 0.f ? x : 0.f;
    default: return x;
  }
}

template <int CTRL> __device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}

// Sum over aligned groups of Q lanes (Q a power of two, wave-uniform); every
// lane of the group receives the total.
__device__ __forceinline__ float group_sum(float v, int Q) {
  if (Q >= 2) v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]: lane ^ 1
  if (Q >= 4) v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]: lane ^ 2
  if (Q >= 8) v += dpp<0x141>(v);  // row_half_mirror: the other quad of the 8
  if (Q >= 16) v += dpp<0x140>(v); // row_mirror: the other 8 of the row
  if (Q >= 32) v += __shfl_xor(v, 16, 64);
  if (Q >= 64) v += __shfl_xor(v, 32, 64);
  return v;
}

struct Role {
  bool on = false;
  int in = 0, H = 0, Q = 1, Kv = 0, v_off = 0, u = 0, q = 0, span = 1;
};

template <int KPL>
__device__ __forceinline__ Role take_cell(const LstmvCell& c, const float* __restrict__ P, int tid, float (&w)[4][KPL],
                                          float (&b)[4]) {
  Role r;
  const int span = c.H * c.Q;
  if (tid < c.lane0 || tid >= c.lane0 + span) return r;
  r.on = true;
  r.in = c.in;
  r.H = c.H;
  r.Q = c.Q;
  r.Kv = c.Kv;
  r.v_off = c.v_off;
  r.span = span;
  r.u = (tid - c.lane0) / c.Q;
  r.q = (tid - c.lane0) - r.u * c.Q;
  const float4* src = reinterpret_cast<const float4*>(P + c.w_off + size_t(r.u * c.Q + r.q) * 4 * KPL);
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int j = 0; j < KPL; j += 4) {
      const float4 x = src[(g * KPL + j) >> 2];
      w[g][j] = x.x;
      w[g][j + 1] = x.y;
      w[g][j + 2] = x.z;
      w[g][j + 3] = x.w;
    }
#pragma unroll
  for (int g = 0; g < 4; ++g) b[g] = P[c.b_off + g * c.H + r.u];
  return r;
}

// Gate pre-activations of one row: a[g] = sum_k W[g*H+u][k] v[k] over this
// lane's k slice, summed over the unit's Q lanes.
template <int KPL>
__device__ __forceinline__ void gates(const float* v, const float (&w)[4][KPL], int Q, float (&a)[4]) {
#pragma unroll
  for (int g = 0; g < 4; ++g) a[g] = 0.f;
#pragma unroll
  for (int j = 0; j < KPL; j += 4) {
    const float4 x = *reinterpret_cast<const float4*>(v + j);
#pragma unroll
    for (int g = 0; g < 4; ++g) a[g] += w[g][j] * x.x + w[g][j + 1] * x.y + w[g][j + 2] * x.z + w[g][j + 3] * x.w;
  }
#pragma unroll
  for (int g = 0; g < 4; ++g) a[g] = group_sum(a[g], Q);
}

__device__ __forceinline__ float cell(const float (&a)[4], const float (&b)[4], float& c) {
  const float i = sigm(a[0] + b[0]), f = sigm(a[1] + b[1]), gg = tanh_f(a[2] + b[2]), o = sigm(a[3] + b[3]);
  c = f * c + i * gg;
  return o * tanh_f(c);
}

template <int KPL, int R>
__global__ __launch_bounds__(1024) void lstm_valu_kernel(const double* __restrict__ X, int rows, const LstmvProgram p,
                                                         const float* __restrict__ P, double* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, NT = blockDim.x;
  const int row0 = blockIdx.x * R;
  const int nvalid = min(R, rows - row0);
  const int T = p.T, F = p.F;
  for (int i = tid; i < p.lds_floats; i += NT) lds[i] = 0.f;
  __syncthreads();
  float* xs = lds + p.x_off;  // [R][T][F]
  for (int i = tid; i < R * T * F; i += NT) {
    const int s = i / (T * F);
    xs[i] = s < nvalid ? float(X[size_t(row0) * T * F + i]) : 0.f;
  }
  __syncthreads();

  float w[4][KPL], b[4], cst[R], hl[R];

  // ------------------------------------------------------------ encoder
  for (int l = 0; l < p.n_enc; ++l) {
    Role r;
    int dir = 0;
    {
      const Role r0 = take_cell<KPL>(p.enc[l][0], P, tid, w, b);
      if (r0.on) {
        r = r0;
      } else {
        r = take_cell<KPL>(p.enc[l][1], P, tid, w, b);
        dir = 1;
      }
    }
    const float* src = l == 0 ? xs : lds + p.seq_off[(l - 1) & 1];
    const int src_ld = l == 0 ? F : p.seq_ld;
    const bool keep_seq = l + 1 < p.n_enc;
    float* seq_out = keep_seq ? lds + p.seq_off[l & 1] : nullptr;
    if (r.on) {
#pragma unroll
      for (int s = 0; s < R; ++s) cst[s] = hl[s] = 0.f;
      const int t0 = dir == 0 ? 0 : T - 1;
      for (int e = r.u * r.Q + r.q; e < R * r.in; e += r.span) {
        const int s = e / r.in, k = e - s * r.in;
        lds[r.v_off + s * r.Kv + r.H + k] = src[(s * T + t0) * src_ld + k];
      }
    }
    __syncthreads();
    for (int step = 0; step < T; ++step) {
      const int cur = step & 1, nxt = cur ^ 1;
      if (r.on) {
        const int t = dir == 0 ? step : T - 1 - step;
#pragma unroll
        for (int s = 0; s < R; ++s) {
          float a[4];
          gates<KPL>(lds + r.v_off + (cur * R + s) * r.Kv + r.q * KPL, w, r.Q, a);
          const float h = cell(a, b, cst[s]);
          hl[s] = h;
          if (r.q == 0) {
            lds[r.v_off + (nxt * R + s) * r.Kv + r.u] = h;
            if (keep_seq) seq_out[(s * T + t) * p.seq_ld + dir * r.H + r.u] = h;
          }
        }
        if (step + 1 < T) {  // x of the next step into the next v row
          const int tn = dir == 0 ? step + 1 : T - 2 - step;
          for (int e = r.u * r.Q + r.q; e < R * r.in; e += r.span) {
            const int s = e / r.in, k = e - s * r.in;
            lds[r.v_off + (nxt * R + s) * r.Kv + r.H + k] = src[(s * T + tn) * src_ld + k];
          }
        }
      }
      __syncthreads();
    }
    if (l + 1 == p.n_enc && r.on && r.q == 0) {
#pragma unroll
      for (int s = 0; s < R; ++s) {
        lds[p.hfin_off + s * 2 * r.H + dir * r.H + r.u] = hl[s];
        lds[p.cfin_off + s * 2 * r.H + dir * r.H + r.u] = cst[s];
      }
    }
    __syncthreads();
  }

  // ------------------------------------------------------------ decoder
  int layer = -1;
  Role r;
  for (int l = 0; l < p.n_dec && layer < 0; ++l) {
    r = take_cell<KPL>(p.dec[l], P, tid, w, b);
    if (r.on) layer = l;
  }
  const int He2 = 2 * p.enc[p.n_enc - 1][0].H;
  if (r.on) {  // initial state = [forward | backward] final encoder states
#pragma unroll
    for (int s = 0; s < R; ++s) cst[s] = lds[p.cfin_off + s * He2 + r.u];
    for (int e = r.u * r.Q + r.q; e < R * r.H; e += r.span) {
      const int s = e / r.H, k = e - s * r.H;
      lds[r.v_off + s * r.Kv + k] = lds[p.hfin_off + s * He2 + k];
    }
    if (layer == 0)  // first target = x[:, 0]
      for (int e = r.u * r.Q + r.q; e < R * r.in; e += r.span) {
        const int s = e / r.in, k = e - s * r.in;
        lds[r.v_off + s * r.Kv + r.H + k] = xs[s * T * F + k];
      }
  }
  // Dense output lanes: F outputs x Qy lanes, KPL weights each
  const bool dense = tid >= p.y_lane0 && tid < p.y_lane0 + F * p.Qy;
  int yf = 0, yq = 0;
  float by = 0.f, err[R];
#pragma unroll
  for (int s = 0; s < R; ++s) err[s] = 0.f;
  if (dense) {
    yf = (tid - p.y_lane0) / p.Qy;
    yq = (tid - p.y_lane0) - yf * p.Qy;
    const float4* src = reinterpret_cast<const float4*>(P + p.yw_off + size_t(yf * p.Qy + yq) * KPL);
#pragma unroll
    for (int j = 0; j < KPL; j += 4) {
      const float4 x = src[j >> 2];
      w[0][j] = x.x;
      w[0][j + 1] = x.y;
      w[0][j + 2] = x.z;
      w[0][j + 3] = x.w;
    }
    by = P[p.yb_off + yf];
  }
  __syncthreads();
  const LstmvCell& top = p.dec[p.n_dec - 1];
  const LstmvCell& bottom = p.dec[0];
  for (int t = 1; t < T; ++t) {
    const int cur = (t - 1) & 1, nxt = cur ^ 1;
    for (int l = 0; l < p.n_dec; ++l) {
      if (layer == l) {
        const bool has_next = l + 1 < p.n_dec;
#pragma unroll
        for (int s = 0; s < R; ++s) {
          float a[4];
          gates<KPL>(lds + r.v_off + (cur * R + s) * r.Kv + r.q * KPL, w, r.Q, a);
          const float h = cell(a, b, cst[s]);
          if (r.q == 0) {
            lds[r.v_off + (nxt * R + s) * r.Kv + r.u] = h;
            if (has_next) {  // input of the next layer at this step
              const LstmvCell& nc = p.dec[l + 1];
              lds[nc.v_off + (cur * R + s) * nc.Kv + nc.H + r.u] = h;
            }
          }
        }
      }
      __syncthreads();
    }
    if (dense) {
#pragma unroll
      for (int s = 0; s < R; ++s) {
        const float* vh = lds + top.v_off + (nxt * R + s) * top.Kv + yq * KPL;  // h_top at the row start
        float a = 0.f;
#pragma unroll
        for (int j = 0; j < KPL; j += 4) {
          const float4 x = *reinterpret_cast<const float4*>(vh + j);
          a += w[0][j] * x.x + w[0][j + 1] * x.y + w[0][j + 2] * x.z + w[0][j + 3] * x.w;
        }
        a = group_sum(a, p.Qy);
        const float y = act_out(a + by, p.out_act);
        if (yq == 0) {
          lds[bottom.v_off + (nxt * R + s) * bottom.Kv + bottom.H + yf] = y;
          const float d = xs[(s * T + t) * F + yf] - y;
          err[s] += d * d;
        }
      }
    }
    __syncthreads();
  }
  if (dense && yq == 0) {
#pragma unroll
    for (int s = 0; s < R; ++s) atomicAdd(&lds[p.mse_off + s], err[s]);
  }
  __syncthreads();
  if (tid < nvalid) out[row0 + tid] = double(lds[p.mse_off + tid]) / double(T * F);
}

template <int KPL>
void launch_kpl(const double* X, int rows, const LstmvProgram& p, const float* params, double* out, hipStream_t s) {
  const size_t lds = size_t(p.lds_floats) * sizeof(float);
  const dim3 grid((rows + p.R - 1) / p.R), block(p.threads);
  switch (p.R) {
    case 1: hipLaunchKernelGGL((lstm_valu_kernel<KPL, 1>), grid, block, lds, s, X, rows, p, params, out); break;
    case 2: hipLaunchKernelGGL((lstm_valu_kernel<KPL, 2>), grid, block, lds, s, X, rows, p, params, out); break;
    default: hipLaunchKernelGGL((lstm_valu_kernel<KPL, 4>), grid, block, lds, s, X, rows, p, params, out); break;
  }
}

}  // namespace

void lstm_valu_mse(const double* X, int rows, const LstmvProgram& prog, const float* params, double* out,
                   hipStream_t s) {
  if (rows <= 0 || !prog.ok) return;
  switch (prog.KPL) {
    case 8: launch_kpl<8>(X, rows, prog, params, out, s); break;
    case 16: launch_kpl<16>(X, rows, prog, params, out, s); break;
    default: launch_kpl<32>(X, rows, prog, params, out, s); break;
  }
}

}  // namespace sca::kern
