// Dependent-chain latencies of one wave64 on MI355X (gfx950), in shader
// clocks (s_memtime) per operation: the numbers the one-wave latency-bound
// kernels (Mahalanobis eigen-solver, small-batch LSTM) are designed against.
// Each test is a chain of N operations where every operation consumes the
// previous result; one workgroup of 64 threads, nothing else on the GPU.
//   hipcc --offload-arch=gfx950 -O3 -o wave_latency tools/micro/wave_latency.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int CTRL> __device__ __forceinline__ double dpp64(double v) {
  const int2 h = __builtin_bit_cast(int2, v);
  int2 o;
  o.x = __builtin_amdgcn_update_dpp(0, h.x, CTRL, 0xF, 0xF, false);
  o.y = __builtin_amdgcn_update_dpp(0, h.y, CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, o);
}
__device__ __forceinline__ double readlane64(double v, int l) {
  const int2 h = __builtin_bit_cast(int2, v);
  int2 o;
  o.x = __builtin_amdgcn_readlane(h.x, l);
  o.y = __builtin_amdgcn_readlane(h.y, l);
  return __builtin_bit_cast(double, o);
}
__device__ __forceinline__ double wave_sum_dpp(double v) {
  v += dpp64<0xB1>(v);
  v += dpp64<0x4E>(v);
  v += dpp64<0x141>(v);
  v += dpp64<0x140>(v);
  return (readlane64(v, 0) + readlane64(v, 16)) + (readlane64(v, 32) + readlane64(v, 48));
}
template <int CTRL> __device__ __forceinline__ double mdpp64(double v) {  // no old-value operand
  const int2 h = __builtin_bit_cast(int2, v);
  int2 o;
  o.x = __builtin_amdgcn_mov_dpp(h.x, CTRL, 0xF, 0xF, true);
  o.y = __builtin_amdgcn_mov_dpp(h.y, CTRL, 0xF, 0xF, true);
  return __builtin_bit_cast(double, o);
}
// row (16-lane) sums by DPP, then the two cross-row exchanges by
// v_permlane16_swap / v_permlane32_swap (gfx950): VALU only, no SGPR hop
__device__ __forceinline__ double wave_sum_perm(double v) {
  v += mdpp64<0xB1>(v);
  v += mdpp64<0x4E>(v);
  v += mdpp64<0x141>(v);
  v += mdpp64<0x140>(v);
  int2 h = __builtin_bit_cast(int2, v);
  auto a = __builtin_amdgcn_permlane16_swap(h.x, h.x, false, false);
  auto b = __builtin_amdgcn_permlane16_swap(h.y, h.y, false, false);
  v = __builtin_bit_cast(double, make_int2(int(a[0]), int(b[0]))) + __builtin_bit_cast(double, make_int2(int(a[1]), int(b[1])));
  h = __builtin_bit_cast(int2, v);
  a = __builtin_amdgcn_permlane32_swap(h.x, h.x, false, false);
  b = __builtin_amdgcn_permlane32_swap(h.y, h.y, false, false);
  return __builtin_bit_cast(double, make_int2(int(a[0]), int(b[0]))) + __builtin_bit_cast(double, make_int2(int(a[1]), int(b[1])));
}
__device__ __forceinline__ double row_sum_mdpp(double v) {
  v += mdpp64<0xB1>(v);
  v += mdpp64<0x4E>(v);
  v += mdpp64<0x141>(v);
  v += mdpp64<0x140>(v);
  return v;
}
__device__ __forceinline__ double wave_sum_shfl(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double rsq_nr(double x) {
  double r = __builtin_amdgcn_rsq(x);
  r = r * fma(-0.5 * x * r, r, 1.5);
  return r * fma(-0.5 * x * r, r, 1.5);
}
__device__ __forceinline__ double rcp_nr(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = r * fma(-x, r, 2.0);
  return r * fma(-x, r, 2.0);
}

constexpr int kTests = 20;
__global__ __launch_bounds__(64) void lat(double seed, int n, double* out, double* sink) {
  __shared__ double lds[64 * 8];
  __shared__ int ilds[64];
  const int lane = threadIdx.x;
  for (int i = lane; i < 64 * 8; i += 64) lds[i] = 1.0 + 1e-9 * i;
  ilds[lane] = (lane + 1) & 63;
  __syncthreads();
  double x = seed + lane * 1e-12, acc = 0.0;
  uint64_t t0, t1;
  auto run = [&](int id, auto&& body) {
    __builtin_amdgcn_s_waitcnt(0);
    t0 = __builtin_amdgcn_s_memtime();
    body();
    __builtin_amdgcn_s_waitcnt(0);
    t1 = __builtin_amdgcn_s_memtime();
    acc += x;
    if (lane == 0) out[id] = double(t1 - t0) / n;
  };
  run(0, [&] {  // dependent f64 fma
    for (int i = 0; i < n; i += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) x = fma(x, 0.999999, 1e-7);
    }
  });
  run(1, [&] {  // dependent f32 fma
    float y = float(x);
    for (int i = 0; i < n; i += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) y = fmaf(y, 0.999999f, 1e-7f);
    }
    x = y;
  });
  run(2, [&] {  // independent f64 fma (8 chains): issue rate
    double y[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) y[u] = x + u;
    for (int i = 0; i < n; i += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) y[u] = fma(y[u], 0.999999, 1e-7);
    }
    x = y[0] + y[7];
  });
  run(3, [&] {  // DPP + readlane double wave sum
    for (int i = 0; i < n; ++i) x = wave_sum_dpp(x) * (1.0 / 64.0);
  });
  run(4, [&] {  // shuffle double wave sum
    for (int i = 0; i < n; ++i) x = wave_sum_shfl(x) * (1.0 / 64.0);
  });
  run(5, [&] {  // LDS int pointer chase (ds_read_b32 latency)
    int p = lane;
    for (int i = 0; i < n; ++i) p = ilds[p];
    x += p;
  });
  run(6, [&] {  // LDS double read feeding the address of the next
    int p = lane;
    for (int i = 0; i < n; ++i) {
      const double v = lds[p * 8];
      p = (int(v) + p + 1) & 63;
    }
    x += p;
  });
  run(7, [&] {  // readlane64 -> VALU chain
    for (int i = 0; i < n; ++i) x = readlane64(x, i & 63) + 1e-9;
  });
  run(8, [&] {  // rsq + 2 Newton chain
    for (int i = 0; i < n; ++i) x = rsq_nr(x * x + 1.0);
  });
  run(9, [&] {  // IEEE sqrt chain
    for (int i = 0; i < n; ++i) x = sqrt(x + 1.0);
  });
  run(10, [&] {  // IEEE division chain
    for (int i = 0; i < n; ++i) x = 1.0 / (x + 1.0);
  });
  run(11, [&] {  // rcp + 2 Newton chain
    for (int i = 0; i < n; ++i) x = rcp_nr(x + 1.0);
  });
  run(12, [&] {  // ballot + ffs + uniform select chain
    int f = lane;
    for (int i = 0; i < n; ++i) {
      const unsigned long long b = __ballot(lane >= (f & 31));
      f = __ffsll(static_cast<long long>(b)) + (i & 7);
    }
    x += f;
  });
  run(13, [&] {  // LDS store by one lane, read by another (same wave, in order)
    for (int i = 0; i < n; ++i) {
      lds[lane] = x;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      x = lds[(lane + 1) & 63] + 1e-9;
    }
  });
  run(14, [&] {  // s_barrier round trip of one wave
    for (int i = 0; i < n; ++i) {
      __syncthreads();
      x += 1e-9;
    }
  });
  run(15, [&] {  // f64 compare + select chain (pivmin clamp style)
    for (int i = 0; i < n; ++i) x = fabs(x) < 0.5 ? x + 1.0 : x - 0.25;
  });
  run(16, [&] {  // DPP rows + permlane16/32 swaps
    for (int i = 0; i < n; ++i) x = wave_sum_perm(x) * (1.0 / 64.0);
  });
  run(17, [&] {  // 4 DPP stages only (row sums)
    for (int i = 0; i < n; ++i) x = row_sum_mdpp(x) * (1.0 / 16.0);
  });
  run(18, [&] {  // 3 independent DPP+permlane wave sums per step (k = 3 vectors)
    double y = x + 1.0, z = x + 2.0;
    for (int i = 0; i < n; ++i) {
      x = wave_sum_perm(x) * (1.0 / 64.0);
      y = wave_sum_perm(y) * (1.0 / 64.0);
      z = wave_sum_perm(z) * (1.0 / 64.0);
    }
    x += y + z;
  });
  run(19, [&] {  // 8 independent broadcast LDS double reads, then consume (block of 8)
    int p = lane & 1;
    for (int i = 0; i < n; i += 8) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = lds[(p + u) * 8];
      double t = 0.0;
#pragma unroll
      for (int u = 0; u < 8; ++u) t += v[u];
      p = int(t) & 7;
    }
    x += p;
  });
  sink[lane] = acc;
}

int main() {
  double *out, *sink;
  CK(hipMalloc(&out, kTests * sizeof(double)));
  CK(hipMalloc(&sink, 64 * sizeof(double)));
  const int n = 1024;
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(lat, dim3(1), dim3(64), 0, 0, 0.5, n, out, sink);
  CK(hipDeviceSynchronize());
  double h[kTests];
  CK(hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost));
  static const char* names[kTests] = {"fma_f64", "fma_f32", "fma_f64_x8_independent", "wave_sum_dpp_f64",
                                      "wave_sum_shfl_f64", "lds_b32_chase", "lds_b64_chase", "readlane64_chain",
                                      "rsq_newton2_f64", "sqrt_ieee_f64", "div_ieee_f64", "rcp_newton2_f64",
                                      "ballot_ffs", "lds_store_load_roundtrip", "s_barrier_1wave",
                                      "cmp_select_f64", "wave_sum_dpp_permlane_f64", "row_sum_dpp_f64",
                                      "wave_sum_perm_x3_independent", "lds_8_reads_block_per_elem"};
  printf("{");
  for (int i = 0; i < kTests; ++i) printf("%s\"%s\": %.1f", i ? ", " : "", names[i], h[i]);
  printf("}\n");
  return 0;
}
