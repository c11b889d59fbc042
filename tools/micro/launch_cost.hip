// Host-side cost of the micro-batcher's per-batch HIP calls on MI355X:
// hipLaunchKernelGGL, hipEventRecord, hipExtLaunchKernelGGL(stop event),
// hipEventQuery polling -- each timed over many iterations on one stream.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <chrono>
#include <cstdio>

__global__ void tiny(const double* x, double* y, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = x[i] * 2.0;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
  using clk = std::chrono::steady_clock;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  double *x, *y;
  CK(hipHostMalloc(&x, 4096, hipHostMallocMapped));
  CK(hipHostMalloc(&y, 4096, hipHostMallocMapped));
  hipEvent_t ev[4];
  for (auto& evi : ev) CK(hipEventCreateWithFlags(&evi, hipEventDisableTiming));
  const int N = 20000;
  auto us = [](clk::duration d, int n) { return std::chrono::duration<double, std::micro>(d).count() / n; };
  // warm
  for (int i = 0; i < 1000; ++i) hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, x, y, 64);
  CK(hipStreamSynchronize(s));
  // 1: launch only (queue kept short by periodic sync)
  clk::duration tl{};
  for (int i = 0; i < N; ++i) {
    auto t0 = clk::now();
    hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, x, y, 64);
    tl += clk::now() - t0;
    if (i % 4 == 3) CK(hipStreamSynchronize(s));
  }
  // 2: event record only
  clk::duration te{};
  for (int i = 0; i < N; ++i) {
    hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, x, y, 64);
    auto t0 = clk::now();
    CK(hipEventRecord(ev[i & 3], s));
    te += clk::now() - t0;
    if (i % 4 == 3) CK(hipStreamSynchronize(s));
  }
  // 3: ext launch with stop event (one packet)
  clk::duration tx{};
  for (int i = 0; i < N; ++i) {
    auto t0 = clk::now();
    hipExtLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, nullptr, ev[i & 3], 0, x, y, 64);
    tx += clk::now() - t0;
    if (i % 4 == 3) CK(hipStreamSynchronize(s));
  }
  // 4: round trip launch + record + spin on query
  clk::duration tr{}, tq{};
  long polls = 0;
  for (int i = 0; i < N; ++i) {
    auto t0 = clk::now();
    hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, x, y, 64);
    CK(hipEventRecord(ev[0], s));
    auto t1 = clk::now();
    while (hipEventQuery(ev[0]) == hipErrorNotReady) ++polls;
    ++polls;
    tq += clk::now() - t1;
    tr += clk::now() - t0;
  }
  // 5: round trip ext launch + spin on query
  clk::duration tr2{};
  for (int i = 0; i < N; ++i) {
    auto t0 = clk::now();
    hipExtLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, nullptr, ev[0], 0, x, y, 64);
    while (hipEventQuery(ev[0]) == hipErrorNotReady) {}
    tr2 += clk::now() - t0;
  }
  // 6: round trip with a host-memory flag written by the kernel's last store
  printf("{\"launch_us\": %.2f, \"event_record_us\": %.2f, \"ext_launch_with_event_us\": %.2f, "
         "\"roundtrip_launch_record_query_us\": %.2f, \"query_wait_us\": %.2f, \"query_cost_us\": %.3f, "
         "\"roundtrip_ext_launch_query_us\": %.2f}\n",
         us(tl, N), us(te, N), us(tx, N), us(tr, N), us(tq, N), us(tq, int(polls)), us(tr2, N));
  return 0;
}
