// Host cost and end-to-end latency of a chain of K small kernels on MI355X:
// K hipLaunchKernelGGL calls vs one hipGraphLaunch of the same chain captured
// once (does a hipGraph amortise the pump thread's
// per-kernel launch cost for multi-kernel device graphs?).
//   host_us: time in the launch call(s) per batch
//   e2e_us:  launch -> completion observed by hipEventSynchronize, per batch
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

__global__ void tiny(const double* x, double* y, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = x[i] * 2.0 + 1.0;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
  using clk = std::chrono::steady_clock;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  double *buf;
  CK(hipMalloc(&buf, 16 * 4096 * sizeof(double)));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  auto us = [](clk::duration d, int n) { return std::chrono::duration<double, std::micro>(d).count() / n; };
  const int N = 5000;
  for (int K : {1, 2, 4, 8}) {
    auto chain = [&]() {
      for (int k = 0; k < K; ++k) hipLaunchKernelGGL(tiny, dim3(4), dim3(256), 0, s, buf + k * 4096, buf + (k + 1) * 4096, 1024);
    };
    for (int i = 0; i < 200; ++i) chain();
    CK(hipStreamSynchronize(s));
    clk::duration th{}, te{};
    for (int i = 0; i < N; ++i) {
      auto t0 = clk::now();
      chain();
      CK(hipEventRecord(ev, s));
      auto t1 = clk::now();
      CK(hipEventSynchronize(ev));
      th += t1 - t0;
      te += clk::now() - t0;
    }
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    chain();
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int i = 0; i < 200; ++i) CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    clk::duration gh{}, gt{};
    for (int i = 0; i < N; ++i) {
      auto t0 = clk::now();
      CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(ev, s));
      auto t1 = clk::now();
      CK(hipEventSynchronize(ev));
      gh += t1 - t0;
      gt += clk::now() - t0;
    }
    printf("{\"kernels\": %d, \"direct_host_us\": %.2f, \"direct_e2e_us\": %.2f, \"graph_host_us\": %.2f, \"graph_e2e_us\": %.2f}\n",
           K, us(th, N), us(te, N), us(gh, N), us(gt, N));
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  return 0;
}
