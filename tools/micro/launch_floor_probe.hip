// What does a serving launch cost on the GPU side before any real work?
//
//   launch_floor_probe [iters]      (run under rocprofv3 --kernel-trace --stats)
//
// The iris serving kernel (linear_thread_rows<1>) does ~nothing and still
// averages 3.4-4.5 us per dispatch in rocprof, the xgb1000 whole-ensemble
// kernel 7.4-8.0 us.  Each variant below is its own template instance, so
// rocprof's per-kernel stats separate them.  Every launch is followed by a
// host wait for the stream (the serving pattern: one batch, the host reads
// the reply, the next batch):
//   <0> empty kernel (1 workgroup of 64)
//   <1> one lane writes one double to device memory
//   <2> one lane writes one double to pinned coherent host memory
//   <3> 9 x 32 doubles read from pinned host memory, 9 doubles written to
//       pinned host memory (the iris / tree serving shape)
//   <4> the same batch read from BAR-written fine-grained HBM, reply to host
//   <5> = <3> with 1024-thread workgroups (the tree kernel's block size)
//   <6> = <0> launched back to back, no host wait in between (the floor of
//       a dispatch that does not wait on the host)
// Host-observed launch -> completion (p50 / p99) is printed per variant.
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                      \
  do {                                                             \
    hipError_t e_ = (x);                                           \
    if (e_ != hipSuccess) {                                        \
      std::printf("%s FAILED: %s\n", #x, hipGetErrorString(e_));   \
      std::exit(1);                                                \
    }                                                              \
  } while (0)

using clk = std::chrono::steady_clock;

template <int V>
__global__ void probe(const double* __restrict__ x, int rows, int cols, double* __restrict__ y) {
  if constexpr (V == 0 || V == 6) {
    return;
  } else if constexpr (V == 1 || V == 2) {
    if (threadIdx.x == 0) y[0] = 1.0;
  } else {
    const int r = int(threadIdx.x);
    if (r < rows) {
      double s = 0.0;
      for (int c = 0; c < cols; ++c) s += x[size_t(r) * cols + c];
      y[r] = s;
    }
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 4000;
  const int rows = 9, cols = 32;
  const size_t n = size_t(rows) * cols;
  CK(hipSetDevice(0));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const unsigned hflags = hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent;
  double *hx, *hy, *dy, *vx;
  CK(hipHostMalloc(reinterpret_cast<void**>(&hx), n * sizeof(double), hflags));
  CK(hipHostMalloc(reinterpret_cast<void**>(&hy), 64 * sizeof(double), hflags));
  CK(hipMalloc(reinterpret_cast<void**>(&dy), 64 * sizeof(double)));
  CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&vx), n * sizeof(double), hipDeviceMallocFinegrained));
  std::vector<double> src(n, 1.0);
  auto run = [&](int v, const char* name) {
    std::vector<double> rt;
    for (int it = 0; it < iters + 50; ++it) {
      if (v == 3 || v == 5) std::memcpy(hx, src.data(), n * sizeof(double));
      if (v == 4) {
        std::memcpy(vx, src.data(), n * sizeof(double));
        _mm_sfence();
      }
      const auto t0 = clk::now();
      switch (v) {
        case 0: probe<0><<<1, 64, 0, st>>>(hx, rows, cols, hy); break;
        case 1: probe<1><<<1, 64, 0, st>>>(hx, rows, cols, dy); break;
        case 2: probe<2><<<1, 64, 0, st>>>(hx, rows, cols, hy); break;
        case 3: probe<3><<<1, 64, 0, st>>>(hx, rows, cols, hy); break;
        case 4: probe<4><<<1, 64, 0, st>>>(vx, rows, cols, hy); break;
        case 5: probe<5><<<1, 1024, 0, st>>>(hx, rows, cols, hy); break;
        default: probe<6><<<1, 64, 0, st>>>(hx, rows, cols, hy); break;
      }
      if (v != 6 || it == iters + 49) CK(hipStreamSynchronize(st));
      const auto t1 = clk::now();
      if (it >= 50 && v != 6) rt.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    if (rt.empty()) rt.push_back(0.0);
    std::sort(rt.begin(), rt.end());
    std::printf("{\"variant\": %d, \"name\": \"%s\", \"host_roundtrip_p50_us\": %.2f, \"p99_us\": %.2f}\n", v, name,
                rt[rt.size() / 2], rt[std::min(rt.size() - 1, size_t(rt.size() * 0.99))]);
    std::fflush(stdout);
  };
  run(0, "empty");
  run(1, "write device");
  run(2, "write host");
  run(3, "host rows -> host reply");
  run(4, "BAR rows -> host reply");
  run(5, "host rows, 1024 threads");
  run(6, "empty, back to back");
  CK(hipStreamDestroy(st));
  return 0;
}
