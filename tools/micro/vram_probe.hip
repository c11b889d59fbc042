// Where should a serving kernel's small input batch live?
//
//   vram_probe [iters] [rows] [cols]
//
// The batcher parses request rows on the CPU and the kernel reads them once.
// Today they sit in pinned host memory (hipHostMalloc) and the kernel reads
// them over PCIe.  This probe compares, per launch of a kernel that only
// reads the batch and reduces it:
//   host   rows written by the CPU into pinned host memory (hipHostMallocDefault)
//   hostc  the same with the batcher's flags (Mapped | Portable | Coherent:
//          PinnedBuffer in csrc/gpu/hip_util.h, the current serving path)
//   vram   rows written by the CPU straight into fine-grained device memory
//          (hipExtMallocWithFlags(hipDeviceMallocFinegrained), CPU-mapped
//          through the BAR), then sfence
//   dev    rows already in ordinary device memory (no CPU write: the floor)
// Each iteration writes fresh values and checks the GPU's sum against the
// CPU's (a stale line anywhere fails the run).  Reported: host-side launch +
// sync round trip (p50/p99), CPU write time of the batch, and mismatches.
// Kernel durations come from `rocprofv3 --kernel-trace --stats` over the
// same run (the three kernels are separate template instances).
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <setjmp.h>
#include <signal.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::printf("%s FAILED: %s\n", #x, hipGetErrorString(e_));                \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

using clk = std::chrono::steady_clock;

template <int SRC>
__global__ __launch_bounds__(256) void sum_batch(const double* __restrict__ x, int n, double* __restrict__ out) {
  __shared__ double part[4];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) s += x[i];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = part[0] + part[1] + part[2] + part[3];
}

static sigjmp_buf g_jmp;
static void on_segv(int) { siglongjmp(g_jmp, 1); }

static bool cpu_can_write(double* p, size_t n) {
  struct sigaction sa {}, old {};
  sa.sa_handler = on_segv;
  sigaction(SIGSEGV, &sa, &old);
  sigaction(SIGBUS, &sa, nullptr);
  bool ok = false;
  if (sigsetjmp(g_jmp, 1) == 0) {
    for (size_t i = 0; i < n; ++i) p[i] = 0.0;
    _mm_sfence();
    ok = true;
  }
  sigaction(SIGSEGV, &old, nullptr);
  signal(SIGBUS, SIG_DFL);
  return ok;
}

// WC-friendly copy: 16-byte non-temporal stores, then sfence.
static void stream_copy(double* dst, const double* src, size_t n) {
  size_t i = 0;
  for (; i + 2 <= n; i += 2) _mm_stream_pd(dst + i, _mm_loadu_pd(src + i));
  for (; i < n; ++i) dst[i] = src[i];
  _mm_sfence();
}

struct Stats {
  std::vector<double> rt, wr;
  int bad = 0;
  void print(const char* name) {
    std::sort(rt.begin(), rt.end());
    std::sort(wr.begin(), wr.end());
    auto q = [](const std::vector<double>& v, double f) { return v.empty() ? 0.0 : v[std::min(v.size() - 1, size_t(v.size() * f))]; };
    std::printf("{\"src\": \"%s\", \"iters\": %zu, \"roundtrip_p50_us\": %.2f, \"roundtrip_p99_us\": %.2f, "
                "\"cpu_write_p50_us\": %.3f, \"cpu_write_p99_us\": %.3f, \"mismatches\": %d}\n",
                name, rt.size(), q(rt, 0.5), q(rt, 0.99), q(wr, 0.5), q(wr, 0.99), bad);
    std::fflush(stdout);
  }
};

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 4000;
  const int rows = argc > 2 ? std::atoi(argv[2]) : 9;
  const int cols = argc > 3 ? std::atoi(argv[3]) : 32;
  const size_t n = size_t(rows) * cols;
  if (n == 0 || n > (1u << 20)) { std::printf("bad shape\n"); return 2; }
  CK(hipSetDevice(0));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  double *host = nullptr, *hostc = nullptr, *fine = nullptr, *dev = nullptr, *out = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&host), n * sizeof(double), hipHostMallocDefault));
  CK(hipHostMalloc(reinterpret_cast<void**>(&hostc), n * sizeof(double),
                   hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent));
  CK(hipHostMalloc(reinterpret_cast<void**>(&out), 64, hipHostMallocDefault));
  CK(hipMalloc(reinterpret_cast<void**>(&dev), n * sizeof(double)));
  hipError_t fe = hipExtMallocWithFlags(reinterpret_cast<void**>(&fine), n * sizeof(double), hipDeviceMallocFinegrained);
  std::printf("{\"fine_grained_alloc\": \"%s\"}\n", hipGetErrorString(fe));
  if (fe == hipSuccess) {
    hipPointerAttribute_t a{};
    hipError_t ae = hipPointerGetAttributes(&a, fine);
    std::printf("{\"attr\": \"%s\", \"type\": %d, \"host_ptr\": \"%p\", \"dev_ptr\": \"%p\", \"ptr\": \"%p\", "
                "\"flags\": %u}\n", hipGetErrorString(ae), int(a.type), a.hostPointer, a.devicePointer,
                static_cast<void*>(fine), a.allocationFlags);
  }
  int large_bar = -1;
  (void)hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, 0);
  std::printf("{\"is_large_bar\": %d}\n", large_bar);
  bool fine_ok = fe == hipSuccess && cpu_can_write(fine, n);
  std::printf("{\"fine_grained_cpu_writable\": %s}\n", fine_ok ? "true" : "false");
  std::fflush(stdout);

  std::vector<double> src(n);
  auto fill = [&](int it) {
    for (size_t i = 0; i < n; ++i) src[i] = double((it * 7 + int(i) * 3) % 1000);
  };
  auto expect = [&]() {
    double s = 0.0;
    for (double v : src) s += v;
    return s;
  };
  auto run = [&](int which, const char* name) {
    Stats S;
    for (int it = 0; it < iters + 50; ++it) {
      fill(it);
      const double want = expect();
      out[0] = -1.0;
      auto t0 = clk::now();
      const double* x = dev;
      if (which == 0) {
        std::memcpy(host, src.data(), n * sizeof(double));
        x = host;
      } else if (which == 3) {
        std::memcpy(hostc, src.data(), n * sizeof(double));
        x = hostc;
      } else if (which == 1) {
        stream_copy(fine, src.data(), n);
        x = fine;
      } else {
        CK(hipMemcpy(dev, src.data(), n * sizeof(double), hipMemcpyHostToDevice));  // untimed below
        t0 = clk::now();
      }
      auto t1 = clk::now();
      if (which == 0) sum_batch<0><<<1, 256, 0, st>>>(x, int(n), out);
      else if (which == 1) sum_batch<1><<<1, 256, 0, st>>>(x, int(n), out);
      else if (which == 3) sum_batch<3><<<1, 256, 0, st>>>(x, int(n), out);
      else sum_batch<2><<<1, 256, 0, st>>>(x, int(n), out);
      CK(hipStreamSynchronize(st));
      auto t2 = clk::now();
      if (it >= 50) {
        S.wr.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
        S.rt.push_back(std::chrono::duration<double, std::micro>(t2 - t1).count());
        if (out[0] != want) ++S.bad;
      }
    }
    S.print(name);
  };
  run(0, "host");
  run(3, "hostc");
  if (fine_ok) run(1, "vram");
  run(2, "dev");
  if (fine_ok) run(1, "vram");
  run(3, "hostc");
  run(0, "host");
  CK(hipStreamDestroy(st));
  return 0;
}
