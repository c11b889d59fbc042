// Cross-process data-plane probe for the fabric's IPC transport
// (csrc/parallel/fabric.cc): two processes on the SAME MI355X, each with its
// own HIP context, exchange buffers and ordering signals.
//
//   ipc_probe A <shm-name> <iters>     (creates the shared page)
//   ipc_probe B <shm-name> <iters>     (opens it)
//
// Started side by side by tools/micro/ipc_probe.py (neither process forks or
// execs after touching the GPU).  Tests, in order:
//   T1 hipIpcGetMemHandle / hipIpcOpenMemHandle: B reads A's pattern, writes
//      its own, A checks it
//   T2 hipIpcGetEventHandle / hipIpcOpenEventHandle: B's stream waits for A's
//      slow kernel through the event (host time of the wait call reported)
//   T3 a host page shared by both (shm + hipHostRegister): B's stream writes a
//      flag after its kernel stored into A's buffer; A's host sees the flag,
//      then the data
//   T4 hipStreamWaitValue64 on that page: A's stream waits for a flag B's host
//      sets; A's host releases the wait itself after 2 s if it never comes
//   T5 round trip (the fabric's message pattern): A copies X into B's slot and
//      writes a doorbell; B's stream waits, runs y = x + 1 into its Y slot and
//      writes a reply flag; A's stream waits, copies Y back; per-iteration
//      latency with a host sync, then pipelined throughput
// Every GPU-side wait has a host-side escape: the flag it waits on lives in
// host memory, and the waiting process writes it itself when the peer is late.
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#define CK(x)                                                                                    \
  do {                                                                                           \
    hipError_t e_ = (x);                                                                         \
    if (e_ != hipSuccess) {                                                                      \
      std::printf("%s: %s FAILED: %s\n", role, #x, hipGetErrorString(e_));                       \
      std::fflush(stdout);                                                                       \
      fail(#x);                                                                                  \
    }                                                                                            \
  } while (0)

using clk = std::chrono::steady_clock;

struct alignas(4096) Shared {
  std::atomic<int> stage_a, stage_b;
  int fail_a, fail_b;
  hipIpcMemHandle_t mem_a, mem_b_x, mem_b_y;
  hipIpcEventHandle_t ev_a;
  int ev_ok;
  alignas(64) uint64_t flags[64];  // GPU-visible (both processes register this page)
};
enum { F_T3 = 0, F_T4_GO = 8, F_T4_DONE = 16, F_X = 24, F_Y = 32 };

static const char* role = "?";
static Shared* S = nullptr;
static void fail(const char* what) {
  if (S) (role[0] == 'A' ? S->fail_a : S->fail_b) = 1;
  std::printf("%s: abort at %s\n", role, what);
  std::fflush(stdout);
  std::_Exit(3);
}

static double us_since(clk::time_point t) { return std::chrono::duration<double, std::micro>(clk::now() - t).count(); }

static void wait_stage(std::atomic<int>& s, int v, const char* what, int timeout_ms = 10000) {
  auto t = clk::now();
  while (s.load(std::memory_order_acquire) < v) {
    if (us_since(t) > timeout_ms * 1000.0) {
      std::printf("%s: timeout waiting for %s\n", role, what);
      fail(what);
    }
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

static bool wait_flag(volatile uint64_t* f, uint64_t v, int timeout_ms) {
  auto t = clk::now();
  while (__atomic_load_n(f, __ATOMIC_ACQUIRE) < v)
    if (us_since(t) > timeout_ms * 1000.0) return false;
  return true;
}

__global__ void fill_kernel(uint32_t* p, uint32_t v, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v + uint32_t(i);
}

__global__ void slow_store_kernel(uint32_t* p, uint32_t v, uint64_t ticks) {
  // wall_clock64 runs at a fixed 100 MHz on CDNA
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  if (threadIdx.x == 0) p[0] = v;
}

__global__ void plus_one_kernel(const double* x, double* y, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = x[i] + 1.0;
}

static Shared* map_shared(const char* name, bool create) {
  int fd = -1;
  auto t = clk::now();
  while (fd < 0) {
    fd = shm_open(name, create ? (O_CREAT | O_EXCL | O_RDWR) : O_RDWR, 0600);
    if (fd < 0 && (create || us_since(t) > 10e6)) {
      std::printf("%s: shm_open(%s): %s\n", role, name, std::strerror(errno));
      std::exit(2);
    }
    if (fd < 0) std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
  if (create && ftruncate(fd, sizeof(Shared)) != 0) std::exit(2);
  if (!create) {  // wait for the creator's ftruncate
    struct stat st {};
    while (fstat(fd, &st) == 0 && size_t(st.st_size) < sizeof(Shared)) std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
  void* p = mmap(nullptr, sizeof(Shared), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) std::exit(2);
  return static_cast<Shared*>(p);
}

int main(int argc, char** argv) {
  if (argc < 4) {
    std::printf("usage: ipc_probe A|B <shm> <iters>\n");
    return 2;
  }
  const bool A = argv[1][0] == 'A';
  role = A ? "A" : "B";
  const int iters = std::max(10, std::atoi(argv[3]));
  S = map_shared(argv[2], A);
  volatile uint64_t* flags = S->flags;

  CK(hipSetDevice(0));
  int can_wait = -1;
  CK(hipDeviceGetAttribute(&can_wait, hipDeviceAttributeCanUseStreamWaitValue, 0));
  const char* cpw = std::getenv("GPU_STREAMOPS_CP_WAIT");
  std::printf("%s: pid %d, hipDeviceAttributeCanUseStreamWaitValue=%d GPU_STREAMOPS_CP_WAIT=%s\n", role, getpid(),
              can_wait, cpw ? cpw : "(unset)");
  CK(hipHostRegister((void*)S, sizeof(Shared), hipHostRegisterMapped | hipHostRegisterPortable));
  uint64_t* dflags = nullptr;
  CK(hipHostGetDevicePointer((void**)&dflags, (void*)S->flags, 0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int N = 1 << 16;  // 256 KB of uint32

  if (A) {
    // ---------------- T1
    uint32_t* bufA;
    CK(hipMalloc(&bufA, N * sizeof(uint32_t)));
    fill_kernel<<<N / 256, 256, 0, s>>>(bufA, 0xA0000000u, N);
    CK(hipStreamSynchronize(s));
    CK(hipIpcGetMemHandle(&S->mem_a, bufA));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventInterprocess | hipEventDisableTiming));
    hipError_t eh = hipIpcGetEventHandle(&S->ev_a, ev);
    S->ev_ok = eh == hipSuccess;
    std::printf("A: hipIpcGetEventHandle -> %s\n", hipGetErrorString(eh));
    S->stage_a.store(1, std::memory_order_release);
    wait_stage(S->stage_b, 1, "B T1");
    std::vector<uint32_t> h(N);
    CK(hipMemcpy(h.data(), bufA, N * sizeof(uint32_t), hipMemcpyDeviceToHost));
    int bad = 0;
    for (int i = 0; i < N; ++i) bad += h[i] != 0xB0000000u + uint32_t(i);
    std::printf("A: T1 IPC mem: B's writes into A's buffer: %s (%d bad)\n", bad ? "FAIL" : "ok", bad);

    // ---------------- T2: slow kernel (~2 ms) then record; B waits on its stream
    CK(hipMemset(bufA, 0, 64));
    if (S->ev_ok) {
      slow_store_kernel<<<1, 64, 0, s>>>(bufA, 4242u, 200000);  // 2 ms at 100 MHz
      CK(hipEventRecord(ev, s));
    }
    S->stage_a.store(2, std::memory_order_release);
    wait_stage(S->stage_b, 2, "B T2");
    CK(hipStreamSynchronize(s));

    // ---------------- T3: B's stream stores into bufA then writes flag F_T3
    S->stage_a.store(3, std::memory_order_release);
    const bool t3 = wait_flag(flags + F_T3, 1, 5000);
    uint32_t v3 = 0;
    if (t3) CK(hipMemcpy(&v3, bufA, 4, hipMemcpyDeviceToHost));
    std::printf("A: T3 GPU write of a host-shared flag seen by the other process: %s (data %u, want 777)\n",
                t3 ? "ok" : "TIMEOUT", v3);
    wait_stage(S->stage_b, 3, "B T3");

    // ---------------- T4: A's stream waits on F_T4_GO (set by B's host), then writes F_T4_DONE
    auto t4 = clk::now();
    CK(hipStreamWaitValue64(s, dflags + F_T4_GO, 1, hipStreamWaitValueGte, ~0ull));
    fill_kernel<<<1, 64, 0, s>>>(bufA, 9000u, 64);
    CK(hipStreamWriteValue64(s, dflags + F_T4_DONE, 1, 0));
    const double enq = us_since(t4);
    S->stage_a.store(4, std::memory_order_release);
    bool t4ok = wait_flag(flags + F_T4_DONE, 1, 2000);
    if (!t4ok) {
      __atomic_store_n(flags + F_T4_GO, 1ull, __ATOMIC_RELEASE);  // escape: release our own stream
      t4ok = false;
    }
    const double waited = us_since(t4);
    CK(hipStreamSynchronize(s));
    std::printf("A: T4 hipStreamWaitValue64 on host-shared flag released by B's host: %s (enqueue %.1f us, "
                "done after %.0f us; B sets the flag ~1000 us in)\n",
                t4ok ? "ok" : "TIMEOUT (released by A's own host)", enq, waited);
    wait_stage(S->stage_b, 4, "B T4");

    // ---------------- T5: round trips
    void *bx = nullptr, *by = nullptr;
    CK(hipIpcOpenMemHandle(&bx, S->mem_b_x, hipIpcMemLazyEnablePeerAccess));
    CK(hipIpcOpenMemHandle(&by, S->mem_b_y, hipIpcMemLazyEnablePeerAccess));
    const int n = 512;  // 4 KB of fp64 per message
    double *xa, *ya;
    CK(hipMalloc(&xa, n * sizeof(double)));
    CK(hipMalloc(&ya, n * sizeof(double)));
    std::vector<double> hx(n), hy(n);
    for (int mode = 0; mode < 2; ++mode) {  // 0: latency (sync each), 1: pipelined
      const uint64_t base = uint64_t(mode) * 1000000ull;
      std::vector<double> lat;
      auto t0 = clk::now();
      int errs = 0;
      for (int i = 1; i <= iters; ++i) {
        const uint64_t seq = base + uint64_t(i);
        auto ti = clk::now();
        for (int k = 0; k < n; ++k) hx[k] = double(i) + k;
        if (mode == 0) CK(hipMemcpyAsync(xa, hx.data(), n * sizeof(double), hipMemcpyHostToDevice, s));
        else fill_kernel<<<1, 64, 0, s>>>((uint32_t*)xa, uint32_t(i), 64);  // cheap device-side X change
        CK(hipMemcpyAsync(bx, xa, n * sizeof(double), hipMemcpyDeviceToDevice, s));
        CK(hipStreamWriteValue64(s, dflags + F_X, seq, 0));
        CK(hipStreamWaitValue64(s, dflags + F_Y, seq, hipStreamWaitValueGte, ~0ull));
        CK(hipMemcpyAsync(ya, by, n * sizeof(double), hipMemcpyDeviceToDevice, s));
        if (mode == 0) {
          CK(hipMemcpyAsync(hy.data(), ya, n * sizeof(double), hipMemcpyDeviceToHost, s));
          // bounded host wait for the stream: escape if the reply never comes
          if (!wait_flag(flags + F_Y, seq, 3000)) {
            std::printf("A: T5 reply %llu TIMEOUT, releasing\n", (unsigned long long)seq);
            __atomic_store_n(flags + F_Y, ~0ull >> 1, __ATOMIC_RELEASE);
            CK(hipStreamSynchronize(s));
            fail("T5 reply");
          }
          CK(hipStreamSynchronize(s));
          lat.push_back(us_since(ti));
          for (int k = 0; k < n; ++k) errs += hy[k] != hx[k] + 1.0;
        } else if (i % 64 == 0 || i == iters) {
          if (!wait_flag(flags + F_Y, seq, 5000)) {
            std::printf("A: T5 pipelined reply %llu TIMEOUT, releasing\n", (unsigned long long)seq);
            __atomic_store_n(flags + F_Y, ~0ull >> 1, __ATOMIC_RELEASE);
            CK(hipStreamSynchronize(s));
            fail("T5 pipelined");
          }
        }
      }
      CK(hipStreamSynchronize(s));
      const double tot = us_since(t0);
      if (mode == 0) {
        std::sort(lat.begin(), lat.end());
        std::printf("A: T5 round trip (H2D x, copy into B, B waits+kernel+flag, A waits, copy back, D2H), %d iters: "
                    "p50 %.1f us p90 %.1f us p99 %.1f us max %.1f us; data errors %d\n",
                    iters, lat[lat.size() / 2], lat[lat.size() * 9 / 10], lat[lat.size() * 99 / 100], lat.back(),
                    errs);
      } else {
        std::printf("A: T5 pipelined (device-only, sync every 64): %.2f us per round trip over %d\n", tot / iters,
                    iters);
      }
      S->stage_a.store(5 + mode, std::memory_order_release);
      wait_stage(S->stage_b, 5 + mode, "B T5");
    }
    CK(hipIpcCloseMemHandle(bx));
    CK(hipIpcCloseMemHandle(by));
    S->stage_a.store(100, std::memory_order_release);
    wait_stage(S->stage_b, 100, "B exit");
    CK(hipHostUnregister((void*)S));
    shm_unlink(argv[2]);
    std::printf("A: done\n");
    return 0;
  }

  // ======================= B
  wait_stage(S->stage_a, 1, "A T1");
  uint32_t* a = nullptr;
  CK(hipIpcOpenMemHandle((void**)&a, S->mem_a, hipIpcMemLazyEnablePeerAccess));
  std::vector<uint32_t> h(N);
  CK(hipMemcpy(h.data(), a, N * sizeof(uint32_t), hipMemcpyDeviceToHost));
  int bad = 0;
  for (int i = 0; i < N; ++i) bad += h[i] != 0xA0000000u + uint32_t(i);
  std::printf("B: T1 IPC mem: read A's pattern: %s (%d bad)\n", bad ? "FAIL" : "ok", bad);
  fill_kernel<<<N / 256, 256, 0, s>>>(a, 0xB0000000u, N);
  CK(hipStreamSynchronize(s));
  const int n = 512;
  double *x, *y;
  CK(hipMalloc(&x, n * sizeof(double)));
  CK(hipMalloc(&y, n * sizeof(double)));
  CK(hipIpcGetMemHandle(&S->mem_b_x, x));
  CK(hipIpcGetMemHandle(&S->mem_b_y, y));
  S->stage_b.store(1, std::memory_order_release);

  // T2
  wait_stage(S->stage_a, 2, "A T2");
  if (S->ev_ok) {
    hipEvent_t ev;
    hipError_t e = hipIpcOpenEventHandle(&ev, S->ev_a);
    std::printf("B: hipIpcOpenEventHandle -> %s\n", hipGetErrorString(e));
    if (e == hipSuccess) {
      auto t = clk::now();
      CK(hipStreamWaitEvent(s, ev, 0));
      const double call = us_since(t);
      uint32_t v = 0;
      CK(hipMemcpyAsync(&v, a, 4, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
      std::printf("B: T2 IPC event wait: %s (saw %u, want 4242; hipStreamWaitEvent host call %.1f us, total %.0f us)\n",
                  v == 4242u ? "ok" : "FAIL", v, call, us_since(t));
      CK(hipEventDestroy(ev));
    }
  }
  S->stage_b.store(2, std::memory_order_release);

  // T3
  wait_stage(S->stage_a, 3, "A T3");
  fill_kernel<<<1, 1, 0, s>>>(a, 777u, 1);
  CK(hipStreamWriteValue64(s, dflags + F_T3, 1, 0));
  CK(hipStreamSynchronize(s));
  S->stage_b.store(3, std::memory_order_release);

  // T4
  wait_stage(S->stage_a, 4, "A T4");
  std::this_thread::sleep_for(std::chrono::microseconds(1000));
  __atomic_store_n(flags + F_T4_GO, 1ull, __ATOMIC_RELEASE);
  S->stage_b.store(4, std::memory_order_release);

  // T5: B's slots (exported to A before T1 completes)
  for (int mode = 0; mode < 2; ++mode) {
    const uint64_t base = uint64_t(mode) * 1000000ull;
    // B enqueues up to 4 iterations ahead (its stream waits on the doorbell);
    // its host checks the replies with a bounded wait and releases its own
    // stream if A stops sending.
    for (int i = 1; i <= iters; ++i) {
      const uint64_t seq = base + uint64_t(i);
      if (i > 4 && !wait_flag(flags + F_Y, seq - 4, 5000)) {
        std::printf("B: T5 A stopped sending at %llu, releasing\n", (unsigned long long)seq);
        __atomic_store_n(flags + F_X, ~0ull >> 1, __ATOMIC_RELEASE);
        CK(hipStreamSynchronize(s));
        fail("T5 B");
      }
      CK(hipStreamWaitValue64(s, dflags + F_X, seq, hipStreamWaitValueGte, ~0ull));
      plus_one_kernel<<<(n + 255) / 256, 256, 0, s>>>(x, y, n);
      CK(hipStreamWriteValue64(s, dflags + F_Y, seq, 0));
    }
    if (!wait_flag(flags + F_Y, base + uint64_t(iters), 10000)) {
      __atomic_store_n(flags + F_X, ~0ull >> 1, __ATOMIC_RELEASE);
      CK(hipStreamSynchronize(s));
      fail("T5 B drain");
    }
    CK(hipStreamSynchronize(s));
    wait_stage(S->stage_a, 5 + mode, "A T5");
    S->stage_b.store(5 + mode, std::memory_order_release);
  }
  wait_stage(S->stage_a, 100, "A exit");
  CK(hipHostUnregister((void*)S));
  S->stage_b.store(100, std::memory_order_release);
  std::printf("B: done\n");
  return 0;
}
