// Does an XCD's L2 keep a kernel's data for the NEXT launch?
//
//   xcd_l2_probe [launches] [slice_kb]
//
// slice_kb (default 256): each launch chases through EVERY line of its slice,
// so the data one XCD touches per launch is the slice, and 8 x slice_kb is the
// rotating working set (> 4 MB from slice_kb = 1024: the rot modes then miss
// the XCD's L2 by construction, the same modes still fit it).
//
// The tree kernels re-read the same ~3 MB ensemble on every batch; whether a
// launch finds it in its XCD's 4 MB L2 or must go to the Infinity Cache / HBM
// decides the length of each descent's dependent-load chain.  Eight slices of
// 256 KB, each a random cycle over its 128-B lines.  One lane per workgroup
// chases 256 hops through ONE slice and times it with the 100 MHz wall clock.
// The slice is picked from the workgroup's XCD as read from HW_REG_XCC_ID
// (slice = (xcc + rot) % 8), so placement is exact whatever order the
// dispatcher deals workgroups in.  Modes (each reports ns per hop, mean over
// workgroups, for launches 2..N):
//   same/b2b    rot = 0, launches back to back on one stream (the slice an
//               XCD reads is the one it read last launch: L2-hot if kept)
//   same/sync   rot = 0, hipStreamSynchronize between launches (the serving
//               pattern: the host waits for every batch)
//   rot/b2b     rot = launch index: every launch reads a slice another XCD
//               read last time (not in this XCD's L2; Infinity Cache at best)
//   cold        rot = 0 after a 512 MB streaming write evicted everything
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#define CK(x)                                                      \
  do {                                                             \
    hipError_t e_ = (x);                                           \
    if (e_ != hipSuccess) {                                        \
      std::printf("%s FAILED: %s\n", #x, hipGetErrorString(e_));   \
      std::exit(1);                                                \
    }                                                              \
  } while (0)

constexpr int kLineWords = 32;  // 128-B lines of uint32
constexpr int kBlocks = 64;     // 8 per XCD
int g_slice_words = (256 << 10) / 4;

__global__ __launch_bounds__(64) void chase(const uint32_t* __restrict__ buf, int rot, int slice_words, int hops,
                                            unsigned long long* out) {
  uint32_t xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  xcc &= 7u;
  const uint32_t* base = buf + size_t((xcc + uint32_t(rot)) & 7u) * size_t(slice_words);
  if (threadIdx.x == 0) {
    const unsigned long long t0 = wall_clock64();
    uint32_t i = 0;
    for (int h = 0; h < hops; ++h) i = base[i];
    const unsigned long long t1 = wall_clock64();
    out[blockIdx.x * 2] = (t1 - t0) + (i == 0xffffffffu ? 1ull : 0ull);
    out[blockIdx.x * 2 + 1] = xcc;
  }
}

__global__ void scribble(uint4* p, size_t n) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
    p[i] = make_uint4(uint32_t(i), 1, 2, 3);
}

int main(int argc, char** argv) {
  const int launches = argc > 1 ? std::atoi(argv[1]) : 50;
  const int slice_kb = argc > 2 ? std::atoi(argv[2]) : 256;
  if (slice_kb < 4 || slice_kb > 8192) { std::printf("slice_kb 4..8192\n"); return 2; }
  g_slice_words = slice_kb * 1024 / 4;
  const int kSliceWords = g_slice_words;
  const int kHops = kSliceWords / kLineWords;  // every line of the slice once per launch
  CK(hipSetDevice(0));
  // eight slices, each one random cycle over its lines
  std::vector<uint32_t> h(size_t(8) * kSliceWords, 0);
  std::mt19937 rng(7);
  const int lines = kSliceWords / kLineWords;
  for (int s = 0; s < 8; ++s) {
    std::vector<int> perm(lines);
    std::iota(perm.begin(), perm.end(), 0);
    std::shuffle(perm.begin() + 1, perm.end(), rng);
    for (int k = 0; k < lines; ++k) {
      const int from = perm[k], to = perm[(k + 1) % lines];
      h[size_t(s) * kSliceWords + size_t(from) * kLineWords] = uint32_t(to * kLineWords);
    }
  }
  uint32_t* buf = nullptr;
  unsigned long long* out = nullptr;
  uint4* big = nullptr;
  const size_t big_n = (size_t(512) << 20) / sizeof(uint4);
  CK(hipMalloc(reinterpret_cast<void**>(&buf), h.size() * 4));
  CK(hipMemcpy(buf, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  CK(hipHostMalloc(reinterpret_cast<void**>(&out), kBlocks * 2 * sizeof(unsigned long long), hipHostMallocDefault));
  CK(hipMalloc(reinterpret_cast<void**>(&big), big_n * sizeof(uint4)));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  auto ns_per_hop = [&]() {
    double s = 0;
    for (int b = 0; b < kBlocks; ++b) s += double(out[b * 2]);
    return s / kBlocks * 10.0 / kHops;  // 100 MHz ticks -> ns
  };
  auto run = [&](const char* name, bool rotate, bool sync, bool evict) {
    std::vector<double> v;
    int xcc_seen = 0;
    for (int l = 0; l < launches; ++l) {
      if (evict) scribble<<<1024, 256, 0, st>>>(big, big_n);
      chase<<<kBlocks, 64, 0, st>>>(buf, rotate ? l : 0, kSliceWords, kHops, out);
      if (sync || evict || l == launches - 1) CK(hipStreamSynchronize(st));
      if (sync || evict) {
        if (l > 0) v.push_back(ns_per_hop());
        int mask = 0;
        for (int b = 0; b < kBlocks; ++b) mask |= 1 << int(out[b * 2 + 1]);
        xcc_seen = __builtin_popcount(unsigned(mask));
      }
    }
    if (v.empty()) v.push_back(ns_per_hop());  // back to back: the last launch
    std::sort(v.begin(), v.end());
    std::printf("{\"slice_kb\": %d, \"mode\": \"%s\", \"ns_per_hop_p50\": %.1f, \"ns_per_hop_min\": %.1f, \"ns_per_hop_max\": %.1f, "
                "\"xccs_seen\": %d}\n", slice_kb, name, v[v.size() / 2], v.front(), v.back(), xcc_seen);
    std::fflush(stdout);
  };
  run("same/sync", false, true, false);
  run("same/b2b", false, false, false);
  run("rot/b2b", true, false, false);
  run("rot/sync", true, true, false);
  run("cold", false, false, true);
  run("same/sync", false, true, false);
  CK(hipStreamDestroy(st));
  return 0;
}
