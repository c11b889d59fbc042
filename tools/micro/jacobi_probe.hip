// Times the Mahalanobis detector's Jacobi solver (jacobi_solve<NT>) in
// isolation: a cold solve of a random covariance, then warm solves after
// rank-1 updates.  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17
//   -I csrc/kernels tools/micro/jacobi_probe.hip -o /tmp/jacobi_probe
#include "../../csrc/kernels/mahalanobis.hip"

#include <chrono>
#include <cstdio>
#include <random>
#include <vector>

namespace sca::kern {
template <int NT>
__global__ __launch_bounds__(NT) void jac_probe(const double* C, double* eig, int p, int k, int reps,
                                                long long* cycles) {
  __shared__ double A[kMahaMaxP * kLdA], V[kMahaMaxP * kLd], W[kMahaMaxP * kLd];
  __shared__ double lamv[kMahaMaxP];
  __shared__ int sel[kMahaMaxK];
  long long total = 0;
  for (int r = 0; r < reps; ++r) {
    for (int e = threadIdx.x; e < p * p; e += NT) A[(e / p) * kLdA + e % p] = C[e];
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    const bool warm = eig[kMahaEigTail] == double(p);
    __syncthreads();
    jacobi_solve<NT>(A, V, W, sel, p, k, eig, eig + kMahaEigTail, lamv, eig + kMahaEigLam, warm,
                     eig + kMahaEigMeta + 3);
    total += __builtin_amdgcn_s_memrealtime() - t0;
    __syncthreads();
  }
  if (threadIdx.x == 0) cycles[0] = total;
}
}  // namespace sca::kern

int main(int argc, char** argv) {
  const int p = argc > 1 ? atoi(argv[1]) : 20;
  std::mt19937_64 g(1);
  std::normal_distribution<double> nd;
  std::vector<double> X(size_t(400) * p), C(size_t(p) * p, 0.0);
  for (auto& x : X) x = nd(g);
  for (int a = 0; a < p; ++a)
    for (int b = 0; b < p; ++b) {
      double s = 0;
      for (int i = 0; i < 400; ++i) s += X[i * p + a] * X[i * p + b];
      C[a * p + b] = s / 399.0;
    }
  double *dC, *deig;
  long long* dcy;
  hipMalloc(&dC, C.size() * 8);
  hipMalloc(&deig, sca::kern::kMahaEigDoubles * 8);
  hipMalloc(&dcy, 8);
  hipMemcpy(dC, C.data(), C.size() * 8, hipMemcpyHostToDevice);
  hipMemset(deig, 0, sca::kern::kMahaEigDoubles * 8);
  for (int pass = 0; pass < 2; ++pass) {  // pass 0: cold (tail empty); pass 1: warm from pass 0's basis
    const int reps = pass == 0 ? 1 : 10;
    if (p <= 16)
      hipLaunchKernelGGL(sca::kern::jac_probe<64>, dim3(1), dim3(64), 0, nullptr, dC, deig, p, 3, reps, dcy);
    else
      hipLaunchKernelGGL(sca::kern::jac_probe<256>, dim3(1), dim3(256), 0, nullptr, dC, deig, p, 3, reps, dcy);
    hipDeviceSynchronize();
    long long cy;
    std::vector<double> meta(8);
    hipMemcpy(&cy, dcy, 8, hipMemcpyDeviceToHost);
    hipMemcpy(meta.data(), deig + sca::kern::kMahaEigMeta, 64, hipMemcpyDeviceToHost);
    printf("p=%d %s: %.1f us per solve (s_memrealtime, 100 MHz), sweeps so far %.0f over %.0f solves\n", p,
           pass ? "warm" : "cold", cy / double(reps) * 0.01, meta[3], meta[4]);
    if (pass == 0) hipMemset(deig + sca::kern::kMahaEigMeta + 3, 0, 16);
  }
  return 0;
}
