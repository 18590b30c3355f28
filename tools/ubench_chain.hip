// Dev microbenchmark: the phases of the panel chain's 64x64 step in one
// 512-thread workgroup (lds_potrf64_lookahead, lds_trtri64_mfma, the two 64^3
// LDS products), timed with s_memrealtime (100 MHz) inside the kernel.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "../math_amd/csrc/tri_small.h"

__global__ __launch_bounds__(512) void k_chain_phases(const double* g, unsigned long long* ts, int* st,
                                                      double* sink) {
  __shared__ double D[SMG_NB * SMG_NBP], X[SMG_NB * SMG_NBP], Y[SMG_NB * SMG_NBP];
  __shared__ double T[768];
  if (blockIdx.x > 0) {  // load generator: the owners' 64^3 LDS MFMA products, back to back
    lds_load_block(D, g, 64, 64, false);
    lds_load_block(Y, g, 64, 64, false);
    __syncthreads();
    for (int it = 0; it < 60; ++it) lds_mma64_8w<false, true>(X, D, Y, 1e-3, 1.0);
    if (threadIdx.x == 0) sink[blockIdx.x] = X[0];
    return;
  }
  for (int rep = 0; rep < 4; ++rep) {
    lds_load_block(D, g, 64, 64, true);
    lds_load_block(Y, g, 64, 64, false);
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    lds_potrf64_lookahead(D, st);
    __syncthreads();
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    lds_trtri64_mfma(D, X, T);
    __syncthreads();
    const unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
    lds_mma64_8w<false, true>(Y, Y, X);
    const unsigned long long t3 = __builtin_amdgcn_s_memrealtime();
    lds_mma64_8w<false, true>(D, Y, Y, -1.0, 1.0);
    const unsigned long long t4 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
      ts[rep * 4 + 0] = t1 - t0;
      ts[rep * 4 + 1] = t2 - t1;
      ts[rep * 4 + 2] = t3 - t2;
      ts[rep * 4 + 3] = t4 - t3;
    }
    __syncthreads();
  }
}

int main() {
  const int n = 64;
  std::vector<double> A(n * n);
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) A[i + j * n] = (i == j ? n : 0.0) + 1.0 / (1.0 + i + j);
  double* g;
  unsigned long long* ts;
  int* st;
  hipMalloc(&g, 8 * n * n);
  hipMalloc(&ts, 8 * 16);
  hipMalloc(&st, 4);
  hipMemcpy(g, A.data(), 8 * n * n, hipMemcpyHostToDevice);
  hipMemset(st, 0, 4);
  double* sink;
  hipMalloc(&sink, 8 * 1024);
  for (int grid : {1, 64, 256}) {
    hipLaunchKernelGGL(k_chain_phases, dim3(grid), dim3(512), 0, 0, g, ts, st, sink);
    hipDeviceSynchronize();
    unsigned long long h[16];
    hipMemcpy(h, ts, sizeof(h), hipMemcpyDeviceToHost);
    for (int r = 0; r < 4; ++r)
      printf("grid %3d rep %d: potrf %.2f us  trtri %.2f us  mma(L) %.2f us  mma(sym) %.2f us\n", grid, r,
             h[4 * r] / 100.0, h[4 * r + 1] / 100.0, h[4 * r + 2] / 100.0, h[4 * r + 3] / 100.0);
  }
  return 0;
}
