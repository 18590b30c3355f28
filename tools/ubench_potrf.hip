// Dev microbenchmark: phases of the single-wave diagonal-block kernels.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "../math_amd/csrc/tri_small.h"

__global__ __launch_bounds__(64) void k_phase(double* g, double* dinv, long long* cyc, int* st) {
  __shared__ double col[SMG_NB];
  __shared__ double Lrow[SMG_NB * SMG_NBP];
  __shared__ double Xcol[SMG_NB * SMG_NBP];
  long long t0 = __builtin_amdgcn_s_memtime();
  wave_potrf64_reg(g, 64, 64, false, g, 64, col, Lrow, st, true);
  __builtin_amdgcn_s_waitcnt(0);
  long long t1 = __builtin_amdgcn_s_memtime();
  wave_trtri64_lds(Lrow, Xcol, dinv, 64, 64);
  __builtin_amdgcn_s_waitcnt(0);
  long long t2 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    cyc[0] = t1 - t0;
    cyc[1] = t2 - t1;
  }
}

__global__ __launch_bounds__(256) void k_lds_old(double* g, long long* cyc, int* st) {
  __shared__ double D[SMG_NB * SMG_NBP], X[SMG_NB * SMG_NBP], T[768];
  lds_load_block(D, g, 64, 64, true);
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime();
  lds_potrf_inv64(D, X, T, st);
  long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
  lds_store_block(X, g, 64, 64, true);
}

int main() {
  double *d, *dinv;
  long long* cyc;
  int* st;
  hipMalloc(&d, 1 << 20);
  hipMalloc(&dinv, 1 << 20);
  hipMalloc(&cyc, 64 * sizeof(long long));
  hipMalloc(&st, 64);
  std::vector<double> h(4096);
  for (int j = 0; j < 64; ++j)
    for (int i = 0; i < 64; ++i) h[i + 64 * j] = (i == j ? 64.0 : 0.0) + 1.0 / (1 + i + j);
  long long c[4];
  for (int rep = 0; rep < 3; ++rep) {
    hipMemcpy(d, h.data(), 4096 * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_phase, dim3(1), dim3(64), 0, 0, d, dinv, cyc, st);
    hipDeviceSynchronize();
    hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    printf("reg factor: %lld cycles, lds trtri: %lld cycles\n", c[0], c[1]);
    hipMemcpy(d, h.data(), 4096 * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_lds_old, dim3(1), dim3(256), 0, 0, d, cyc, st);
    hipDeviceSynchronize();
    hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    printf("old lds potrf+inv: %lld cycles\n", c[0]);
  }
  return 0;
}
