// Dev microbenchmark: latency of the 64x64 diagonal-block building blocks
// (tri_small.h) inside one 512-thread workgroup, phase by phase, timed with
// s_memrealtime (100 MHz) around each phase; REPS repetitions, mean in us.
#include "../math_amd/csrc/tri_small.h"
#include <cstdio>
#include <vector>

#define NPH 8
__global__ __launch_bounds__(512) void k_diag(const double* A, int* status, unsigned long long* t,
                                              int reps) {
  __shared__ double D[SMG_NB * SMG_NBP];
  __shared__ double X[SMG_NB * SMG_NBP];
  __shared__ double Y[SMG_NB * SMG_NBP];
  __shared__ double Tt[3 * 256];
  unsigned long long acc[NPH] = {0};
  for (int r = 0; r < reps; ++r) {
    lds_load_block(D, A, 64, 64, true);
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    lds_potrf64_lookahead(D, status);
    __syncthreads();
    unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    lds_trtri64_mfma(D, X, Tt);
    __syncthreads();
    unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
    lds_mma64_8w<false, true>(Y, D, X);
    __syncthreads();
    unsigned long long t3 = __builtin_amdgcn_s_memrealtime();
    lds_load_block(D, A, 64, 64, true);
    __syncthreads();
    unsigned long long t4 = __builtin_amdgcn_s_memrealtime();
    lds_potrf64_blocked(D, status);
    __syncthreads();
    unsigned long long t5 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x < 64) wave_potrf64_reg(A, 64, 64, false, nullptr, 0, Tt, D, status, true);
    __syncthreads();
    unsigned long long t6 = __builtin_amdgcn_s_memrealtime();
    lds_load_block((r & 1) ? D : Y, A, 64, 64, true);
    __syncthreads();
    unsigned long long t7 = __builtin_amdgcn_s_memrealtime();
    lds_potrf_inv64_blk((r & 1) ? D : Y, X, 64, nullptr, 0, nullptr, 0, status, true);
    __syncthreads();
    unsigned long long t8 = __builtin_amdgcn_s_memrealtime();
    acc[0] += t1 - t0; acc[1] += t2 - t1; acc[2] += t3 - t2; acc[3] += t5 - t4;
    acc[4] += t6 - t5; acc[5] += t7 - t6; acc[6] += t8 - t7; acc[7] += t4 - t3;
  }
  if (threadIdx.x == 0)
    for (int p = 0; p < NPH; ++p) t[p] = acc[p];
  if (threadIdx.x == 0 && Y[7] == 12345.0 && X[9] == 4321.0) t[0] = 0;  // keep Y / X live
}

int main() {
  const int n = 64, reps = 50;
  std::vector<double> A(n * n);
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) A[i + j * n] = (i == j ? n : 0.0) + 1.0 / (1.0 + i + j);
  double* dA;
  int* st;
  unsigned long long* dt;
  (void)hipMalloc(&dA, 8 * n * n);
  (void)hipMalloc(&st, 4);
  (void)hipMalloc(&dt, 8 * NPH);
  (void)hipMemcpy(dA, A.data(), 8 * n * n, hipMemcpyHostToDevice);
  (void)hipMemset(st, 0, 4);
  hipLaunchKernelGGL(k_diag, dim3(1), dim3(512), 0, 0, dA, st, dt, 2);
  hipLaunchKernelGGL(k_diag, dim3(1), dim3(512), 0, 0, dA, st, dt, reps);
  unsigned long long h[NPH];
  (void)hipMemcpy(h, dt, 8 * NPH, hipMemcpyDeviceToHost);
  const char* nm[NPH] = {"potrf64_lookahead", "trtri64_mfma", "mma64_8w", "potrf64_blocked",
                         "potrf64_reg(1 wave)", "barrier", "potrf_inv64_blk", "load_block"};
  for (int p = 0; p < NPH; ++p) printf("%-20s %8.2f us\n", nm[p], h[p] / 100.0 / reps);
  return 0;
}
