// Dev microbenchmark: smg_gemm on the shapes of one blocked-Cholesky step
// (tools/ubench_shapes.h) plus an empty-kernel floor.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../include/smg_hip.h"
#include "ubench_shapes.h"

__global__ void k_empty() {}

int main(int argc, char** argv) {
  const int only = argc > 1 ? atoi(argv[1]) : -1;
  smg_ctx* ctx = nullptr;
  smg_ctx_create(0, 1ull << 30, &ctx);
  hipStream_t s = (hipStream_t)smg_ctx_stream(ctx);
  const int n = 4096;
  double *A, *B, *C;
  hipMalloc(&A, sizeof(double) * n * n);
  hipMalloc(&B, sizeof(double) * n * n);
  hipMalloc(&C, sizeof(double) * n * n);
  smg_fill_unif(ctx, A, (long long)n * n, 1, -1.0, 1.0, 1.0);
  smg_fill_unif(ctx, B, (long long)n * n, 2, -1.0, 1.0, 1.0);
  smg_fill_unif(ctx, C, (long long)n * n, 3, -1.0, 1.0, 1.0);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int reps = 50;
  for (int w = 0; w < 5; ++w) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
  hipEventRecord(e0, s);
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
  hipEventRecord(e1, s);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  printf("%-34s %8.2f us\n", "empty kernel", ms * 1000 / reps);
  for (int si = 0; si < ub_nshapes; ++si) {
    const ub_shape& sh = ub_shapes[si];
    if (only >= 0 && int(si) != only) continue;
    const int lda = n, ldb = n, ldc = n;
    for (int w = 0; w < 3; ++w)
      smg_gemm_tri(ctx, sh.ta, sh.tb, sh.uplo, sh.tri, sh.m, sh.n, sh.k, -1e-3, A, lda, B, ldb, 1.0, C, ldc);
    const int rr = sh.k == 4096 ? 5 : reps;
    hipEventRecord(e0, s);
    for (int r = 0; r < rr; ++r)
      smg_gemm_tri(ctx, sh.ta, sh.tb, sh.uplo, sh.tri, sh.m, sh.n, sh.k, -1e-3, A, lda, B, ldb, 1.0, C, ldc);
    hipEventRecord(e1, s);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1000 / rr;
    const double fl = ub_flops(sh);
    printf("%-34s %8.2f us  %6.2f TF/s  \n", sh.name, us, fl / us * 1e-6);
  }
  smg_ctx_destroy(ctx);
}
