// Dev microbenchmark: smg_gemm on the shapes of one blocked-Cholesky step
// (n = 4096, b = 64, block column j = 2048) plus an empty-kernel floor.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../include/smg_hip.h"

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
  hipMemset(A, 0, sizeof(double) * n * n);
  hipMemset(B, 0, sizeof(double) * n * n);
  hipMemset(C, 0, sizeof(double) * n * n);
  struct S { const char* name; int ta, tb, uplo, m, nn, k; };
  std::vector<S> shapes = {
      {"fwd L21 NT (2048,64,64)", 0, 1, 0, 2048, 64, 64},
      {"fwd SYRK (2048,2048,64)", 0, 1, 1, 2048, 2048, 64},
      {"rev Cadj*Dinv NN (2048,64,64)", 0, 0, 0, 2048, 64, 64},
      {"rev Badj NN (2048,2048,64)", 0, 0, 0, 2048, 2048, 64},
      {"rev Dadj TN (64,64,2048)", 1, 0, 0, 64, 64, 2048},
      {"rev Radj TN (64,2048,2048)", 1, 0, 0, 64, 2048, 2048},
      {"rev fused TN (64,2112,2048)", 1, 0, 0, 64, 2112, 2048},
      {"rev Radj sym NN (64,2048,64)", 0, 0, 0, 64, 2048, 64},
      {"big NN (4096,4096,4096)", 0, 0, 0, 4096, 4096, 4096},
      {"SYRK256 (2048,2048,256)", 0, 1, 1, 2048, 2048, 256},
      {"SYRK256 (1024,1024,256)", 0, 1, 1, 1024, 1024, 256},
      {"SYRK256 (3584,3584,256)", 0, 1, 1, 3584, 3584, 256},
      {"rev B NN (1792,2048,256)", 0, 0, 0, 1792, 2048, 256},
      {"rev TN (256,2304,1792)", 1, 0, 0, 256, 2304, 1792},
      {"sym256 TN (256,256,256)", 1, 0, 0, 256, 256, 256},
      {"rev TN (256,256,3840)", 1, 0, 0, 256, 256, 3840},
      {"rev TN (256,3840,256)", 1, 0, 0, 256, 3840, 256},
      {"rev TN (256,2048,2048)", 1, 0, 0, 256, 2048, 2048},
      {"rev NN Cadj W (3584,256,256)", 0, 0, 0, 3584, 256, 256},
      {"rev NN B (3584,256,256)", 0, 0, 0, 3584, 256, 256},
      {"rev NN PR (256,3584,256)", 0, 0, 0, 256, 3584, 256},
  };
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
  for (size_t si = 0; si < shapes.size(); ++si) {
    auto& sh = shapes[si];
    if (only >= 0 && int(si) != only) continue;
    const int lda = n, ldb = n, ldc = n;
    for (int w = 0; w < 3; ++w)
      smg_gemm(ctx, sh.ta, sh.tb, sh.uplo, sh.m, sh.nn, sh.k, -1.0, A, lda, B, ldb, 1.0, C, ldc);
    const int rr = sh.k == 4096 ? 5 : reps;
    hipEventRecord(e0, s);
    for (int r = 0; r < rr; ++r)
      smg_gemm(ctx, sh.ta, sh.tb, sh.uplo, sh.m, sh.nn, sh.k, -1.0, A, lda, B, ldb, 1.0, C, ldc);
    hipEventRecord(e1, s);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1000 / rr;
    const double fl = sh.uplo ? (double)sh.k * sh.m * (sh.m + 1) : 2.0 * sh.m * sh.nn * sh.k;
    printf("%-34s %8.2f us  %6.2f TF/s  \n", sh.name, us, fl / us * 1e-6);
  }
  smg_ctx_destroy(ctx);
}
