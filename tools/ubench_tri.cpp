// Dev microbenchmark: N x N x N products with triangular operands (the HVP
// Cholesky-tangent node's shapes) against the full product, through
// smg_gemm_tri; operands with stored zeros outside their triangles.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include "../include/smg_hip.h"

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4096;
  smg_ctx* ctx = nullptr;
  smg_ctx_create(0, 1ull << 30, &ctx);
  hipStream_t s = (hipStream_t)smg_ctx_stream(ctx);
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
  struct sh { const char* name; int ta, tb, uplo, tri; double frac; };
  const sh shapes[] = {
      {"NN full", 0, 0, 0, 0, 1.0},
      {"NN tri A lower", 0, 0, 0, 1, 0.5},
      {"NN tri A upper", 0, 0, 0, 2, 0.5},
      {"NN tri B lower", 0, 0, 0, 4, 0.5},
      {"TN tri A upper (op)", 1, 0, 0, 2, 0.5},
      {"NT mode3 tri B upper", 0, 1, 3, 8, 1.0 / 6},
      {"NN lower out", 0, 0, 1, 0, 0.5},
      {"NN mode3 tri B lower", 0, 0, 3, 4, 1.0 / 3},
      {"NN lower tri A,B lower", 0, 0, 1, 5, 1.0 / 6},
  };
  for (const sh& q : shapes) {
    for (int w = 0; w < 2; ++w)
      smg_gemm_tri(ctx, q.ta, q.tb, q.uplo, q.tri, n, n, n, 1.0, A, n, B, n, 0.0, C, n);
    const int rr = 5;
    hipEventRecord(e0, s);
    for (int r = 0; r < rr; ++r) smg_gemm_tri(ctx, q.ta, q.tb, q.uplo, q.tri, n, n, n, 1.0, A, n, B, n, 0.0, C, n);
    hipEventRecord(e1, s);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1000 / rr;
    const double fl = 2.0 * n * (double)n * n * q.frac;
    printf("%-26s %9.1f us  %6.2f TF/s (useful)\n", q.name, us, fl / us * 1e-6);
  }
  smg_ctx_destroy(ctx);
}
