// Dev microbenchmark: the progressive K^{-1} share C += W_k^T W_k (lower,
// K = 512) as the TN product the factorisation issues against the NT product
// on a transposed copy of W_k (+ the transpose), alone on the device, and the
// right-looking Y part's NN shape.  Prints us per call and TF/s.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../include/smg_hip.h"

int main() {
  smg_ctx* ctx = nullptr;
  if (smg_ctx_create(0, 1ull << 30, &ctx)) return 1;
  hipStream_t s = (hipStream_t)smg_ctx_stream(ctx);
  const int n = 4096, P = 512;
  double *W, *V, *C;
  hipMalloc(&W, sizeof(double) * n * n);
  hipMalloc(&V, sizeof(double) * n * n);
  hipMalloc(&C, sizeof(double) * n * n);
  smg_fill_unif(ctx, W, (long long)n * n, 1, -1.0, 1.0, 1.0);
  smg_fill_unif(ctx, C, (long long)n * n, 3, -1.0, 1.0, 1.0);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto time = [&](const char* what, double flops, auto&& f) {
    for (int w = 0; w < 3; ++w) f();
    const int reps = 10;
    hipEventRecord(e0, s);
    for (int r = 0; r < reps; ++r) f();
    hipEventRecord(e1, s);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1000 / reps;
    printf("%-44s %8.1f us  %6.1f TF/s\n", what, us, flops / us * 1e-6);
  };
  for (int r1 : {1024, 2048, 3072, 4096}) {
    const double fl = (double)r1 * (r1 + 1) * P;  // lower triangle, 2 flop per MAC
    char b[96];
    // W_k: rows r0 .. r1 of W (P x r1, ld n); the TN share
    const double* Wk = W + (r1 - P);
    snprintf(b, sizeof b, "share TN   r1=%d", r1);
    time(b, fl, [&] { smg_gemm(ctx, 1, 0, 1, r1, r1, P, 1.0, Wk, n, Wk, n, 1.0, C, n); });
    snprintf(b, sizeof b, "transpose + share NT r1=%d", r1);
    time(b, fl, [&] {
      smg_transpose(ctx, P, r1, Wk, n, V, r1, 0.0);
      smg_gemm(ctx, 0, 1, 1, r1, r1, P, 1.0, V, r1, V, r1, 1.0, C, n);
    });
    snprintf(b, sizeof b, "share NT only r1=%d", r1);
    time(b, fl, [&] { smg_gemm(ctx, 0, 1, 1, r1, r1, P, 1.0, V, r1, V, r1, 1.0, C, n); });
    if (r1 + P < n) {  // Y part 4: Y[r1+P:, 0:r1] += L[r1+P:, k] W_k
      const int m = n - r1 - P;
      snprintf(b, sizeof b, "Y part 4 NN m=%d n=%d", m, r1);
      time(b, 2.0 * m * r1 * P, [&] { smg_gemm(ctx, 0, 0, 0, m, r1, P, 1.0, W, n, Wk, n, 1.0, C, n); });
    }
  }
  smg_ctx_destroy(ctx);
  return 0;
}
