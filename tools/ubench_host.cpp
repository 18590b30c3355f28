// Dev microbenchmark: host enqueue time of the N = 4096 Cholesky forward
// (the GP step's factorisation, with and without the progressive K^{-1}
// row work on the side stream) against its device time, and the bare
// hipLaunchKernel cost on one stream / alternating two streams with events.
// Answers "is the panel loop host-bound": a host enqueue close to the device
// time means the next panel's launch is late.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "smg_hip.h"

__global__ void k_empty(int* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 1 << 30) p[0] = 1;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4096;
  smg_ctx* ctx = nullptr;
  if (smg_ctx_create(0, 1ull << 28, &ctx)) return 1;
  {  // bare launches
    hipStream_t s0, s1;
    hipStreamCreateWithFlags(&s0, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
    hipEvent_t ev;
    hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    for (int w = 0; w < 100; ++w) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s0, nullptr);
    hipStreamSynchronize(s0);
    double t0 = now_us();
    for (int w = 0; w < 1000; ++w) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s0, nullptr);
    double t1 = now_us();
    hipStreamSynchronize(s0);
    double t2 = now_us();
    printf("one stream: %.2f us per launch (host), %.2f us per launch (device drained)\n", (t1 - t0) / 1000,
           (t2 - t0) / 1000);
    t0 = now_us();
    for (int w = 0; w < 500; ++w) {
      hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, w & 1 ? s1 : s0, nullptr);
      hipEventRecord(ev, w & 1 ? s1 : s0);
      hipStreamWaitEvent(w & 1 ? s0 : s1, ev, 0);
    }
    t1 = now_us();
    hipStreamSynchronize(s0);
    hipStreamSynchronize(s1);
    t2 = now_us();
    printf("two streams + event hand-off: %.2f us per step (host), %.2f us (drained)\n", (t1 - t0) / 500,
           (t2 - t0) / 500);
  }
  std::vector<double> A((size_t)n * n);
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) A[i + (size_t)j * n] = (i == j ? n : 0.0) + 1.0 / (1.0 + i + j);
  double *dA, *dL, *aux, *ws;
  hipMalloc(&dA, 8ull * n * n);
  hipMalloc(&dL, 8ull * n * n);
  hipMalloc(&aux, 8ull * smg_cholesky_aux_doubles(n));
  hipMalloc(&ws, 8ull * smg_cholesky_mvn_rev_ws_doubles(n));
  hipMemcpy(dA, A.data(), 8ull * n * n, hipMemcpyHostToDevice);
  for (int prog = 0; prog < 2; ++prog) {
    double host = 0, total = 0;
    const int reps = 30;
    for (int r = -5; r < reps; ++r) {
      smg_sync(ctx);
      double t0 = now_us();
      int started = 0, st = 0;
      int rc = prog ? smg_cholesky_fwd_checked_mark_inv(ctx, dA, n, n, dL, n, aux, ws, &started)
                    : smg_cholesky_fwd_checked_mark(ctx, dA, n, n, dL, n, aux);
      double t1 = now_us();
      smg_status_mark_wait(ctx, &st);
      smg_join_async(ctx);
      smg_sync(ctx);
      double t2 = now_us();
      if (rc || st) {
        printf("rc %d status %d\n", rc, st);
        return 1;
      }
      if (r >= 0) {
        host += t1 - t0;
        total += t2 - t0;
      }
    }
    printf("cholesky fwd n=%d %s: host enqueue %.1f us, enqueue->done %.1f us\n", n,
           prog ? "+ K^-1 rows (mark_inv)" : "(mark)", host / reps, total / reps);
  }
  smg_ctx_destroy(ctx);
  return 0;
}
