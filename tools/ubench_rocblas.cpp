// Reference point only (not used by the product): rocBLAS DGEMM / DSYRK
// throughput on the GP N = 4096 shapes (tools/ubench_shapes.h), to size the
// headroom of the hand-written GEMM.  Lower-trapezoid shapes run as full
// DGEMMs (timed; TF/s counted on the trapezoid's flops like the product's).
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <cstdio>
#include <vector>
#include "ubench_shapes.h"
int main() {
  rocblas_handle h;
  rocblas_create_handle(&h);
  const int n = 4096;
  double *A, *B, *C;
  hipMalloc(&A, 8ull * n * n); hipMalloc(&B, 8ull * n * n); hipMalloc(&C, 8ull * n * n);
  std::vector<double> hv((size_t)n * n);
  for (size_t i = 0; i < hv.size(); ++i) hv[i] = ((i * 2654435761u) % 2000) * 1e-3 - 1.0;
  hipMemcpy(A, hv.data(), 8ull * n * n, hipMemcpyHostToDevice);
  hipMemcpy(B, hv.data(), 8ull * n * n, hipMemcpyHostToDevice);
  hipMemcpy(C, hv.data(), 8ull * n * n, hipMemcpyHostToDevice);
  const double al = -1e-3, be = 1.0;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  auto op = [](int t) { return t ? rocblas_operation_transpose : rocblas_operation_none; };
  for (int si = 0; si < ub_nshapes; ++si) {
    const ub_shape& s = ub_shapes[si];
    const bool syrk = s.uplo && s.m == s.n;
    auto run = [&] {
      if (syrk)
        rocblas_dsyrk(h, rocblas_fill_lower, rocblas_operation_none, s.m, s.k, &al, A, n, &be, C, n);
      else
        rocblas_dgemm(h, op(s.ta), op(s.tb), s.m, s.n, s.k, &al, A, n, B, n, &be, C, n);
    };
    for (int w = 0; w < 3; ++w) run();
    const int reps = s.k == 4096 ? 5 : 50;
    hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) run();
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1000 / reps;
    printf("%-34s %8.2f us  %6.2f TF/s  %s\n", s.name, us, ub_flops(s) / us * 1e-6, syrk ? "dsyrk" : "dgemm");
  }
}
