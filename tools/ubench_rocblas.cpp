// Reference point only (not used by the product): rocBLAS DGEMM throughput on
// the Cholesky update shapes, to size the headroom of the hand-written GEMM.
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <cstdio>
int main() {
  rocblas_handle h;
  rocblas_create_handle(&h);
  const int n = 4096;
  double *A, *B, *C;
  hipMalloc(&A, 8ull * n * n); hipMalloc(&B, 8ull * n * n); hipMalloc(&C, 8ull * n * n);
  hipMemset(A, 0, 8ull * n * n); hipMemset(B, 0, 8ull * n * n); hipMemset(C, 0, 8ull * n * n);
  struct S { const char* nm; rocblas_operation ta, tb; int m, nn, k; };
  S sh[] = {{"NN 4096^3", rocblas_operation_none, rocblas_operation_none, 4096, 4096, 4096},
            {"NN (1792,2048,256)", rocblas_operation_none, rocblas_operation_none, 1792, 2048, 256},
            {"NT (2048,2048,256)", rocblas_operation_none, rocblas_operation_transpose, 2048, 2048, 256},
            {"TN (256,2304,1792)", rocblas_operation_transpose, rocblas_operation_none, 256, 2304, 1792},
            {"NN (2048,2048,64)", rocblas_operation_none, rocblas_operation_none, 2048, 2048, 64}};
  const double al = -1.0, be = 1.0;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (auto& s : sh) {
    for (int w = 0; w < 3; ++w)
      rocblas_dgemm(h, s.ta, s.tb, s.m, s.nn, s.k, &al, A, n, B, n, &be, C, n);
    const int reps = s.k == 4096 ? 5 : 50;
    hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) rocblas_dgemm(h, s.ta, s.tb, s.m, s.nn, s.k, &al, A, n, B, n, &be, C, n);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1000 / reps;
    printf("%-22s %9.2f us %7.2f TF/s\n", s.nm, us, 2.0 * s.m * s.nn * s.k / us * 1e-6);
  }
}
