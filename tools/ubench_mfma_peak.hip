// Dev microbenchmark: whole-chip fp64 MFMA throughput (v_mfma_f64_16x16x4f64)
// vs waves per SIMD, timed with hipEvents (no s_memtime clock assumptions).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
template <int NACC>
__global__ void k_mfma(double* out, int iters) {
  d4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = d4{0, 0, 0, 0};
  double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 12345.0) out[0] = s;
}
template <int NACC>
void run(int wpc) {  // waves per CU
  double* out;
  (void)hipMalloc(&out, 8);
  const int iters = 8192 / NACC;
  const int wgs = 256 * (wpc / 4 > 0 ? wpc / 4 : 1);
  const int threads = wpc < 4 ? 64 * wpc : 256;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(k_mfma<NACC>, dim3(wgs), dim3(threads), 0, 0, out, iters);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k_mfma<NACC>, dim3(wgs), dim3(threads), 0, 0, out, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double fl = 2048.0 * iters * NACC * (threads / 64) * wgs;
  printf("nacc=%d waves/CU=%2d: %8.1f us  %6.1f TF/s\n", NACC, wgs * threads / 64 / 256, ms * 1e3,
         fl / (ms * 1e-3) * 1e-12);
  (void)hipFree(out);
}
int main() {
  for (int w : {4, 8, 16, 32}) { run<1>(w); run<4>(w); run<8>(w); }
  return 0;
}
