// Dev microbenchmark: v_mfma_f64_16x16x4f64 cycles per instruction on one SIMD
// versus the number of independent accumulators (dependent-chain latency) and
// waves per SIMD.  Prints cycles/MFMA per wave as measured by s_memtime.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void k_chain(double* out, long long* cyc, int iters) {
  d4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = d4{0, 0, 0, 0};
  double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NACC>
void run(int waves_per_wg, int wgs) {
  double* out; long long* cyc;
  hipMalloc(&out, sizeof(double) * wgs * 64 * waves_per_wg);
  hipMalloc(&cyc, sizeof(long long) * wgs);
  const int iters = 4096 / NACC;
  hipLaunchKernelGGL(k_chain<NACC>, dim3(wgs), dim3(64 * waves_per_wg), 0, 0, out, cyc, iters);
  hipLaunchKernelGGL(k_chain<NACC>, dim3(wgs), dim3(64 * waves_per_wg), 0, 0, out, cyc, iters);
  hipDeviceSynchronize();
  long long h;
  hipMemcpy(&h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  // s_memtime ticks at the shader clock per the microarch guide
  printf("nacc=%d waves/WG=%d WGs=%d: %.1f cyc per MFMA per wave\n", NACC, waves_per_wg, wgs,
         double(h) / (iters * NACC));
  hipFree(out); hipFree(cyc);
}

int main() {
  for (int w : {1, 4, 8}) {
    run<1>(w, 1); run<2>(w, 1); run<4>(w, 1); run<8>(w, 1);
  }
  return 0;
}
