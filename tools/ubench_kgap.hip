// Dev microbenchmark (round 6): the device-side gap between two kernels on
// one stream (s_memrealtime, 100 MHz) after the first wrote B bytes with
// ordinary / nontemporal / device-scope (sc1) stores.
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ unsigned long long g_t[4];
template <int MODE>
__global__ void k_write(double* p, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    if (MODE == 0) p[i] = 1.0;
    if (MODE == 1) __builtin_nontemporal_store(1.0, p + i);
    if (MODE == 2) __hip_atomic_store(p + i, 1.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(&g_t[0], __builtin_amdgcn_s_memrealtime());
}
__global__ void k_probe() {
  if (threadIdx.x == 0) g_t[1] = __builtin_amdgcn_s_memrealtime();
}
int main() {
  double* p;
  const long long maxb = 256ll << 20;
  hipMalloc(&p, maxb);
  hipStream_t s;
  hipStreamCreate(&s);
  const char* nm[3] = {"ordinary", "nontemporal", "sc1"};
  for (int mode = 0; mode < 3; ++mode)
    for (long long mb : {0ll, 1ll, 4ll, 16ll, 64ll, 256ll}) {
      double best = 1e30, sum = 0;
      for (int r = 0; r < 6; ++r) {
        unsigned long long z[4] = {0, 0, 0, 0};
        hipMemcpyToSymbol(HIP_SYMBOL(g_t), z, sizeof(z));
        const long long n = (mb << 20) / 8;
        if (mode == 0) hipLaunchKernelGGL(k_write<0>, dim3(1024), dim3(256), 0, s, p, n);
        if (mode == 1) hipLaunchKernelGGL(k_write<1>, dim3(1024), dim3(256), 0, s, p, n);
        if (mode == 2) hipLaunchKernelGGL(k_write<2>, dim3(1024), dim3(256), 0, s, p, n);
        hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, s);
        hipStreamSynchronize(s);
        unsigned long long t[4];
        hipMemcpyFromSymbol(t, HIP_SYMBOL(g_t), sizeof(t));
        const double gap = (double)(t[1] - t[0]) / 100.0;
        if (r > 0) { best = gap < best ? gap : best; sum += gap; }
      }
      printf("%-12s %4lld MB written: gap to the next kernel %.2f us (best) %.2f (mean)\n", nm[mode], mb, best, sum / 5);
    }
}
