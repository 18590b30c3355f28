// PMC calibration (guide: "other access widths are uncalibrated: calibrate on
// a known byte count"): 8-byte-per-lane coalesced streaming read and write of
// a buffer far larger than the 256 MiB Infinity Cache.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_read8(const double* __restrict__ x, long long n, double* out) {
  double s = 0.0;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    s += x[i];
  if (s == 1234.5) out[0] = s;
}
__global__ void k_write8(double* __restrict__ x, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    x[i] = (double)i;
}

int main() {
  const long long n = 1ll << 27;  // 1 GiB of doubles
  double *x, *o;
  hipMalloc(&x, n * 8);
  hipMalloc(&o, 64);
  hipLaunchKernelGGL(k_write8, dim3(4096), dim3(256), 0, 0, x, n);
  hipLaunchKernelGGL(k_read8, dim3(4096), dim3(256), 0, 0, x, n, o);
  hipDeviceSynchronize();
  printf("bytes %lld\n", n * 8);
}
