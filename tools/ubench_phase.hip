// Dev microbenchmark: phase times (s_memtime) of lds_potrf64_lookahead's pieces.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../math_amd/csrc/tri_small.h"

__device__ __forceinline__ long long stamp() {
  __builtin_amdgcn_s_waitcnt(0);
  asm volatile("" ::: "memory");
  long long t = __builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  return t;
}

template <int WHICH>
__global__ __launch_bounds__(512) void k_phase(double* g, long long* cyc) {
  __shared__ double D[SMG_NB * SMG_NBP];
  lds_load_block(D, g, 64, 64, true);
  __syncthreads();
  bool bad = false;
  long long t0 = stamp();
  if (threadIdx.x < 64) {
    if (WHICH == 0) wave_panel8_local(D, 0, bad);
    if (WHICH == 1) {
      double a[8];
      for (int t = 0; t < 8; ++t) a[t] = D[(threadIdx.x & 63) * SMG_NBP + t];
      wave_factor8_reg(a, 0, bad);
      wave_store8(D, a, 0);
    }
  }
  long long t1 = stamp();
  __syncthreads();
  long long t2 = stamp();
  if (WHICH == 2) lds_potrf64_lookahead(D, (int*)(cyc + 60));
  long long t3 = stamp();
  if (threadIdx.x == 0) { cyc[0] = t1 - t0; cyc[1] = t2 - t1; cyc[2] = t3 - t2; }
  if (bad) g[0] = 0;
}

int main() {
  double* d;
  long long* cyc;
  hipMalloc(&d, 1 << 20);
  hipMalloc(&cyc, 4096);
  std::vector<double> h(4096);
  for (int j = 0; j < 64; ++j) for (int i = 0; i < 64; ++i) h[i + 64 * j] = (i == j ? 64.0 : 0.0) + 1.0 / (1 + i + j);
  long long c[4];
  auto run = [&](const char* nm, void (*k)(double*, long long*)) {
    for (int r = 0; r < 2; ++r) {
      hipMemcpy(d, h.data(), 4096 * 8, hipMemcpyHostToDevice);
      hipLaunchKernelGGL(k, dim3(1), dim3(512), 0, 0, d, cyc);
      hipDeviceSynchronize();
      hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    }
    printf("%-22s w0 %lld  barrier %lld  full %lld\n", nm, c[0], c[1], c[2]);
  };
  run("panel8 per-lane", k_phase<0>);
  run("panel8 readlane", k_phase<1>);
  run("lookahead potrf", k_phase<2>);
}
