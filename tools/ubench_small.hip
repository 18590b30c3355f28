// Microbenchmarks for the latency-bound single-workgroup kernels (dev tool).
//   (a) v_mfma_f64_16x16x4_f64 issue rate (one wave, 4 independent accumulators)
//   (b) lds_mma64 (64^3 product from LDS, 4 waves)
//   (c) lds_potrf_inv64 (current 64x64 factor + inverse)
//   (d) register-resident single-wave 64x64 Cholesky (unrolled right-looking)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "../math_amd/csrc/tri_small.h"

__global__ void k_mfma_rate(double* out, long long* cyc, int iters) {
  double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
  d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
  }
  long long t1 = clock64();
  out[threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void k_fma_rate(double* out, long long* cyc, int iters) {
  double a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, m = 1.0000001, s = 1e-9;
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
    a0 = fma(a0, m, s); a1 = fma(a1, m, s); a2 = fma(a2, m, s); a3 = fma(a3, m, s);
    a0 = fma(a0, m, s); a1 = fma(a1, m, s); a2 = fma(a2, m, s); a3 = fma(a3, m, s);
  }
  long long t1 = clock64();
  out[threadIdx.x] = a0 + a1 + a2 + a3;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ __launch_bounds__(256) void k_mma64(double* g, long long* cyc) {
  __shared__ double A[SMG_NB * SMG_NBP], B[SMG_NB * SMG_NBP], C[SMG_NB * SMG_NBP];
  for (int e = threadIdx.x; e < SMG_NB * SMG_NBP; e += 256) { A[e] = g[e % 4096]; B[e] = 1.0 / (e + 1); C[e] = 0; }
  __syncthreads();
  long long t0 = clock64();
  for (int r = 0; r < 10; ++r) lds_mma64<true, false>(C, A, B, 1.0, 1.0);
  long long t1 = clock64();
  if (threadIdx.x == 0) cyc[0] = (t1 - t0) / 10;
  g[threadIdx.x] = C[threadIdx.x];
}

__global__ __launch_bounds__(256) void k_potrf64(double* g, long long* cyc, int* status) {
  __shared__ double D[SMG_NB * SMG_NBP], X[SMG_NB * SMG_NBP], T[768];
  lds_load_block(D, g, 64, 64, true);
  __syncthreads();
  long long t0 = clock64();
  lds_potrf_inv64(D, X, T, status);
  long long t1 = clock64();
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
  lds_store_block(X, g, 64, 64, true);
}

// one wave, row i in registers, fully unrolled right-looking
__global__ __launch_bounds__(64) void k_potrf_reg(double* g, long long* cyc) {
  const int l = threadIdx.x;
  double a[64];
#pragma unroll
  for (int c = 0; c < 64; ++c) a[c] = g[l + 64 * c];
  long long t0 = clock64();
#pragma unroll
  for (int j = 0; j < 64; ++j) {
    const double piv = bcast(a[j], j);
    double r = __builtin_amdgcn_rsq(piv);
    r = r * (1.5 - 0.5 * piv * r * r);
    const double lij = (l == j) ? piv * r : a[j] * r;
    a[j] = lij;
#pragma unroll
    for (int c = j + 1; c < 64; ++c) a[c] -= lij * bcast(lij, c);
  }
  long long t1 = clock64();
  if (l == 0) cyc[0] = t1 - t0;
#pragma unroll
  for (int c = 0; c < 64; ++c) g[l + 64 * c] = a[c];
}

int main() {
  double* d;
  long long* cyc;
  int* st;
  hipMalloc(&d, 1 << 22);
  hipMalloc(&cyc, 4096 * sizeof(long long));
  hipMalloc(&st, 64);
  std::vector<double> h(4096);
  for (int j = 0; j < 64; ++j)
    for (int i = 0; i < 64; ++i) h[i + 64 * j] = (i == j ? 64.0 : 0.0) + 1.0 / (1 + i + j);
  long long c[4];
  auto run = [&](const char* name, auto launch) {
    hipMemcpy(d, h.data(), 4096 * 8, hipMemcpyHostToDevice);
    launch();
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipMemcpy(d, h.data(), 4096 * 8, hipMemcpyHostToDevice);
    hipEventRecord(e0);
    for (int r = 0; r < 20; ++r) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    printf("%-14s cycles(in-kernel)=%lld  wall/launch=%.2f us\n", name, c[0], ms * 1000 / 20);
  };
  run("mfma_f64x1000", [&] { hipLaunchKernelGGL(k_mfma_rate, dim3(1), dim3(64), 0, 0, d, cyc, 250); });
  run("fma_f64x8000", [&] { hipLaunchKernelGGL(k_fma_rate, dim3(1), dim3(64), 0, 0, d, cyc, 1000); });
  run("lds_mma64", [&] { hipLaunchKernelGGL(k_mma64, dim3(1), dim3(256), 0, 0, d, cyc); });
  run("potrf_inv64", [&] { hipLaunchKernelGGL(k_potrf64, dim3(1), dim3(256), 0, 0, d, cyc, st); });
  run("potrf_reg", [&] { hipLaunchKernelGGL(k_potrf_reg, dim3(1), dim3(64), 0, 0, d, cyc); });
  run("empty-ish", [&] { hipLaunchKernelGGL(k_mfma_rate, dim3(1), dim3(64), 0, 0, d, cyc, 1); });
  // clock: 1000 MFMAs vs wall
  return 0;
}
