// Dev microbenchmark: phase times (s_memtime) of lds_potrf64_lookahead's pieces.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cmath>
#include <algorithm>
#include "../math_amd/csrc/tri_small.h"

__device__ __forceinline__ long long stamp() {
  __builtin_amdgcn_s_waitcnt(0);
  asm volatile("" ::: "memory");
  long long t = __builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  return t;
}

typedef __attribute__((address_space(3))) double lds_dbl;
// the panel kernel's form: out of line, address_space(3) pointers
__device__ __noinline__ void cf_pair(lds_dbl* D, int* st) { lds_potrf64_lookahead<true>(D, st); }
__device__ __noinline__ void cf_old(lds_dbl* D, int* st) { lds_potrf64_lookahead<false>(D, st); }

template <int WHICH>
__global__ __launch_bounds__(512) void k_phase(double* g, long long* cyc) {
  __shared__ double D[SMG_NB * SMG_NBP];
  lds_load_block(D, g, 64, 64, true);
  __syncthreads();
  bool bad = false;
  long long t0 = stamp();
  if (threadIdx.x < 64) {
    if (WHICH == 0) wave_panel8_local(D, 0, bad);
    if (WHICH == 1 || WHICH == 6) {
      double a[8];
      for (int t = 0; t < 8; ++t) a[t] = D[(threadIdx.x & 63) * SMG_NBP + t];
      if (WHICH == 1)
        wave_factor8_reg(a, 0, bad);
      else
        wave_factor8_pair(a, 0, bad);
      wave_store8(D, a, 0);
    }
  }
  long long t1 = stamp();
  __syncthreads();
  long long t2 = stamp();
  const long long r2 = __builtin_amdgcn_s_memrealtime();
  if (WHICH == 8) cf_pair((lds_dbl*)D, (int*)(cyc + 60));
  if (WHICH == 9) cf_old((lds_dbl*)D, (int*)(cyc + 60));
  if (WHICH == 2) lds_potrf64_lookahead(D, (int*)(cyc + 60));
  if (WHICH == 3) lds_potrf64_lookahead(D, (int*)(cyc + 60));
  if (WHICH == 7) lds_potrf64_lookahead<true>(D, (int*)(cyc + 60));
  if (WHICH == 4 || WHICH == 5) {
    __shared__ double X[SMG_NB * SMG_NBP];
    __shared__ double T[768];
    if (WHICH == 4) {
      lds_potrf64_lookahead(D, (int*)(cyc + 60));
      __syncthreads();
      lds_trtri64_mfma(D, X, T);
    } else {
      lds_potrf64_lookahead(D, (int*)(cyc + 60));
      __syncthreads();
      lds_trtri64_mfma(D, X, T);
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 64 * 64; e += blockDim.x) g[8192 + e] = X[(e >> 6) * SMG_NBP + (e & 63)];
  }
  long long t3 = stamp();
  const long long r3 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { cyc[0] = t1 - t0; cyc[1] = t2 - t1; cyc[2] = t3 - t2; cyc[3] = r3 - r2; }
  __syncthreads();
  for (int e = threadIdx.x; e < 64 * 64; e += blockDim.x) g[4096 + e] = D[(e >> 6) * SMG_NBP + (e & 63)];
  if (bad) g[0] = 0;
}

int main() {
  double* d;
  long long* cyc;
  hipMalloc(&d, 1 << 20);
  hipMalloc(&cyc, 4096);
  std::vector<double> h(4096);
  for (int j = 0; j < 64; ++j) for (int i = 0; i < 64; ++i) h[i + 64 * j] = (i == j ? 64.0 : 0.0) + 1.0 / (1 + i + j);
  long long c[4] = {0, 0, 0, 0};
  std::vector<double> o2(4096), o3(4096);
  auto run = [&](const char* nm, void (*k)(double*, long long*), std::vector<double>* out = nullptr) {
    for (int r = 0; r < 2; ++r) {
      hipMemcpy(d, h.data(), 4096 * 8, hipMemcpyHostToDevice);
      hipLaunchKernelGGL(k, dim3(1), dim3(512), 0, 0, d, cyc);
      hipDeviceSynchronize();
      hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    }
    printf("%-22s w0 %lld  barrier %lld  full %lld  (%.2f us real)\n", nm, c[0], c[1], c[2], c[3] / 100.0);
    if (out) hipMemcpy(out->data(), d + 4096, 4096 * 8, hipMemcpyDeviceToHost);
  };
  run("panel8 per-lane", k_phase<0>);
  run("panel8 readlane", k_phase<1>);
  run("panel8 pairs", k_phase<6>);
  std::vector<double> o7(4096);
  for (int rep = 0; rep < 3; ++rep) run("lookahead potrf pairs", k_phase<7>, &o7);
  for (int rep = 0; rep < 2; ++rep) {
    run("out-of-line pairs", k_phase<8>);
    run("out-of-line per-pivot", k_phase<9>);
  }
  for (int rep = 0; rep < 3; ++rep) {
    run("lookahead potrf", k_phase<2>, &o2);
    run("pre-broadcast potrf", k_phase<3>, &o3);
  }
  std::vector<double> x4(4096), x5(4096), l4(4096), l5(4096);
  for (int rep = 0; rep < 3; ++rep) {
    run("potrf + trtri", k_phase<4>, &l4);
    hipMemcpy(x4.data(), d + 8192, 4096 * 8, hipMemcpyDeviceToHost);
    run("fused potrf_trtri", k_phase<5>, &l5);
    hipMemcpy(x5.data(), d + 8192, 4096 * 8, hipMemcpyDeviceToHost);
  }
  {
    int dl = 0, dx = 0;
    double ex = 0;
    for (int e = 0; e < 4096; ++e) {
      if ((e >> 6) >= (e & 63) && l4[e] != l5[e]) ++dl;
      if (x4[e] != x5[e]) ++dx;
      // X L = I check on the fused result
    }
    for (int r = 0; r < 64; ++r)
      for (int c = 0; c < 64; ++c) {
        double v = 0;
        for (int k = 0; k < 64; ++k) v += x5[r * 64 + k] * (k >= c ? l5[k * 64 + c] : 0.0);
        ex = std::max(ex, std::abs(v - (r == c ? 1.0 : 0.0)));
      }
    printf("fused vs separate: L entries differing %d, X entries differing %d, |XL - I| %.2e\n", dl, dx, ex);
  }
  int diff = 0;
  for (int e = 0; e < 4096; ++e)
    if ((e >> 6) >= (e & 63) && o2[e] != o3[e]) ++diff;
  printf("lower-triangle entries differing: %d\n", diff);
  {  // pairs vs per-pivot factor: max |diff| and |L L^T - A|
    double md = 0, res = 0;
    for (int r = 0; r < 64; ++r)
      for (int c = 0; c <= r; ++c) {
        md = std::max(md, std::abs(o7[r * 64 + c] - o2[r * 64 + c]));
        double v = 0;
        for (int k = 0; k <= c; ++k) v += o7[r * 64 + k] * o7[c * 64 + k];
        res = std::max(res, std::abs(v - h[r + 64 * c]));
      }
    printf("pairs vs per-pivot: max |dL| %.2e, |L L^T - A| %.2e\n", md, res);
  }
}
