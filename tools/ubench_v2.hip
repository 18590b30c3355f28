// Dev microbenchmark: 64x64 diagonal-block potrf + inverse variants (timing
// and max difference between the fused per-column and the blocked variant).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
#include "../math_amd/csrc/tri_small.h"
template <int MODE>
__global__ __launch_bounds__(512) void k_v2(double* g, double* L, double* dinv, long long* cyc, int* st) {
  __shared__ double D[SMG_NB * SMG_NBP];
  __shared__ double X[SMG_NB * SMG_NBP];
  long long t0 = __builtin_amdgcn_s_memtime();
  lds_load_block(D, g, 64, 64, true);
  for (int e = threadIdx.x; e < SMG_NB * SMG_NBP; e += blockDim.x) X[e] = (e / SMG_NBP == e % SMG_NBP) ? 1.0 : 0.0;
  __syncthreads();
  long long t1 = __builtin_amdgcn_s_memtime();
  if (MODE == 0) lds_potrf_inv64_v2(D, X, 64, L, 64, dinv, 64, st, true);
  if (MODE == 1) lds_potrf_inv64_blk(D, X, 64, L, 64, dinv, 64, st, true);
  if (MODE == 2) { lds_potrf64_blocked(D, st); }
  if (MODE == 3) { lds_potrf64_blocked(D, st); __shared__ double T[512]; lds_trtri64_blocked(D, X, T); }
  if (MODE == 4) { lds_potrf64_lookahead(D, st); }
  if (MODE == 5) { lds_potrf64_lookahead(D, st); __shared__ double T2[768]; lds_trtri64_mfma(D, X, T2); }
  if (MODE == 5 || MODE == 1) {
    __syncthreads();
    for (int e = threadIdx.x; e < 4096; e += blockDim.x) {
      const int c = e / 64, r = e % 64;
      if (MODE == 5) { L[r + 64 * c] = r >= c ? D[r * SMG_NBP + c] : 0.0; dinv[r + 64 * c] = r >= c ? X[r * SMG_NBP + c] : 0.0; }
    }
  }
  __syncthreads();
  long long t2 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { cyc[0] = t1 - t0; cyc[1] = t2 - t1; }
}
int main() {
  double *d, *L, *dinv; long long* cyc; int* st;
  hipMalloc(&d, 1 << 20); hipMalloc(&L, 1 << 20); hipMalloc(&dinv, 1 << 20); hipMalloc(&cyc, 512); hipMalloc(&st, 64);
  std::vector<double> h(4096);
  for (int j = 0; j < 64; ++j) for (int i = 0; i < 64; ++i) h[i + 64 * j] = (i == j ? 64.0 : 0.0) + 1.0 / (1 + i + j);
  long long c[2];
  std::vector<double> Lr[2], Xr[2];
  auto run = [&](int slot, const char* name, void (*k)(double*, double*, double*, long long*, int*)) {
    for (int r = 0; r < 3; ++r) {
      hipMemcpy(d, h.data(), 4096 * 8, hipMemcpyHostToDevice);
      hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
      hipEventRecord(e0);
      hipLaunchKernelGGL(k, dim3(1), dim3(512), 0, 0, d, L, dinv, cyc, st);
      hipEventRecord(e1); hipEventSynchronize(e1); float ms; hipEventElapsedTime(&ms, e0, e1);
      hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
      printf("%-14s load %lld cyc, body %lld cyc, event %.1f us\n", name, c[0], c[1], ms * 1000);
    }
    if (slot >= 0) {
      Lr[slot].resize(4096); Xr[slot].resize(4096);
      hipMemcpy(Lr[slot].data(), L, 4096 * 8, hipMemcpyDeviceToHost);
      hipMemcpy(Xr[slot].data(), dinv, 4096 * 8, hipMemcpyDeviceToHost);
    }
  };
  run(0, "v2 fused", k_v2<0>); run(-1, "blk potrf", k_v2<2>); run(-1, "blk potrf+inv", k_v2<3>);
  run(-1, "la potrf", k_v2<4>); run(1, "la+mfma inv", k_v2<5>);
  double dl = 0, dx = 0;
  for (int e = 0; e < 4096; ++e) {
    dl = fmax(dl, fabs(Lr[0][e] - Lr[1][e]) / (fabs(Lr[0][e]) + 1e-300) * (Lr[0][e] != 0));
    dx = fmax(dx, fabs(Xr[0][e] - Xr[1][e]) / (fabs(Xr[0][e]) + 1e-300) * (Xr[0][e] != 0));
  }
  // L * X should be I
  double ei = 0;
  for (int i = 0; i < 64; ++i) for (int j = 0; j < 64; ++j) {
    double s = 0; for (int k = 0; k < 64; ++k) s += Lr[1][i + 64 * k] * Xr[1][k + 64 * j];
    ei = fmax(ei, fabs(s - (i == j)));
  }
  printf("max rel diff L %.3e X %.3e ; |L X - I| %.3e\n", dl, dx, ei);
}
