// Dev microbenchmark (round 6): where the chain's 64 x 64 factor
// (lds_potrf64_lookahead<true>'s structure) spends its time: s_memtime stamps
// of wave 0 and wave 1 at every phase boundary of every 8-column panel.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../math_amd/csrc/tri_small.h"

__device__ __forceinline__ long long now() {
  long long t = __builtin_amdgcn_s_memtime();
  return t;
}
// MODE 0: as the library; 1: no (A) work; 2: no wave-0 factor (loads/stores only); 3: no (B) MFMA work
template <int MODE>
__global__ __launch_bounds__(512) void k_tr(const double* g, long long* tr, int* status) {
  __shared__ double D[SMG_NB * SMG_NBP];
  lds_load_block(D, g, 64, 64, true);
  __syncthreads();
  const int i = threadIdx.x & 63, gw = threadIdx.x >> 6;
  bool bad = false;
  int k = 0;
  auto mark = [&]() {
    if (i == 0 && gw < 2) tr[gw * 64 + k] = now();
    ++k;
  };
  mark();
  if (gw == 0) {
    if (MODE == 2) { double a[8]; for (int t = 0; t < 8; ++t) a[t] = D[i * SMG_NBP + t]; wave_store8(D, a, 0); }
    else wave_panel8_rl<true>(D, 0, bad);
  }
  mark();
  __syncthreads();
  mark();
  for (int p = 0; p < 7; ++p) {
    const int j0 = 8 * p, c1 = j0 + 8, c2 = j0 + 16;
    if (gw > 0 && MODE != 1) {
      const int e = threadIdx.x - 64;
      const int r = c1 + (e >> 3), c = c1 + (e & 7);
      if (r < 64 && r >= c) {
        double v = D[r * SMG_NBP + c];
#pragma unroll
        for (int t = 0; t < 8; ++t) v -= D[r * SMG_NBP + j0 + t] * D[c * SMG_NBP + j0 + t];
        D[r * SMG_NBP + c] = v;
      }
    }
    mark();
    __syncthreads();
    mark();
    if (gw == 0) {
      if (MODE == 2) { double a[8]; for (int t = 0; t < 8; ++t) a[t] = D[i * SMG_NBP + c1 + t]; wave_store8(D, a, c1); }
      else wave_panel8_rl<true>(D, c1, bad);
    } else if (c2 < 64 && MODE != 3) {
      const int t0 = c2 >> 4, nt = 4 - t0, ntiles = nt * (nt + 1) / 2;
      const int fr = i & 15, fk = i >> 4;
      for (int q = gw - 1; q < ntiles; q += 7) {
        int ti = 0, rem = q;
        while (rem > ti) { rem -= ti + 1; ++ti; }
        const int tj = rem + t0;
        ti += t0;
        d4 acc = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k0 = 0; k0 < 8; k0 += 4) {
          const double av = D[(16 * ti + fr) * SMG_NBP + j0 + k0 + fk];
          const double bv = D[(16 * tj + fr) * SMG_NBP + j0 + k0 + fk];
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
        }
        const int col = 16 * tj + fr;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * ti + fk + 4 * r;
          if (col >= c2 && row >= col) D[row * SMG_NBP + col] -= acc[r];
        }
      }
    }
    mark();
    __syncthreads();
    mark();
  }
  if (bad) atomicOr(status, 1);
}

int main() {
  double* dA;
  long long* dt;
  int* st;
  hipMalloc(&dA, 4096 * 8);
  hipMalloc(&dt, 128 * 8);
  hipMalloc(&st, 4);
  std::vector<double> h(4096);
  for (int j = 0; j < 64; ++j)
    for (int i = 0; i < 64; ++i) h[i + 64 * j] = (i == j ? 64.0 : 0.0) + 1.0 / (1 + i + j);
  hipMemcpy(dA, h.data(), 4096 * 8, hipMemcpyHostToDevice);
  void (*ks[4])(const double*, long long*, int*) = {k_tr<0>, k_tr<1>, k_tr<2>, k_tr<3>};
  const char* nm[4] = {"library structure", "no (A) work", "no wave-0 factor", "no (B) MFMA"};
  for (int m = 0; m < 4; ++m) {
    std::vector<long long> t(128);
    for (int rep = 0; rep < 3; ++rep) {
      hipLaunchKernelGGL(ks[m], dim3(1), dim3(512), 0, 0, dA, dt, st);
      hipDeviceSynchronize();
    }
    hipMemcpy(t.data(), dt, 128 * 8, hipMemcpyDeviceToHost);
    const int K = 3 + 7 * 4;
    std::printf("%s: total %lld cycles\n", nm[m], t[K - 1] - t[0]);
    // per-panel phases (wave 0): A (mark A), barrier1, B, barrier2
    std::printf("  w0 prologue factor %lld, barrier %lld\n", t[1] - t[0], t[2] - t[1]);
    for (int p = 0; p < 7; ++p) {
      const int b = 3 + 4 * p;
      std::printf("  p%d: w0 [A %lld, bar %lld, B %lld, bar %lld]  w1 [A %lld, bar %lld, B %lld, bar %lld]\n", p,
                  t[b] - t[b - 1], t[b + 1] - t[b], t[b + 2] - t[b + 1], t[b + 3] - t[b + 2], t[64 + b] - t[64 + b - 1],
                  t[64 + b + 1] - t[64 + b], t[64 + b + 2] - t[64 + b + 1], t[64 + b + 3] - t[64 + b + 2]);
    }
  }
  return 0;
}
