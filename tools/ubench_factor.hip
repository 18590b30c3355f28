// Dev microbenchmark (round 6): the chain's 64 x 64 factor variants
// (lds_potrf64_v3<PANEL, AMFMA>, tri_small.h) against the library's
// lds_potrf64_lookahead<true>: cycles (s_memtime, 2.4 GHz) and accuracy
// against a long-double Cholesky, on a well-conditioned block and on a GP
// kernel block (close points, small jitter).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cmath>
#include <algorithm>
#include "../math_amd/csrc/tri_small.h"

typedef __attribute__((address_space(3))) double lds_dbl;
__device__ __forceinline__ long long stamp() {
  __builtin_amdgcn_s_waitcnt(0);
  asm volatile("" ::: "memory");
  long long t = __builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  return t;
}
template <int V> __device__ __noinline__ void fac(lds_dbl* D, int* st) {
  if (V == 0) lds_potrf64_lookahead<true>(D, st);
  if (V == 1) lds_potrf64_v3<1, false>(D, st);
  if (V == 2) lds_potrf64_v3<2, false>(D, st);
  if (V == 3) lds_potrf64_v3<0, true>(D, st);
  if (V == 4) lds_potrf64_v3<1, true>(D, st);
  if (V == 5) lds_potrf64_v3<2, true>(D, st);
  if (V == 6) lds_potrf64_v3<3, false>(D, st);
}
template <int V>
__global__ __launch_bounds__(512) void k_fac(const double* g, double* out, long long* cyc, int* st) {
  __shared__ double D[SMG_NB * SMG_NBP];
  lds_load_block(D, g, 64, 64, true);
  __syncthreads();
  const long long t0 = stamp();
  fac<V>((lds_dbl*)D, st);
  __syncthreads();
  const long long t1 = stamp();
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
  for (int e = threadIdx.x; e < 64 * 64; e += blockDim.x) out[e] = D[(e >> 6) * SMG_NBP + (e & 63)];
}

template <int V>
__global__ __launch_bounds__(512) void k_leaf(const double* g, double* out, long long* cyc) {
  __shared__ double D[SMG_NB * SMG_NBP];
  __shared__ double X[SMG_NB * SMG_NBP];
  lds_load_block(D, g, 64, 64, true);
  for (int e = threadIdx.x; e < SMG_NB * SMG_NBP; e += blockDim.x) X[e] = 0.0;
  __syncthreads();
  lds_potrf64_lookahead<true>((lds_dbl*)D, (int*)(cyc + 8));
  __syncthreads();
  const long long t0 = stamp();
  const int w = threadIdx.x >> 6;
  if (V == 0 && w < 4) trtri_leaf16((const lds_dbl*)D, (lds_dbl*)X, w);
  if (V >= 1 && w == 0) trtri_leaf16((const lds_dbl*)D, (lds_dbl*)X, 3);
  __syncthreads();
  const long long t1 = stamp();
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
  for (int e = threadIdx.x; e < 64 * 64; e += blockDim.x) out[e] = X[(e >> 6) * SMG_NBP + (e & 63)];
}

int main() {
  const char* names[7] = {"lookahead pairs (lib)", "pairs + rsq_h", "uniform + rsq_h", "pairs + MFMA (A)",
                          "pairs rsq_h + MFMA (A)", "uniform + MFMA (A)", "pair2 (own entries bcast)"};
  void (*ks[7])(const double*, double*, long long*, int*) = {k_fac<0>, k_fac<1>, k_fac<2>, k_fac<3>, k_fac<4>, k_fac<5>, k_fac<6>};
  double *dA, *dO;
  long long* dc;
  int* dst;
  hipMalloc(&dA, 4096 * 8);
  hipMalloc(&dO, 4096 * 8);
  hipMalloc(&dc, 64);
  hipMalloc(&dst, 4);
  for (int mat = 0; mat < 2; ++mat) {
    std::vector<double> h(4096);
    std::vector<double> xs(64);
    for (int i = 0; i < 64; ++i) xs[i] = 10.0 * i / 64 + 0.01 * std::sin(7.0 * i);
    for (int j = 0; j < 64; ++j)
      for (int i = 0; i < 64; ++i)
        h[i + 64 * j] = mat == 0 ? (i == j ? 64.0 : 0.0) + 1.0 / (1 + i + j)
                                 : std::exp(-(xs[i] - xs[j]) * (xs[i] - xs[j]) / (2 * 0.3 * 0.3)) + (i == j ? 1e-4 : 0.0);
    // long-double reference Cholesky (row-major L)
    std::vector<long double> Lr(4096, 0.0L);
    for (int j = 0; j < 64; ++j) {
      long double s = h[j + 64 * j];
      for (int k = 0; k < j; ++k) s -= Lr[j * 64 + k] * Lr[j * 64 + k];
      Lr[j * 64 + j] = std::sqrt(s);
      for (int i = j + 1; i < 64; ++i) {
        long double v = h[i + 64 * j];
        for (int k = 0; k < j; ++k) v -= Lr[i * 64 + k] * Lr[j * 64 + k];
        Lr[i * 64 + j] = v / Lr[j * 64 + j];
      }
    }
    long double lmax = 0;
    for (auto v : Lr) lmax = std::max(lmax, std::fabs(v));
    hipMemcpy(dA, h.data(), 4096 * 8, hipMemcpyHostToDevice);
    std::printf("%s block:\n", mat == 0 ? "diagonally dominant" : "GP kernel (l = 0.3, jitter 1e-4)");
    for (int v = 0; v < 7; ++v) {
      long long best = 1LL << 60;
      std::vector<double> o(4096);
      for (int rep = 0; rep < 5; ++rep) {
        hipMemset(dst, 0, 4);
        hipLaunchKernelGGL(ks[v], dim3(1), dim3(512), 0, 0, dA, dO, dc, dst);
        hipDeviceSynchronize();
        long long c;
        hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
        best = std::min(best, c);
      }
      int st;
      hipMemcpy(&st, dst, 4, hipMemcpyDeviceToHost);
      hipMemcpy(o.data(), dO, 4096 * 8, hipMemcpyDeviceToHost);
      long double err = 0;
      for (int r = 0; r < 64; ++r)
        for (int c = 0; c <= r; ++c) err = std::max(err, std::fabs((long double)o[r * 64 + c] - Lr[r * 64 + c]));
      std::printf("  %-24s %6lld cycles (%.2f us)  max|L - L_ref| / max|L| %.2e  status %d\n", names[v], best,
                  best / 2400.0, (double)(err / lmax), st);
    }
  }
  {  // leaf inverses: the library's trtri_leaf16 vs the pipelined one (4 waves / one wave)
    std::vector<double> h(4096), o0(4096), o1(4096);
    for (int j = 0; j < 64; ++j)
      for (int i = 0; i < 64; ++i) h[i + 64 * j] = (i == j ? 64.0 : 0.0) + 1.0 / (1 + i + j);
    hipMemcpy(dA, h.data(), 4096 * 8, hipMemcpyHostToDevice);
    void (*kl[4])(const double*, double*, long long*) = {k_leaf<0>, k_leaf<1>, k_leaf<2>, k_leaf<3>};
    const char* nl[4] = {"trtri_leaf16 x4 waves", "trtri_leaf16 leaf 3", "(same)", "(same)"};
    for (int v = 0; v < 4; ++v) {
      long long best = 1LL << 60;
      for (int rep = 0; rep < 5; ++rep) {
        hipLaunchKernelGGL(kl[v], dim3(1), dim3(512), 0, 0, dA, dO, dc);
        hipDeviceSynchronize();
        long long c;
        hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
        best = std::min(best, c);
      }
      hipMemcpy(v == 0 ? o0.data() : o1.data(), dO, 4096 * 8, hipMemcpyDeviceToHost);
      int diff = 0;
      double md = 0.0;
      if (v >= 1)
        for (int e = 0; e < 4096; ++e) {
          diff += o0[e] != o1[e];
          md = std::max(md, std::fabs(o0[e] - o1[e]));
        }
      if (v >= 1) std::printf("  (%d entries differ, max |d| %.2e)\n", diff, md);
      {  // |X_k L_k - I| per leaf, L from the factor (dumped by k_fac<0> on the same input)
        std::vector<double> Lf(4096);
        hipLaunchKernelGGL(ks[0], dim3(1), dim3(512), 0, 0, dA, dO, dc, dst);
        hipDeviceSynchronize();
        hipMemcpy(Lf.data(), dO, 4096 * 8, hipMemcpyDeviceToHost);
        const std::vector<double>& Xo = v == 0 ? o0 : o1;
        double res = 0;
        for (int k = 0; k < 4; ++k)
          for (int r = 0; r < 16; ++r)
            for (int c = 0; c < 16; ++c) {
              double acc = 0;
              for (int q = 0; q < 16; ++q)
                acc += Xo[(16 * k + r) * 64 + 16 * k + q] * (q >= c ? Lf[(16 * k + q) * 64 + 16 * k + c] : 0.0);
              res = std::max(res, std::fabs(acc - (r == c ? 1.0 : 0.0)));
            }
        std::printf("  |X L - I| = %.2e\n", res);
      }
      std::printf("  %-24s %6lld cycles (%.2f us)%s\n", nl[v], best, best / 2400.0,
                  v >= 1 ? (diff ? "  DIFFERENT bits" : "  same bits") : "");
    }
  }
  return 0;
}
