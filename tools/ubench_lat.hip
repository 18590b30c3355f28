// Dev microbenchmark (round 6): issue cost and latency of the cross-lane
// primitives the chain's pivot factor uses (one wave, s_memtime cycles).
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ __forceinline__ long long now() { return __builtin_amdgcn_s_memtime(); }
__device__ __forceinline__ double bcast(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double bperm(double v, int lane) {
  const int lo = __builtin_amdgcn_ds_bpermute(lane * 4, __double2loint(v));
  const int hi = __builtin_amdgcn_ds_bpermute(lane * 4, __double2hiint(v));
  return __hiloint2double(hi, lo);
}
template <int T>
__global__ void k(double* out, long long* cyc, double seed) {
  __shared__ double S[64 * 8];
  const int l = threadIdx.x;
  double v[16];
  for (int q = 0; q < 16; ++q) v[q] = seed + l + q;
  __builtin_amdgcn_s_waitcnt(0);
  const long long t0 = now();
  double acc = 0.0;
  if (T == 0) {  // 64 independent double broadcasts (readlane), summed
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc += bcast(v[q], q + 16 * r);
  } else if (T == 1) {  // dependent chain: x = bcast(x * 1.0000001, lane) 64 times
    double x = v[0];
#pragma unroll
    for (int r = 0; r < 64; ++r) x = bcast(x, r) + l * 1e-9;
    acc = x;
  } else if (T == 2) {  // dependent fp64 FMA chain, 64 long
    double x = v[0];
#pragma unroll
    for (int r = 0; r < 64; ++r) x = __builtin_fma(x, 1.0000001, l * 1e-9);
    acc = x;
  } else if (T == 3) {  // 64 independent fp64 FMAs (16 chains of 4)
    double x[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) x[q] = v[q];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int q = 0; q < 16; ++q) x[q] = __builtin_fma(x[q], 1.0000001, l * 1e-9);
#pragma unroll
    for (int q = 0; q < 16; ++q) acc += x[q];
  } else if (T == 4) {  // 64 independent double broadcasts through ds_bpermute
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc += bperm(v[q], q + 16 * r);
  } else if (T == 5) {  // dependent chain through ds_bpermute
    double x = v[0];
#pragma unroll
    for (int r = 0; r < 64; ++r) x = bperm(x, r) + l * 1e-9;
    acc = x;
  } else if (T == 6) {  // LDS round trip chain: write own, read lane r's, 64 times
    double x = v[0];
    for (int r = 0; r < 64; ++r) {
      S[l] = x + l * 1e-9;
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
      x = S[r];
      __builtin_amdgcn_wave_barrier();
    }
    acc = x;
  } else if (T == 7) {  // v_rsq_f64 dependent chain
    double x = v[0] + 1.0;
#pragma unroll
    for (int r = 0; r < 64; ++r) x = __builtin_amdgcn_rsq(x) + 1.0;
    acc = x;
  }
  __builtin_amdgcn_s_waitcnt(0);
  int dep = __builtin_amdgcn_readfirstlane(__double2loint(acc));
  asm volatile("s_mov_b32 %0, %0" : "+s"(dep));
  const long long t1 = now();
  if (dep == 12345) out[0] = 0;
  out[l] = acc;
  if (l == 0) cyc[T] = t1 - t0;
}
int main() {
  double* o;
  long long* c;
  hipMalloc(&o, 64 * 8);
  hipMalloc(&c, 64 * 8);
  const char* nm[8] = {"64 indep readlane bcasts", "64 dep readlane bcast+add", "64 dep fp64 fma",
                       "64 indep fp64 fma", "64 indep bpermute bcasts", "64 dep bpermute bcast+add",
                       "64 dep LDS write/read round trips", "64 dep v_rsq_f64 + add"};
  void (*ks[8])(double*, long long*, double) = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>, k<6>, k<7>};
  for (int t = 0; t < 8; ++t) {
    long long best = 1LL << 60, v;
    for (int r = 0; r < 5; ++r) {
      hipLaunchKernelGGL(ks[t], dim3(1), dim3(64), 0, 0, o, c, 1.0);
      hipDeviceSynchronize();
      hipMemcpy(&v, c + t, 8, hipMemcpyDeviceToHost);
      if (v < best) best = v;
    }
    printf("%-36s %6lld cycles  (%.1f per op)\n", nm[t], best, best / 64.0);
  }
}
