// Cross-workgroup hand-off primitives of the persistent kernels (the
// Cholesky panel kernel, the persistent triangular solves).
//
// The fence-free form of MI355X_MICROARCH.md's hand-off table (row 1): the
// producer stores every payload byte with device-scope (sc1) stores
// (st_dev), EVERY storing wave waits for its own stores (s_waitcnt
// vmcnt(0)), a workgroup barrier, then ONE lane stores the flag sc1; the
// consumer polls the flag with sc1 loads, a workgroup barrier, and then reads
// every payload byte with sc1 loads (ld_dev).  No release fence (an L2
// write-back, ~1.7 us) and no acquire fence (an L1 invalidate, ~1.7 us) on
// either side of a hand-off.  Requirements kept by the callers: payload in
// hipMalloc memory, one workgroup per CU, every load of handed-off bytes an
// ld_dev.  Flags carry the launch's epoch (no reset launch between uses).
// Every wait gives up after ~4 s and latches SMG_ERR_SYNC, so a protocol
// fault can never hang the device.
#pragma once
#include "smg_internal.h"

__device__ __forceinline__ void st_dev(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ double ld_dev(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// all threads of the workgroup call it (barrier inside)
__device__ inline void panel_publish(int* flag, int epoch) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 payload stores have landed
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// all threads of the workgroup call it (barrier inside)
__device__ inline void panel_wait(const int* flag, int epoch, int* status) {
  if (threadIdx.x == 0) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 400000000ull) {
        atomicOr(status, (int)SMG_ERR_SYNC);
        break;
      }
    }
  }
  __syncthreads();  // the other waves read the payload after the polling wave saw the flag
}

// panel_wait over flags[first], flags[first + stride], ..., flags[last]
// (at most 64 flags): wave 0 polls them in parallel, one lane per flag, then
// one barrier for the whole set
__device__ inline void panel_wait_all(const int* flags, int first, int last, int stride, int epoch,
                                      int* status) {
  if (threadIdx.x < 64) {
    const int c = first + (int)threadIdx.x;
    const bool mine = c <= last;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    bool seen = !mine;
    while (true) {
      if (!seen) seen = __hip_atomic_load(&flags[c * stride], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch;
      if (__all(seen)) break;
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 400000000ull) {
        if (threadIdx.x == 0) atomicOr(status, (int)SMG_ERR_SYNC);
        break;
      }
    }
  }
  __syncthreads();  // the other waves read the payload after the polling wave saw the flag
}
