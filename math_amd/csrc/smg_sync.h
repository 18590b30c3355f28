// Cross-workgroup hand-off primitives of the persistent kernels (the
// Cholesky panel kernel, the persistent triangular solves).
//
// Producers store payload with device-scope (sc1) stores, so no XCD's L2
// holds dirty payload and the release fence before a flag has nothing to
// write back; the flag is a release store of the launch's epoch (no reset
// launch between uses).  Consumers spin on a relaxed device-scope load (no
// L2 invalidation per poll) and take ONE acquire fence once the flag is seen.
// Every wait gives up after ~4 s and latches SMG_ERR_SYNC, so a protocol
// fault can never hang the device.
#pragma once
#include "smg_internal.h"

__device__ __forceinline__ void st_dev(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// all threads of the workgroup call it (barrier inside)
__device__ inline void panel_publish(int* flag, int epoch) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
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
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

// panel_wait over flags[first], flags[first + stride], ..., flags[last]
// (at most 64 flags): wave 0 polls them in parallel, one lane per flag, then
// one barrier and ONE acquire fence for the whole set (so that the payload
// loads issued after it can be prefetched without a fence between them)
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
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}
