// Context, device arena, transfers, status latch, profiling, reductions.
// The arena mirrors stack_alloc (memory/stack_alloc.hpp:72-287): a list of
// device blocks, each twice the previous, bump allocation, marks = positions.
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "smg_internal.h"

namespace {

constexpr size_t kAlign = 256;

__global__ void k_reduce_partials(const double* __restrict__ p, int nparts,
                                  int width, double* out, int accumulate) {
  // one block per output column; fixed-order tree => deterministic
  __shared__ double lds[16];
  const int c = blockIdx.x;
  double s = 0.0;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) s += p[(size_t)i * width + c];
  s = block_sum(s, lds);
  if (threadIdx.x == 0) out[c] = accumulate ? out[c] + s : s;
}

// copy n device doubles to pinned host memory with system-scope stores, then
// publish seq to the host completion word (smg_publish_to_host)
__global__ __launch_bounds__(256) void k_publish(const double* __restrict__ src, long long n, double* dst,
                                                 long long* done, long long seq) {
  for (long long i = threadIdx.x; i < n; i += blockDim.x)
    __hip_atomic_store(dst + i, src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// zero up to ZR_MAX device ranges in one launch (16-byte stores; a range of
// an odd number of doubles gets its last one from the range's first lane):
// the adjoint zeroings and workspace clears without a runtime fill per buffer
constexpr int ZR_MAX = 16;
struct zero_ranges {
  double* p[ZR_MAX];
  unsigned long long n[ZR_MAX];  // doubles
  int count;
};
__global__ __launch_bounds__(256) void k_zero_ranges(zero_ranges z) {
  const unsigned long long tid = blockIdx.x * 256ull + threadIdx.x, stride = gridDim.x * 256ull;
  const double2 zz = {0.0, 0.0};
  for (int r = 0; r < z.count; ++r) {
    double* q = z.p[r];
    unsigned long long n = z.n[r];
    if (reinterpret_cast<uintptr_t>(q) & 8) {  // (a head double up to the 16-byte boundary)
      if (tid == 0) q[0] = 0.0;
      ++q;
      --n;
    }
    double2* p = reinterpret_cast<double2*>(q);
    const unsigned long long n2 = n >> 1;
    for (unsigned long long i = tid; i < n2; i += stride) p[i] = zz;
    if ((n & 1) && tid == 0) q[n - 1] = 0.0;
  }
}

// small device -> pinned host copies (the context's host staging buffer) as a
// kernel with system-scope stores instead of a runtime copy launch
__global__ __launch_bounds__(256) void k_copy_to_host(const double* __restrict__ src, long long n, double* dst) {
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += gridDim.x * 256ll)
    __hip_atomic_store(dst + i, src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// copy the status word to host memory (pinned, device-visible) and clear it:
// one launch instead of a runtime copy and fill
__global__ void k_status_take(int* st, int* host_dst) {
  if (threadIdx.x == 0) {
    __hip_atomic_store(host_dst, st[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    st[0] = 0;
  }
}

__global__ void k_status_copy(const int* st, int* host_dst) {
  if (threadIdx.x == 0) __hip_atomic_store(host_dst, st[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

constexpr int GATHER_MAX = 64;  // scalars per launch (kernel-argument array)
struct gather_args {
  const double* p[GATHER_MAX];
};
__global__ __launch_bounds__(64) void k_gather_scalars(gather_args a, int n, double* dst, const int* status,
                                                       int* status_out, long long* done, long long seq) {
  const int i = threadIdx.x;
  if (i < n) __hip_atomic_store(dst + i, *a.p[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (i == 0 && status_out) __hip_atomic_store(status_out, *status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (i == 0 && done) __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

smg_prof_scope::smg_prof_scope(smg_ctx* c, int f) : ctx(c), fam(f), on(c && c->prof_on) {
  if (!on) return;
  if (ctx->prof_pool.size() < 2) {
    for (int i = 0; i < 64; ++i) {
      hipEvent_t e;
      if (hipEventCreate(&e) == hipSuccess) ctx->prof_pool.push_back(e);
    }
  }
  a = ctx->prof_pool.back();
  ctx->prof_pool.pop_back();
  b = ctx->prof_pool.back();
  ctx->prof_pool.pop_back();
  hipEventRecord(a, ctx->stream);
}

smg_prof_scope::~smg_prof_scope() {
  if (!on) return;
  hipEventRecord(b, ctx->stream);
  ctx->prof_pending.push_back({a, b, fam});
}

static void prof_drain(smg_ctx* ctx) {
  for (auto& s : ctx->prof_pending) {
    float ms = 0.f;
    if (hipEventSynchronize(s.stop) == hipSuccess &&
        hipEventElapsedTime(&ms, s.start, s.stop) == hipSuccess) {
      ctx->prof_ms[s.family] += ms;
      ctx->prof_count[s.family] += 1;
    }
    ctx->prof_pool.push_back(s.start);
    ctx->prof_pool.push_back(s.stop);
  }
  ctx->prof_pending.clear();
}

double* smg_ws(smg_ctx* ctx, int id, size_t doubles) {
  if (doubles > ctx->ws_doubles[id]) {
    if (ctx->ws[id]) {
      hipStreamSynchronize(ctx->stream);
      if (ctx->side) hipStreamSynchronize(ctx->side);
      if (ctx->main_stream) hipStreamSynchronize(ctx->main_stream);
      hipFree(ctx->ws[id]);
    }
    size_t n = doubles < (1u << 18) ? (1u << 18) : doubles + doubles / 4;
    if (hipMalloc(&ctx->ws[id], n * sizeof(double)) != hipSuccess) {
      hipGetLastError();
      ctx->ws[id] = nullptr;
      ctx->ws_doubles[id] = 0;
      ctx->host_status |= SMG_ERR_OOM;
      return nullptr;
    }
    ctx->ws_doubles[id] = n;
  }
  return ctx->ws[id];
}

int smg_side_begin(smg_ctx* ctx) {
  if (ctx->side) return SMG_OK;
  if (hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking) != hipSuccess) {
    ctx->side = nullptr;
    ctx->host_status |= SMG_ERR_HIP;
    return SMG_ERR_HIP;
  }
  return SMG_OK;
}

int smg_inv_events(smg_ctx* ctx) {
  for (hipEvent_t* e : {&ctx->inv_ev, &ctx->inv_ev_main, &ctx->inv_ev_aux, &ctx->inv_ev_w})
    if (!*e && hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) {
      *e = nullptr;
      ctx->host_status |= SMG_ERR_HIP;
      return SMG_ERR_HIP;
    }
  return SMG_OK;
}

static hipEvent_t pooled_event(smg_ctx* ctx, std::vector<hipEvent_t>& pool, int i) {
  while ((int)pool.size() <= i) {
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
      ctx->host_status |= SMG_ERR_HIP;
      return nullptr;
    }
    pool.push_back(e);
  }
  return pool[i];
}

hipEvent_t smg_event(smg_ctx* ctx, int i) { return pooled_event(ctx, ctx->ev_pool, i); }

hipEvent_t smg_fork_event(smg_ctx* ctx, int i) { return pooled_event(ctx, ctx->ev_fork, i); }

void smg_reduce_partials(smg_ctx* ctx, const double* partials, int nparts,
                         int width, double* out, int accumulate) {
  hipLaunchKernelGGL(k_reduce_partials, dim3(width), dim3(256), 0, ctx->stream,
                     partials, nparts, width, out, accumulate);
}

extern "C" {

int smg_device_count(int* n) {
  smg_ctx* ctx = nullptr;
  SMG_HIP_TRY(hipGetDeviceCount(n));
  return SMG_OK;
}

int smg_ctx_create(int device, size_t initial, smg_ctx** out) {
  if (!out) return SMG_ERR_ARG;
  *out = nullptr;
  smg_ctx* ctx = nullptr;
  SMG_HIP_TRY(hipSetDevice(device));
  ctx = new smg_ctx();
  ctx->device = device;
  ctx->cur_block = 0;
  ctx->offset = 0;
  ctx->host_status = 0;
  ctx->status_armed = 0;
  ctx->pin_io = nullptr;
  ctx->pin_io_size = 0;
  ctx->res_h = nullptr;
  ctx->res_h_size = 0;
  ctx->done_h = nullptr;
  ctx->done_seq = 0;
  ctx->red_counter_d = nullptr;
  for (int i = 0; i < SMG_WS_COUNT; ++i) {
    ctx->ws[i] = nullptr;
    ctx->ws_doubles[i] = 0;
  }
  ctx->prof_on = 0;
  ctx->comm = nullptr;
  ctx->status_ev = nullptr;
  ctx->status_mark = 0;
  ctx->zero_stream = nullptr;
  ctx->zero_ev_main = ctx->zero_ev_done = nullptr;
  ctx->zero_pending = 0;
  ctx->inv_ev = ctx->inv_ev_main = ctx->inv_ev_aux = ctx->inv_ev_w = nullptr;
  ctx->inv_pending = 0;
  ctx->inv_w_recorded = 0;
  ctx->side = nullptr;
  ctx->main_stream = nullptr;
  for (int i = 0; i < SMG_FAM_COUNT; ++i) {
    ctx->prof_ms[i] = 0;
    ctx->prof_count[i] = 0;
    ctx->prof_flops[i] = 0;
  }
  // the main stream at the highest priority: when one of its launches (a
  // Cholesky panel on the critical path) becomes ready together with a side
  // stream's (the trailing update behind it), the panel's workgroups are
  // dispatched first instead of waiting for CUs the GEMM took
  int prio_least = 0, prio_greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest) != hipSuccess) prio_greatest = 0;
  if (hipStreamCreateWithPriority(&ctx->stream, hipStreamNonBlocking, prio_greatest) != hipSuccess) {
    delete ctx;
    return SMG_ERR_HIP;
  }
  if (initial < (size_t)(64u << 20)) initial = (size_t)(64u << 20);
  char* base = nullptr;
  if (hipMalloc(&base, initial) != hipSuccess) {
    hipStreamDestroy(ctx->stream);
    delete ctx;
    return SMG_ERR_OOM;
  }
  ctx->blocks.push_back({base, initial});
  // status word at [0]; the panel-kernel flags from byte 256 on
  if (hipMalloc(&ctx->status_d, SMG_STATUS_BYTES) != hipSuccess ||
      hipHostMalloc(&ctx->status_h, 256, hipHostMallocDefault) != hipSuccess) {
    delete ctx;
    return SMG_ERR_HIP;
  }
  hipMemset(ctx->status_d, 0, SMG_STATUS_BYTES);
  ctx->flags_d = ctx->status_d + 64;
  ctx->flag_epoch = 0;
  ctx->inv_ctr_d = reinterpret_cast<unsigned*>(ctx->flags_d + 4096);
  ctx->inv_launches = 0;
  ctx->inv_per_cu = ctx->inv_cus = -1;
  ctx->inv_mode = 0;
  ctx->host_scratch_size = 1u << 20;
  if (hipHostMalloc(&ctx->host_scratch, ctx->host_scratch_size, hipHostMallocDefault) != hipSuccess) {
    delete ctx;
    return SMG_ERR_HIP;
  }
  if (hipHostMalloc(&ctx->done_h, 256, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess ||
      hipMalloc(&ctx->red_counter_d, 256) != hipSuccess) {
    delete ctx;
    return SMG_ERR_HIP;
  }
  *(volatile long long*)ctx->done_h = 0;
  hipMemset(ctx->red_counter_d, 0, 256);
  hipDeviceSynchronize();
  *out = ctx;
  return SMG_OK;
}

int smg_ctx_destroy(smg_ctx* ctx) {
  if (!ctx) return SMG_OK;
  hipSetDevice(ctx->device);
  hipStreamSynchronize(ctx->stream);
  prof_drain(ctx);
  smg_comm_destroy(ctx);
  for (auto& b : ctx->blocks) hipFree(b.base);
  for (auto e : ctx->prof_pool) hipEventDestroy(e);
  for (auto e : ctx->ev_pool) hipEventDestroy(e);
  for (auto e : ctx->ev_fork) hipEventDestroy(e);
  for (auto e : ctx->marker_ev) hipEventDestroy(e);
  if (ctx->status_ev) hipEventDestroy(ctx->status_ev);
  if (ctx->zero_stream) {
    hipStreamSynchronize(ctx->zero_stream);
    hipEventDestroy(ctx->zero_ev_main);
    hipEventDestroy(ctx->zero_ev_done);
    hipStreamDestroy(ctx->zero_stream);
  }
  if (ctx->side) {
    hipStreamSynchronize(ctx->side);
    hipStreamDestroy(ctx->side);
  }
  if (ctx->copy_stream) {
    hipStreamSynchronize(ctx->copy_stream);
    hipStreamDestroy(ctx->copy_stream);
  }
  for (hipEvent_t e : {ctx->inv_ev, ctx->inv_ev_main, ctx->inv_ev_aux, ctx->inv_ev_w})
    if (e) hipEventDestroy(e);
  for (int i = 0; i < SMG_WS_COUNT; ++i)
    if (ctx->ws[i]) hipFree(ctx->ws[i]);
  hipFree(ctx->status_d);
  hipHostFree(ctx->status_h);
  hipHostFree(ctx->host_scratch);
  if (ctx->pin_io) hipHostFree(ctx->pin_io);
  if (ctx->res_h) hipHostFree(ctx->res_h);
  hipHostFree(ctx->done_h);
  hipFree(ctx->red_counter_d);
  hipStreamDestroy(ctx->stream);
  delete ctx;
  return SMG_OK;
}

int smg_ctx_device(const smg_ctx* ctx) { return ctx ? ctx->device : -1; }
void* smg_ctx_stream(smg_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

void* smg_arena_alloc(smg_ctx* ctx, size_t bytes) {
  if (!ctx) return nullptr;
  bytes = (bytes + kAlign - 1) & ~(kAlign - 1);
  if (bytes == 0) bytes = kAlign;
  smg_arena_block* b = &ctx->blocks[ctx->cur_block];
  if (ctx->offset + bytes <= b->size) {
    void* p = b->base + ctx->offset;
    ctx->offset += bytes;
    return p;
  }
  // move_to_next_block (stack_alloc.hpp:94-119)
  size_t nb = ctx->cur_block + 1;
  while (nb < ctx->blocks.size() && ctx->blocks[nb].size < bytes) ++nb;
  if (nb >= ctx->blocks.size()) {
    size_t newsize = ctx->blocks.back().size * 2;
    if (newsize < bytes) newsize = bytes;
    char* base = nullptr;
    if (hipMalloc(&base, newsize) != hipSuccess) {
      // retry with exactly what is needed before giving up
      if (newsize == bytes || hipMalloc(&base, bytes) != hipSuccess) {
        hipGetLastError();
        ctx->host_status |= SMG_ERR_OOM;
        return nullptr;
      }
      newsize = bytes;
    }
    ctx->blocks.push_back({base, newsize});
    nb = ctx->blocks.size() - 1;
  }
  ctx->cur_block = nb;
  ctx->offset = bytes;
  return ctx->blocks[nb].base;
}

// mark encodes (block, offset): block in the top 16 bits
size_t smg_arena_mark(smg_ctx* ctx) {
  return ((size_t)ctx->cur_block << 48) | ctx->offset;
}

int smg_arena_rewind(smg_ctx* ctx, size_t mark) {
  size_t blk = mark >> 48, off = mark & ((1ull << 48) - 1);
  if (blk >= ctx->blocks.size()) return SMG_ERR_ARG;
  // the freed memory is handed out again: no zeroing of it may still be
  // queued or running behind the main stream
  if (int e = smg_join_async(ctx)) return e;
  ctx->cur_block = blk;
  ctx->offset = off;
  return SMG_OK;
}

int smg_arena_recover_all(smg_ctx* ctx) {
  if (int e = smg_join_async(ctx)) return e;
  ctx->cur_block = 0;
  ctx->offset = 0;
  return SMG_OK;
}

size_t smg_arena_used(const smg_ctx* ctx) {
  size_t s = 0;
  for (size_t i = 0; i < ctx->cur_block; ++i) s += ctx->blocks[i].size;
  return s + ctx->offset;
}

size_t smg_arena_reserved(const smg_ctx* ctx) {
  size_t s = 0;
  for (auto& b : ctx->blocks) s += b.size;
  return s;
}

// every stream that may still have a copy into / out of pinned host memory
// in flight (the streamed factor's panel copies run on the zeroing stream)
static void sync_all_streams(smg_ctx* ctx) {
  hipStreamSynchronize(ctx->stream);
  if (ctx->main_stream && ctx->main_stream != ctx->stream) hipStreamSynchronize(ctx->main_stream);
  if (ctx->side) hipStreamSynchronize(ctx->side);
  if (ctx->zero_stream) hipStreamSynchronize(ctx->zero_stream);
  if (ctx->copy_stream) hipStreamSynchronize(ctx->copy_stream);
}

void* smg_host_scratch(smg_ctx* ctx, size_t bytes) {
  if (bytes > ctx->host_scratch_size) {
    sync_all_streams(ctx);
    hipHostFree(ctx->host_scratch);
    size_t n = ctx->host_scratch_size;
    while (n < bytes) n *= 2;
    if (hipHostMalloc(&ctx->host_scratch, n, hipHostMallocDefault) != hipSuccess) {
      ctx->host_scratch = nullptr;
      ctx->host_scratch_size = 0;
      return nullptr;
    }
    ctx->host_scratch_size = n;
  }
  return ctx->host_scratch;
}

void* smg_pinned_io(smg_ctx* ctx, size_t bytes) {
  if (!ctx) return nullptr;
  if (bytes > ctx->pin_io_size) {
    sync_all_streams(ctx);
    if (ctx->pin_io) hipHostFree(ctx->pin_io);
    size_t n = ctx->pin_io_size ? ctx->pin_io_size : (size_t)1 << 16;
    while (n < bytes) n *= 2;
    // coarse-grained: kernel stores leave the L2 as whole lines at the
    // system-scope release, instead of one PCIe write per store
    if (hipHostMalloc(&ctx->pin_io, n, hipHostMallocNonCoherent | hipHostMallocMapped) != hipSuccess) {
      hipGetLastError();
      ctx->pin_io = nullptr;
      ctx->pin_io_size = 0;
      return nullptr;
    }
    ctx->pin_io_size = n;
  }
  return ctx->pin_io;
}

void* smg_pinned_result(smg_ctx* ctx, size_t bytes) {
  if (!ctx) return nullptr;
  if (bytes > ctx->res_h_size) {
    sync_all_streams(ctx);
    if (ctx->res_h) hipHostFree(ctx->res_h);
    size_t n = ctx->res_h_size ? ctx->res_h_size : (size_t)1 << 12;
    while (n < bytes) n *= 2;
    if (hipHostMalloc(&ctx->res_h, n, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
      hipGetLastError();
      ctx->res_h = nullptr;
      ctx->res_h_size = 0;
      return nullptr;
    }
    ctx->res_h_size = n;
  }
  return ctx->res_h;
}

int smg_wait_done(smg_ctx* ctx, long long seq) {
  // the kernel publishes seq after a system-scope release; spin briefly (the
  // common case completes in microseconds), then fall back to the stream
  // sync so a failed launch still returns
  volatile long long* d = ctx->done_h;
  for (long long spin = 0; spin < (1ll << 22); ++spin)
    if (*d >= seq) return SMG_OK;
  SMG_HIP_TRY(hipStreamSynchronize(ctx->stream));
  return *d >= seq ? SMG_OK : SMG_ERR_HIP;
}

int smg_publish_to_host(smg_ctx* ctx, const double* src, long long n, double* dst) {
  if (!ctx || n < 0 || (n > 0 && (!src || !dst))) return SMG_ERR_ARG;
  const long long seq = ++ctx->done_seq;
  hipLaunchKernelGGL(k_publish, dim3(1), dim3(256), 0, ctx->stream, src, n, dst, ctx->done_h, seq);
  SMG_LAUNCH_CHECK();
  return smg_wait_done(ctx, seq);
}

int smg_gather_scalars(smg_ctx* ctx, const double* const* src, int n, double* dst, int* status_out) {
  if (!ctx || n < 0 || (n > 0 && (!src || !dst))) return SMG_ERR_ARG;
  if (n == 0 && !status_out) return SMG_OK;
  long long seq = 0;
  for (int b = 0; b < n || (b == 0 && status_out); b += GATHER_MAX) {
    const int m = n - b < GATHER_MAX ? n - b : GATHER_MAX;
    gather_args a;
    for (int i = 0; i < m; ++i) a.p[i] = src[b + i];
    const bool last = b + GATHER_MAX >= n;
    int* so = last ? status_out : nullptr;
    if (last) seq = ++ctx->done_seq;
    hipLaunchKernelGGL(k_gather_scalars, dim3(1), dim3(64), 0, ctx->stream, a, m, dst + b, ctx->status_d, so,
                       last ? ctx->done_h : nullptr, seq);
    SMG_LAUNCH_CHECK();
    if (last) break;
  }
  if (status_out) ctx->status_armed = 0;
  return smg_wait_done(ctx, seq);
}

int smg_memcpy_h2d(smg_ctx* ctx, void* dst, const void* src, size_t bytes) {
  if (!bytes) return SMG_OK;
  SMG_HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
  return SMG_OK;
}


// dst inside the context's pinned host staging buffer (device-accessible)
static bool in_host_scratch(const smg_ctx* ctx, const void* p, size_t bytes) {
  const char* b = static_cast<const char*>(ctx->host_scratch);
  const char* c = static_cast<const char*>(p);
  return b && c >= b && c + bytes <= b + ctx->host_scratch_size;
}

int smg_d2h_impl(smg_ctx* ctx, hipStream_t stream, void* dst, const void* src, size_t bytes) {
  (void)ctx;  // (the copy engine: a kernel-driven copy measured no faster, round 5)
  SMG_HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, stream));
  return SMG_OK;
}

int smg_memcpy_d2h(smg_ctx* ctx, void* dst, const void* src, size_t bytes) {
  if (!bytes) return SMG_OK;
  if (bytes >= 65536) return smg_d2h_impl(ctx, ctx->stream, dst, src, bytes);
  if (bytes <= 65536 && !((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src) | bytes) & 7) &&
      in_host_scratch(ctx, dst, bytes)) {
    const long long n = (long long)(bytes / 8);
    hipLaunchKernelGGL(k_copy_to_host, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream,
                       static_cast<const double*>(src), n, static_cast<double*>(dst));
    SMG_LAUNCH_CHECK();
    return SMG_OK;
  }
  SMG_HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
  return SMG_OK;
}

int smg_memcpy_d2d(smg_ctx* ctx, void* dst, const void* src, size_t bytes) {
  if (!bytes) return SMG_OK;
  SMG_HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, ctx->stream));
  return SMG_OK;
}

int smg_memset(smg_ctx* ctx, void* dst, int v, size_t bytes) {
  if (!bytes) return SMG_OK;
  if (v == 0) {
    const std::pair<void*, size_t> r(dst, bytes);
    return smg_zero_ranges_impl(ctx, ctx->stream, &r, 1);
  }
  SMG_HIP_TRY(hipMemsetAsync(dst, v, bytes, ctx->stream));
  return SMG_OK;
}

}  // extern "C"

int smg_zero_ranges_impl(smg_ctx* ctx, hipStream_t stream, const std::pair<void*, size_t>* r, int count,
                         unsigned max_grid) {
  zero_ranges z{};
  size_t most = 0;
  auto launch = [&]() -> int {
    if (!z.count) return SMG_OK;
    const size_t g = (most / 2 + 255) / 256;
    hipLaunchKernelGGL(k_zero_ranges, dim3(g < max_grid ? (g < 1 ? 1 : (unsigned)g) : max_grid), dim3(256), 0, stream,
                       z);
    SMG_LAUNCH_CHECK();
    z.count = 0;
    most = 0;
    return SMG_OK;
  };
  for (int i = 0; i < count; ++i) {
    const size_t b = r[i].second;
    if (!b) continue;
    if ((reinterpret_cast<uintptr_t>(r[i].first) & 7) || (b & 7)) {  // (not a range of doubles)
      SMG_HIP_TRY(hipMemsetAsync(r[i].first, 0, b, stream));
      continue;
    }
    z.p[z.count] = static_cast<double*>(r[i].first);
    z.n[z.count] = b / 8;
    most = b / 8 > most ? b / 8 : most;
    if (++z.count == ZR_MAX)
      if (int rc = launch()) return rc;
  }
  return launch();
}

extern "C" {

int smg_zero_stream_begin(smg_ctx* ctx) {
  if (ctx->zero_stream) return SMG_OK;
  if (hipStreamCreateWithFlags(&ctx->zero_stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->zero_ev_main, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->zero_ev_done, hipEventDisableTiming) != hipSuccess) {
    hipGetLastError();
    ctx->zero_stream = nullptr;
    return SMG_ERR_HIP;
  }
  return SMG_OK;
}

int smg_marker_event(smg_ctx* ctx, int slot, hipEvent_t* ev) {
  if (slot < 0 || slot >= 64) return SMG_ERR_ARG;
  while ((int)ctx->marker_ev.size() <= slot) {
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
      ctx->host_status |= SMG_ERR_HIP;
      return SMG_ERR_HIP;
    }
    ctx->marker_ev.push_back(e);
  }
  *ev = ctx->marker_ev[slot];
  return SMG_OK;
}

int smg_memset_async(smg_ctx* ctx, void* dst, size_t bytes) {
  if (!ctx) return SMG_ERR_ARG;
  if (!bytes) return SMG_OK;
  if (!dst) return SMG_ERR_ARG;
  if (smg_zero_stream_begin(ctx) != SMG_OK) {  // no second stream: in order
    const std::pair<void*, size_t> r(dst, bytes);
    return smg_zero_ranges_impl(ctx, ctx->stream, &r, 1);
  }
  // issued by smg_zero_flush: at the next latency-bound entry, the join, or a
  // rewind (the memory then still belongs to this tape)
  ctx->zero_queue.emplace_back(dst, bytes);
  return SMG_OK;
}

int smg_zero_flush(smg_ctx* ctx) {
  if (ctx->zero_queue.empty()) return SMG_OK;
  // after everything already enqueued on the main stream (the memory may have
  // belonged to a recovered tape whose kernels are still queued there)
  hipStream_t main = (ctx->side && ctx->stream == ctx->side) ? ctx->main_stream : ctx->stream;
  SMG_HIP_TRY(hipEventRecord(ctx->zero_ev_main, main));
  SMG_HIP_TRY(hipStreamWaitEvent(ctx->zero_stream, ctx->zero_ev_main, 0));
  // at most 128 workgroups: these zeroings (the N^2 adjoints of a GP's K, K + dI
  // and L: 400 MB at N = 4096) run beside the first panel, and at full width
  // they had stretched it 177 -> 230 us; GP 367 -> 369-372 evals/s against 2048
  // (same box; 64 / 32: the same within noise)
  if (int rc = smg_zero_ranges_impl(ctx, ctx->zero_stream, ctx->zero_queue.data(), (int)ctx->zero_queue.size(), 128u))
    return rc;
  SMG_HIP_TRY(hipEventRecord(ctx->zero_ev_done, ctx->zero_stream));
  ctx->zero_queue.clear();
  ctx->zero_pending = 1;
  return SMG_OK;
}

int smg_join_async(smg_ctx* ctx) {
  if (!ctx) return SMG_ERR_ARG;
  if (ctx->inv_pending) {  // an smg_cholesky_inv_t_async still on the side stream
    SMG_HIP_TRY(hipStreamWaitEvent(ctx->stream, ctx->inv_ev, 0));
    ctx->inv_pending = 0;
  }
  if (int e = smg_zero_flush(ctx)) return e;
  if (!ctx->zero_pending) return SMG_OK;
  SMG_HIP_TRY(hipStreamWaitEvent(ctx->stream, ctx->zero_ev_done, 0));
  ctx->zero_pending = 0;
  return SMG_OK;
}

int smg_marker_record(smg_ctx* ctx, int slot) {
  if (!ctx) return SMG_ERR_ARG;
  hipEvent_t e;
  if (int rc = smg_marker_event(ctx, slot, &e)) return rc;
  SMG_HIP_TRY(hipEventRecord(e, ctx->stream));
  return SMG_OK;
}

int smg_marker_wait(smg_ctx* ctx, int slot) {
  if (!ctx || slot < 0 || slot >= (int)ctx->marker_ev.size()) return SMG_ERR_ARG;
  SMG_HIP_TRY(hipEventSynchronize(ctx->marker_ev[slot]));
  return SMG_OK;
}

int smg_set_inv_block_mode(smg_ctx* ctx, int mode) {
  if (!ctx || mode < 0 || mode > 1) return SMG_ERR_ARG;
  ctx->inv_mode = mode;
  return SMG_OK;
}

int smg_sync_all(smg_ctx* ctx) {
  if (!ctx) return SMG_ERR_ARG;
  sync_all_streams(ctx);
  SMG_HIP_TRY(hipGetLastError());
  if (ctx->prof_on) prof_drain(ctx);
  return SMG_OK;
}

int smg_sync(smg_ctx* ctx) {
  SMG_HIP_TRY(hipStreamSynchronize(ctx->stream));
  if (ctx->prof_on) prof_drain(ctx);
  return SMG_OK;
}

int smg_status(smg_ctx* ctx, int* status) {
  hipLaunchKernelGGL(k_status_take, dim3(1), dim3(64), 0, ctx->stream, ctx->status_d, ctx->status_h);
  SMG_LAUNCH_CHECK();
  SMG_HIP_TRY(hipStreamSynchronize(ctx->stream));
  if (ctx->prof_on) prof_drain(ctx);
  int s = ctx->status_h[0] | ctx->host_status;
  ctx->host_status = 0;
  ctx->status_armed = 0;
  if (status) *status = s;
  return SMG_OK;
}

}  // extern "C"

int smg_status_mark_impl(smg_ctx* ctx) {
  if (!ctx->status_ev && hipEventCreateWithFlags(&ctx->status_ev, hipEventDisableTiming) != hipSuccess) {
    ctx->status_ev = nullptr;
    return SMG_ERR_HIP;
  }
  hipLaunchKernelGGL(k_status_take, dim3(1), dim3(64), 0, ctx->stream, ctx->status_d, ctx->status_h + 1);
  SMG_LAUNCH_CHECK();
  SMG_HIP_TRY(hipEventRecord(ctx->status_ev, ctx->stream));
  ctx->status_mark = 1;
  return SMG_OK;
}

extern "C" {

int smg_status_mark_wait(smg_ctx* ctx, int* status) {
  if (!ctx) return SMG_ERR_ARG;
  if (!ctx->status_mark || ctx->prof_on) {  // no mark (or profiling): the whole-stream status read
    ctx->status_mark = 0;
    return smg_status(ctx, status);
  }
  SMG_HIP_TRY(hipEventSynchronize(ctx->status_ev));
  int s = ctx->status_h[1] | ctx->host_status;
  ctx->host_status = 0;
  ctx->status_mark = 0;
  ctx->status_armed = 0;  // the launches that could latch it ran before the mark
  if (status) *status = s;
  return SMG_OK;
}

int smg_status_armed(smg_ctx* ctx, int* armed) {
  if (!ctx || !armed) return SMG_ERR_ARG;
  *armed = ctx->status_armed;
  return SMG_OK;
}

int smg_status_enqueue(smg_ctx* ctx, int* host_dst) {
  if (!ctx || !host_dst) return SMG_ERR_ARG;
  if (in_host_scratch(ctx, host_dst, sizeof(int))) {
    hipLaunchKernelGGL(k_status_copy, dim3(1), dim3(64), 0, ctx->stream, ctx->status_d, host_dst);
    SMG_LAUNCH_CHECK();
  } else {
    SMG_HIP_TRY(hipMemcpyAsync(host_dst, ctx->status_d, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  }
  ctx->status_armed = 0;
  return SMG_OK;
}

namespace {
__global__ void k_status_or(int* st, int bits) {
  if (threadIdx.x == 0) st[0] |= bits;
}
}  // namespace

int smg_status_inject(smg_ctx* ctx, int bits) {
  if (!ctx) return SMG_ERR_ARG;
  hipLaunchKernelGGL(k_status_or, dim3(1), dim3(64), 0, ctx->stream, ctx->status_d, bits);
  SMG_LAUNCH_CHECK();
  ctx->status_armed = 1;
  return SMG_OK;
}

int smg_profile_enable(smg_ctx* ctx, int on) {
  hipStreamSynchronize(ctx->stream);
  prof_drain(ctx);
  ctx->prof_on = on;
  for (int i = 0; i < SMG_FAM_COUNT; ++i) {
    ctx->prof_ms[i] = 0;
    ctx->prof_count[i] = 0;
    ctx->prof_flops[i] = 0;
  }
  return SMG_OK;
}

int smg_profile_read(smg_ctx* ctx, int family, double* ms, long long* count) {
  if (family < 0 || family >= SMG_FAM_COUNT) return SMG_ERR_ARG;
  hipStreamSynchronize(ctx->stream);
  prof_drain(ctx);
  if (ms) *ms = ctx->prof_ms[family];
  if (count) *count = ctx->prof_count[family];
  return SMG_OK;
}

int smg_profile_flops(smg_ctx* ctx, int family, double* flops) {
  if (!ctx || family < 0 || family >= SMG_FAM_COUNT || !flops) return SMG_ERR_ARG;
  *flops = ctx->prof_flops[family];
  return SMG_OK;
}

}  // extern "C"

namespace {
__device__ __forceinline__ unsigned long long splitmix(unsigned long long seed, long long i) {
  unsigned long long z = seed + (unsigned long long)(i + 1) * 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
__global__ void k_fill_unif(double* out, long long n, unsigned long long seed, double a, double b,
                            double scale) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const double u = (double)(splitmix(seed, i) >> 11) * (1.0 / 9007199254740992.0);
    const double v = __dadd_rn(a, __dmul_rn(b - a, u));  // no contraction: matches oracle/gen.h
    out[i] = scale == 1.0 ? v : __dmul_rn(v, scale);
  }
}
__global__ void k_fill_bern(int* out, long long n, unsigned long long seed, double p) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const double u = (double)(splitmix(seed, i) >> 11) * (1.0 / 9007199254740992.0);
    out[i] = u < p ? 1 : 0;
  }
}
}  // namespace

extern "C" int smg_fill_unif(smg_ctx* ctx, double* out, long long n, unsigned long long seed,
                             double a, double b, double scale) {
  if (!ctx || n < 0 || (n > 0 && !out)) return SMG_ERR_ARG;
  if (!n) return SMG_OK;
  hipLaunchKernelGGL(k_fill_unif, dim3(8192), dim3(256), 0, ctx->stream, out, n, seed, a, b, scale);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}
extern "C" int smg_fill_bernoulli(smg_ctx* ctx, int* out, long long n, unsigned long long seed,
                                  double p) {
  if (!ctx || n < 0 || (n > 0 && !out)) return SMG_ERR_ARG;
  if (!n) return SMG_OK;
  hipLaunchKernelGGL(k_fill_bern, dim3(8192), dim3(256), 0, ctx->stream, out, n, seed, p);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}
