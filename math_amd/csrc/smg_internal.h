// Internal declarations shared by the libsmg_hip.so translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <utility>
#include <vector>

#include "../../include/smg_hip.h"

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2v __attribute__((ext_vector_type(2)));

struct smg_arena_block {
  char* base;
  size_t size;
};

struct smg_prof_slot {
  hipEvent_t start, stop;
  int family;
};

// device status allocation: the status word, then the panel-kernel flags
// (+ the counter ring of k_inv_block512's grid barriers: SMG_INV_CTRS slots)
constexpr int SMG_INV_CTRS = 64;
constexpr size_t SMG_STATUS_BYTES = 256 + 4096 * sizeof(int) + SMG_INV_CTRS * sizeof(int);

struct smg_ctx {
  int device;
  hipStream_t stream;       // the tape's stream: every entry point's work is ordered on it
  // look-ahead side stream of the blocked factorizations (created lazily);
  // work issued there is joined back into `stream` before the entry returns
  hipStream_t side;
  hipStream_t main_stream;  // saved while `stream` temporarily points at `side`
  std::vector<hipEvent_t> ev_pool;
  std::vector<hipEvent_t> ev_fork;  // smg_fork_event
  std::vector<hipEvent_t> marker_ev;  // smg_marker_record / smg_marker_wait (host pipelining)
  // device bump arena: blocks double in size (memory/stack_alloc.hpp:94-119)
  std::vector<smg_arena_block> blocks;
  size_t cur_block;
  size_t offset;  // within cur_block
  // status word (device) + pinned host mirror
  int* status_d;
  int* status_h;
  int host_status;  // host-detected errors (OOM, HIP)
  // set when a launch that can latch the status word (the persistent solves
  // and panels: SMG_ERR_SYNC on a timed-out hand-off) is enqueued; cleared
  // when the status is read (smg_status / smg_status_enqueue)
  int status_armed;
  // status mark (smg_cholesky_fwd_checked_mark / smg_status_mark_wait): the
  // status word copied into status_h[1] and reset at a point inside an entry,
  // with an event the host waits on instead of the whole stream
  hipEvent_t status_ev;
  int status_mark;
  // zeroing stream (smg_memset_async / smg_join_async): large adjoint buffers
  // are cleared there, overlapping the forward pass, and joined into `stream`
  // before the reverse sweep
  hipStream_t zero_stream;
  // the streamed factor's panel packs and device->host copies (created on
  // first use): off the zeroing stream, whose block-row chain the side
  // stream's K^{-1} shares and with them the trailing updates wait for
  hipStream_t copy_stream;
  hipEvent_t zero_ev_main, zero_ev_done;
  int zero_pending;
  // zeroings requested but not yet issued: they are issued at the next
  // latency-bound entry (the Cholesky panels, the persistent solves) so they
  // overlap those rather than the HBM-bound element-wise kernels before them,
  // and at the latest by smg_join_async / an arena rewind (smg_zero_flush)
  std::vector<std::pair<void*, size_t>> zero_queue;
  // smg_cholesky_inv_t_async: L^{-T} formed on `side` while the main stream
  // runs the (latency-bound) MVN solves; `inv_ev` is recorded after it and
  // joined into `stream` by smg_cholesky_mvn_rev_v or smg_join_async
  hipEvent_t inv_ev, inv_ev_main, inv_ev_aux;
  int inv_pending;
  // W = L^{-1} complete (all block rows) for the latest progressive
  // factorisation; each recording first waits for the previous one, so
  // waiting on it covers every earlier factorisation's W too
  hipEvent_t inv_ev_w;
  int inv_w_recorded;
  // cross-workgroup flags of the persistent panel kernels (device, zeroed at
  // creation; a launch's flags count as set when they hold its epoch)
  int* flags_d;
  int flag_epoch;
  // k_inv_block512 (cholesky.hip): a ring of monotonic grid-barrier counters
  // after the flags, and the launches issued so far (slot = launch % ring)
  unsigned* inv_ctr_d;
  long long inv_launches;
  int inv_per_cu, inv_cus;  // k_inv_block512's occupancy per CU and the CUs (-1: not yet queried)
  int inv_mode;      // 1: the block inverses by the six-launch chain (smg_set_inv_block_mode, a test hook)
  // pinned host scratch
  void* host_scratch;
  size_t host_scratch_size;
  // zero-copy io: pinned, host-coherent memory the kernels of the latency-
  // bound entries (smg_normal_lpdf_fused) read and write directly, plus the
  // completion word they publish (host spins on it instead of a stream sync)
  void* pin_io;
  size_t pin_io_size;
  void* res_h;           // fine-grained pinned results (smg_pinned_result)
  size_t res_h_size;
  long long* done_h;     // host-coherent completion word
  long long done_seq;
  unsigned int* red_counter_d;  // last-block-done counter of the fused reductions (device, self-resetting)
  // persistent device workspaces (grow on demand; NOT arena-managed)
  double* ws[12];  // SMG_WS_COUNT
  size_t ws_doubles[12];
  // profiling
  int prof_on;
  std::vector<smg_prof_slot> prof_pending;
  std::vector<hipEvent_t> prof_pool;
  double prof_ms[SMG_FAM_COUNT];
  double prof_flops[SMG_FAM_COUNT];
  long long prof_count[SMG_FAM_COUNT];
  // RCCL communicator (opaque)
  void* comm;
};

// latch helpers
#define SMG_HIP_TRY(expr)                          \
  do {                                             \
    hipError_t _e = (expr);                        \
    if (_e != hipSuccess) {                        \
      if (ctx) ctx->host_status |= SMG_ERR_HIP;    \
      return SMG_ERR_HIP;                          \
    }                                              \
  } while (0)

#define SMG_LAUNCH_CHECK()                         \
  do {                                             \
    hipError_t _e = hipGetLastError();             \
    if (_e != hipSuccess) {                        \
      ctx->host_status |= SMG_ERR_HIP;             \
      return SMG_ERR_HIP;                          \
    }                                              \
  } while (0)

// profiling scope: records events around a region of launches on ctx->stream
struct smg_prof_scope {
  smg_ctx* ctx;
  int fam;
  hipEvent_t a, b;
  bool on;
  smg_prof_scope(smg_ctx* c, int f);
  ~smg_prof_scope();
};

// named persistent workspaces (grow on demand; a growth synchronises the
// stream, so steady-state evaluations never reallocate)
enum { SMG_WS_GEMM = 0, SMG_WS_RED = 1, SMG_WS_TMP = 2, SMG_WS_TMP2 = 3, SMG_WS_ALIAS = 4,
       SMG_WS_GEMM_SIDE = 5, SMG_WS_INV = 6, SMG_WS_CW = 7, SMG_WS_RHS = 8,
       SMG_WS_GLM = 9,  // the GLM parameters [alpha, beta] (not the Cholesky aux's TMP2)
       SMG_WS_GEMM_ZERO = 10,  // split-K slabs of the GEMMs on the zeroing stream
       SMG_WS_MVN = 11,        // the tile partials of the MVN's passes over W = L^{-1} (mvn_inv.hip)
       SMG_WS_COUNT = 12 };
static_assert(SMG_WS_COUNT == sizeof(((smg_ctx*)nullptr)->ws) / sizeof(double*), "workspace slots");
double* smg_ws(smg_ctx* ctx, int id, size_t doubles);
// spin on the host-coherent completion word until it reaches seq (then the
// stream sync as a bounded fallback)
extern "C" int smg_wait_done(smg_ctx* ctx, long long seq);

// side-stream helpers (ctx.hip): events come from a per-context pool
int smg_side_begin(smg_ctx* ctx);          // ensure `side` exists
int smg_inv_events(smg_ctx* ctx);          // ensure the inv_ev* events exist
hipEvent_t smg_event(smg_ctx* ctx, int i); // i-th pooled event (grown on demand)
// i-th event of a second pool, for the fork / join pairs of the products that
// run two independent launches on the main and side streams at once (their
// indices never meet chol_fwd's, which grow with the panel count)
hipEvent_t smg_fork_event(smg_ctx* ctx, int i);
// RAII: issue the enclosed launches on the side stream
struct smg_on_side {
  smg_ctx* ctx;
  explicit smg_on_side(smg_ctx* c) : ctx(c) {
    ctx->main_stream = ctx->stream;
    ctx->stream = ctx->side;
  }
  ~smg_on_side() { ctx->stream = ctx->main_stream; }
};

// chol_mvn.hip: K^{-1} for the closed-form reverse formed progressively
// during the factorisation, block row k of W = L^{-1} once panel k is final
// (queued by chol_fwd on `side`); ws: smg_cholesky_mvn_rev_ws_doubles(n)
bool smg_inv_prog_ok(int n);
int smg_inv_prog_init(smg_ctx* ctx, int n, double* ws);
// part 0..3 of block row k (W_kk, W_{k,0:k}, the K^{-1} share, Y_{k+1});
// inverses_here: part 0 forms the block row's 128/256/512 inverses first,
// then records inv_ev_aux.  smg_inv_prog_cost: its device time estimate, us.
int smg_inv_prog_row(smg_ctx* ctx, const double* L, int ldl, double* aux, int n, double* ws, int k, int part,
                     bool inverses_here);
double smg_inv_prog_cost(int n, int k, int part, bool inverses_here);
// block inverses of the rows [row0, row0 + nrows) (multiples of 512), T: a
// workspace (NULL: SMG_WS_TMP); Wout (ld n, may be NULL): the 512-level
// block also written there when one launch forms it (*wrote)
int smg_block_inverses_rows(smg_ctx* ctx, const double* L, int ldl, double* aux, int n, int row0, int nrows,
                            double* T, double* Wout = nullptr, bool* wrote = nullptr);
// C = beta C (lower != 0: lower triangle only)
int smg_scale_impl(smg_ctx* ctx, int m, int n, double beta, double* C, int ldc, int lower);

// blocked triangular helpers (tri.hip, trsv.hip)
// B <- op(tri(A))^{-1} B in place; or, with X, X <- op(tri(A))^{-1} B out of
// place (B is then the right-hand side's workspace, overwritten): each
// block's X_p = W_p R_p is written straight to X, no in-place copy-back
int smg_trsm_impl(smg_ctx* ctx, int lower, int trans, const double* A, int lda, const double* W,
                  int ldw, double* B, int ldb, int m, int n, double* X = nullptr, int ldx = 0,
                  const double* aux = nullptr);
// B (n x n) += S, S symmetric with only its upper triangle stored
extern "C" int smg_add_sym_from_upper(smg_ctx* ctx, int n, const double* S, int lds, double* B, int ldb);
int smg_copy_impl(smg_ctx* ctx, int m, int n, const double* A, int lda, double* B, int ldb,
                  double alpha, int accumulate);
int smg_status_mark_impl(smg_ctx* ctx);
// zero `count` device ranges (pointer, bytes) on `stream`: batched launches of
// one kernel (ranges of doubles on 16 bytes), the runtime fill otherwise (ctx.hip)
int smg_zero_ranges_impl(smg_ctx* ctx, hipStream_t stream, const std::pair<void*, size_t>* r, int count,
                         unsigned max_grid = 2048);
// device -> host copy of `bytes` on `stream` (ctx.hip)
extern "C" int smg_d2h_impl(smg_ctx* ctx, hipStream_t stream, void* dst, const void* src, size_t bytes);
// issue the queued smg_memset_async zeroings on the zeroing stream (ctx.hip)
extern "C" int smg_zero_flush(smg_ctx* ctx);
// ensure the zeroing stream (also the device->host stream of the streamed
// Cholesky output) and host-pipelining marker `slot` exist (ctx.hip)
extern "C" int smg_zero_stream_begin(smg_ctx* ctx);
extern "C" int smg_marker_event(smg_ctx* ctx, int slot, hipEvent_t* ev);
// dst[tril_off(n, j) + i - j] = A(i, j) for j in [j0, j1), i >= j (matrix_util.hip)
extern "C" int smg_pack_tril_cols(smg_ctx* ctx, int n, const double* A, int lda, int j0, int j1, double* dst);
int smg_trtri_blocks_impl(smg_ctx* ctx, const double* L, int ldl, int n, double* W);
int smg_block_inverses_impl(smg_ctx* ctx, const double* L, int ldl, double* aux, int n);
int smg_trsv_lower_impl(smg_ctx* ctx, int trans, const double* L, int ldl, const double* W64,
                        const double* W256, const double* W512, int ldw, const double* x, double* y,
                        double* r, int n);

// internal GEMM entry used by other units (no argument re-validation).
// tri: triangular operands (SMG_TRI_* bits of smg_hip.h, in op() orientation);
// every tile's K loop is cut to the range where both operands can be nonzero
// (the caller guarantees stored zeros outside each triangle)
int smg_gemm_impl(smg_ctx* ctx, int transA, int transB, int uplo, int m, int n,
                  int k, double alpha, const double* A, int lda, const double* B,
                  int ldb, double beta, double* C, int ldc, int tri = 0);
// the same with beta taken as 0 from row bz (bz > 0) / column -bz (bz < 0) of C on
int smg_gemm_bz_impl(smg_ctx* ctx, int ta, int tb, int uplo, int m, int n, int k, double alpha, const double* A,
                     int lda, const double* B, int ldb, double beta, double* C, int ldc, int tri, int bz);

// C = alpha op(A) op(B) + beta C and C2 = tril(C) with halved diagonal (one pass)
int smg_gemm_dual_impl(smg_ctx* ctx, int ta, int tb, int m, int n, int k, double alpha, const double* A, int lda,
                       const double* B, int ldb, double beta, double* C, int ldc, double* C2, int ldc2,
                       int tri = 0);

// C = alpha op(A) op(B) + beta C symmetric (lower computed, stored mirrored)
// and P = Phi(C) (strict lower, halved diagonal; upper zero inside the
// diagonal 64-blocks only) (one pass, gemm.hip)
int smg_gemm_sym_phi_impl(smg_ctx* ctx, int ta, int tb, int n, int k, double alpha, const double* A, int lda,
                          const double* B, int ldb, double beta, double* C, int ldc, double* P, int ldp, int tri);

int smg_gemm_batched_impl(smg_ctx* ctx, int ta, int tb, int m, int n, int k, double alpha,
                          const double* A, int lda, long long sA, const double* B, int ldb,
                          long long sB, double beta, double* C, int ldc, long long sC, int batch);

// deterministic device reductions: out[0] (+)= sum of per-block partials
// partial layout: nparts doubles (or nparts x width for vector partials)
void smg_reduce_partials(smg_ctx* ctx, const double* partials, int nparts,
                         int width, double* out, int accumulate);

static inline int smg_ceil_div(long long a, long long b) { return (int)((a + b - 1) / b); }

// wave (64-lane) reductions
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
  return v;
}

// block-wide sum of one value per thread (blockDim.x multiple of 64, <= 1024)
// fixed order => deterministic
__device__ __forceinline__ double block_sum(double v, double* lds /* >= 16 */) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) lds[w] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0)
    for (int i = 0; i < nw; ++i) s += lds[i];
  return s;  // valid in thread 0 only
}

// grid-stride walk over a column-major m x n index space: (i, j) advance by
// the grid stride with one compare instead of a 64-bit division per element
// (a division per element cost element-wise passes ~40% of their bandwidth)
struct smg_mn {
  long long e, tot;
  int i, j, m, si, sj, st;
  __device__ __forceinline__ smg_mn(int m_, int n_) : m(m_) {
    tot = (long long)m_ * n_;
    e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    st = gridDim.x * blockDim.x;
    j = m_ > 0 ? (int)(e / m_) : 0;
    i = m_ > 0 ? (int)(e - (long long)j * m_) : 0;
    sj = m_ > 0 ? st / m_ : 0;
    si = st - sj * m_;
  }
  __device__ __forceinline__ bool ok() const { return e < tot; }
  __device__ __forceinline__ void next() {
    e += st;
    i += si;
    j += sj;
    if (i >= m) {
      i -= m;
      ++j;
    }
  }
};
