// cholesky_decompose forward and Murray's blocked reverse on MI355X.
//
// Reference: stan/math/rev/mat/fun/cholesky_decompose.hpp
//   forward  :378-392  (check_symmetric, Eigen LLT, check_pos_definite)
//   reverse  :118-165  (cholesky_block::chain, Murray 2016)
//
// Forward: right-looking blocked factorisation with SMG_NB = 64 diagonal
// blocks.  Per block: one workgroup factors the diagonal block in LDS and
// writes both L11 and its inverse (kept in Dinv for TRSM / TRSV / reverse);
// the panel L21 = A21 L11^{-T} and the trailing SYRK A22 -= L21 L21^T run on
// the fp64 MFMA GEMM (lower-triangle tiles only).
//
// Reverse: the same block partition walked backwards.  With R, D, B, C the
// blocks left of / on / below-left of / below the diagonal block:
//   C_adj = C_adj D^{-1};  B_adj -= C_adj R;  D_adj -= C_adj^T C
//   D_adj = D^{-T} sym(D^T tril(D_adj)) D^{-1}          (symbolic_rev, :101-111)
//   R_adj -= C_adj^T B + sym(D_adj) R;  D_adj: diag *= 1/2, strict upper = 0
// The partition differs from the reference's bottom-aligned block_size_ only
// in where the block seams fall; Murray's recurrence is exact for any
// partition, so results agree to round-off.  Aadj(lower) += L_adj(lower).
#include <chrono>
#include "smg_internal.h"
#include "tri_small.h"
#include "smg_sync.h"
#include <cstdlib>
#include <vector>

namespace {

// one 64 x 64 tile pair per workgroup: tile (bi, bj) of the lower triangle
// and its mirror (bj, bi), both read coalesced (column segments), the mirror
// transposed through LDS; every element is read once
__global__ __launch_bounds__(256) void k_check_symmetric(const double* __restrict__ A, int lda,
                                                         int n, int* status) {
  // CONSTRAINT_TOLERANCE = 1e-8 absolute (prim/mat/err/constraint_tolerance.hpp:12)
  __shared__ double T[64][65];
  int bi, bj;
  {  // blockIdx.x -> (bi, bj), bj <= bi, row-major over the lower triangle
    const int t = blockIdx.x;
    int r = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
    while ((r + 1) * (r + 2) / 2 <= t) ++r;
    while (r * (r + 1) / 2 > t) --r;
    bi = r;
    bj = t - r * (r + 1) / 2;
  }
  const int i0 = 64 * bi, j0 = 64 * bj;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // mirror tile: rows j0.., cols i0.. -> T[c][r] = A(j0 + r, i0 + c)
  for (int c = w; c < 64; c += 4) {
    const int gr = j0 + lane, gc = i0 + c;
    T[c][lane] = (gr < n && gc < n) ? A[gr + (size_t)gc * lda] : 0.0;
  }
  __syncthreads();
  bool bad = false;
  for (int c = w; c < 64; c += 4) {  // A(i0 + lane, j0 + c) vs A(j0 + c, i0 + lane) = T[lane][c]
    const int gr = i0 + lane, gc = j0 + c;
    if (gr < n && gc < n && gr > gc)
      // !(|d| <= tol) so that NaN entries fail too (check_symmetric.hpp:45-46)
      bad |= !(fabs(A[gr + (size_t)gc * lda] - T[lane][c]) <= 1e-8);
  }
  if (__any(bad) && lane == 0) atomicOr(status, (int)SMG_ERR_NOT_SYMMETRIC);
}

// k_check_symmetric fused with the copy of A's lower triangle into L (zeros
// above): one pass over A instead of two.  Tile pair (bi, bj), bj <= bi:
// L's lower tile (bi, bj) from A's, L's upper tile (bj, bi) zero.
__global__ __launch_bounds__(256) void k_check_symmetric_copy(const double* __restrict__ A, int lda,
                                                              int n, int* status,
                                                              double* __restrict__ L, int ldl) {
  __shared__ double T[64][65];
  int bi, bj;
  {
    const int t = blockIdx.x;
    int r = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
    while ((r + 1) * (r + 2) / 2 <= t) ++r;
    while (r * (r + 1) / 2 > t) --r;
    bi = r;
    bj = t - r * (r + 1) / 2;
  }
  const int i0 = 64 * bi, j0 = 64 * bj;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int c = w; c < 64; c += 4) {
    const int gr = j0 + lane, gc = i0 + c;
    T[c][lane] = (gr < n && gc < n) ? A[gr + (size_t)gc * lda] : 0.0;
  }
  __syncthreads();
  bool bad = false;
  for (int c = w; c < 64; c += 4) {
    const int gr = i0 + lane, gc = j0 + c;
    if (gr < n && gc < n) {
      const double a = A[gr + (size_t)gc * lda];
      if (gr > gc) bad |= !(fabs(a - T[lane][c]) <= 1e-8);
      L[gr + (size_t)gc * ldl] = gr >= gc ? a : 0.0;
    }
    if (bi != bj && j0 + lane < n && i0 + c < n) L[(j0 + lane) + (size_t)(i0 + c) * ldl] = 0.0;
  }
  if (__any(bad) && lane == 0) atomicOr(status, (int)SMG_ERR_NOT_SYMMETRIC);
}

// The same pass for n % 64 == 0 with 16-byte aligned columns: each lane moves
// two rows per 16-byte access, and all sixteen loads of a lane (eight from the
// mirror tile U = A[j0.., i0..], eight from the tile itself) are issued before
// the first use.  U(r, c) sits in LDS at c*64 + (r ^ (c & 62)): the 16-byte
// stores of a column and the transposed reads of a row are both bank-spread.
__global__ __launch_bounds__(256) void k_check_symmetric_copy2(const double* __restrict__ A,
                                                               int lda, int n, int* status,
                                                               double* __restrict__ L, int ldl) {
  __shared__ double T[64 * 64];
  int bi, bj;
  {
    const int t = blockIdx.x;
    int r = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
    while ((r + 1) * (r + 2) / 2 <= t) ++r;
    while (r * (r + 1) / 2 > t) --r;
    bi = r;
    bj = t - r * (r + 1) / 2;
  }
  const int i0 = 64 * bi, j0 = 64 * bj;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int rr = 2 * (lane & 31), cb = 2 * w + (lane >> 5);
  double2 u[8], a[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int c = 8 * p + cb;
    u[p] = *reinterpret_cast<const double2*>(A + (j0 + rr) + (size_t)(i0 + c) * lda);
  }
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int c = 8 * p + cb;
    a[p] = *reinterpret_cast<const double2*>(A + (i0 + rr) + (size_t)(j0 + c) * lda);
  }
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int c = 8 * p + cb;
    *reinterpret_cast<double2*>(&T[c * 64 + (rr ^ (c & 62))]) = u[p];
  }
  __syncthreads();
  bool bad = false;
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int c = 8 * p + cb;
    const int gc = j0 + c;
    const double t0 = T[rr * 64 + (c ^ rr)], t1 = T[(rr + 1) * 64 + (c ^ rr)];
    double2 v = a[p];
    if (i0 + rr > gc) bad |= !(fabs(v.x - t0) <= 1e-8);
    if (i0 + rr + 1 > gc) bad |= !(fabs(v.y - t1) <= 1e-8);
    if (i0 + rr < gc) v.x = 0.0;
    if (i0 + rr + 1 < gc) v.y = 0.0;
    *reinterpret_cast<double2*>(L + (i0 + rr) + (size_t)gc * ldl) = v;
    if (bi != bj)
      *reinterpret_cast<double2*>(L + (j0 + rr) + (size_t)(i0 + c) * ldl) = make_double2(0.0, 0.0);
  }
  if (__any(bad) && lane == 0) atomicOr(status, (int)SMG_ERR_NOT_SYMMETRIC);
}

__global__ void k_copy_lower(const double* __restrict__ A, int lda, int n,
                             double* __restrict__ L, int ldl) {
  for (smg_mn it(n, n); it.ok(); it.next()) {
    const long long e = it.e;
    const int i = it.i, j = it.j;
    L[i + (size_t)j * ldl] = (i >= j) ? A[i + (size_t)j * lda] : 0.0;
  }
}

__global__ void k_add_lower(const double* __restrict__ X, int ldx, int n,
                            double* __restrict__ Y, int ldy) {
  for (smg_mn it(n, n); it.ok(); it.next()) {
    const long long e = it.e;
    const int i = it.i, j = it.j;
    if (i >= j) Y[i + (size_t)j * ldy] += X[i + (size_t)j * ldx];
  }
}

// k_add_lower in the column form (16-byte accesses, whole columns per
// workgroup, only the row pairs at or below the diagonal touched)
__global__ __launch_bounds__(256) void k_add_lower_col2(const double* __restrict__ X, int ldx, int n,
                                                        double* __restrict__ Y, int ldy) {
  const int np = n >> 1;
  for (int j = blockIdx.x; j < n; j += gridDim.x) {
    const double2* x = reinterpret_cast<const double2*>(X + (size_t)j * ldx);
    double2* y = reinterpret_cast<double2*>(Y + (size_t)j * ldy);
    const int p1 = j >> 1;  // first pair holding a row >= j
    for (int p0 = p1 + threadIdx.x; p0 < np; p0 += 4 * 256) {
      double2 a[4], b[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int p = p0 + 256 * k;
        if (p < np) {
          a[k] = x[p];
          b[k] = y[p];
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int p = p0 + 256 * k;
        if (p < np) {
          if (2 * p >= j) b[k].x += a[k].x;
          b[k].y += a[k].y;  // row 2p + 1 >= j for every p >= j / 2
          y[p] = b[k];
        }
      }
    }
  }
}

// factor the diagonal block in place and write its inverse (dense, upper
// zeros, so GEMMs may read it as a plain matrix); ONE wave
__global__ __launch_bounds__(512) void k_potrf_diag(double* __restrict__ L, int ldl, int b,
                                                    double* __restrict__ Dinv, int ldd,
                                                    int* status) {
  __shared__ double D[SMG_NB * SMG_NBP];
  __shared__ double X[SMG_NB * SMG_NBP];
  lds_load_block(D, L, ldl, b, true);
  __syncthreads();
  lds_potrf_inv64_blk(D, X, b, L, ldl, Dinv, ldd, status, true);
}

// ---------------------------------------------------------------------------
// Persistent panel factorisation: ONE launch factors a panel of up to
// PANEL_MAX_STEPS diagonal blocks (columns [J, K), all rows below), where the
// blocked loop above would issue potrf / TRSM / trapezoid-update launches
// per 64-column step.  Workgroup 0 is the diagonal chain; row tile t >= 1
// (64 rows from J + 64 t in the panel, 32-row tiles below it: panel_tiles)
// belongs to workgroup 2 + (t - 1) mod (gown - 2)
// (workgroup 1 inverts the factored diagonal blocks),
// which applies every step's update to it, so the only cross-workgroup
// dependencies are
//   * the factored diagonal block j (L_jj, which every tile solves against): flag diag[j];
//   * the panel-region rows L_cj (c < nb) that update tile t's column block c:
//     flag row[j][c];
//   * tile j + 2's step-j updates, which the chain's step j + 1 reads:
//     flag done[j][j + 2].
// A workgroup only ever waits on tiles c < nb <= 8 owned by workgroups
// 0 .. 7, which are dispatched first, so the grid needs no co-residency.  The
// critical path per step is the next diagonal tile's own L_tj + A_tt update
// (two 64^3 LDS products) and its factorisation; the other tiles' updates
// overlap it.  Flags carry the launch's epoch (no reset launch); every wait
// gives up after ~4 s and latches SMG_ERR_SYNC so a protocol fault can never
// hang the device.
constexpr int PANEL_MAX_STEPS = 8;
constexpr int PANEL_MAX_GRID = 256;
constexpr int PANEL_BELOW_ROWS = 32;  // row tiles below the panel (panel_tiles)

// dev instrumentation (tools/ubench_panel.hip): per-workgroup event log of
// (s_memrealtime, code); compiled out of the library
#ifdef SMG_PANEL_TRACE
__device__ unsigned long long g_panel_trace[PANEL_MAX_GRID * 128];
__device__ int g_panel_trace_n[PANEL_MAX_GRID];
#define PANEL_EV(code)                                                              \
  if (threadIdx.x == 0) {                                                           \
    const int k_ = g_panel_trace_n[blockIdx.x]++;                                   \
    if (k_ < 64) {                                                                  \
      g_panel_trace[blockIdx.x * 128 + 2 * k_] = __builtin_amdgcn_s_memrealtime(); \
      g_panel_trace[blockIdx.x * 128 + 2 * k_ + 1] = (code);                        \
    }                                                                               \
  }
#else
#define PANEL_EV(code)
#endif

// dev instrumentation (tools/ubench_timeline.cpp): device-clock start / end
// of every panel launch (slot = epoch mod 64) and host-placed stamps, to see
// the panels' gaps inside a whole evaluation without a profiler (which
// serialises dispatches); compiled out of the library
#ifdef SMG_PANEL_TIMELINE
__device__ unsigned long long g_panel_tl[3 * 64];
struct panel_tl_end {
  int e;
  __device__ ~panel_tl_end() {
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(&g_panel_tl[2 * (e & 63) + 1], __builtin_amdgcn_s_memrealtime());
  }
};
#define PANEL_TL()                                                                               \
  if (blockIdx.x == 0 && threadIdx.x == 0) g_panel_tl[2 * (epoch & 63)] = __builtin_amdgcn_s_memrealtime(); \
  panel_tl_end tl_end_{epoch};
__global__ void k_tl_stamp(int slot) {
  if (threadIdx.x == 0) g_panel_tl[128 + slot] = __builtin_amdgcn_s_memrealtime();
}
// host steady-clock time (us) of each panel launch call, by epoch
double g_panel_host_us[64];
static inline void panel_host_stamp(int epoch) {
  g_panel_host_us[epoch & 63] =
      std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
extern "C" void smg_dev_timeline_host(double* out) {
  for (int i = 0; i < 64; ++i) out[i] = g_panel_host_us[i];
}
extern "C" int smg_dev_timeline(smg_ctx* ctx, int stamp_slot, unsigned long long* out) {
  if (stamp_slot >= 0) {
    hipLaunchKernelGGL(k_tl_stamp, dim3(1), dim3(64), 0, ctx->stream, stamp_slot & 63);
    return 0;
  }
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_panel_tl), sizeof(g_panel_tl)) == hipSuccess ? 0 : SMG_ERR_HIP;
}
#else
#define PANEL_TL()
static inline void panel_host_stamp(int) {}
#endif

// hand-off primitives (st_dev / panel_publish / panel_wait): smg_sync.h

// The chain's LDS phases out of line: each compiles with its own register
// budget instead of under the whole kernel's pressure (228 VGPRs, ~110 SGPR
// spills inlined); the LDS pointers are typed address_space(3) so the
// callees keep ds_ instructions (a generic pointer would turn them into flat
// accesses).  Same arithmetic in the same order as inlined.
typedef __attribute__((address_space(3))) double lds_dbl;
// the chain's factorisation: 8-column panels whose pivots are taken two at a
// time (wave_factor8_pair2: the 2 x 2 leading minors' two roots side by side,
// rsq_h roots, the later columns updated with the factor's own entries
// broadcast from the lanes that form them)
__device__ __noinline__ void chain_factor(lds_dbl* D, int* status) { lds_potrf64_v3<3, false>(D, status); }
// the chain's leaves also stored (sc1) into the diagonal 16 x 16 blocks of
// Dinv_j (G = Dinv + cj, ld ldg; the inverter later writes the same bits
// there), published with diag[j]: the panel tiles load them instead of
// recomputing them
__device__ __noinline__ void chain_leaves_pub(const lds_dbl* D, lds_dbl* X, double* G, int ldg, int b) {
  const int w = threadIdx.x >> 6;
  if (w >= 4) return;
  trtri_leaf16(D, X, w);
  leaf16_store((const lds_dbl*)X, G, ldg, b, w);
}
// the chain's global work beside its leaf inverses, by waves 4-7 (256
// threads; waves 0-3 form the leaves): L_jj stored (lower, zeros above),
// then -- when a next tile follows -- its operands A_{t,j} and A_tt loaded
// (each wave polls the owner's done flag itself: no barrier with the leaf
// waves) and staged into Y and Zn; all of it hidden under the leaves, which
// had run with these four waves idle (the stores, the loads and their LDS
// staging had been 2 us of each chain step)
__device__ __noinline__ void chain_side(const lds_dbl* Dc, lds_dbl* Y, lds_dbl* Zn, double* L, int ldl, int cj,
                                        int bj, int rt0, int rt, int bt, int more, const int* flag, int epoch,
                                        int* status) {
  const int tid = (int)threadIdx.x - 256;
  double ra[16], rz[16];
  unsigned oka = 0, okz = 0;
  if (more) {  // the loads first (their latency is the long pole), then L_jj's stores under them
    if (flag && (threadIdx.x & 63) == 0) {
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > 400000000ull) {
          atomicOr(status, (int)SMG_ERR_SYNC);
          break;
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int e = tid + 256 * q;
      const int c = e >> 6, r = e & 63;
      ra[q] = ld_dev(&L[rt0 + min(r, rt - 1) + (size_t)(cj + min(c, bj - 1)) * ldl]);
      rz[q] = ld_dev(&L[rt0 + min(r, bt - 1) + (size_t)(rt0 + min(c, bt - 1)) * ldl]);
      oka |= (r < rt && c < bj) ? (1u << q) : 0u;
      okz |= (r < bt && c < bt && r >= c) ? (1u << q) : 0u;
    }
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int e = tid + 256 * q;
    const int c = e >> 6, r = e & 63;
    if (r < bj && c < bj) st_dev(&L[cj + r + (size_t)(cj + c) * ldl], r >= c ? Dc[r * SMG_NBP + c] : 0.0);
  }
  if (!more) return;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int e = tid + 256 * q;
    const int c = e >> 6, r = e & 63;
    Y[r * SMG_NBP + c] = ((oka >> q) & 1u) ? ra[q] : 0.0;
    Zn[r * SMG_NBP + c] = ((okz >> q) & 1u) ? rz[q] : 0.0;
  }
}
__device__ __noinline__ void chain_trsm(lds_dbl* Y, const lds_dbl* D, const lds_dbl* X) { lds_trsm64_rt(Y, D, X); }
// X = L^{-1} (64 x 64) given its four 16 x 16 leaf inverses on X's diagonal
// blocks: lds_trtri64_mfma's phases p = 1..3 (the same arithmetic and order:
// the same bits); the blocks above the diagonal are not written (a
// triangle store writes zeros there); T: 3 x 256 doubles
__device__ __noinline__ void chain_last_inverse(const lds_dbl* D, lds_dbl* X, lds_dbl* T) {
  const int w = threadIdx.x >> 6;
  __syncthreads();  // the leaves in X complete (and Y free)
  for (int p = 1; p < 4; ++p) {
    if (w < p) {
      d4 acc = d4{0.0, 0.0, 0.0, 0.0}, acc2 = acc;
      trtri_t_acc(D, (const lds_dbl*)X, p, w, 16 * w, 16 * p, acc, acc2);
      trtri_t_store(T, w, acc, acc2);
    }
    __syncthreads();
    if (w < p) trtri_x_tile(X, T, p, w);
    __syncthreads();
  }
}
__device__ __noinline__ void chain_syrk(lds_dbl* Zn, const lds_dbl* Y, int b) { lds_syrk64_8w_next(Zn, Y, b); }
__device__ __noinline__ void owner_update(lds_dbl* Z, const lds_dbl* D, const lds_dbl* B) {
  lds_mma64_8w<false, true, lds_dbl*, const lds_dbl*>(Z, D, B, -1.0, 1.0);
}
#define CHAIN_FACTOR(D, st) chain_factor((lds_dbl*)(D), (st))
#define CHAIN_LEAVES_PUB(D, X, G, ldg, b) chain_leaves_pub((const lds_dbl*)(D), (lds_dbl*)(X), (G), (ldg), (b))
#define CHAIN_TRSM(Y, D, X) chain_trsm((lds_dbl*)(Y), (const lds_dbl*)(D), (const lds_dbl*)(X))
__device__ __noinline__ void below_trsm(lds_dbl* Y, const lds_dbl* D, const lds_dbl* X) {
  lds_trsm64_rt(Y, D, X, PANEL_BELOW_ROWS / 16);
}
__device__ __noinline__ void below_ltj(lds_dbl* Y, const lds_dbl* X) {
  lds_mma32_8w<lds_dbl*, const lds_dbl*>(Y, Y, X);
}
__device__ __noinline__ void below_update(lds_dbl* Z, const lds_dbl* D, const lds_dbl* B) {
  lds_mma32_8w<lds_dbl*, const lds_dbl*>(Z, D, B, -1.0, 1.0);
}
#define CHAIN_SYRK(Zn, Y, b) chain_syrk((lds_dbl*)(Zn), (const lds_dbl*)(Y), (b))

#define OWNER_UPDATE(Z, D, B) owner_update((lds_dbl*)(Z), (const lds_dbl*)(D), (const lds_dbl*)(B))
#define BELOW_LTJ(Y, X) below_ltj((lds_dbl*)(Y), (const lds_dbl*)(X))
#define BELOW_TRSM(Y, D, X) below_trsm((lds_dbl*)(Y), (const lds_dbl*)(D), (const lds_dbl*)(X))
#define BELOW_UPDATE(Z, D, B) below_update((lds_dbl*)(Z), (const lds_dbl*)(D), (const lds_dbl*)(B))

// rows x cols block of a col-major matrix -> registers (8 per thread, 512
// threads); branch-free: clamped addresses, out-of-range (and, with lower,
// strict-upper) elements masked at the LDS store
struct panel_regs {
  double v[8];
  unsigned ok;
};
// R = 64: a 64-row tile (8 elements per thread); R = 32: the 32-row tiles
// below the panel (4 per thread), rows 0 .. 31 of the same LDS layout
template <int R = 64>
__device__ inline void panel_gload(panel_regs& Rg, const double* A, int ld, int rows, int cols,
                                   bool lower) {
  Rg.ok = 0;
#pragma unroll
  for (int q = 0; q < R / 8; ++q) {
    const int e = threadIdx.x + SMG_DIAG_THREADS * q;
    const int c = e / R, r = e % R;
    Rg.v[q] = ld_dev(&A[min(r, rows - 1) + (size_t)min(c, cols - 1) * ld]);  // handed-off data: sc1
    Rg.ok |= (r < rows && c < cols && (!lower || r >= c)) ? (1u << q) : 0u;
  }
}
template <int R = 64, typename P = double*>
__device__ inline void panel_lstore(P D, const panel_regs& Rg) {
#pragma unroll
  for (int q = 0; q < R / 8; ++q) {
    const int e = threadIdx.x + SMG_DIAG_THREADS * q;
    D[(e % R) * SMG_NBP + e / R] = ((Rg.ok >> q) & 1u) ? Rg.v[q] : 0.0;
  }
}
template <int R = 64, typename CP = const double*>
__device__ inline void panel_gstore(CP D, double* A, int ld, int rows, int cols,
                                    bool lower) {
#pragma unroll
  for (int q = 0; q < R / 8; ++q) {
    const int e = threadIdx.x + SMG_DIAG_THREADS * q;
    const int c = e / R, r = e % R;
    if (r < rows && c < cols && (!lower || r >= c)) st_dev(&A[r + (size_t)c * ld], D[r * SMG_NBP + c]);
  }
}
// the 4 diagonal 16 x 16 leaf inverses of Dinv_j (G, ld ldg; identity
// beyond b, as the chain's identity-padded factor gives them) into the
// diagonal blocks of Y (2 per thread; r fastest: 128-byte column runs)
struct panel_leaves {
  double v[2];
};
__device__ inline void panel_gload_leaves(panel_leaves& Rg, const double* G, int ldg, int b) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int e = threadIdx.x + SMG_DIAG_THREADS * q;
    const int w = e >> 8, c = (e >> 4) & 15, r = e & 15;
    const int i = 16 * w + r, j = 16 * w + c;
    const double v = ld_dev(&G[min(i, b - 1) + (size_t)min(j, b - 1) * ldg]);
    Rg.v[q] = (i < b && j < b) ? v : (i == j ? 1.0 : 0.0);
  }
}
template <typename P = double*>
__device__ inline void panel_lstore_leaves(P Y, const panel_leaves& Rg) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int e = threadIdx.x + SMG_DIAG_THREADS * q;
    const int w = e >> 8, c = (e >> 4) & 15, r = e & 15;
    Y[(16 * w + r) * SMG_NBP + 16 * w + c] = Rg.v[q];
  }
}

// a b x b lower triangle (loaded with lower = true) into LDS with identity
// padding beyond b: the factor's leaf inverses stay finite
template <typename P = double*>
__device__ inline void panel_lstore_id(P D, const panel_regs& R, int b) {
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int e = threadIdx.x + SMG_DIAG_THREADS * q;
    const int r = e & 63, c = e >> 6;
    D[r * SMG_NBP + c] = ((R.ok >> q) & 1u) ? R.v[q] : (r == c && r >= b ? 1.0 : 0.0);
  }
}
// b x b lower triangle of D with zeros above (the factored block / inverse)
__device__ inline void panel_gstore_tri(const double* D, double* A, int ld, int b) {
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int e = threadIdx.x + SMG_DIAG_THREADS * q;
    const int c = e >> 6, r = e & 63;
    if (r < b && c < b) st_dev(&A[r + (size_t)c * ld], r >= c ? D[r * SMG_NBP + c] : 0.0);
  }
}

// Row tiles of a panel: t < nb are the panel's 64-row tiles (rows J + 64 t),
// the rows below the panel come in 32-row tiles (rows J + 64 nb + 32 (t - nb)):
// their owners' seven column updates per step, not the chain, bounded the
// panel's end at 64 rows, and their rows are independent (no extra hand-off)
__host__ __device__ inline int panel_tiles(int n, int J, int nb) {
  const int below0 = J + SMG_NB * nb;
  return nb + (n > below0 ? (n - below0 + PANEL_BELOW_ROWS - 1) / PANEL_BELOW_ROWS : 0);
}

// column block c of panel tile t is updated by t's helper workgroup
// (round 6: two helpers per tile from t = 4 on -- A the odd, B the even
// column blocks c <= t - 2 -- so the owner keeps only c = t - 1 and its own
// diagonal block: the late tiles' owners had fallen ~10 us behind the chain
// over the first steps, which stalled it at step 5, where it needs tile 6)
// 0: the owner updates column block c of panel tile t; 1 / 2: helper A / B
__device__ __forceinline__ int panel_helper(int t, int c, int nb, int nha, int nhb) {
  if (t >= nb || c > t - 2 || c < 1) return 0;  // (block 0 takes no updates)
  if (c & 1) return (t >= 3 && t - 3 < nha) ? 1 : 0;
  return (t >= 4 && t - 4 < nhb) ? 2 : 0;
}

// A workgroup whose only tile t (>= nb) lies below the panel: every step of
// that tile with its column blocks held in registers for the whole panel (the
// accumulator layout of lds_mma32_8w: 4 doubles per lane per 32 x 64 block),
// loaded once; each step's update A_tc -= L_tj L_cj^T is subtracted from them
// in place, and block j goes out once, as L_tj -- instead of every later block
// being loaded and stored again at every step (the kernel fetched 2.6x and
// wrote 2.1x its algorithmic bytes).  Out of line, with the LDS products
// inlined: its own register budget (the resident blocks live across the steps).
__device__ __noinline__ void below_resident(double* __restrict__ L, int ldl, int n, int J, int K,
                                            double* __restrict__ Dinv, int ldd, int* flags, int epoch, int* status,
                                            int nb, int t, lds_dbl* D, lds_dbl* X, lds_dbl* Y) {
  constexpr int S = PANEL_MAX_STEPS;
  constexpr int R = PANEL_BELOW_ROWS;
  static_assert(R == 32, "the resident layout is lds_mma32_8w's");
  int* diag = flags;
  int* row = flags + S;
  int* dinvf = flags + S + 3 * S * S;
  const int rt0 = J + SMG_NB * nb + R * (t - nb), rt = min(R, n - rt0);
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ar = 16 * (w & 1) + (l >> 4), ac = 16 * (w >> 1) + (l & 15);  // + 4 q: this lane's rows
  double Rres[S][4];
#pragma unroll
  for (int c = 0; c < S; ++c) {  // the whole tile (final: rows are independent), once
    const int cc = J + SMG_NB * c, bc = min(SMG_NB, K - cc);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = ar + 4 * q;
      const bool in = c < nb && r < rt && ac < bc;
      const int col = c < nb ? cc + min(ac, bc - 1) : J;  // (clamped in range: loads are unconditional)
      const double v = ld_dev(&L[rt0 + min(r, rt - 1) + (size_t)col * ldl]);
      Rres[c][q] = in ? v : 0.0;
    }
  }
  for (int j = 0; j < nb; ++j) {
    const int cj = J + SMG_NB * j;
    const int bj = min(SMG_NB, K - cj);
    __syncthreads();  // LDS of the previous step fully consumed
    PANEL_EV((j << 16) | (t << 8) | 5);
#pragma unroll
    for (int c = 0; c < S; ++c)  // block j into D (its current A_tj)
      if (c == j)
#pragma unroll
        for (int q = 0; q < 4; ++q) D[(ar + 4 * q) * SMG_NBP + ac] = Rres[c][q];
    panel_regs Rd;
    if (j + 1 < nb) {
      panel_wait(&dinvf[j], epoch, status);
      PANEL_EV((j << 16) | (t << 8) | 6);
      panel_gload(Rd, Dinv + cj, ldd, bj, bj, true);
      panel_lstore(X, Rd);
      __syncthreads();
      lds_mma32_8w<lds_dbl*, const lds_dbl*>(D, D, X);  // L_tj = A_tj Dinv_j^T
    } else {  // the last step: solve against L_jj (the chain's end, not the inverter's, bounds it)
      panel_wait(&diag[j], epoch, status);
      PANEL_EV((j << 16) | (t << 8) | 6);
      panel_gload(Rd, L + cj + (size_t)cj * ldl, ldl, bj, bj, true);  // L_jj
      panel_leaves Rv;
      panel_gload_leaves(Rv, Dinv + cj, ldd, bj);  // the chain's leaf inverses
      panel_lstore_id(X, Rd, bj);
      panel_lstore_leaves(Y, Rv);
      __syncthreads();
      lds_trsm64_rt(D, (const lds_dbl*)X, (const lds_dbl*)Y, R / 16);
      __syncthreads();
    }
    panel_gstore<R>((const lds_dbl*)D, L + rt0 + (size_t)cj * ldl, ldl, rt, bj, false);
    PANEL_EV((j << 16) | (t << 8) | 7);
    if (j + 1 >= nb) break;
    panel_wait_all(row + j * S, j + 1, nb - 1, 1, epoch, status);
    panel_regs Ryn;
    auto issue = [&](int c) {
      const int cc = J + SMG_NB * c;
      panel_gload(Ryn, L + cc + (size_t)cj * ldl, ldl, min(SMG_NB, K - cc), bj, false);
    };
    issue(j + 1);
    for (int c = j + 1; c < nb; ++c) {
      __syncthreads();  // previous product's Y consumed
      panel_lstore(Y, Ryn);
      __syncthreads();
      if (c + 1 < nb) issue(c + 1);  // in flight during this product
      const d4 acc = lds_mma32_8w_acc((const lds_dbl*)D, (const lds_dbl*)Y);  // this wave's tile of L_tj L_cj^T
#pragma unroll
      for (int cr = 0; cr < S; ++cr)
        if (cr == c)
#pragma unroll
          for (int q = 0; q < 4; ++q) Rres[cr][q] -= acc[q];
      PANEL_EV((j << 16) | (t << 8) | (16 + c));
    }
  }
}

// below_resident for a PAIR of adjacent 32-row tiles (one 64-row band, rows
// rt0 ..): two resident sets in the same accumulator layout (rows 0-31 and
// 32-63 of D), L_tj for both by one 64-row product, each later update's L_cj
// loaded and staged once for both halves.  Half the workgroups of the rows
// below (the first panel: 56 instead of 112), each one CU held through the
// panel for little MFMA work; the freed CUs go to the trailing updates and
// the K^{-1} parts beside the panels.
__device__ __noinline__ void below_resident2(double* __restrict__ L, int ldl, int n, int J, int K,
                                             double* __restrict__ Dinv, int ldd, int* flags, int epoch, int* status,
                                             int nb, int rt0, int t, lds_dbl* D, lds_dbl* X, lds_dbl* Y,
                                             lds_dbl* Z) {
  constexpr int S = PANEL_MAX_STEPS;
  int* diag = flags;
  int* row = flags + S;
  int* dinvf = flags + S + 3 * S * S;
  const int rt = min(2 * PANEL_BELOW_ROWS, n - rt0);
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ar = 16 * (w & 1) + (l >> 4), ac = 16 * (w >> 1) + (l & 15);  // + 4 q (+ 32 for the second half)
  double Ra[S][4], Rb[S][4];
#pragma unroll
  for (int c = 0; c < S; ++c) {  // the whole band (final: rows are independent), once
    const int cc = J + SMG_NB * c, bc = min(SMG_NB, K - cc);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = ar + 4 * q, r2 = r + 32;
      const int col = c < nb ? cc + min(ac, bc - 1) : J;
      const double va = ld_dev(&L[rt0 + min(r, rt - 1) + (size_t)col * ldl]);
      const double vb = ld_dev(&L[rt0 + min(r2, rt - 1) + (size_t)col * ldl]);
      Ra[c][q] = (c < nb && r < rt && ac < bc) ? va : 0.0;
      Rb[c][q] = (c < nb && r2 < rt && ac < bc) ? vb : 0.0;
    }
  }
  for (int j = 0; j < nb; ++j) {
    const int cj = J + SMG_NB * j;
    const int bj = min(SMG_NB, K - cj);
    __syncthreads();  // LDS of the previous step fully consumed
    PANEL_EV((j << 16) | (t << 8) | 5);
#pragma unroll
    for (int c = 0; c < S; ++c)  // block j of both halves into D (its current A_tj)
      if (c == j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          D[(ar + 4 * q) * SMG_NBP + ac] = Ra[c][q];
          D[(32 + ar + 4 * q) * SMG_NBP + ac] = Rb[c][q];
        }
    panel_regs Rd;
    if (j + 1 < nb) {
      panel_wait(&dinvf[j], epoch, status);
      PANEL_EV((j << 16) | (t << 8) | 6);
      panel_gload(Rd, Dinv + cj, ldd, bj, bj, true);
      panel_lstore(X, Rd);
      __syncthreads();
      lds_mma64_8w<false, true, lds_dbl*, const lds_dbl*>(D, D, X);  // L_tj = A_tj Dinv_j^T (64 rows)
    } else {  // the last step: solve against L_jj
      panel_wait(&diag[j], epoch, status);
      PANEL_EV((j << 16) | (t << 8) | 6);
      panel_gload(Rd, L + cj + (size_t)cj * ldl, ldl, bj, bj, true);  // L_jj
      panel_leaves Rv;
      panel_gload_leaves(Rv, Dinv + cj, ldd, bj);  // the chain's leaf inverses
      panel_lstore_id(X, Rd, bj);
      panel_lstore_leaves(Y, Rv);
      __syncthreads();
      lds_trsm64_rt(D, (const lds_dbl*)X, (const lds_dbl*)Y, 4);
      __syncthreads();
    }
    panel_gstore<64>((const lds_dbl*)D, L + rt0 + (size_t)cj * ldl, ldl, rt, bj, false);
    PANEL_EV((j << 16) | (t << 8) | 7);
    if (j + 1 >= nb) break;
    panel_wait_all(row + j * S, j + 1, nb - 1, 1, epoch, status);
    // L_cj staged into Y / Z alternately: the next block is stored while this
    // one's products run, one barrier per update
    panel_regs Ryn;
    auto issue = [&](int c) {
      const int cc = J + SMG_NB * c;
      panel_gload(Ryn, L + cc + (size_t)cj * ldl, ldl, min(SMG_NB, K - cc), bj, false);
    };
    issue(j + 1);
    __syncthreads();  // (D's L_tj stored above: every wave past its reads of Y)
    panel_lstore(Y, Ryn);
    if (j + 2 < nb) issue(j + 2);
    __syncthreads();
    for (int c = j + 1; c < nb; ++c) {
      const lds_dbl* B = ((c - j - 1) & 1) ? (const lds_dbl*)Z : (const lds_dbl*)Y;
      // both halves' products in one k loop: two independent accumulator
      // chains per wave (one after the other, each wave's 16 dependent MFMAs
      // had made an update ~4 us)
      d4 acc_a = d4{0.0, 0.0, 0.0, 0.0}, acc_b = d4{0.0, 0.0, 0.0, 0.0};
      {
        const int fr = l & 15, fk = l >> 4;
        const int ia = 16 * (w & 1) + fr, jb = 16 * (w >> 1) + fr;
#pragma unroll 4
        for (int k0 = 0; k0 < SMG_NB; k0 += 4) {
          const int kk = k0 + fk;
          const double bv = B[jb * SMG_NBP + kk];
          acc_a = __builtin_amdgcn_mfma_f64_16x16x4f64(D[ia * SMG_NBP + kk], bv, acc_a, 0, 0, 0);
          acc_b = __builtin_amdgcn_mfma_f64_16x16x4f64(D[(32 + ia) * SMG_NBP + kk], bv, acc_b, 0, 0, 0);
        }
      }
      if (c + 1 < nb) {  // the next block into the other buffer (read two updates ago, past a barrier)
        panel_lstore(((c - j - 1) & 1) ? Y : Z, Ryn);
        if (c + 2 < nb) issue(c + 2);
      }
#pragma unroll
      for (int cr = 0; cr < S; ++cr)
        if (cr == c)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            Ra[cr][q] -= acc_a[q];
            Rb[cr][q] -= acc_b[q];
          }
      __syncthreads();
      PANEL_EV((j << 16) | (t << 8) | (16 + c));
    }
  }
}

__global__ __launch_bounds__(512) void k_chol_panel(double* __restrict__ L, int ldl, int n, int J,
                                                    int K, double* __restrict__ Dinv, int ldd,
                                                    int* flags, int epoch, int* status, int gown, int nha,
                                                    int paired) {
  __shared__ double D[SMG_NB * SMG_NBP];
  __shared__ double X[SMG_NB * SMG_NBP];
  __shared__ double Y[SMG_NB * SMG_NBP];
  __shared__ double Z[SMG_NB * SMG_NBP];
  PANEL_TL();
  constexpr int S = PANEL_MAX_STEPS;
  int* diag = flags;           // diag[j]: L_jj stored
  int* row = flags + S;        // row[j S + t]: L_tj stored (panel tiles t < nb)
  int* done = flags + S + S * S;  // done[j S + t]: tile t's step-j updates stored
  int* hflag = flags + S + 2 * S * S;  // hflag[j S + t]: tile t's helper finished step j
  int* dinvf = flags + S + 3 * S * S;  // dinvf[j]: Dinv_j stored (the inverter workgroup)
  int* hflagb = flags + S + 4 * S * S;  // hflagb[j S + t]: tile t's helper B finished step j
  const int nb = (K - J + SMG_NB - 1) / SMG_NB;
  const int T = panel_tiles(n, J, nb);
  const unsigned bid = blockIdx.x;
  // Column helpers: panel tile t >= 3 (t < nb) gets helper A (workgroup
  // gown + t - 3) for its odd column blocks c <= t - 2, tile t >= 4 helper B
  // (workgroup gown + nha + t - 4) for the even ones (panel_helper); the
  // owner of t does c = t - 1, t and its L_tj, and waits for the helper's
  // flag of step j - 1 (hflag / hflagb) before reading a helped column j.
  // The owners of the last panel tiles were the chain's bottleneck (their
  // seven column updates per step).
  // workgroup 1 is the inverter: Dinv_j = L_jj^{-1} (the aux level SMG_NB)
  // once the chain publishes L_jj; the tiles below the panel multiply by it
  // (their column updates, not the chain, bound the panel's end, so their
  // cheaper product beats the solve), the panel tiles solve against L_jj
  // (the chain needs their updates sooner).  Owners are workgroups
  // 2 .. gown - 1, column helpers gown ...
  const int nhb = (int)gridDim.x - gown - nha;
  if (bid == 1) {
    // ... and, behind each Dinv_j, the aux 128 level of the previous full
    // block pair (j - 2, j - 1): X = [[D1, 0], [-D2 L21 D1, D2]] (two 64^3
    // LDS products; Y = D1, Z = D2 kept from the pair's own steps), so the
    // doubling after the panel starts at 256 (chol_block_inverses skip128)
    __shared__ double Tin[3 * 256];
    double* W128 = Dinv + (size_t)ldd * SMG_AUX_W128;
    auto pair128 = [&](int j2) {  // blocks j2 - 1, j2 (Y, Z); both full
      const int c1 = J + SMG_NB * (j2 - 1), c2 = c1 + SMG_NB;
      panel_wait(&row[(j2 - 1) * S + j2], epoch, status);  // L_{j2, j2-1}, stored by tile j2's owner
      panel_regs Rl;
      panel_gload(Rl, L + c2 + (size_t)c1 * ldl, ldl, SMG_NB, SMG_NB, false);
      __syncthreads();
      panel_lstore(D, Rl);
      __syncthreads();
      lds_mma64_8w<false, false>(D, D, Y);        // T = L21 D1
      lds_mma64_8w<false, false>(D, Z, D, -1.0);  // X21 = -D2 T
      panel_gstore(Y, W128 + c1, ldd, SMG_NB, SMG_NB, false);
      panel_gstore(Z, W128 + c2 + (size_t)SMG_NB * ldd, ldd, SMG_NB, SMG_NB, false);
      panel_gstore(D, W128 + c2, ldd, SMG_NB, SMG_NB, false);
#pragma unroll
      for (int q = 0; q < 8; ++q) {  // the zero upper-right block
        const int e = threadIdx.x + SMG_DIAG_THREADS * q;
        W128[c1 + (e & 63) + (size_t)(SMG_NB + (e >> 6)) * ldd] = 0.0;
      }
    };
    auto full = [&](int j) { return j < nb && K - (J + SMG_NB * j) >= SMG_NB; };
    // the last block pair (nb - 2, nb - 1) after the chain's last step is the
    // launch's tail: its T = L21 D1 needs only L_{nb-1,nb-2} (tile nb-1's
    // owner, step nb - 2) and D1, so it is formed into Z (free: the previous
    // pair is done) BEFORE the wait for L_{nb-1,nb-1}, leaving X21 = -D2 T
    // after it (one 64^3 product instead of two, and no load, past the chain)
    const bool early = nb >= 2 && (nb & 1) == 0 && full(nb - 1) && full(nb - 2);
    for (int j = 0; j < nb; ++j) {
      const int cj = J + SMG_NB * j, bj = min(SMG_NB, K - cj);
      if (early && j == nb - 1) {
        panel_wait(&row[(j - 1) * S + j], epoch, status);  // L_{j,j-1}, stored by tile j's owner
        panel_regs Rt;
        panel_gload(Rt, L + cj + (size_t)(cj - SMG_NB) * ldl, ldl, SMG_NB, SMG_NB, false);
        __syncthreads();
        panel_lstore(D, Rt);
        __syncthreads();
        lds_mma64_8w<false, false>(Z, D, Y);  // T = L21 D1 (Y = D1)
        __syncthreads();
      }
      if (early && j == nb - 1) {  // the chain forms this last Dinv from its own leaves (chain_last_inverse)
        panel_wait(&dinvf[j], epoch, status);
        panel_regs Rx;
        panel_gload(Rx, Dinv + cj, ldd, bj, bj, true);
        __syncthreads();
        panel_lstore(X, Rx);
        __syncthreads();
        PANEL_EV((j << 16) | (j << 8) | 31);
      } else {
        panel_wait(&diag[j], epoch, status);
        panel_regs Rl;
        panel_gload(Rl, L + cj + (size_t)cj * ldl, ldl, bj, bj, true);
        __syncthreads();
        panel_lstore_id(D, Rl, bj);
        __syncthreads();
        lds_trtri64_mfma(D, X, Tin);
        __syncthreads();
        PANEL_EV((j << 16) | (j << 8) | 30);
        panel_gstore_tri(X, Dinv + cj, ldd, bj);
        panel_publish(&dinvf[j], epoch);
        PANEL_EV((j << 16) | (j << 8) | 31);
      }
      if (early && j == nb - 1) {  // X21 = -D2 T (X = D2), the pair's three blocks + the zero one
        const int c1 = cj - SMG_NB;
        lds_mma64_8w<false, false>(D, X, Z, -1.0);
        panel_gstore(Y, W128 + c1, ldd, SMG_NB, SMG_NB, false);
        panel_gstore(X, W128 + cj + (size_t)SMG_NB * ldd, ldd, SMG_NB, SMG_NB, false);
        panel_gstore(D, W128 + cj, ldd, SMG_NB, SMG_NB, false);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int e = threadIdx.x + SMG_DIAG_THREADS * q;
          W128[c1 + (e & 63) + (size_t)(SMG_NB + (e >> 6)) * ldd] = 0.0;
        }
      }
      if ((j & 1) == 0 && j >= 2 && full(j - 1)) pair128(j - 1);  // after Dinv_j: off the tiles' path
      PANEL_EV((j << 16) | (j << 8) | 32);
      __syncthreads();
      for (int e = threadIdx.x; e < SMG_NB * SMG_NBP; e += SMG_DIAG_THREADS) ((j & 1) ? Z : Y)[e] = X[e];
      __syncthreads();
    }
    if (!early && (nb & 1) == 0 && full(nb - 1)) pair128(nb - 1);
    return;
  }

  if (bid >= gown) {
    const int hb = (int)bid - gown, kind = hb < nha ? 1 : 2;
    const int t = kind == 1 ? 3 + hb : 4 + (hb - nha);
    if (t >= nb) return;
    int* hf = kind == 1 ? hflag : hflagb;
    const int rt0 = J + SMG_NB * t, rt = min(SMG_NB, n - rt0);
    for (int j = 0; j + 2 <= t; ++j) {
      const int cj = J + SMG_NB * j, bj = min(SMG_NB, K - cj);
      int c0 = j + 1;
      while (c0 <= t - 2 && panel_helper(t, c0, nb, nha, nhb) != kind) ++c0;
      if (c0 <= t - 2) {
        panel_wait(&row[j * S + t], epoch, status);  // the owner's L_tj
        PANEL_EV((j << 16) | (t << 8) | 20);
        panel_regs Rl;
        panel_gload(Rl, L + rt0 + (size_t)cj * ldl, ldl, rt, bj, false);
        panel_wait_all(row + j * S, c0, t - 2, 1, epoch, status);
        PANEL_EV((j << 16) | (t << 8) | 21);
        __syncthreads();
        panel_lstore(D, Rl);
        for (int c = c0; c <= t - 2; ++c) {
          if (panel_helper(t, c, nb, nha, nhb) != kind) continue;
          const int cc = J + SMG_NB * c, bc = min(SMG_NB, K - cc);
          panel_regs Ry, Rz;
          panel_gload(Rz, L + rt0 + (size_t)cc * ldl, ldl, rt, bc, false);
          panel_gload(Ry, L + cc + (size_t)cj * ldl, ldl, bc, bj, false);
          __syncthreads();  // previous product's Y / Z consumed (and D stored)
          panel_lstore(Y, Ry);
          panel_lstore(Z, Rz);
          __syncthreads();
          OWNER_UPDATE(Z, D, Y);
          panel_gstore(Z, L + rt0 + (size_t)cc * ldl, ldl, rt, bc, false);
        }
      }
      panel_publish(&hf[j * S + t], epoch);
      PANEL_EV((j << 16) | (t << 8) | 22);
    }
    return;
  }

  if (bid == 0) {
    // the diagonal chain: factor block j, then apply step j to tile j + 1
    // (a private L_{j+1,j} and the A_{j+1,j+1} update) so that block j + 1 is
    // ready in LDS without a hand-off.  Tile j + 1's owner computes the same
    // L_{j+1,j} (same inputs, same code: the same bits) and stores /
    // publishes it, so no store or publish of it sits on the chain.  The
    // chain reads A_{j+1,j} before publishing diag[j]; the owner overwrites
    // it with L_{j+1,j} only after seeing diag[j].
    double* Dc = D;  // current diagonal block (LDS)
    double* Zn = Z;  // next one
    {
      panel_regs R0;
      const int b0 = min(SMG_NB, K - J);
      panel_gload(R0, L + J + (size_t)J * ldl, ldl, b0, b0, true);
      panel_lstore_id(Dc, R0, b0);
    }
    __syncthreads();
    for (int j = 0; j < nb; ++j) {
      const int cj = J + SMG_NB * j;
      const int bj = min(SMG_NB, K - cj);
      PANEL_EV((j << 16) | (j << 8) | 2);
      const bool more = j + 1 < nb;
      const int t = j + 1, rt0 = J + SMG_NB * t, rt = min(SMG_NB, n - rt0);
      const int bt = min(SMG_NB, K - rt0);
      // L_jj is what the other tiles wait for (they solve against it): waves
      // 0-3 form and store its leaf inverses while waves 4-7 store L_jj and
      // stage the next tile's operands (chain_side); one publish covers both.
      // No 64 x 64 inverse on the chain: L_{t,j} = A_{t,j} L_jj^{-T} by the
      // leaf inverses and one row-tile solve (the inverter workgroup forms
      // Dinv_j beside it)
      CHAIN_FACTOR(Dc, status);
      __syncthreads();
      PANEL_EV((j << 16) | (j << 8) | 14);
      if (threadIdx.x < 256)
        CHAIN_LEAVES_PUB(Dc, X, Dinv + cj, ldd, bj);
      else
        chain_side((const lds_dbl*)Dc, (lds_dbl*)Y, (lds_dbl*)Zn, L, ldl, cj, bj, rt0, rt, bt, more ? 1 : 0,
                   j >= 1 ? &done[(j - 1) * S + t] : nullptr, epoch, status);
      PANEL_EV((j << 16) | (j << 8) | 10);
      panel_publish(&diag[j], epoch);
      PANEL_EV((j << 16) | (j << 8) | 4);
      if (!more) {
        // the last block's Dinv from the leaves already in X (the inverter's
        // phases after its leaves; T in Y), stored and published for the
        // inverter's last 128-level pair: ~7 us sooner than the inverter's
        // own load, leaves and phases after diag[j] (the launch's tail)
        const bool chain_inv = nb >= 2 && (nb & 1) == 0 && K - (J + SMG_NB * (nb - 2)) >= 2 * SMG_NB;
        if (chain_inv) {
          chain_last_inverse((const lds_dbl*)Dc, (lds_dbl*)X, (lds_dbl*)Y);
          panel_gstore_tri(X, Dinv + cj, ldd, bj);
          panel_publish(&dinvf[j], epoch);
          PANEL_EV((j << 16) | (j << 8) | 33);
        }
        break;
      }
      PANEL_EV((j << 16) | (t << 8) | 12);
      CHAIN_TRSM(Y, Dc, X);  // L_{t,j} = A_{t,j} L_jj^{-T} (private)
      __syncthreads();
      PANEL_EV((j << 16) | (t << 8) | 13);
      // A_tt -= L_tj L_tj^T, written as the factorisation's input: lower
      // triangle, zero strict upper, identity padding beyond bt
      CHAIN_SYRK(Zn, Y, bt);
      double* tmp = Dc;
      Dc = Zn;
      Zn = tmp;
      PANEL_EV((j << 16) | (t << 8) | 9);
    }
    return;
  }

  // the other workgroups: tiles t >= 1, owner(t) = 2 + (t - 1) mod (gown - 2);
  // every step of tile t.  At step t - 1 of a panel tile (t < nb) the owner
  // only computes, stores and publishes L_{t,t-1}: the chain applies the
  // A_tt update privately.
  // A workgroup whose only tile is one below the panel keeps that tile's
  // column blocks in registers for the whole panel (the accumulator layout of
  // lds_mma32_8w: 4 doubles per lane per 32 x 64 block): loaded once, each
  // step's update A_tc -= L_tj L_cj^T subtracted from the MFMA accumulator in
  // place, and block j written out once, as L_tj -- instead of loading and
  // storing every later block at every step (the kernel fetched 2.6x and
  // wrote 2.1x its algorithmic bytes)
  // paired: workgroups nb + 1 .. gown - 1 each hold a pair of 32-row tiles
  // below the panel (below_resident2); the owners 2 .. nb the panel tiles
  if (paired && (int)bid >= nb + 1) {
    const int p = (int)bid - (nb + 1);
    below_resident2(L, ldl, n, J, K, Dinv, ldd, flags, epoch, status, nb,
                    J + SMG_NB * nb + 2 * PANEL_BELOW_ROWS * p, nb + 2 * p, (lds_dbl*)D, (lds_dbl*)X, (lds_dbl*)Y,
                    (lds_dbl*)Z);
    return;
  }
  if (!paired && bid - 1 >= nb && bid - 1 + (gown - 2) >= T) {
    below_resident(L, ldl, n, J, K, Dinv, ldd, flags, epoch, status, nb, (int)bid - 1, (lds_dbl*)D, (lds_dbl*)X,
                   (lds_dbl*)Y);
    return;
  }
  const int Tloop = paired ? nb : T;  // (paired: the owners' tiles are the panel's only)
  for (int j = 0; j < nb; ++j) {
    const int cj = J + SMG_NB * j;
    const int bj = min(SMG_NB, K - cj);
    for (int t = 1 + (bid - 2); t < Tloop; t += gown - 2) {
      if (t <= j) continue;  // done
      if (t >= nb) {  // a 32-row tile below the panel: L_tj = A_tj Dinv_j^T, then A_tc -= L_tj L_cj^T (c < nb)
        constexpr int R = PANEL_BELOW_ROWS;
        const int rt0 = J + SMG_NB * nb + R * (t - nb), rt = min(R, n - rt0);
        __syncthreads();  // LDS of the previous item fully consumed
        PANEL_EV((j << 16) | (t << 8) | 5);
        panel_regs Ra, Rd;
        panel_gload<R>(Ra, L + rt0 + (size_t)cj * ldl, ldl, rt, bj, false);  // own data, final
        if (j + 1 < nb) {
          panel_wait(&dinvf[j], epoch, status);
          PANEL_EV((j << 16) | (t << 8) | 6);
          panel_gload(Rd, Dinv + cj, ldd, bj, bj, true);
          panel_lstore<R>(D, Ra);
          panel_lstore(X, Rd);
          __syncthreads();
          BELOW_LTJ(D, X);
        } else {  // the last step: solve against L_jj (the chain's end, not the inverter's, bounds it)
          panel_wait(&diag[j], epoch, status);
          PANEL_EV((j << 16) | (t << 8) | 6);
          panel_gload(Rd, L + cj + (size_t)cj * ldl, ldl, bj, bj, true);  // L_jj
          panel_leaves Rv;
          panel_gload_leaves(Rv, Dinv + cj, ldd, bj);  // the chain's leaf inverses
          panel_lstore<R>(D, Ra);
          panel_lstore_id(X, Rd, bj);
          panel_lstore_leaves(Y, Rv);
          __syncthreads();
          BELOW_TRSM(D, X, Y);
          __syncthreads();
        }
        panel_gstore<R>(D, L + rt0 + (size_t)cj * ldl, ldl, rt, bj, false);
        PANEL_EV((j << 16) | (t << 8) | 7);
        if (j + 1 >= nb) continue;
        panel_wait_all(row + j * S, j + 1, nb - 1, 1, epoch, status);
        panel_regs Ryn, Rzn;
        auto issue = [&](int c) {
          const int cc = J + SMG_NB * c;
          panel_gload<R>(Rzn, L + rt0 + (size_t)cc * ldl, ldl, rt, min(SMG_NB, K - cc), false);
          panel_gload(Ryn, L + cc + (size_t)cj * ldl, ldl, min(SMG_NB, K - cc), bj, false);
        };
        issue(j + 1);
        for (int c = j + 1; c < nb; ++c) {
          const int cc = J + SMG_NB * c;
          __syncthreads();  // previous product's Y / Z consumed
          panel_lstore(Y, Ryn);
          panel_lstore<R>(Z, Rzn);
          __syncthreads();
          if (c + 1 < nb) issue(c + 1);  // in flight during this product
          BELOW_UPDATE(Z, D, Y);
          panel_gstore<R>(Z, L + rt0 + (size_t)cc * ldl, ldl, rt, min(SMG_NB, K - cc), false);
          PANEL_EV((j << 16) | (t << 8) | (16 + c));
        }
        continue;
      }
      const bool next = t == j + 1;  // the chain's next diagonal tile
      const int rt0 = J + SMG_NB * t;
      const int rt = min(SMG_NB, n - rt0);
      __syncthreads();  // LDS of the previous item fully consumed
      PANEL_EV((j << 16) | (t << 8) | 5);
      panel_regs Ra, Rd;
      // a helped column is final once the helper has finished step j - 1
      if (const int hk = panel_helper(t, j, nb, nha, nhb))
        panel_wait(&(hk == 1 ? hflag : hflagb)[(j - 1) * S + t], epoch, status);
      panel_gload(Ra, L + rt0 + (size_t)cj * ldl, ldl, rt, bj, false);  // own data, final
      // a panel tile: solve against L_jj (the chain's own solve for tile j + 1: the same bits)
      panel_wait(&diag[j], epoch, status);
      PANEL_EV((j << 16) | (t << 8) | 6);
      panel_gload(Rd, L + cj + (size_t)cj * ldl, ldl, bj, bj, true);  // L_jj
      panel_leaves Rv;
      panel_gload_leaves(Rv, Dinv + cj, ldd, bj);  // the chain's leaf inverses
      panel_lstore(D, Ra);
      panel_lstore_id(X, Rd, bj);
      panel_lstore_leaves(Y, Rv);
      __syncthreads();
      CHAIN_TRSM(D, X, Y);
      __syncthreads();
      panel_gstore(D, L + rt0 + (size_t)cj * ldl, ldl, rt, bj, false);
      PANEL_EV((j << 16) | (t << 8) | 7);
      panel_publish(&row[j * S + t], epoch);
      if (next) continue;
      // A_tc -= L_tj L_cj^T for the panel's later column blocks c <= t.  The
      // rows L_cj (c < t) are published by their owners at about the same
      // time, so ONE wait covers all of them; the operands of update c + 1
      // are then loaded while update c's product runs.
      const int clast = t;
      const int cwait = t - 1;  // L_tt's row is this tile's own
      if (j + 1 <= cwait) panel_wait_all(row + j * S, j + 1, cwait, 1, epoch, status);
      panel_regs Ryn, Rzn;
      auto issue = [&](int c) {
        const int cc = J + SMG_NB * c;
        const bool own = c == t;
        panel_gload(Rzn, L + rt0 + (size_t)cc * ldl, ldl, rt, min(SMG_NB, K - cc), own);
        if (!own) panel_gload(Ryn, L + cc + (size_t)cj * ldl, ldl, min(SMG_NB, K - cc), bj, false);
      };
      auto next_col = [&](int c) {  // the next column from c on that this workgroup updates
        while (c <= clast && panel_helper(t, c, nb, nha, nhb)) ++c;
        return c;
      };
      int cfirst = next_col(j + 1);
      if (cfirst <= clast) issue(cfirst);
      for (int c = cfirst; c <= clast; c = next_col(c + 1)) {
        const int cc = J + SMG_NB * c;
        const int bc = min(SMG_NB, K - cc);
        const bool own = c == t;  // L_cj is L_tj itself; A_tt: lower triangle
        __syncthreads();  // previous product's Y / Z consumed
        if (!own) panel_lstore(Y, Ryn);
        panel_lstore(Z, Rzn);
        __syncthreads();
        const int cn = next_col(c + 1);
        if (cn <= clast) issue(cn);  // in flight during this product
        OWNER_UPDATE(Z, D, own ? D : Y);
        panel_gstore(Z, L + rt0 + (size_t)cc * ldl, ldl, rt, bc, own);
        PANEL_EV((j << 16) | (t << 8) | (16 + c));
      }
      if (t == j + 2) panel_publish(&done[j * S + t], epoch);
    }
  }
}

// inverse of a lower-triangular diagonal block (no factorisation)
__global__ __launch_bounds__(512) void k_trtri_diag(const double* __restrict__ L, int ldl,
                                                    int b, double* __restrict__ Dinv, int ldd) {
  __shared__ double D[SMG_NB * SMG_NBP];
  __shared__ double X[SMG_NB * SMG_NBP];
  lds_load_block(D, L, ldl, b, true);
  __syncthreads();
  lds_potrf_inv64_blk(D, X, b, nullptr, 0, Dinv, ldd, nullptr, false);
}

// symbolic_rev (cholesky_decompose.hpp:101-111) on one diagonal block:
//   S = D^T tril(Dadj); S = sym_from_lower(S); S = Dinv^T S Dinv
// writes Ssym (b x b dense, ld b) and Dadj <- tril(S) with halved diagonal.
__global__ __launch_bounds__(512) void k_symbolic_rev(const double* __restrict__ L, int ldl,
                                                      const double* __restrict__ Dinv, int ldd,
                                                      double* __restrict__ Dadj, int lda,
                                                      int b, double* __restrict__ Ssym) {
  __shared__ double D[SMG_NB * SMG_NBP];   // D, later temp
  __shared__ double G[SMG_NB * SMG_NBP];   // tril(Dadj), later S
  __shared__ double W[SMG_NB * SMG_NBP];   // Dinv (lower)
  // zero padding beyond b keeps every 64x64 product exact on the b x b block;
  // the three block loads are issued back to back (one global-latency exposure)
  lds_load_block0(D, L, ldl, b, true);
  lds_load_block0(G, Dadj, lda, b, true);
  lds_load_block0(W, Dinv, ldd, b, true);
  __syncthreads();
  lds_mma64_8w<true, false>(G, D, G);  // S = D^T tril(Dadj)
  // mirror the lower triangle into the upper (:106-107)
  for (int e = threadIdx.x; e < SMG_NB * SMG_NB; e += blockDim.x) {
    const int r = e / SMG_NB, c = e % SMG_NB;
    if (r < c) G[r * SMG_NBP + c] = G[c * SMG_NBP + r];
  }
  __syncthreads();
  lds_mma64_8w<true, false>(D, W, G);   // T = Dinv^T S
  lds_mma64_8w<false, false>(G, D, W);  // S = T Dinv
  // outputs: selfadjointView<Lower> of S, and tril(S) with halved diagonal (:160-161)
  for (int e = threadIdx.x; e < b * b; e += blockDim.x) {
    const int c = e / b, r = e % b;
    const double low = (r >= c) ? G[r * SMG_NBP + c] : G[c * SMG_NBP + r];
    Ssym[r + (size_t)c * b] = low;
    double v = 0.0;
    if (r > c) v = low;
    else if (r == c) v = 0.5 * low;
    Dadj[r + (size_t)c * lda] = v;
  }
}

// P (n x n dense) = X + X^T from the lower triangle of X with halved diagonal
__global__ void k_sym_from_half(const double* __restrict__ X, int ldx, int n, double* __restrict__ P) {
  for (smg_mn it(n, n); it.ok(); it.next()) {
    const long long e = it.e;
    const int i = it.i, j = it.j;
    P[e] = i > j ? X[i + (size_t)j * ldx] : (i < j ? X[j + (size_t)i * ldx] : 2.0 * X[i + (size_t)i * ldx]);
  }
}

// Recursive-doubling step of the block inverses of a lower-triangular L:
// from the s x s inverses Wi (rows aligned with L, ld ldi, s columns) to the
// 2s x 2s inverses Wo (ld ldo, 2s columns) of the nb full 2s-blocks:
// this kernel copies the diagonal s-blocks and zeroes the upper-right one;
// the lower-left X21 = -X22 (L21 X11) comes from two batched GEMMs.
__global__ void k_inv_double_diag(int nb, int s2, const double* __restrict__ Wi, int ldi,
                                  double* __restrict__ Wo, int ldo) {
  const int s = s2 / 2;
  const long long tot = (long long)nb * s2 * s2;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < tot;
       e += (long long)gridDim.x * blockDim.x) {
    const int q = (int)(e / ((long long)s2 * s2));
    const int rem = (int)(e % ((long long)s2 * s2));
    const int c = rem / s2, r = rem % s2;
    const int row = q * s2 + r;
    double v;
    if (r < s && c < s) v = Wi[row + (size_t)c * ldi];
    else if (r >= s && c >= s) v = Wi[row + (size_t)(c - s) * ldi];
    else if (r < s) v = 0.0;
    else continue;  // lower-left: written by the GEMMs
    Wo[row + (size_t)c * ldo] = v;
  }
}

// The 256- and 512-level inverses of ONE 512-row block row from its 128-level
// ones in one launch: chol_block_inverses' doubling steps
//   level 256 (pairs q = 0, 1):  T_q = L21_q X11_q,  X21_q = -X22_q T_q
//   level 512:                   T = L21 W256_0,     X21 = -W256_1 T
// as four phases over IB_WG workgroups with a grid-wide counter between them
// (the fence-free hand-off of smg_sync.h: sc1 payload stores, every wave's
// vmcnt(0), a barrier, one counter add; sc1 loads after the poll).  The
// counter needs the 64 workgroups co-resident: the kernel is used only when
// the device can hold them beside the persistent panel kernel (inv_fused_ok:
// occupancy x CUs, checked once per context); else the six launches.  A
// ticketed work queue (each workgroup takes its next item from an atomic
// counter, waits only for lower tickets: deadlock-free at any residency) was
// measured 41-56 -> 67-83 us per launch (returning device-scope atomics on one
// address serialise beyond the XCD L2s) and GP 383 -> 358 evals/s; dropped.  Six
// dependent launches of 32-128 tiles each took 66 us after the last panel,
// sharing their CUs with the K^{-1} shares.  Every phase is 32 x 32 output
// tiles on 16 x 16 x 4 f64 MFMAs (one 16 x 16 quadrant per wave); the
// diagonal-block copies of both levels ride along.  Aux strips: ld n; L at
// the block row's diagonal origin.
constexpr int IB_WG = 64;
constexpr int IB_PHASES = 4;

__device__ inline void ib_sync(unsigned* ctr, unsigned target, int* status) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 stores have landed
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while ((int)(__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 400000000ull) {
        atomicOr(status, (int)SMG_ERR_SYNC);
        break;
      }
    }
  }
  __syncthreads();
}

// C[32 x 32 at C] = alpha A[32 x K] B[K x 32] (column-major, sc1 loads and
// stores); wave w takes the 16 x 16 quadrant (w & 1, w >> 1)
__device__ inline void ib_tile(const double* A, int lda, const double* B, int ldb, int K, double alpha, double* C,
                               int ldc, double* C2 = nullptr, int ldc2 = 0) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wi = (w & 1) * 16, wj = (w >> 1) * 16;
  const int fr = lane & 15, fk = lane >> 4;
  const double* a = A + wi + fr + (size_t)fk * lda;
  const double* b = B + fk + (size_t)(wj + fr) * ldb;
  d4 acc = {0.0, 0.0, 0.0, 0.0};
  constexpr int U = 16;  // k-steps of 4 whose loads are all issued before their MFMAs
  for (int k = 0; k < K; k += 4 * U) {
    double av[U], bv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      av[u] = ld_dev(a + (size_t)(k + 4 * u) * lda);
      bv[u] = ld_dev(b + k + 4 * u);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u], bv[u], acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    st_dev(C + (wi + fk + 4 * r) + (size_t)(wj + fr) * ldc, alpha * acc[r]);
    if (C2) st_dev(C2 + (wi + fk + 4 * r) + (size_t)(wj + fr) * ldc2, alpha * acc[r]);
  }
}

// dst[rows x cols] = src (or zero when src is null); the workgroup's share
// `part` of `parts` of the elements, sc1 loads / stores
__device__ inline void ib_copy(const double* src, int lds, double* dst, int ldd, int rows, int cols, int part,
                               int parts, double* dst2 = nullptr, int ldd2 = 0) {
  const int tot = rows * cols;
  for (int e = part * 256 + (int)threadIdx.x; e < tot; e += parts * 256) {
    const int r = e % rows, c = e / rows;
    const double v = src ? ld_dev(src + r + (size_t)c * lds) : 0.0;
    st_dev(dst + r + (size_t)c * ldd, v);
    if (dst2) st_dev(dst2 + r + (size_t)c * ldd2, v);
  }
}

__global__ __launch_bounds__(256) void k_inv_block512(const double* __restrict__ Lb, int ldl, const double* Wi,
                                                      double* W256, double* W512, int ldw, double* T,
                                                      unsigned* ctr, unsigned base, int* status, double* W2,
                                                      int ldw2) {
  // W2 (optional, ld ldw2): a second copy of the 512-level result (the
  // progressive W's diagonal block: no separate copy launch)
  const int g = blockIdx.x;
  // phase 1: T_q = L21_q X11_q (2 x 16 tiles, K = 128); the level-256 diagonal copies
  if (g < 32) {
    const int q = g >> 4, t = g & 15, ti = (t & 3) * 32, tj = (t >> 2) * 32;
    const int o = q * 256;
    ib_tile(Lb + (o + 128 + ti) + (size_t)o * ldl, ldl, Wi + o + (size_t)tj * ldw, ldw, 128, 1.0,
            T + q * 128 * 128 + ti + (size_t)tj * 128, 128);
  } else {  // X11 (rows o.., cols 0..128), X22 (rows o + 128.., cols 128..256), the upper-right block zero
    const int p = g - 32;  // 32 workgroups: (q, piece) = (p >> 4, p & 15)
    const int q = p >> 4, o = q * 256, piece = p & 15;
    ib_copy(Wi + o, ldw, W256 + o, ldw, 128, 128, piece, 16);
    ib_copy(Wi + o + 128, ldw, W256 + o + 128 + (size_t)128 * ldw, ldw, 128, 128, piece, 16);
    ib_copy(nullptr, 0, W256 + o + (size_t)128 * ldw, ldw, 128, 128, piece, 16);
  }
  ib_sync(ctr, base + 1 * IB_WG, status);
  // phase 2: X21_q = -X22_q T_q (2 x 16 tiles, K = 128)
  if (g < 32) {
    const int q = g >> 4, t = g & 15, ti = (t & 3) * 32, tj = (t >> 2) * 32;
    const int o = q * 256;
    ib_tile(Wi + o + 128 + ti, ldw, T + q * 128 * 128 + (size_t)tj * 128, 128, 128, -1.0,
            W256 + o + 128 + ti + (size_t)tj * ldw, ldw);
  }
  ib_sync(ctr, base + 2 * IB_WG, status);
  // phase 3: T = L21 W256_0 (64 tiles, K = 256; T reused: phase 2 has read it);
  // the level-512 diagonal copies
  {
    const int ti = (g & 7) * 32, tj = (g >> 3) * 32;
    ib_tile(Lb + 256 + ti, ldl, W256 + (size_t)tj * ldw, ldw, 256, 1.0, T + ti + (size_t)tj * 256, 256);
    ib_copy(W256, ldw, W512, ldw, 256, 256, g, IB_WG, W2, ldw2);
    ib_copy(W256 + 256, ldw, W512 + 256 + (size_t)256 * ldw, ldw, 256, 256, g, IB_WG,
            W2 ? W2 + 256 + (size_t)256 * ldw2 : nullptr, ldw2);
    ib_copy(nullptr, 0, W512 + (size_t)256 * ldw, ldw, 256, 256, g, IB_WG, W2 ? W2 + (size_t)256 * ldw2 : nullptr,
            ldw2);
  }
  ib_sync(ctr, base + 3 * IB_WG, status);
  // phase 4: X21 = -W256_1 T (64 tiles, K = 256)
  {
    const int ti = (g & 7) * 32, tj = (g >> 3) * 32;
    ib_tile(W256 + 256 + ti, ldw, T + (size_t)tj * 256, 256, 256, -1.0, W512 + 256 + ti + (size_t)tj * ldw, ldw,
            W2 ? W2 + 256 + ti + (size_t)tj * ldw2 : nullptr, ldw2);
  }
  // (the fourth count: the next launch on this slot starts from base + IB_PHASES * IB_WG)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// G = tril(X) (n x n dense, ld n)
__global__ void k_tril_copy(const double* __restrict__ X, int ldx, int n, double* __restrict__ G) {
  for (smg_mn it(n, n); it.ok(); it.next()) {
    const long long e = it.e;
    const int i = it.i, j = it.j;
    G[e] = i >= j ? X[i + (size_t)j * ldx] : 0.0;
  }
}

// S (n x n, ld n): upper triangle <- lower triangle (sym_from_lower)
__global__ void k_mirror_lower(double* __restrict__ S, int n) {
  for (smg_mn it(n, n); it.ok(); it.next()) {
    const long long e = it.e;
    const int i = it.i, j = it.j;
    if (i < j) S[i + (size_t)j * n] = S[j + (size_t)i * n];
  }
}

// Dadj (ld lda) <- tril(S) with halved diagonal; strict upper untouched
__global__ void k_half_lower(const double* __restrict__ S, int n, double* __restrict__ Dadj, int lda) {
  for (smg_mn it(n, n); it.ok(); it.next()) {
    const long long e = it.e;
    const int i = it.i, j = it.j;
    if (i > j) Dadj[i + (size_t)j * lda] = S[e];
    else if (i == j) Dadj[i + (size_t)j * lda] = 0.5 * S[e];
  }
}

inline int grid_for(long long tot) {
  long long g = (tot + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (int)g;
}

// Murray's reverse on an n x n (sub)matrix with SMG_NB blocks, in place:
// on exit the lower triangle of La holds Abar of chol(this block) with the
// reference's convention (halved diagonal, :160-161).  Dv: the SMG_NB-block
// inverses of L's diagonal blocks (rows aligned with L, leading dimension ldd).
int chol_rev_blocks(smg_ctx* ctx, const double* L, int ldl, const double* Dv, int ldd, double* La,
                    int ldla, int n) {
  double* Ssym = smg_ws(ctx, SMG_WS_TMP, (size_t)SMG_NB * SMG_NB);
  if (!Ssym) return SMG_ERR_OOM;
  const int nblk = (n + SMG_NB - 1) / SMG_NB;
  for (int p = nblk - 1; p >= 0; --p) {
    const int j = p * SMG_NB;
    const int b = min(SMG_NB, n - j);
    const int k = j + b, m = n - k;
    const double* Di = Dv + j;
    double* Cadj = La + k + (size_t)j * ldla;
    double* Badj = La + k;
    double* Dadj = La + j + (size_t)j * ldla;
    double* Radj = La + j;
    const double* R = L + j;
    const double* Bv = L + k;
    int rc;
    if (m > 0) {
      // C_adj = C_adj D^{-1}
      rc = smg_gemm_impl(ctx, 0, 0, 0, m, b, b, 1.0, Cadj, ldla, Di, ldd, 0.0, Cadj, ldla);
      if (rc) return rc;
      if (j > 0) {  // B_adj -= C_adj R
        rc = smg_gemm_impl(ctx, 0, 0, 0, m, j, b, -1.0, Cadj, ldla, R, ldl, 1.0, Badj, ldla);
        if (rc) return rc;
      }
      // [R_adj | D_adj] -= C_adj^T [B | C]: both operands are contiguous column
      // ranges (L[k:, 0:k] and Abar[j:k, 0:k]), so one GEMM (one split-K
      // reduction) does both updates; R_adj's does not depend on the symbolic step
      rc = smg_gemm_impl(ctx, 1, 0, 0, b, k, m, -1.0, Cadj, ldla, Bv, ldl, 1.0, Radj, ldla);
      if (rc) return rc;
    }
    hipLaunchKernelGGL(k_symbolic_rev, dim3(1), dim3(SMG_DIAG_THREADS), 0, ctx->stream,
                       L + j + (size_t)j * ldl, ldl, Di, ldd, Dadj, ldla, b, Ssym);
    if (j > 0) {
      // R_adj -= sym(D_adj) R
      rc = smg_gemm_impl(ctx, 0, 0, 0, b, j, b, -1.0, Ssym, b, R, ldl, 1.0, Radj, ldla);
      if (rc) return rc;
    }
  }
  return SMG_OK;
}

// k_inv_block512's counter barriers need its IB_WG workgroups co-resident.
// Nothing it runs beside waits on it, so they all get a slot once those
// kernels drain -- unless the device cannot hold IB_WG of them at all next to
// a panel launch of this factorisation, whose workgroups take one CU each
// (LDS-bound; its VGPRs fill the SIMDs): the CUs the widest panel grid (the
// first panel's) leaves must hold IB_WG.  The occupancy is queried once per
// context; the test hook smg_set_inv_block_mode forces the six-launch chain.
bool inv_fused_ok(smg_ctx* ctx, int n) {
  if (ctx->inv_mode == 1) return false;
  if (ctx->inv_per_cu < 0) {
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_inv_block512, 256, 0) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess)
      per_cu = cus = 0;
    ctx->inv_per_cu = per_cu;
    ctx->inv_cus = cus;
  }
  const int nb0 = smg_ceil_div(min(n, SMG_NBF), SMG_NB), t0 = panel_tiles(n, 0, nb0);
  const int panel_grid = min(nb0 + 1 + (t0 - nb0 + 1) / 2, PANEL_MAX_GRID + 1) + (nb0 > 3 ? nb0 - 3 : 0) +
                         (nb0 > 4 ? nb0 - 4 : 0);
  return (long long)ctx->inv_per_cu * max(0, ctx->inv_cus - panel_grid) >= IB_WG;
}

// Inverses of the full 128-, 256- and 512-row diagonal blocks of L by
// recursive doubling from the SMG_NB-block inverses: aux (ld n) holds the
// levels at the SMG_AUX_W* column offsets (smg_cholesky_aux_doubles).
// (rows [row0, row0 + nrows) only, nrows < 0: all; T: workspace of
// nrows / 2 x 256 doubles, NULL: SMG_WS_TMP)
// (Wout, ld n: when the one-launch form runs, it also writes the 512-level
// block there and sets *wrote)
int chol_block_inverses(smg_ctx* ctx, const double* L, int ldl, double* aux, int n, int row0 = 0,
                        int nrows = -1, double* Tbuf = nullptr, bool skip128 = false, double* Wout = nullptr,
                        bool* wrote = nullptr) {
  if (wrote) *wrote = false;
  if (nrows < 0) nrows = n;
  L += (size_t)row0 * (ldl + 1);
  // skip128: the 128 level is already there (the panel kernel's inverter forms it)
  const double* Wi = skip128 ? aux + (size_t)n * SMG_AUX_W128 + row0 : aux + row0;
  int ldi = n;
  static_assert(SMG_NBR == 512 && SMG_NB == 64, "k_inv_block512's phases");
  if (skip128 && nrows == SMG_NBR && inv_fused_ok(ctx, n)) {  // one block row: one launch (k_inv_block512)
    double* T = Tbuf ? Tbuf : smg_ws(ctx, SMG_WS_TMP, (size_t)256 * 256);
    if (!T) return SMG_ERR_OOM;
    const long long e = ctx->inv_launches;  // (counted once the launch is in: a failed one adds nothing to its slot)
    unsigned* ctr = ctx->inv_ctr_d + e % SMG_INV_CTRS;
    const unsigned base = (unsigned)((unsigned long long)(e / SMG_INV_CTRS) * (IB_PHASES * IB_WG));
    ctx->status_armed = 1;
    hipLaunchKernelGGL(k_inv_block512, dim3(IB_WG), dim3(256), 0, ctx->stream, L, ldl, Wi,
                       aux + (size_t)n * SMG_AUX_W256 + row0, aux + (size_t)n * SMG_AUX_W512 + row0, n, T, ctr,
                       base, ctx->status_d, Wout, n);
    SMG_LAUNCH_CHECK();
    ctx->inv_launches = e + 1;
    if (wrote) *wrote = Wout != nullptr;
    return SMG_OK;
  }
  for (int s2 = skip128 ? 4 * SMG_NB : 2 * SMG_NB; s2 <= SMG_NBR; s2 *= 2) {
    const int s = s2 / 2, nb = nrows / s2;
    if (nb == 0) return SMG_OK;
    const int off = s2 == 128 ? SMG_AUX_W128 : (s2 == 256 ? SMG_AUX_W256 : SMG_AUX_W512);
    double* Wo = aux + (size_t)n * off + row0;
    const int ldw = n;
    hipLaunchKernelGGL(k_inv_double_diag, dim3(grid_for((long long)nb * s2 * s2)), dim3(256), 0,
                       ctx->stream, nb, s2, Wi, ldi, Wo, ldw);
    double* T = Tbuf ? Tbuf : smg_ws(ctx, SMG_WS_TMP, (size_t)nb * s * s);
    if (!T) return SMG_ERR_OOM;
    // T_q = L21_q X11_q ;  X21_q = -X22_q T_q
    int rc = smg_gemm_batched_impl(ctx, 0, 0, s, s, s, 1.0, L + s, ldl, (long long)s2 * (ldl + 1),
                                   Wi, ldi, s2, 0.0, T, s, (long long)s * s, nb);
    if (rc) return rc;
    rc = smg_gemm_batched_impl(ctx, 0, 0, s, s, s, -1.0, Wi + s, ldi, s2, T, s, (long long)s * s,
                               0.0, Wo + s, ldw, s2, nb);
    if (rc) return rc;
    Wi = Wo;
    ldi = ldw;
  }
  return SMG_OK;
}

// Two-level Murray reverse: outer blocks of SMG_NBR columns make the three
// big updates rank-SMG_NBR (compute-bound GEMMs).  The diagonal block's
// symbolic adjoint (:101-111) is applied in closed form to the whole
// SMG_NBR block: P = D^{-T} sym(D^T tril(Dadj)) D^{-1} with the block inverse
// from chol_block_inverses (a ragged last block falls back to the exact
// inner recursion chol_rev_blocks); P also feeds R_adj -= P R.
int chol_rev_two_level(smg_ctx* ctx, const double* L, int ldl, const double* aux, int n,
                       double* La, int ldla) {
  const int nbo = (n + SMG_NBR - 1) / SMG_NBR;
  const double* Dv = aux;                           // SMG_NB-block inverses, ld n
  const int ldd = n;
  const double* W = aux + (size_t)n * SMG_AUX_W512;  // SMG_NBR-block inverses, ld n
  int rc;
  const size_t bb = (size_t)SMG_NBR * SMG_NBR;
  // B_adj -= C_adj R (rows K:, columns 0:J) runs on the side stream, in
  // parallel with [R_adj | D_adj] -= C_adj^T [B | C], the symbolic step and
  // R_adj -= P R (rows J:K) on the main stream: disjoint outputs, and neither
  // reads what the other writes.  The next block's C_adj (rows J:, columns
  // J-NB2:J) includes B_adj's rows, hence the wait at the top of each step.
  const bool side = smg_side_begin(ctx) == SMG_OK;
  int nev = 0;
  hipEvent_t F = nullptr;
  // the C_adj D^{-1} workspace at its largest (m grows as P falls), so that
  // no block reallocates it (a reallocation synchronises the streams)
  if (n > SMG_NBR && !smg_ws(ctx, SMG_WS_CW, (size_t)(n - SMG_NBR) * SMG_NBR)) return SMG_ERR_OOM;
  for (int P = nbo - 1; P >= 0; --P) {
    if (F) {
      SMG_HIP_TRY(hipStreamWaitEvent(ctx->stream, F, 0));
      F = nullptr;
    }
    const int J = P * SMG_NBR;
    const int K = min(J + SMG_NBR, n), bs = K - J, m = n - K;
    const bool full = bs == SMG_NBR;
    double* Ca = La + K + (size_t)J * ldla;
    double* Da = La + J + (size_t)J * ldla;
    const double* Ld = L + J + (size_t)J * ldl;
    const double* Wp = W + J;  // this block's inverse, ld n
    // C_adj D^{-1} of a full block goes to a workspace (Cw, ld m) that the two
    // updates read; its copy back into La (read again only by the final
    // accumulation into A's adjoint) runs on the side stream behind B_adj
    const double* Cr = Ca;
    int ldcr = ldla;
    double* Cw = nullptr;
    if (m > 0) {
      if (full) {  // C_adj = C_adj D^{-1}
        Cw = smg_ws(ctx, SMG_WS_CW, (size_t)m * bs);
        if (!Cw) return SMG_ERR_OOM;
        rc = smg_gemm_impl(ctx, 0, 0, 0, m, bs, bs, 1.0, Ca, ldla, Wp, n, 0.0, Cw, m, 4);  // D^{-1} lower
        if (rc) return rc;
        Cr = Cw;
        ldcr = m;
      } else {  // ragged: blocked right solve with the SMG_NB inverses
        const int nbi = (bs + SMG_NB - 1) / SMG_NB;
        for (int q = nbi - 1; q >= 0; --q) {
          const int jq = q * SMG_NB, bq = min(SMG_NB, bs - jq), rest = bs - jq - bq;
          if (rest > 0) {
            rc = smg_gemm_impl(ctx, 0, 0, 0, m, bq, rest, -1.0, Ca + (size_t)(jq + bq) * ldla, ldla,
                               Ld + (jq + bq) + (size_t)jq * ldl, ldl, 1.0, Ca + (size_t)jq * ldla,
                               ldla);
            if (rc) return rc;
          }
          rc = smg_gemm_impl(ctx, 0, 0, 0, m, bq, bq, 1.0, Ca + (size_t)jq * ldla, ldla,
                             Dv + J + jq, ldd, 0.0, Ca + (size_t)jq * ldla, ldla);
          if (rc) return rc;
        }
      }
      if (J > 0) {  // B_adj -= C_adj R
        if (side) {
          hipEvent_t E = smg_event(ctx, nev++);
          if (!E) return SMG_ERR_HIP;
          SMG_HIP_TRY(hipEventRecord(E, ctx->stream));
          SMG_HIP_TRY(hipStreamWaitEvent(ctx->side, E, 0));
          {
            smg_on_side on(ctx);
            rc = smg_gemm_impl(ctx, 0, 0, 0, m, J, bs, -1.0, Cr, ldcr, L + J, ldl, 1.0, La + K, ldla);
            if (!rc && Cw) rc = smg_copy_impl(ctx, m, bs, Cw, m, Ca, ldla, 1.0, 0);
          }
          if (rc) return rc;
          Cw = nullptr;  // copied back on the side stream
          F = smg_event(ctx, nev++);
          if (!F) return SMG_ERR_HIP;
          SMG_HIP_TRY(hipEventRecord(F, ctx->side));
        } else {
          rc = smg_gemm_impl(ctx, 0, 0, 0, m, J, bs, -1.0, Cr, ldcr, L + J, ldl, 1.0, La + K, ldla);
          if (rc) return rc;
        }
      }
      // [R_adj | D_adj] -= C_adj^T [B | C]
      rc = smg_gemm_impl(ctx, 1, 0, 0, bs, K, m, -1.0, Cr, ldcr, L + K, ldl, 1.0, La + J, ldla);
      if (rc) return rc;
      if (Cw) {  // no side-stream copy was queued
        rc = smg_copy_impl(ctx, m, bs, Cw, m, Ca, ldla, 1.0, 0);
        if (rc) return rc;
      }
    }
    double* Pm;
    if (full) {
      double* G = smg_ws(ctx, SMG_WS_TMP, 3 * bb);
      if (!G) return SMG_ERR_OOM;
      double* S = G + bb;
      double* T = S + bb;
      const int gb = grid_for((long long)bb);
      // D^T tril(Dadj) read straight from Dadj, no tril copy: for an output
      // entry (i, j), i >= j, an entry Dadj_kj of the strict upper (k < j,
      // written by the [R_adj | D_adj] update) meets (D^T)_ik = D_ki, a stored
      // zero of L since k < j <= i (finite times zero: the same sums).
      // The operands' triangles bound each tile's K range (gemm tri flags):
      // D^T upper (2) x tril(Dadj) lower (4), lower output only (mirrored
      // next); D^{-T} upper (2); D^{-1} lower (4).  Measured on MI355X (GP
      // N = 4096, same-box A/B): 221.3 -> 225.4 evals/s
      // (uplo 3: the lower half computed and stored mirrored, the
      // sym_from_lower pass folded into the epilogue; the last product also
      // writes D_adj = tril(P) with halved diagonal from its epilogue)
      rc = smg_gemm_impl(ctx, 1, 0, 3, bs, bs, bs, 1.0, Ld, ldl, Da, ldla, 0.0, S, bs, 6);
      if (rc) return rc;
      rc = smg_gemm_impl(ctx, 1, 0, 0, bs, bs, bs, 1.0, Wp, n, S, bs, 0.0, T, bs, 2);  // D^{-T} S
      if (rc) return rc;
      rc = smg_gemm_dual_impl(ctx, 0, 0, bs, bs, bs, 1.0, T, bs, Wp, n, 0.0, S, bs, Da, ldla, 4);  // ... D^{-1}
      if (rc) return rc;
      (void)gb;
      Pm = S;
    } else {
      rc = chol_rev_blocks(ctx, Ld, ldl, Dv + J, ldd, Da, ldla, bs);
      if (rc) return rc;
      Pm = smg_ws(ctx, SMG_WS_ALIAS, (size_t)bs * bs);
      if (!Pm) return SMG_ERR_OOM;
      hipLaunchKernelGGL(k_sym_from_half, dim3(grid_for((long long)bs * bs)), dim3(256), 0,
                         ctx->stream, Da, ldla, bs, Pm);
    }
    if (J > 0) {  // R_adj -= P R
      rc = smg_gemm_impl(ctx, 0, 0, 0, bs, J, bs, -1.0, Pm, bs, L + J, ldl, 1.0, La + J, ldla);
      if (rc) return rc;
    }
  }
  if (F) SMG_HIP_TRY(hipStreamWaitEvent(ctx->stream, F, 0));
  return SMG_OK;
}

// the factor streamed to the host panel by panel (smg_cholesky_fwd_checked_mark_stream)
// W = L^{-1} complete on stream s (the progressive rows' last part 1):
// ctx->inv_ev_w, chained behind its previous recording
int record_w_ready(smg_ctx* ctx, hipStream_t s) {
  if (ctx->inv_w_recorded) SMG_HIP_TRY(hipStreamWaitEvent(s, ctx->inv_ev_w, 0));
  SMG_HIP_TRY(hipEventRecord(ctx->inv_ev_w, s));
  ctx->inv_w_recorded = 1;
  return SMG_OK;
}

struct chol_stream_sink {
  double* packed;   // device, tril_count(n) doubles
  double* host;     // host (pinned), the same
  int marker_base;  // marker slot of panel 0
};
int chol_fwd(smg_ctx* ctx, const double* A, int lda, int n, double* L, int ldl, double* Dinv,
             bool check_sym, bool mark = false, double* inv_ws = nullptr, int* inv_started = nullptr,
             const chol_stream_sink* sink = nullptr, bool w_only = false);

}  // namespace

// the 128- / 256- / 512-row diagonal-block inverses of a lower L from the
// 64-row ones (aux: n x SMG_AUX_COLS, ld n, 64-row level filled)
int smg_block_inverses_impl(smg_ctx* ctx, const double* L, int ldl, double* aux, int n) {
  return chol_block_inverses(ctx, L, ldl, aux, n);
}
int smg_block_inverses_rows(smg_ctx* ctx, const double* L, int ldl, double* aux, int n, int row0, int nrows,
                            double* T, double* Wout, bool* wrote) {
  return chol_block_inverses(ctx, L, ldl, aux, n, row0, nrows, T, true, Wout, wrote);  // (behind chol_fwd's panels)
}

extern "C" {

int smg_cholesky_block_size(int n) { return SMG_NB; }

int smg_inv_block_fused(smg_ctx* ctx, int n) { return ctx && n > 0 ? (inv_fused_ok(ctx, n) ? 1 : 0) : -1; }

// aux = the 64-, 128-, 256- and 512-row diagonal-block inverses, n rows each, ld n
long long smg_cholesky_aux_doubles(int n) {
  return (long long)(n > 0 ? n : 0) * SMG_AUX_COLS;
}

int smg_check_symmetric(smg_ctx* ctx, const double* A, int lda, int n) {
  if (!ctx || n < 0 || (n > 0 && (!A || lda < n))) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  const int tb = smg_ceil_div(n, 64);
  hipLaunchKernelGGL(k_check_symmetric, dim3(tb * (tb + 1) / 2), dim3(256), 0, ctx->stream, A, lda,
                     n, ctx->status_d);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_cholesky_fwd(smg_ctx* ctx, const double* A, int lda, int n, double* L, int ldl,
                     double* Dinv) {
  return chol_fwd(ctx, A, lda, n, L, ldl, Dinv, false);
}

int smg_cholesky_fwd_checked(smg_ctx* ctx, const double* A, int lda, int n, double* L, int ldl,
                             double* Dinv) {
  return chol_fwd(ctx, A, lda, n, L, ldl, Dinv, true);
}

int smg_cholesky_fwd_checked_mark(smg_ctx* ctx, const double* A, int lda, int n, double* L, int ldl,
                                  double* Dinv) {
  return chol_fwd(ctx, A, lda, n, L, ldl, Dinv, true, true);
}

int smg_cholesky_fwd_checked_mark_inv(smg_ctx* ctx, const double* A, int lda, int n, double* L, int ldl,
                                      double* Dinv, double* ws, int* started) {
  if (!started) return SMG_ERR_ARG;
  *started = 0;
  if (ws && !Dinv) return SMG_ERR_ARG;
  return chol_fwd(ctx, A, lda, n, L, ldl, Dinv, true, true, ws, started);
}

int smg_cholesky_fwd_checked_mark_winv(smg_ctx* ctx, const double* A, int lda, int n, double* L, int ldl,
                                       double* Dinv, double* ws, int* started) {
  if (!started) return SMG_ERR_ARG;
  *started = 0;
  if (!ws || !Dinv) return SMG_ERR_ARG;
  return chol_fwd(ctx, A, lda, n, L, ldl, Dinv, true, true, ws, started, nullptr, true);
}

int smg_cholesky_inverse_wait(smg_ctx* ctx) {
  if (!ctx) return SMG_ERR_ARG;
  if (!ctx->inv_w_recorded) return SMG_ERR_ARG;
  SMG_HIP_TRY(hipStreamWaitEvent(ctx->stream, ctx->inv_ev_w, 0));
  return SMG_OK;
}

int smg_cholesky_stream_panels(int n) { return n <= 0 ? 0 : smg_ceil_div(n, n > SMG_NBF ? SMG_NBF : n); }

int smg_cholesky_fwd_checked_mark_stream(smg_ctx* ctx, const double* A, int lda, int n, double* L, int ldl,
                                         double* Dinv, double* ws, int* started, double* packed, double* host_dst,
                                         int marker_base) {
  if (!started || !packed || !host_dst || marker_base < 0) return SMG_ERR_ARG;
  *started = 0;
  if (ws && !Dinv) return SMG_ERR_ARG;
  if (marker_base + smg_cholesky_stream_panels(n) > 64) return SMG_ERR_ARG;
  if (!ctx || smg_zero_stream_begin(ctx) != SMG_OK) return SMG_ERR_HIP;
  const chol_stream_sink sink{packed, host_dst, marker_base};
  const int rc = chol_fwd(ctx, A, lda, n, L, ldl, Dinv, true, true, ws, started, &sink);
  // an error after some panel copies were queued: they still target host_dst,
  // which the caller may free or regrow once this returns
  if (rc != SMG_OK) {
    hipStreamSynchronize(ctx->zero_stream);
    if (ctx->copy_stream) hipStreamSynchronize(ctx->copy_stream);
  }
  return rc;
}

int smg_cholesky_stream_panel_cols(int n, int p, int* j0, int* j1) {
  const int np = smg_cholesky_stream_panels(n);
  if (!j0 || !j1 || p < 0 || p >= np) return SMG_ERR_ARG;
  const int nb2 = n > SMG_NBF ? SMG_NBF : n;  // chol_fwd's panel width
  *j0 = p * nb2;
  *j1 = min(n, *j0 + nb2);
  return SMG_OK;
}

}  // extern "C"

namespace {

int chol_fwd(smg_ctx* ctx, const double* A, int lda, int n, double* L, int ldl, double* Dinv,
             bool check_sym, bool mark, double* inv_ws, int* inv_started, const chol_stream_sink* sink,
             bool w_only) {
  if (!ctx || n < 0 || (n > 0 && (!A || !L || lda < n || ldl < n))) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  smg_prof_scope prof(ctx, SMG_FAM_CHOL_FWD);
  double* aux = Dinv;
  if (!aux) {
    aux = smg_ws(ctx, SMG_WS_TMP2, (size_t)smg_cholesky_aux_doubles(n));
    if (!aux) return SMG_ERR_OOM;
  }
  Dinv = aux;  // the SMG_NB level comes first
  const int tb = smg_ceil_div(n, 64);
  if (A != L || lda != ldl) {
    if (check_sym && n % 64 == 0 && lda % 2 == 0 && ldl % 2 == 0 &&
        ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(L)) & 15) == 0)
      hipLaunchKernelGGL(k_check_symmetric_copy2, dim3(tb * (tb + 1) / 2), dim3(256), 0,
                         ctx->stream, A, lda, n, ctx->status_d, L, ldl);
    else if (check_sym)
      hipLaunchKernelGGL(k_check_symmetric_copy, dim3(tb * (tb + 1) / 2), dim3(256), 0, ctx->stream, A,
                         lda, n, ctx->status_d, L, ldl);
    else
      hipLaunchKernelGGL(k_copy_lower, dim3(grid_for((long long)n * n)), dim3(256), 0, ctx->stream,
                         A, lda, n, L, ldl);
  } else if (check_sym) {
    hipLaunchKernelGGL(k_check_symmetric, dim3(tb * (tb + 1) / 2), dim3(256), 0, ctx->stream, A, lda,
                       n, ctx->status_d);
  }
  // queued adjoint zeroings overlap the latency-bound panels, not the copy
  if (int e = smg_zero_flush(ctx)) return e;
  // Two-level right-looking: panels of SMG_NBF columns factored with SMG_NB
  // steps whose updates stay inside the panel (all rows below), then ONE
  // rank-SMG_NBF update of the trailing matrix per panel (compute-bound, vs a
  // memory-bound rank-SMG_NB update per step).  n <= 2 SMG_NBF: one level.
  //
  // Look-ahead: panel p's trailing update is split into
  //   (a) the next panel's columns  A[K:, K:K2] -= P P[0:K2-K]^T  (main stream)
  //   (b) the rest                  A[K2:, K2:] -= P2 P2^T        (side stream)
  // so that (b), the bulk of the rank-NB2 work, runs on the CUs the next
  // panel's chain leaves idle while (a), on the chain's critical path, runs
  // alone.  Ordering (E = (a) done, F = (b) done):
  //   main: panel_p, wait F_{p-1}, (a)_p, rec E_p, panel_{p+1} ...
  //   side: wait E_p, (b)_p, rec F_p
  // (a)_p and (b)_{p-1} both update columns K_p:K_{p+1}, hence the wait;
  // (b)_p is disjoint from panel p+1's columns.
  // (panels never exceed SMG_NBF = PANEL_MAX_STEPS x SMG_NB columns: the
  // flag arrays of k_chol_panel hold PANEL_MAX_STEPS steps)
  static_assert(SMG_NBF <= PANEL_MAX_STEPS * SMG_NB, "panel width");
  const int NB2 = n > SMG_NBF ? SMG_NBF : n;
  const bool look = NB2 < n && smg_side_begin(ctx) == SMG_OK;
  // K^{-1} for the closed-form reverse under an MVN (chol_mvn.hip), formed
  // progressively: block row k of W = L^{-1} and its rank-512 share of
  // K^{-1} on `side` behind each panel's trailing update (b), so that after
  // the last panel only that panel's own block row remains.  (On a stream of
  // their own the rows ran 2x slower overall: with GPU_MAX_HW_QUEUES = 4 a
  // fifth stream shares a hardware queue with another, here the panels'.)
  const bool prog = inv_ws && look && NB2 == SMG_NBR && smg_inv_prog_ok(n) && smg_inv_events(ctx) == SMG_OK;
  if (prog) {  // side follows the work queued so far (earlier readers of ws)
    SMG_HIP_TRY(hipEventRecord(ctx->inv_ev_main, ctx->stream));
    SMG_HIP_TRY(hipStreamWaitEvent(ctx->side, ctx->inv_ev_main, 0));
    smg_on_side on(ctx);
    if (int rc = smg_inv_prog_init(ctx, n, inv_ws)) return rc;
  }
  int nev = 0;       // pooled events used
  hipEvent_t init_ev = nullptr;  // C's zeroing on side (the zeroing stream's parts follow it)
  if (prog) {
    if (!(init_ev = smg_event(ctx, nev++))) return SMG_ERR_HIP;
    SMG_HIP_TRY(hipEventRecord(init_ev, ctx->side));
  }
  hipEvent_t F = nullptr;  // the pending (b) on the side stream
  // the block rows' parts (smg_inv_prog_row) queued on `side` behind each
  // trailing update (b)_p within the slack before (b)_{p+1} becomes ready
  // (the next panel and its look-ahead (a), minus (b)_p itself): queued
  // whole, the growing rows held back (b)_{p+1}, the next (a) waiting for it,
  // and with it the next panel; what does not fit goes after the last panel
  int q_k = 0, q_part = 0;  // the next part to queue (all parts on `side`)
  const int rows_prog = prog ? n / SMG_NBR : 0;
  // With the zeroing stream (idle during the panels): a row's chain of
  // latency-bound parts -- its 256/512-level inverses (~8 small launches),
  // W_{k,0:k} and Y_{k+1} -- runs there as soon as its panel is done (pe_ev);
  // only the K^{-1} shares (part 2, the bulk) go on `side` within the slack,
  // each after its row's W (w_ev).  C's accumulation order stays the rows'.
  const bool zero_parts = prog && smg_zero_stream_begin(ctx) == SMG_OK;
  std::vector<hipEvent_t> pe_ev(rows_prog, nullptr), w_ev(rows_prog, nullptr);
  int z_k = 0, s_k = 0;  // next row for the zeroing stream's parts / the next share
  auto queue_zero = [&](int kmax) -> int {
    while (z_k <= kmax && z_k < rows_prog - 1) {
      if (!pe_ev[z_k] || !(w_ev[z_k] = smg_event(ctx, nev++))) return SMG_ERR_HIP;
      if (z_k == 0) SMG_HIP_TRY(hipStreamWaitEvent(ctx->zero_stream, init_ev, 0));
      SMG_HIP_TRY(hipStreamWaitEvent(ctx->zero_stream, pe_ev[z_k], 0));
      hipStream_t keep = ctx->stream;
      ctx->stream = ctx->zero_stream;
      int rc = smg_inv_prog_row(ctx, L, ldl, aux, n, inv_ws, z_k, 0, true);
      if (!rc) rc = smg_inv_prog_row(ctx, L, ldl, aux, n, inv_ws, z_k, 1, true);
      if (!rc && hipEventRecord(w_ev[z_k], ctx->zero_stream) != hipSuccess) rc = SMG_ERR_HIP;
      if (!rc) rc = smg_inv_prog_row(ctx, L, ldl, aux, n, inv_ws, z_k, 3, true);  // the next row's Y
      if (!rc) rc = smg_inv_prog_row(ctx, L, ldl, aux, n, inv_ws, z_k, 4, true);  // the later rows' Y
      ctx->stream = keep;
      if (rc) return rc;
      ++z_k;
    }
    return SMG_OK;
  };
  auto queue_shares = [&](double budget_us) -> int {  // budget < 0: every row queued on zero so far
    if (w_only) return SMG_OK;  // (W alone: no K^{-1} shares)
    // (a share may overrun the budget by this much -- r05z5, three same-box pairs: 40 379.8, 0 374.4,
    // 80 374.5, 150 375.3 evals/s)
    constexpr double tol = 40.0;
    while (s_k < z_k) {
      const double c = smg_inv_prog_cost(n, s_k, 2, true);
      if (budget_us >= 0 && c > budget_us + tol) break;
      budget_us -= c;
      SMG_HIP_TRY(hipStreamWaitEvent(ctx->side, w_ev[s_k], 0));
      smg_on_side on(ctx);
      if (int rc = smg_inv_prog_row(ctx, L, ldl, aux, n, inv_ws, s_k, 2, true)) return rc;
      ++s_k;
    }
    return SMG_OK;
  };
  auto queue_parts = [&](int kmax, double budget_us) -> int {  // budget < 0: all of rows <= kmax
    if (zero_parts) {
      if (int rc = queue_zero(kmax)) return rc;
      return queue_shares(budget_us);
    }
    static const int order[5] = {0, 1, 3, 4, 2};  // W_k first, then its Y contributions, its share last
    const int nparts = w_only ? 4 : 5;
    while (q_k <= kmax && q_k < rows_prog - 1) {
      const double c = smg_inv_prog_cost(n, q_k, order[q_part], true);
      if (budget_us >= 0 && c > budget_us + 40.0) break;
      budget_us -= c;
      smg_on_side on(ctx);
      if (int rc = smg_inv_prog_row(ctx, L, ldl, aux, n, inv_ws, q_k, order[q_part], true)) return rc;
      if (++q_part == nparts) {
        q_part = 0;
        ++q_k;
      }
    }
    return SMG_OK;
  };
  for (int J = 0; J < n; J += NB2) {
    const int K = min(J + NB2, n);
    {  // the whole panel in one persistent launch (k_chol_panel)
      // workgroup 0 = diagonal chain; tiles 1 .. T-1 over the others
      const int T = panel_tiles(n, J, smg_ceil_div(K - J, SMG_NB));
      // chain, inverter, owners of tiles 1..T-1; paired: owners of the panel
      // tiles 1..nb-1 and one workgroup per pair of 32-row tiles below
      const int nbq = smg_ceil_div(K - J, SMG_NB);
      const int npairs = (T - nbq + 1) / 2;
      const int paired = nbq + 1 + npairs <= PANEL_MAX_GRID + 1 - (nbq > 3 ? 2 * nbq - 7 : 0) ? 1 : 0;
      const int grid = paired ? nbq + 1 + npairs : (T < PANEL_MAX_GRID ? T : PANEL_MAX_GRID) + 1;
      const int epoch = ++ctx->flag_epoch;
      ctx->status_armed = 1;
      // column helpers for panel tiles 3 .. nb-1
      const int nbp = smg_ceil_div(K - J, SMG_NB);
      int nha = nbp > 3 ? nbp - 3 : 0, nhb = nbp > 4 ? nbp - 4 : 0;  // helpers A (tiles 3..), B (tiles 4..)
      if (grid + nha + nhb > PANEL_MAX_GRID + 1 || nbp > T) nha = nhb = 0;
      smg_prof_scope pprof(ctx, SMG_FAM_PANEL);  // (the launch alone: bench.py's dominant-kernel roofline)
      if (ctx->prof_on) {  // in-panel work: the diagonal block's factor + the rows below's solve
        const double m = n - J, b = K - J;
        ctx->prof_flops[SMG_FAM_PANEL] += m * b * b - 2.0 * b * b * b / 3.0;
      }
      panel_host_stamp(epoch);
      hipLaunchKernelGGL(k_chol_panel, dim3(grid + nha + nhb), dim3(SMG_DIAG_THREADS), 0, ctx->stream, L, ldl,
                         n, J, K, Dinv, n, ctx->flags_d, epoch, ctx->status_d, grid, nha, paired);
    }
    if (zero_parts && J / NB2 < rows_prog) {  // this panel is final: its block row's inverses may start
      if (!(pe_ev[J / NB2] = smg_event(ctx, nev++))) return SMG_ERR_HIP;
      SMG_HIP_TRY(hipEventRecord(pe_ev[J / NB2], ctx->stream));
    }
    if (sink) {  // columns [J, K) are final: packed and copied to the host on the copy stream
      // (on the zeroing stream each copy held back the block-row chain queued behind it, the K^{-1}
      // shares waiting for that, and the trailing updates queued after those: in a gp_eigen trace the
      // eight panels spanned 4.8 ms with the copies at 28 GB/s, 3.3 ms at 55 GB/s on a stream of their own)
      if (!ctx->copy_stream && hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking) != hipSuccess) {
        ctx->copy_stream = nullptr;
        return SMG_ERR_HIP;
      }
      hipStream_t cs = ctx->copy_stream;
      hipEvent_t Pe = smg_event(ctx, nev++), Me = nullptr;
      if (!Pe) return SMG_ERR_HIP;
      if (int rc = smg_marker_event(ctx, sink->marker_base + J / NB2, &Me)) return rc;
      SMG_HIP_TRY(hipEventRecord(Pe, ctx->stream));
      SMG_HIP_TRY(hipStreamWaitEvent(cs, Pe, 0));
      hipStream_t keep = ctx->stream;
      ctx->stream = cs;
      const int prc = smg_pack_tril_cols(ctx, n, L, ldl, J, K, sink->packed);
      ctx->stream = keep;
      if (prc) return prc;
      const size_t o0 = (size_t)J * n - (size_t)J * (J - 1) / 2, o1 = (size_t)K * n - (size_t)K * (K - 1) / 2;
      if (int rc = smg_d2h_impl(ctx, cs, sink->host + o0, sink->packed + o0, (o1 - o0) * sizeof(double))) return rc;
      SMG_HIP_TRY(hipEventRecord(Me, cs));
    }
    if (K >= n) break;
    const int m = n - K;
    const double* P = L + K + (size_t)J * ldl;
    if (!look) {  // trailing A[K:, K:] -= L[K:, J:K] L[K:, J:K]^T (lower)
      int rc = smg_gemm_impl(ctx, 0, 1, 1, m, m, K - J, -1.0, P, ldl, P, ldl, 1.0,
                             L + K + (size_t)K * ldl, ldl);
      if (rc) return rc;
      continue;
    }
    const int K2 = min(K + NB2, n);
    hipEvent_t E = smg_event(ctx, nev++);
    if (!E) return SMG_ERR_HIP;
    if (F) SMG_HIP_TRY(hipStreamWaitEvent(ctx->stream, F, 0));
    int rc = 0;
    // (a) the next panel's columns (lower trapezoid), main stream
    if ((rc = smg_gemm_impl(ctx, 0, 1, 1, m, K2 - K, K - J, -1.0, P, ldl, P, ldl, 1.0, L + K + (size_t)K * ldl, ldl)))
      return rc;
    SMG_HIP_TRY(hipEventRecord(E, ctx->stream));
    F = nullptr;
    if (K2 < n) {  // (b) the rest, side stream
      const int m2 = n - K2;
      const double* P2 = L + K2 + (size_t)J * ldl;
      SMG_HIP_TRY(hipStreamWaitEvent(ctx->side, E, 0));
      // (b) in two: (b1), the columns of the panel after next (all the next
      // look-ahead (a) waits for: F), and (b2), the rest behind it (GP
      // 355-358 -> 358-360 evals/s in a same-box A/B)
      const int K3 = min(K2 + NB2, n);
      {
        smg_on_side on(ctx);
        rc = smg_gemm_impl(ctx, 0, 1, 1, m2, K3 - K2, K - J, -1.0, P2, ldl, P2, ldl, 1.0,
                           L + K2 + (size_t)K2 * ldl, ldl);
      }
      if (rc) return rc;
      F = smg_event(ctx, nev++);
      if (!F) return SMG_ERR_HIP;
      SMG_HIP_TRY(hipEventRecord(F, ctx->side));
      if (K3 < n) {  // (b2)
        const int m3 = n - K3;
        const double* P3 = L + K3 + (size_t)J * ldl;
        smg_on_side on(ctx);
        if ((rc = smg_gemm_impl(ctx, 0, 1, 1, m3, m3, K - J, -1.0, P3, ldl, P3, ldl, 1.0, L + K3 + (size_t)K3 * ldl,
                                ldl)))
          return rc;
      }
    } else if (prog) {  // no (b): the side stream still follows this panel
      SMG_HIP_TRY(hipStreamWaitEvent(ctx->side, E, 0));
    }
    if (prog) {  // (F is recorded before them: the next (a) does not wait for them)
      // slack: the next panel (~22 us per 64-column step) and its (a), at
      // ~30 TF/s, minus (b) at ~40 TF/s
      const double m2 = n - K2, kk = K - J;
      const double slack = 22.0 * (K2 - K) / SMG_NB + 6.0 + (double)(n - K) * (K2 - K) * kk / 30e6 -
                           (K2 < n ? 6.0 + m2 * m2 * kk / 40e6 : 0.0);
      // queued against HALF that estimate: since the K^{-1} / Y parts stopped clearing their outputs and
      // the block-row inverses became one launch, the full estimate measures slower
      // (same-box A/Bs of the scale, r05y / r05z2 / r05z3: 0.5 380.5 and 379.9, 0.65 379.0, 1.0 374.8
      // and 376.0, 0.4 371, 0.25 373.6, 0 370.6 evals/s)
      if ((rc = queue_parts(J / NB2, 0.5 * slack))) return rc;
    }
  }
  if (prog) {  // the rest of the rows but the last
    if (int rc0 = queue_parts(rows_prog - 2, -1.0)) return rc0;
  }
  // every launch that can latch the status (the symmetric check, the panels'
  // not-PD and hand-off bits) is enqueued: the status mark goes here, so a
  // host waiting on it does not also wait for the block inverses below
  if (mark) {
    const int rc = smg_status_mark_impl(ctx);
    if (rc) return rc;
  }
  if (F) SMG_HIP_TRY(hipStreamWaitEvent(ctx->stream, F, 0));
  // the 128-, 256- and 512-block inverses (reverse pass, triangular solves);
  // progressive: every block row's but the last were formed on `side`, the
  // last one's here on the main stream (idle after the last panel), then the
  // last block row of W and its K^{-1} update go to `side`, overlapping the
  // MVN's forward solves and the host's work up to the reverse
  int rc;
  if (prog) {
    const int r0 = n - SMG_NBR;
    SMG_HIP_TRY(hipStreamWaitEvent(ctx->stream, ctx->inv_ev_aux, 0));
    bool wkk = false;  // W_last's diagonal block written by the inverse launch itself
    if ((rc = chol_block_inverses(ctx, L, ldl, aux, n, r0, SMG_NBR, nullptr, true, inv_ws + r0 + (size_t)r0 * n,
                                  &wkk)))
      return rc;
    SMG_HIP_TRY(hipEventRecord(ctx->inv_ev_main, ctx->stream));
    const int klast = n / SMG_NBR - 1;
    if (zero_parts) {  // W_last on the zeroing stream behind the last Y, its share on side
      SMG_HIP_TRY(hipStreamWaitEvent(ctx->zero_stream, ctx->inv_ev_main, 0));
      hipStream_t keep = ctx->stream;
      ctx->stream = ctx->zero_stream;
      rc = wkk ? SMG_OK : smg_inv_prog_row(ctx, L, ldl, aux, n, inv_ws, klast, 0, false);
      if (!rc) rc = smg_inv_prog_row(ctx, L, ldl, aux, n, inv_ws, klast, 1, false);
      ctx->stream = keep;
      if (rc) return rc;
      if ((rc = record_w_ready(ctx, ctx->zero_stream))) return rc;
      SMG_HIP_TRY(hipStreamWaitEvent(ctx->side, ctx->inv_ev_w, 0));
      smg_on_side on(ctx);
      if (!w_only && (rc = smg_inv_prog_row(ctx, L, ldl, aux, n, inv_ws, klast, 2, false))) return rc;
    } else {
      SMG_HIP_TRY(hipStreamWaitEvent(ctx->side, ctx->inv_ev_main, 0));
      smg_on_side on(ctx);
      for (int part = 0; part < (w_only ? 2 : 3); ++part) {  // (the last row adds to no later row's Y)
        if (part == 0 && wkk) continue;
        if ((rc = smg_inv_prog_row(ctx, L, ldl, aux, n, inv_ws, klast, part, false))) return rc;
        if (part == 1 && (rc = record_w_ready(ctx, ctx->side))) return rc;
      }
    }
    // its writes to ws are joined before anything on the main stream may
    // touch ws (smg_cholesky_mvn_rev_v / smg_join_async)
    SMG_HIP_TRY(hipEventRecord(ctx->inv_ev, ctx->side));
    ctx->inv_pending = 1;
    *inv_started = w_only ? 3 : 2;
  } else if ((rc = chol_block_inverses(ctx, L, ldl, aux, n, 0, -1, nullptr, true))) {
    return rc;
  }
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

}  // namespace

extern "C" {

int smg_cholesky_rev(smg_ctx* ctx, const double* L, int ldl, const double* Dinv, double* La,
                     int ldla, int n, double* Aadj, int ldaa) {
  if (!ctx || n < 0 || (n > 0 && (!L || !La || !Aadj || ldl < n || ldla < n || ldaa < n)))
    return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  smg_prof_scope prof(ctx, SMG_FAM_CHOL_REV);
  const double* aux = Dinv;
  if (!aux) {  // no forward aux: rebuild the block inverses from L
    double* w = smg_ws(ctx, SMG_WS_TMP2, (size_t)smg_cholesky_aux_doubles(n));
    if (!w) return SMG_ERR_OOM;
    for (int j = 0; j < n; j += SMG_NB) {
      const int b = min(SMG_NB, n - j);
      hipLaunchKernelGGL(k_trtri_diag, dim3(1), dim3(SMG_DIAG_THREADS), 0, ctx->stream,
                         L + j + (size_t)j * ldl, ldl, b, w + j, n);
    }
    int rc = chol_block_inverses(ctx, L, ldl, w, n);
    if (rc) return rc;
    aux = w;
  }
  int rc = n > 2 * SMG_NBR ? chol_rev_two_level(ctx, L, ldl, aux, n, La, ldla)
                           : chol_rev_blocks(ctx, L, ldl, aux, n, La, ldla, n);
  if (rc) return rc;
  if (n % 2 == 0 && ldla % 2 == 0 && ldaa % 2 == 0 &&
      ((reinterpret_cast<uintptr_t>(La) | reinterpret_cast<uintptr_t>(Aadj)) & 15) == 0)
    hipLaunchKernelGGL(k_add_lower_col2, dim3(n < 2048 ? n : 2048), dim3(256), 0, ctx->stream, La,
                       ldla, n, Aadj, ldaa);
  else
    hipLaunchKernelGGL(k_add_lower, dim3(grid_for((long long)n * n)), dim3(256), 0, ctx->stream,
                       La, ldla, n, Aadj, ldaa);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

}  // extern "C"
