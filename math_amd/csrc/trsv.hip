// Triangular solves with ONE right-hand side (the two solves of
// multi_normal_cholesky_lpdf, prim/mat/prob/multi_normal_cholesky_lpdf.hpp:
// 117-131), blocked on diagonal blocks whose inverses W_p the Cholesky
// forward already produced (the aux buffer: 64-, 128- and 256-row levels).
//
//   forward  y = L^{-1} x : for p = 0..:  y_p = W_p r_p;   r[k:] -= L[k:, p] y_p
//   backward y = L^{-T} x : for p = ..0:  y_p = W_p^T r_p; r[:j] -= L[p, :j]^T y_p
//
// One launch per block step: every workgroup recomputes the diagonal product
// redundantly from L2 (no inter-workgroup hand-off inside a launch),
// workgroup 0 publishes y_p, and each workgroup updates its slice of the
// residual.  Reads of L are coalesced in both directions.  With the 256-row
// inverses a solve takes n/256 steps instead of n/64 (the steps are
// latency-bound launches, so the count is what matters); a ragged tail uses
// the 64-row level.
#include "smg_internal.h"
#include "smg_sync.h"
#include "tri_small.h"

namespace {

constexpr int ROWS = 256;  // residual rows (forward) / entries (backward) per workgroup

// yp = W_p rp (trans == 0) or W_p^T rp (trans == 1); rp, yp in LDS; 256 threads
template <int TB>
__device__ inline void diag_apply(const double* __restrict__ W, int ldw, int j, int b, int trans,
                                  const double* rp, double* yp, double* part) {
  const int t = threadIdx.x;
  if (TB == 64) {
    // row / column t&63 of W_p, quarter t>>6 of the other index
    const int r = t & 63, q = t >> 6;
    double s = 0.0;
    if (r < b) {
      if (!trans) {
#pragma unroll 4
        for (int c = 16 * q; c < 16 * q + 16 && c < b; ++c) s += W[j + r + (size_t)c * ldw] * rp[c];
      } else {
#pragma unroll 4
        for (int c = 16 * q; c < 16 * q + 16 && c < b; ++c) s += W[j + c + (size_t)r * ldw] * rp[c];
      }
    }
    part[q * 64 + r] = s;
    __syncthreads();
    if (t < 64) yp[t] = (part[t] + part[64 + t]) + (part[128 + t] + part[192 + t]);
  } else {
    // 1024 threads: row (column) t = tid & 255, quarter q = tid >> 8 of the
    // other index; W_p is lower triangular
    const int r = t & 255, q = t >> 8;
    double s0 = 0.0, s1 = 0.0;
    if (r < b) {
      const int c0 = 64 * q, c1 = min(64 * q + 64, b);
      if (!trans) {
        const int ce = min(c1, r + 1);
#pragma unroll 4
        for (int c = c0; c < ce; c += 2) {
          s0 += W[j + r + (size_t)c * ldw] * rp[c];
          if (c + 1 < ce) s1 += W[j + r + (size_t)(c + 1) * ldw] * rp[c + 1];
        }
      } else {
        const double* Wc = W + j + (size_t)r * ldw;  // column r of W_p (contiguous)
#pragma unroll 4
        for (int c = max(c0, r); c < c1; c += 2) {
          s0 += Wc[c] * rp[c];
          if (c + 1 < c1) s1 += Wc[c + 1] * rp[c + 1];
        }
      }
    }
    part[q * 256 + r] = s0 + s1;
    __syncthreads();
    if (t < 256) yp[t] = (part[t] + part[256 + t]) + (part[512 + t] + part[768 + t]);
  }
  __syncthreads();
}

// 256 threads for the 64-row level, 1024 for the 256-row level (each row's
// dot product split over 4 threads, partial sums combined in LDS)
template <int TB>
__global__ __launch_bounds__(TB == 64 ? 256 : 1024) void k_trsv_fwd(
    const double* __restrict__ L, int ldl, const double* __restrict__ W, int ldw,
    double* __restrict__ r, double* __restrict__ y, int n, int j, int b) {
  constexpr int NT = TB == 64 ? 256 : 1024;
  __shared__ double rp[TB], yp[256], part[NT];
  const int t = threadIdx.x;
  if (t < TB) rp[t] = t < b ? r[j + t] : 0.0;
  __syncthreads();
  diag_apply<TB>(W, ldw, j, b, 0, rp, yp, part);
  if (blockIdx.x == 0 && t < b) y[j + t] = yp[t];
  const int k = j + b;
  const int row = t & (ROWS - 1), q = t / ROWS;  // q = 0 for the 64-row level
  const int i = k + blockIdx.x * ROWS + row;
  constexpr int NQ = NT / ROWS;
  const int c0 = (b * q) / NQ, c1 = (b * (q + 1)) / NQ;
  double s0 = 0.0, s1 = 0.0;
  if (i < n) {
    const double* Lc = L + i + (size_t)j * ldl;
#pragma unroll 4
    for (int c = c0; c < c1; c += 2) {
      s0 += Lc[(size_t)c * ldl] * yp[c];
      if (c + 1 < c1) s1 += Lc[(size_t)(c + 1) * ldl] * yp[c + 1];
    }
  }
  if (NQ == 1) {
    if (i < n) r[i] -= s0 + s1;
    return;
  }
  __syncthreads();
  part[t] = s0 + s1;
  __syncthreads();
  if (q == 0 && i < n) r[i] -= (part[row] + part[ROWS + row]) + (part[2 * ROWS + row] + part[3 * ROWS + row]);
}

template <int TB>
__global__ __launch_bounds__(TB == 64 ? 256 : 1024) void k_trsv_bwd(
    const double* __restrict__ L, int ldl, const double* __restrict__ W, int ldw,
    double* __restrict__ r, double* __restrict__ y, int j, int b) {
  constexpr int NT = TB == 64 ? 256 : 1024;
  __shared__ double rp[TB], yp[256], part[NT];
  const int t = threadIdx.x;
  if (t < TB) rp[t] = t < b ? r[j + t] : 0.0;
  __syncthreads();
  diag_apply<TB>(W, ldw, j, b, 1, rp, yp, part);
  if (blockIdx.x == 0 && t < b) y[j + t] = yp[t];
  // r[i] -= sum_c L[j + c, i] yp[c]: thread (i, q) walks part q of the
  // contiguous segment L[j:j+b, i] of column i
  const int col = t & (ROWS - 1), q = t / ROWS;
  const int i = blockIdx.x * ROWS + col;
  constexpr int NQ = NT / ROWS;
  const int c0 = (b * q) / NQ, c1 = (b * (q + 1)) / NQ;
  double s0 = 0.0, s1 = 0.0;
  if (i < j) {
    const double* Lc = L + j + (size_t)i * ldl;
#pragma unroll 4
    for (int c = c0; c < c1; c += 2) {
      s0 += Lc[c] * yp[c];
      if (c + 1 < c1) s1 += Lc[c + 1] * yp[c + 1];
    }
  }
  if (NQ == 1) {
    if (i < j) r[i] -= s0 + s1;
    return;
  }
  __syncthreads();
  part[t] = s0 + s1;
  __syncthreads();
  if (q == 0 && i < j) r[i] -= (part[col] + part[ROWS + col]) + (part[2 * ROWS + col] + part[3 * ROWS + col]);
}

// ---- 256-row level: two launches per step ---------------------------------
// (1) y_p = W_p r_p (or W_p^T r_p), published to y; 16 workgroups of 256
//     threads, 16 outputs each, so W_p (256 KB) streams through 16 CUs
__global__ __launch_bounds__(256) void k_trsv_diag256(const double* __restrict__ W, int ldw,
                                                      const double* __restrict__ r,
                                                      double* __restrict__ y, int j, int b,
                                                      int trans) {
  __shared__ double rp[256], part[256];
  const int t = threadIdx.x;
  rp[t] = t < b ? r[j + t] : 0.0;
  __syncthreads();
  if (!trans) {
    // rows 16g + (t & 15); part (t >> 4) covers columns 16 part .. +15; W lower
    const int row = 16 * blockIdx.x + (t & 15), pc = t >> 4;
    double s = 0.0;
    if (row < b)
#pragma unroll
      for (int c = 16 * pc; c < 16 * pc + 16; ++c)
        if (c <= row) s += W[j + row + (size_t)c * ldw] * rp[c];
    part[t] = s;
    __syncthreads();
    if (t < 16 && 16 * blockIdx.x + t < b) {
      double a = 0.0;
#pragma unroll
      for (int q = 0; q < 16; ++q) a += part[16 * q + t];
      y[j + 16 * blockIdx.x + t] = a;
    }
  } else {
    // column 16g + 4w + cc of W (contiguous), lanes along it, wave reduction
    const int lane = t & 63, w = t >> 6;
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) {
      const int col = 16 * blockIdx.x + 4 * w + cc;
      if (col >= b) break;
      const double* Wc = W + j + (size_t)col * ldw;
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c = lane + 64 * k;
        if (c >= col && c < b) s += Wc[c] * rp[c];
      }
      s = wave_sum(s);
      if (lane == 0) y[j + col] = s;
    }
  }
}

// (2a) forward update r[k:] -= L[k:, j:j+b] y_p: 64 rows per workgroup, each
//      row's dot split over 4 waves (coalesced column reads), LDS combine
__global__ __launch_bounds__(256) void k_trsv_upd_fwd(const double* __restrict__ L, int ldl,
                                                      const double* __restrict__ y,
                                                      double* __restrict__ r, int n, int j,
                                                      int b) {
  __shared__ double yp[256], part[256];
  const int t = threadIdx.x;
  yp[t] = t < b ? y[j + t] : 0.0;
  __syncthreads();
  const int row = t & 63, q = t >> 6;
  const int i = j + b + blockIdx.x * 64 + row;
  const int c0 = (b * q) / 4, c1 = (b * (q + 1)) / 4;
  double s0 = 0.0, s1 = 0.0;
  if (i < n) {
    const double* Lc = L + i + (size_t)j * ldl;
#pragma unroll 4
    for (int c = c0; c < c1; c += 2) {
      s0 += Lc[(size_t)c * ldl] * yp[c];
      if (c + 1 < c1) s1 += Lc[(size_t)(c + 1) * ldl] * yp[c + 1];
    }
  }
  part[t] = s0 + s1;
  __syncthreads();
  if (q == 0 && i < n) r[i] -= (part[row] + part[64 + row]) + (part[128 + row] + part[192 + row]);
}

// (2b) backward update r[i] -= L[j:j+b, i] . y_p for i < j: one wave per
//      column at a time, lanes along the contiguous segment, wave reduction
__global__ __launch_bounds__(256) void k_trsv_upd_bwd(const double* __restrict__ L, int ldl,
                                                      const double* __restrict__ y,
                                                      double* __restrict__ r, int j, int b) {
  __shared__ double yp[256];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  yp[t] = t < b ? y[j + t] : 0.0;
  __syncthreads();
#pragma unroll
  for (int cc = 0; cc < 4; ++cc) {  // 16 columns per workgroup: 4 waves x 4
    const int i = blockIdx.x * 16 + w * 4 + cc;
    if (i >= j) break;
    const double* Lc = L + j + (size_t)i * ldl;
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = lane + 64 * k;
      if (c < b) s += Lc[c] * yp[c];
    }
    s = wave_sum(s);
    if (lane == 0) r[i] -= s;
  }
}

struct trsv_step {
  int j, b, big;
};

// ---- persistent solve: ONE launch per solve (n % 256 == 0) ----------------
// Workgroup s owns the 64-row strip s (rows, forward; columns of L = rows of
// L^T, backward) of 256-row block p = s / 4.  It accumulates its residual
// from every published block of y it depends on (forward: blocks < p, in
// order; backward: blocks > p, from the last), publishes the residual strip
// (rf[s]), then -- once the four strips of block p have -- computes its 64
// entries of y_p = W_p r_p (W_p^T r_p) from the 256-row inverse and
// publishes them (yf[s]).  The critical path per block is one 64 x 256
// residual product and one 64 x 256 diagonal product, with two hand-offs;
// everything else overlaps.  All n / 64 workgroups must be co-resident
// (n / 64 <= 256 CUs; SMG_ERR_SYNC otherwise).
__device__ inline void wait_strips(const int* f, int s0, int cnt, int epoch, int* status) {
  panel_wait_all(f, s0, s0 + cnt - 1, 1, epoch, status);
}

// Column sums of the backward solve's per-lane partials: acc[cc] on lane l of
// wave w is the partial of column 16 (w & 3) + cc over rows 256 (w >> 2) + l,
// + 64, ...; the 64 column sums land in part[0 .. 63].  One LDS transpose and
// a (4 H)-lane reduction instead of 16 full-wave reductions per wave.
template <int H>
__device__ __forceinline__ void cols_reduce(const double (&acc)[16], double (*red)[64][65], double* part) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
#pragma unroll
  for (int cc = 0; cc < 16; ++cc) red[w >> 2][16 * (w & 3) + cc][lane] = acc[cc];
  __syncthreads();
  const int c = t / (4 * H), q = t % (4 * H);
  double v = 0.0;
#pragma unroll
  for (int k = 0; k < 16; ++k) v += red[q >> 2][c][16 * (q & 3) + k];
  v += __shfl_xor(v, 1);
  v += __shfl_xor(v, 2);
  if (H == 2) v += __shfl_xor(v, 4);
  if (q == 0) part[c] = v;
}

// BS: the diagonal-block size of the inverses used (256 or 512); BS threads
// per workgroup, G = BS / 64 strips per block.
template <bool TRANS, int BS>
__global__ __launch_bounds__(BS) void k_trsv_persist(const double* __restrict__ L, int ldl,
                                                     const double* __restrict__ W, int ldw,
                                                     const double* __restrict__ x,
                                                     double* __restrict__ y,
                                                     double* __restrict__ r, int n, int* flags,
                                                     int epoch, int* status) {
  // Operand reads never wait on a flag: this strip's W_p slice is loaded into
  // registers at entry, and each block of L is loaded before the wait for
  // the y block it multiplies, so only LDS traffic and FMAs follow a flag.
  constexpr int G = BS / 64, H = BS / 256;
  __shared__ double vp[BS];
  __shared__ double part[BS];
  __shared__ double red[TRANS ? H : 1][64][65];
  // (one workgroup per CU, the fence-free hand-off's residency rule in
  // smg_sync.h: the 256 VGPRs of wv / lv leave room for BS / 256 waves per
  // SIMD, i.e. this one workgroup)
  const int s = blockIdx.x, p = s / G, sub = s % G, nb = n / BS, ns = n >> 6;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  int* yf = flags;
  int* rf = flags + ns;
  double wv[64], lv[64];
  if (!TRANS) {
    // thread (row 64 s + lane, 64-column slice w of each BS-column block)
    const int i = 64 * s + lane;
    const double* Wr = W + (BS * p + 64 * sub + lane) + (size_t)(64 * w) * ldw;
#pragma unroll
    for (int k = 0; k < 64; ++k) wv[k] = Wr[(size_t)k * ldw];
    double acc0 = 0.0, acc1 = 0.0;
    for (int q = 0; q < p; ++q) {
      const double* Lc = L + i + (size_t)(BS * q + 64 * w) * ldl;
#pragma unroll
      for (int k = 0; k < 64; ++k) lv[k] = Lc[(size_t)k * ldl];
      wait_strips(yf, G * q, G, epoch, status);
      vp[t] = ld_dev(&y[BS * q + t]);
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 64; k += 2) {
        acc0 += lv[k] * vp[64 * w + k];
        acc1 += lv[k + 1] * vp[64 * w + k + 1];
      }
      __syncthreads();  // vp consumed
    }
    part[t] = acc0 + acc1;
    __syncthreads();
    if (w == 0) {
      double sum = 0.0;
#pragma unroll
      for (int g = 0; g < G; ++g) sum += part[64 * g + lane];
      st_dev(&r[i], x[i] - sum);
    }
    panel_publish(&rf[s], epoch);
    // y rows BS p + 64 sub + lane = W_p[64 sub + lane, :] r_p
    wait_strips(rf, G * p, G, epoch, status);
    vp[t] = ld_dev(&r[BS * p + t]);
    __syncthreads();
    acc0 = 0.0;
    acc1 = 0.0;
#pragma unroll
    for (int k = 0; k < 64; k += 2) {
      acc0 += wv[k] * vp[64 * w + k];
      acc1 += wv[k + 1] * vp[64 * w + k + 1];
    }
    part[t] = acc0 + acc1;
    __syncthreads();
    if (w == 0) {
      double sum = 0.0;
#pragma unroll
      for (int g = 0; g < G; ++g) sum += part[64 * g + lane];
      st_dev(&y[i], sum);
    }
    panel_publish(&yf[s], epoch);
  } else {
    // wave w: 16 columns j = 64 s + 16 (w & 3) + cc of L (rows of L^T) over
    // the row half h = w >> 2 of a BS-row block; lanes run down the
    // contiguous column segments (rows 256 h + lane + 64 k of a block)
    const int h = w >> 2;
    const int c0 = 64 * sub + 16 * (w & 3);
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int cc = 0; cc < 16; ++cc)
        wv[16 * k + cc] = W[(BS * p + 256 * h + lane + 64 * k) + (size_t)(c0 + cc) * ldw];
    double acc[16];
#pragma unroll
    for (int cc = 0; cc < 16; ++cc) acc[cc] = 0.0;
    const int j0 = 64 * s + 16 * (w & 3);
    for (int q = nb - 1; q > p; --q) {
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int cc = 0; cc < 16; ++cc)
          lv[16 * k + cc] = L[(BS * q + 256 * h + lane + 64 * k) + (size_t)(j0 + cc) * ldl];
      wait_strips(yf, G * q, G, epoch, status);
      vp[t] = ld_dev(&y[BS * q + t]);
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const double v = vp[256 * h + lane + 64 * k];
#pragma unroll
        for (int cc = 0; cc < 16; ++cc) acc[cc] += lv[16 * k + cc] * v;
      }
      __syncthreads();
    }
    cols_reduce<H>(acc, red, part);
    __syncthreads();
    if (t < 64) st_dev(&r[64 * s + t], x[64 * s + t] - part[t]);
    panel_publish(&rf[s], epoch);
    // y entries BS p + 64 sub + 16 (w & 3) + cc = W_p[:, col] . r_p
    wait_strips(rf, G * p, G, epoch, status);
    vp[t] = ld_dev(&r[BS * p + t]);
    __syncthreads();
#pragma unroll
    for (int cc = 0; cc < 16; ++cc) acc[cc] = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double v = vp[256 * h + lane + 64 * k];
#pragma unroll
      for (int cc = 0; cc < 16; ++cc) acc[cc] += wv[16 * k + cc] * v;
    }
    cols_reduce<H>(acc, red, part);
    __syncthreads();
    if (t < 64) st_dev(&y[BS * p + 64 * sub + t], part[t]);
    panel_publish(&yf[s], epoch);
  }
}

// flags region of the persistent solves (after the panel kernel's)
constexpr int TRSV_FLAG_OFFSET = 256;

}  // namespace

// y = L^{-1} x (trans = 0) or L^{-T} x (trans = 1); L lower.  W64: the 64-row
// diagonal-block inverses (n x 64, ld ldw); W256 / W512: the 256- / 512-row
// ones (ld ldw) or NULL.  r: n-double workspace.  The persistent solve takes
// n / BS block steps, so the 512-row level halves its hand-offs.
int smg_trsv_lower_impl(smg_ctx* ctx, int trans, const double* L, int ldl, const double* W64,
                        const double* W256, const double* W512, int ldw, const double* x, double* y,
                        double* r, int n) {
  if (n <= 0) return SMG_OK;
  // queued adjoint zeroings overlap this latency-bound solve
  if (int e = smg_zero_flush(ctx)) return e;
  const bool fits = n / 64 <= 256 && TRSV_FLAG_OFFSET + 2 * (n / 64) <= 4096;
  // forward only: the backward's 512-row form needs 32 more VGPRs per lane
  // than two waves per SIMD leave and spills (100 vs 83 us at n = 4096);
  // the forward's spills less and gains (65 vs 75 us)
  if (fits && !trans && W512 && n % 512 == 0 && n >= 1024) {
    const int epoch = ++ctx->flag_epoch;
    int* f = ctx->flags_d + TRSV_FLAG_OFFSET;
    ctx->status_armed = 1;
    hipLaunchKernelGGL((k_trsv_persist<false, 512>), dim3(n / 64), dim3(512), 0, ctx->stream, L, ldl,
                       W512, ldw, x, y, r, n, f, epoch, ctx->status_d);
    SMG_LAUNCH_CHECK();
    return SMG_OK;
  }
  if (fits && W256 && n % 256 == 0 && n >= 512) {
    const int epoch = ++ctx->flag_epoch;
    int* f = ctx->flags_d + TRSV_FLAG_OFFSET;
    ctx->status_armed = 1;
    if (trans)
      hipLaunchKernelGGL((k_trsv_persist<true, 256>), dim3(n / 64), dim3(256), 0, ctx->stream, L, ldl,
                         W256, ldw, x, y, r, n, f, epoch, ctx->status_d);
    else
      hipLaunchKernelGGL((k_trsv_persist<false, 256>), dim3(n / 64), dim3(256), 0, ctx->stream, L, ldl,
                         W256, ldw, x, y, r, n, f, epoch, ctx->status_d);
    SMG_LAUNCH_CHECK();
    return SMG_OK;
  }
  hipMemcpyAsync(r, x, sizeof(double) * n, hipMemcpyDeviceToDevice, ctx->stream);
  // block schedule: full 256-row blocks from the top, then 64-row blocks
  trsv_step steps[1024];
  int ns = 0, j = 0;
  if (W256)
    for (; j + 256 <= n && ns < 1024; j += 256) steps[ns++] = {j, 256, 1};
  for (; j < n && ns < 1024; j += SMG_NB) steps[ns++] = {j, min(SMG_NB, n - j), 0};
  if (j < n) return SMG_ERR_ARG;  // > 1024 steps: n beyond what the host layer sizes
  for (int q = 0; q < ns; ++q) {
    const trsv_step st = steps[trans ? ns - 1 - q : q];
    const double* W = st.big ? W256 : W64;
    if (st.big) {
      hipLaunchKernelGGL(k_trsv_diag256, dim3((st.b + 15) / 16), dim3(256), 0, ctx->stream, W, ldw,
                         r, y, st.j, st.b, trans);
      if (!trans) {
        const int rows = n - st.j - st.b;
        if (rows > 0)
          hipLaunchKernelGGL(k_trsv_upd_fwd, dim3((rows + 63) / 64), dim3(256), 0, ctx->stream, L,
                             ldl, y, r, n, st.j, st.b);
      } else if (st.j > 0) {
        hipLaunchKernelGGL(k_trsv_upd_bwd, dim3((st.j + 15) / 16), dim3(256), 0, ctx->stream, L, ldl,
                           y, r, st.j, st.b);
      }
      continue;
    }
    if (!trans) {
      const int rows = n - st.j - st.b;
      const int g = rows > 0 ? (rows + ROWS - 1) / ROWS : 1;
      hipLaunchKernelGGL(k_trsv_fwd<64>, dim3(g), dim3(256), 0, ctx->stream, L, ldl, W, ldw, r, y, n,
                         st.j, st.b);
    } else {
      const int g = st.j > 0 ? (st.j + ROWS - 1) / ROWS : 1;
      hipLaunchKernelGGL(k_trsv_bwd<64>, dim3(g), dim3(256), 0, ctx->stream, L, ldl, W, ldw, r, y,
                         st.j, st.b);
    }
  }
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}
