// multi_normal_cholesky_lpdf's forward on the factor's explicit inverse.
//
// The reference forms inv_L = L^{-1} and takes
//   half = inv_L (y - mu),  scaled_diff = half inv_L
// as two triangular matrix-vector products
// (prim/mat/prob/multi_normal_cholesky_lpdf.hpp:117-131).  When the
// factorisation has formed W = L^{-1} anyway (the progressive K^{-1} of a GP
// whose reverse is predicted to take the closed form, chol_mvn.hip), the
// forward does exactly that: w = W (y - mu), s = W^T w as two HBM-bound
// passes over W's lower triangle instead of two latency-bound persistent
// triangular solves (k_trsv_persist, ~115 us each at n = 4096).
//
// Layout: a pass is a grid of 64 x 64 tiles of W's lower triangle (tile
// (ib, jb), jb <= ib; the diagonal tiles' strict upper is masked to zero,
// W's strict upper outside them is never read).  Each tile writes
// one 64-vector of partial sums: y = W x into P[jb][ib 64 + r] (per column
// tile), y = W^T x into P[ib][jb 64 + c] (per row tile).  The next pass
// (and the finishing kernel) forms its input entries by summing those
// partials in tile order, so the result is deterministic and no separate
// reduction launch sits between the passes.
#include <cmath>

#include "smg_internal.h"

namespace {

constexpr int TB = 64;  // tile edge

// the sum over chunks c in [c0, c1] of P[c][j] for the 64 entries j of
// block jb, into xs[0..64): the 256 threads take the chunks in four
// interleaved groups (independent loads in flight, not one serial chain of
// up to n / 64), combined in a fixed order; red: 4 x 64 doubles of LDS
__device__ __forceinline__ void sum_partials(const double* __restrict__ P, int n, int jb, int c0, int c1,
                                             double* xs, double (*red)[TB]) {
  const int e = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int j = jb * TB + e;
  double a0 = 0.0, a1 = 0.0;
  int c = c0 + g;
  for (; c + 4 <= c1; c += 8) {
    a0 += P[(size_t)c * n + j];
    a1 += P[(size_t)(c + 4) * n + j];
  }
  if (c <= c1) a0 += P[(size_t)c * n + j];
  red[g][e] = a0 + a1;
  __syncthreads();
  if (threadIdx.x < TB) xs[e] = (red[0][e] + red[1][e]) + (red[2][e] + red[3][e]);
}

// x_j for the 64 entries of tile column block jb, into xs[0..64):
//  src 0: y[j] - mu[j] (mu may be null)
//  src 1: sum over column tiles c <= jb of P[c][j] (a W x pass's partials)
__device__ __forceinline__ void tile_input(int src, const double* __restrict__ y, const double* __restrict__ mu,
                                           const double* __restrict__ P, int n, int jb, double* xs,
                                           double (*red)[TB]) {
  const int t = threadIdx.x;
  if (src == 0) {
    if (t < TB) {
      const int j = jb * TB + t;
      xs[t] = mu ? y[j] - mu[j] : y[j];
    }
  } else {
    sum_partials(P, n, jb, 0, jb, xs, red);
  }
}

// tile index -> (ib, jb), jb <= ib, row-major over the lower triangle
__device__ __forceinline__ void tile_of(int t, int& ib, int& jb) {
  int r = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
  while ((r + 1) * (r + 2) / 2 <= t) ++r;
  while (r * (r + 1) / 2 > t) --r;
  ib = r;
  jb = t - r * (r + 1) / 2;
}

// y = W x (TRANS false) or y = W^T x (TRANS true) over the lower tiles of W
// (n x n, ld ldw, n % 64 == 0): partials into P (nb x n, nb = n / 64)
template <bool TRANS>
__global__ __launch_bounds__(256) void k_trmv_tiles(const double* __restrict__ W, int ldw, int n, int src,
                                                    const double* __restrict__ y, const double* __restrict__ mu,
                                                    const double* __restrict__ Pin, double* __restrict__ P) {
  __shared__ double xs[TB];
  __shared__ double red[4][TB];
  __shared__ double tr[TRANS ? TB : 1][TB + 1];
  int ib, jb;
  tile_of(blockIdx.x, ib, jb);
  const int r = threadIdx.x & 63, g = threadIdx.x >> 6;
  // the input entries this tile multiplies: columns of W (W x) or rows (W^T x)
  tile_input(src, y, mu, Pin, n, TRANS ? ib : jb, xs, red);
  // every load of the tile issued before the first use: a wave reads whole
  // 64-row column segments (512 B)
  double wv[16];
  const double* col = W + (size_t)ib * TB + r + (size_t)jb * TB * ldw;
#pragma unroll
  for (int q = 0; q < 16; ++q) wv[q] = col[(size_t)(g + 4 * q) * ldw];
  if (ib == jb) {  // a diagonal tile: its strict upper is not part of the lower matrix
#pragma unroll
    for (int q = 0; q < 16; ++q)
      if (r < g + 4 * q) wv[q] = 0.0;
  }
  __syncthreads();  // (xs complete; red free again)
  if (!TRANS) {
    double acc = 0.0;
#pragma unroll
    for (int q = 0; q < 16; ++q) acc += wv[q] * xs[g + 4 * q];
    red[g][r] = acc;
    __syncthreads();
    if (threadIdx.x < TB)
      P[(size_t)jb * n + ib * TB + threadIdx.x] =
          (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
  } else {
    const double xr = xs[r];
#pragma unroll
    for (int q = 0; q < 16; ++q) tr[g + 4 * q][r] = wv[q] * xr;
    __syncthreads();
    // thread (c = t & 63, g): rows 16 g .. 16 g + 15 of column c
    const int c = threadIdx.x & 63;
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) acc += tr[c][16 * g + k];
    red[g][c] = acc;
    __syncthreads();
    if (threadIdx.x < TB)
      P[(size_t)ib * n + jb * TB + threadIdx.x] =
          (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
  }
}

// w_i = sum_{c <= ib(i)} P1[c][i], s_j = sum_{r >= jb(j)} P2[r][j] into ws
// [w | s] (one workgroup per 64 entries); the value's partials (sum w_i^2,
// sum log(1 / L_ii)) per workgroup
__global__ __launch_bounds__(256) void k_mvn_inv_finish(const double* __restrict__ P1, const double* __restrict__ P2,
                                                        const double* __restrict__ L, int ldl, int n,
                                                        double* __restrict__ ws, double* __restrict__ part) {
  __shared__ double w[TB], s[TB];
  __shared__ double red[4][TB];
  const int b = blockIdx.x, nb = n / TB;
  sum_partials(P1, n, b, 0, b, w, red);
  __syncthreads();
  sum_partials(P2, n, b, b, nb - 1, s, red);
  __syncthreads();
  if (threadIdx.x < TB) {
    const int i = b * TB + threadIdx.x;
    ws[i] = w[threadIdx.x];
    ws[n + i] = s[threadIdx.x];
    double q = w[threadIdx.x] * w[threadIdx.x];
    double ld = log(1.0 / L[i + (size_t)i * ldl]);
    q = wave_sum(q);
    ld = wave_sum(ld);
    if (threadIdx.x == 0) {
      part[2 * b] = q;
      part[2 * b + 1] = ld;
    }
  }
}

// out = the summed partials of a k_trmv_tiles pass: entries of block b from
// column tiles c <= b (W x) or row tiles r >= b (W^T x)
__global__ __launch_bounds__(256) void k_trmv_finish(const double* __restrict__ P, int n, int trans,
                                                     double* __restrict__ out) {
  __shared__ double xs[TB];
  __shared__ double red[4][TB];
  const int b = blockIdx.x, nb = n / TB;
  sum_partials(P, n, b, trans ? b : 0, trans ? nb - 1 : b, xs, red);
  __syncthreads();
  if (threadIdx.x < TB) out[b * TB + threadIdx.x] = xs[threadIdx.x];
}

// A(i, j) += alpha x_i y_j on the lower triangle (i >= j): a workgroup per
// column (grid-stride over columns), rows from the diagonal down
__global__ __launch_bounds__(256) void k_rank1_lower(int n, double alpha, const double* __restrict__ x,
                                                     const double* __restrict__ y, double* __restrict__ A, int lda) {
  for (int j = blockIdx.x; j < n; j += gridDim.x) {
    const double ay = alpha * y[j];
    double* col = A + (size_t)j * lda;
    for (int i = j + (int)threadIdx.x; i < n; i += 256) col[i] += x[i] * ay;
  }
}

__global__ void k_mvn_inv_lp(const double* __restrict__ part, int nparts, int n, double* out) {
  if (threadIdx.x != 0) return;
  double q = 0.0, ld = 0.0;
  for (int b = 0; b < nparts; ++b) {
    q += part[2 * b];
    ld += part[2 * b + 1];
  }
  const double neg_log_sqrt_two_pi = -log(sqrt(2.0 * M_PI));
  out[0] = neg_log_sqrt_two_pi * n - 0.5 * q + ld;
}

}  // namespace

extern "C" {

int smg_mvn_cholesky_fwd_inv(smg_ctx* ctx, const double* y, const double* mu, const double* L, int ldl,
                             const double* W, int ldw, int n, double* ws, double* out_lp) {
  if (!ctx || n < 0 || (n > 0 && (!y || !L || !W || !ws || !out_lp || ldl < n || ldw < n))) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  if (n % TB != 0) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_MVN);
  const int nb = n / TB;
  double* P = smg_ws(ctx, SMG_WS_MVN, 2 * (size_t)nb * n + 2 * (size_t)nb);
  if (!P) return SMG_ERR_OOM;
  double* P1 = P;
  double* P2 = P + (size_t)nb * n;
  double* part = P2 + (size_t)nb * n;
  const int tiles = nb * (nb + 1) / 2;
  // w = W (y - mu), then s = W^T w
  hipLaunchKernelGGL(k_trmv_tiles<false>, dim3(tiles), dim3(256), 0, ctx->stream, W, ldw, n, 0, y, mu, nullptr, P1);
  hipLaunchKernelGGL(k_trmv_tiles<true>, dim3(tiles), dim3(256), 0, ctx->stream, W, ldw, n, 1, nullptr, nullptr, P1,
                     P2);
  hipLaunchKernelGGL(k_mvn_inv_finish, dim3(nb), dim3(256), 0, ctx->stream, P1, P2, L, ldl, n, ws, part);
  hipLaunchKernelGGL(k_mvn_inv_lp, dim3(1), dim3(64), 0, ctx->stream, part, nb, n, out_lp);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_rank1_lower(smg_ctx* ctx, int n, double alpha, const double* x, const double* y, double* A, int lda) {
  if (!ctx || n < 0 || (n > 0 && (!x || !y || !A || lda < n))) return SMG_ERR_ARG;
  if (n == 0 || alpha == 0.0) return SMG_OK;
  hipLaunchKernelGGL(k_rank1_lower, dim3(n < 2048 ? n : 2048), dim3(256), 0, ctx->stream, n, alpha, x, y, A, lda);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_trmv_inv(smg_ctx* ctx, int trans, const double* W, int ldw, int n, const double* x, double* y) {
  if (!ctx || n < 0 || (n > 0 && (!W || !x || !y || ldw < n))) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  if (n % TB != 0) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_TRSV);
  const int nb = n / TB;
  double* P = smg_ws(ctx, SMG_WS_MVN, (size_t)nb * n);
  if (!P) return SMG_ERR_OOM;
  const int tiles = nb * (nb + 1) / 2;
  if (trans)
    hipLaunchKernelGGL(k_trmv_tiles<true>, dim3(tiles), dim3(256), 0, ctx->stream, W, ldw, n, 0, x, nullptr, nullptr,
                       P);
  else
    hipLaunchKernelGGL(k_trmv_tiles<false>, dim3(tiles), dim3(256), 0, ctx->stream, W, ldw, n, 0, x, nullptr, nullptr,
                       P);
  hipLaunchKernelGGL(k_trmv_finish, dim3(nb), dim3(256), 0, ctx->stream, P, n, trans, y);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

}  // extern "C"
