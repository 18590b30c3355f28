// Triangular solves with ONE right-hand side (the two solves of
// multi_normal_cholesky_lpdf, prim/mat/prob/multi_normal_cholesky_lpdf.hpp:
// 117-131), blocked on the SMG_NB diagonal blocks whose inverses W_p the
// Cholesky forward already produced.
//
//   forward  y = L^{-1} x : for p = 0..:  y_p = W_p r_p;   r[k:] -= L[k:, p] y_p
//   backward y = L^{-T} x : for p = ..0:  y_p = W_p^T r_p; r[:j] -= L[p, :j]^T y_p
//
// One launch per block step: every workgroup recomputes the 64 x 64 diagonal
// product redundantly from L2 (no inter-workgroup hand-off inside a launch),
// workgroup 0 publishes y_p, and each workgroup updates its slice of the
// residual.  Reads of L are coalesced in both directions (column segments).
#include "smg_internal.h"
#include "tri_small.h"

namespace {

constexpr int FWD_ROWS = 256;  // residual rows per workgroup (forward)
constexpr int BWD_COLS = 256;  // residual entries per workgroup (backward)

// yp = W_p rp (trans == 0) or W_p^T rp (trans == 1); rp, yp in LDS; 256 threads
__device__ inline void diag_apply(const double* __restrict__ W, int ldw, int j, int b, int trans,
                                  const double* rp, double* yp, double* part) {
  const int t = threadIdx.x;
  if (!trans) {
    // row t&63 of W_p, quarter t>>6 of the columns; W_p(r,c) = W[j + r + c*ldw]
    const int r = t & 63, q = t >> 6;
    double s = 0.0;
    if (r < b)
#pragma unroll 4
      for (int c = 16 * q; c < 16 * q + 16 && c < b; ++c) s += W[j + r + (size_t)c * ldw] * rp[c];
    part[q * 64 + r] = s;
  } else {
    // (W_p^T rp)(r) = sum_c W_p(c, r) rp[c]: thread r walks column r of W_p
    // (contiguous per thread), quarter q of the rows c
    const int r = t & 63, q = t >> 6;
    double s = 0.0;
    if (r < b)
#pragma unroll 4
      for (int c = 16 * q; c < 16 * q + 16 && c < b; ++c) s += W[j + c + (size_t)r * ldw] * rp[c];
    part[q * 64 + r] = s;
  }
  __syncthreads();
  if (t < 64) yp[t] = (part[t] + part[64 + t]) + (part[128 + t] + part[192 + t]);
  __syncthreads();
}

__global__ __launch_bounds__(256) void k_trsv_fwd(const double* __restrict__ L, int ldl,
                                                  const double* __restrict__ W, int ldw,
                                                  double* __restrict__ r, double* __restrict__ y,
                                                  int n, int j, int b) {
  __shared__ double rp[64], yp[64], part[256];
  const int t = threadIdx.x;
  if (t < 64) rp[t] = t < b ? r[j + t] : 0.0;
  __syncthreads();
  diag_apply(W, ldw, j, b, 0, rp, yp, part);
  if (blockIdx.x == 0 && t < b) y[j + t] = yp[t];
  const int k = j + b;
  const int i = k + blockIdx.x * FWD_ROWS + t;
  if (i < n) {
    double s0 = 0.0, s1 = 0.0;
    const double* Lc = L + i + (size_t)j * ldl;
#pragma unroll 4
    for (int c = 0; c + 1 < b; c += 2) {
      s0 += Lc[(size_t)c * ldl] * yp[c];
      s1 += Lc[(size_t)(c + 1) * ldl] * yp[c + 1];
    }
    if (b & 1) s0 += Lc[(size_t)(b - 1) * ldl] * yp[b - 1];
    r[i] -= s0 + s1;
  }
}

__global__ __launch_bounds__(256) void k_trsv_bwd(const double* __restrict__ L, int ldl,
                                                  const double* __restrict__ W, int ldw,
                                                  double* __restrict__ r, double* __restrict__ y,
                                                  int j, int b) {
  __shared__ double rp[64], yp[64], part[256];
  const int t = threadIdx.x;
  if (t < 64) rp[t] = t < b ? r[j + t] : 0.0;
  __syncthreads();
  diag_apply(W, ldw, j, b, 1, rp, yp, part);
  if (blockIdx.x == 0 && t < b) y[j + t] = yp[t];
  // r[i] -= sum_c L[j + c, i] yp[c]: thread i walks the contiguous segment
  // L[j:j+b, i] of column i (whole cache lines per thread)
  const int i = blockIdx.x * BWD_COLS + t;
  if (i < j) {
    const double* Lc = L + j + (size_t)i * ldl;
    double s0 = 0.0, s1 = 0.0;
#pragma unroll 4
    for (int c = 0; c + 1 < b; c += 2) {
      s0 += Lc[c] * yp[c];
      s1 += Lc[c + 1] * yp[c + 1];
    }
    if (b & 1) s0 += Lc[b - 1] * yp[b - 1];
    r[i] -= s0 + s1;
  }
}

}  // namespace

// y = L^{-1} x (trans = 0) or L^{-T} x (trans = 1); L lower, W its SMG_NB
// diagonal-block inverses (n x SMG_NB, ld ldw).  r: n-double workspace.
int smg_trsv_lower_impl(smg_ctx* ctx, int trans, const double* L, int ldl, const double* W,
                        int ldw, const double* x, double* y, double* r, int n) {
  if (n <= 0) return SMG_OK;
  hipMemcpyAsync(r, x, sizeof(double) * n, hipMemcpyDeviceToDevice, ctx->stream);
  const int nblk = (n + SMG_NB - 1) / SMG_NB;
  for (int q = 0; q < nblk; ++q) {
    const int p = trans ? nblk - 1 - q : q;
    const int j = p * SMG_NB, b = min(SMG_NB, n - j);
    if (!trans) {
      const int rows = n - j - b;
      const int g = rows > 0 ? (rows + FWD_ROWS - 1) / FWD_ROWS : 1;
      hipLaunchKernelGGL(k_trsv_fwd, dim3(g), dim3(256), 0, ctx->stream, L, ldl, W, ldw, r, y, n,
                         j, b);
    } else {
      const int g = j > 0 ? (j + BWD_COLS - 1) / BWD_COLS : 1;
      hipLaunchKernelGGL(k_trsv_bwd, dim3(g), dim3(256), 0, ctx->stream, L, ldl, W, ldw, r, y, j, b);
    }
  }
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}
