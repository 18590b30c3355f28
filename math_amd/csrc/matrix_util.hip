// Small dense helpers behind the host layer's matrix functors:
//   transpose  (rev/mat/fun/transpose / Eigen .transpose() in multiply(A, A^T))
//   sym_from_lower (the upper half of a Gram product A A^T computed lower-only)
//   shift      (sum(Matrix<var>) reverse: every operand adjoint += adj,
//               rev/mat/fun/sum.hpp:18-60)
//   dot        (dot_product / the scalar side of multiply(var, Matrix<var>),
//               rev/mat/fun/multiply.hpp:562-600)
//   pack_tril / unpack_tril_add  (the Eigen boundary: a cholesky_decompose
//               factor's or a gp_exp_quad_cov matrix's host varis cover the
//               lower triangle only, packed column by column --
//               rev/mat/fun/cholesky_decompose.hpp:34-48,
//               rev/mat/fun/gp_exp_quad_cov.hpp:235 -- so only it crosses PCIe)
// All deterministic (fixed-order reductions).
#include "smg_internal.h"

namespace {

constexpr int TT = 64;  // transpose tile

// B (n x m) = A^T + beta B; A is m x n.  64 x 64 tiles through LDS so both the
// read of A and the write of B are column-coalesced.
__global__ __launch_bounds__(256) void k_transpose(int m, int n, const double* __restrict__ A,
                                                   int lda, double* __restrict__ B, int ldb,
                                                   double beta) {
  __shared__ double t[TT][TT + 1];
  const int i0 = blockIdx.x * TT, j0 = blockIdx.y * TT;
  const int r = threadIdx.x & 63, c4 = threadIdx.x >> 6;
#pragma unroll 4
  for (int c = c4; c < TT; c += 4) {
    const int i = i0 + r, j = j0 + c;
    t[c][r] = (i < m && j < n) ? A[i + (size_t)j * lda] : 0.0;
  }
  __syncthreads();
#pragma unroll 4
  for (int c = c4; c < TT; c += 4) {
    // B(j0 + r, i0 + c) = A(i0 + c, j0 + r)
    const int bi = j0 + r, bj = i0 + c;
    if (bi < n && bj < m) {
      double* d = B + bi + (size_t)bj * ldb;
      const double v = t[r][c];
      *d = beta == 0.0 ? v : v + beta * *d;
    }
  }
}

// A (n x n, in place): strict upper <- transpose of the strict lower.  Tile
// (bx, by), bx >= by, of the lower triangle is read through LDS and written
// to its mirror tile; on a diagonal tile only the strict upper entries are
// written (every read precedes the barrier)
__global__ __launch_bounds__(256) void k_sym_from_lower(int n, double* __restrict__ A, int lda) {
  const int bx = blockIdx.x, by = blockIdx.y;
  if (bx < by) return;
  __shared__ double t[TT][TT + 1];
  const int i0 = bx * TT, j0 = by * TT;
  const int r = threadIdx.x & 63, c4 = threadIdx.x >> 6;
#pragma unroll 4
  for (int c = c4; c < TT; c += 4) {
    const int i = i0 + r, j = j0 + c;
    t[c][r] = (i < n && j < n) ? A[i + (size_t)j * lda] : 0.0;
  }
  __syncthreads();
#pragma unroll 4
  for (int c = c4; c < TT; c += 4) {
    const int bi = j0 + r, bj = i0 + c;  // A(bi, bj) = A(bj, bi), bi < bj
    if (bi < n && bj < n && bi < bj) A[bi + (size_t)bj * lda] = t[r][c];
  }
}

// B += S with S symmetric and only its upper triangle stored: tile pair
// (bx, by), bx >= by: the upper tile U = S[by.., bx..] is added to B's tile
// (by, bx) as read and, transposed through LDS, to its mirror (bx, by); on a
// diagonal tile each entry (i, j) takes S(min, max)
__global__ __launch_bounds__(256) void k_add_sym_from_upper(int n, const double* __restrict__ S, int lds,
                                                            double* __restrict__ B, int ldb) {
  const int bx = blockIdx.x, by = blockIdx.y;
  if (bx < by) return;
  __shared__ double t[TT][TT + 1];
  const int i0 = by * TT, j0 = bx * TT;  // U's rows i0.., columns j0..
  const int r = threadIdx.x & 63, c4 = threadIdx.x >> 6;
#pragma unroll 4
  for (int c = c4; c < TT; c += 4) {
    const int i = i0 + r, j = j0 + c;
    const double u = (i < n && j < n) ? S[i + (size_t)j * lds] : 0.0;
    t[c][r] = u;
    if (i < n && j < n && (bx != by || i <= j)) B[i + (size_t)j * ldb] += u;
  }
  __syncthreads();
#pragma unroll 4
  for (int c = c4; c < TT; c += 4) {
    const int i = j0 + r, j = i0 + c;  // B(i, j) += S(j, i), i > j
    if (i < n && j < n && i > j) B[i + (size_t)j * ldb] += t[r][c];
  }
}

__global__ void k_shift(int m, int n, double c, double* __restrict__ Y, int ldy, int uplo) {
  for (smg_mn it(m, n); it.ok(); it.next()) {
    const long long e = it.e;
    const int i = it.i, j = it.j;
    if (uplo == 1 && i < j) continue;
    Y[i + (size_t)j * ldy] += c;
  }
}

__global__ void k_dot_part(const double* __restrict__ x, const double* __restrict__ y, long long n,
                           double* part) {
  __shared__ double lds[16];
  double s = 0.0;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    s += x[i] * y[i];
  s = block_sum(s, lds);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// flag <- 1.0 if any element violates the check (all writers store 1.0)
//   kind 0: not nan (check_not_nan)   1: finite (check_finite)
//   2: > 0 (check_positive)           3: finite and > 0 (check_positive_finite)
__global__ void k_check_domain(const double* __restrict__ x, long long n, int kind,
                               double* flag) {
  bool bad = false;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const double v = x[i];
    if (kind == 0) bad |= v != v;
    else if (kind == 1) bad |= !(fabs(v) <= 1.7976931348623157e308);
    else if (kind == 2) bad |= !(v > 0.0);
    else bad |= !(v > 0.0 && v <= 1.7976931348623157e308);
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) *flag = 1.0;
}

__global__ void k_check_bounded_int(const int* __restrict__ y, long long n, int lo, int hi,
                                    double* flag) {
  bool bad = false;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    bad |= y[i] < lo || y[i] > hi;
  if (__any(bad) && (threadIdx.x & 63) == 0) *flag = 1.0;
}

// Y (+)= Phi(X): strict lower of X, diagonal halved, upper zero (the
// tangent of a Cholesky factor, L' = L Phi(L^{-1} A' L^{-T}))
__global__ void k_phi(int n, const double* __restrict__ X, int ldx, double* __restrict__ Y, int ldy,
                      int accumulate) {
  for (smg_mn it(n, n); it.ok(); it.next()) {
    const long long e = it.e;
    const int i = it.i, j = it.j;
    const double v = i > j ? X[i + (size_t)j * ldx] : (i == j ? 0.5 * X[i + (size_t)j * ldx] : 0.0);
    double* y = Y + i + (size_t)j * ldy;
    *y = accumulate ? *y + v : v;
  }
}

__global__ void k_diag_ratio(int n, const double* __restrict__ A, int lda,
                             const double* __restrict__ B, int ldb, double* out) {
  __shared__ double lds[16];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += A[i + (size_t)i * lda] / B[i + (size_t)i * ldb];
  s = block_sum(s, lds);
  if (threadIdx.x == 0) out[0] += s;
}

__global__ void k_diag_ratio_rev(int n, const double* __restrict__ A, int lda,
                                 const double* __restrict__ B, int ldb, double adj, double* Aa,
                                 int ldaa, double* Ba, int ldba) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const double b = B[i + (size_t)i * ldb];
    if (Aa) Aa[i + (size_t)i * ldaa] += adj / b;
    if (Ba) Ba[i + (size_t)i * ldba] -= adj * A[i + (size_t)i * lda] / (b * b);
  }
}

// packed lower triangle, column-major: column j's rows j..n-1 start at
// j n - j (j - 1) / 2
__device__ __forceinline__ long long tril_off(long long n, long long j) { return j * n - j * (j - 1) / 2; }

// mode 0: dst <- tril(A); mode 1: dst <- tril(A) + strict tril(A^T).  One
// 64 x 64 tile of the lower triangle per workgroup; mode 1 reads the mirror
// tile through LDS so both reads are column-coalesced.
__global__ __launch_bounds__(256) void k_pack_tril(int mode, int n, const double* __restrict__ A, int lda,
                                                   double* __restrict__ dst) {
  const int bx = blockIdx.x, by = blockIdx.y;  // tile rows bx, cols by
  if (bx < by) return;
  __shared__ double t[TT][TT + 1];
  const int i0 = bx * TT, j0 = by * TT;
  const int r = threadIdx.x & 63, c4 = threadIdx.x >> 6;
  if (mode == 1) {
#pragma unroll 4
    for (int c = c4; c < TT; c += 4) {  // mirror tile: A(j0 + r, i0 + c) -> t[r][c] = A^T(i0 + c, j0 + r)
      const int i = j0 + r, j = i0 + c;
      t[r][c] = (i < n && j < n) ? A[i + (size_t)j * lda] : 0.0;
    }
    __syncthreads();
  }
#pragma unroll 4
  for (int c = c4; c < TT; c += 4) {
    const int i = i0 + r, j = j0 + c;
    if (i < n && j < n && i >= j) {
      double v = A[i + (size_t)j * lda];
      if (mode == 1 && i != j) v += t[c][r];  // A(j, i)
      dst[tril_off(n, j) + (i - j)] = v;
    }
  }
}

// columns [j0, j1) of the packed lower triangle (a Cholesky panel's final
// columns, streamed to the host while later panels factor): one column per
// workgroup pass, reads and writes both column-contiguous
__global__ __launch_bounds__(256) void k_pack_tril_cols(int n, const double* __restrict__ A, int lda, int j0, int j1,
                                                        double* __restrict__ dst) {
  for (int j = j0 + blockIdx.x; j < j1; j += gridDim.x) {
    const double* a = A + (size_t)j * lda;
    double* d = dst + tril_off(n, j) - j;
    for (int i = j + threadIdx.x; i < n; i += 256) d[i] = a[i];
  }
}

// tril(A) += unpack(src) (modes 0 / 1); A_ii += src[i] (mode 2)
__global__ __launch_bounds__(256) void k_unpack_tril_add(int mode, int n, const double* __restrict__ src,
                                                         double* __restrict__ A, int lda) {
  if (mode == 2) {
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) A[i + (size_t)i * lda] += src[i];
    return;
  }
  for (int j = blockIdx.x; j < n; j += gridDim.x) {
    const double* s = src + tril_off(n, j) - j;
    double* a = A + (size_t)j * lda;
    for (int i = j + threadIdx.x; i < n; i += 256) a[i] += s[i];
  }
}

__global__ __launch_bounds__(256) void k_pack_diag(int n, const double* __restrict__ A, int lda,
                                                   double* __restrict__ dst) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) dst[i] = A[i + (size_t)i * lda];
}

// per-workgroup sums of the strict upper triangle (columns blockIdx.x,
// + gridDim.x, ...; rows < column), in a fixed order
__global__ __launch_bounds__(256) void k_upper_sums(int n, const double* __restrict__ A, int lda,
                                                    double* __restrict__ part) {
  __shared__ double lds[16];
  double v = 0.0;
  for (int j = blockIdx.x; j < n; j += gridDim.x) {
    const double* a = A + (size_t)j * lda;
    for (int i = threadIdx.x; i < j; i += 256) v += a[i];
  }
  v = block_sum(v, lds);
  if (threadIdx.x == 0) part[blockIdx.x] = v;
}

inline int grid_for(long long tot, int cap = 4096) {
  long long g = (tot + 255) / 256;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

extern "C" {

int smg_transpose(smg_ctx* ctx, int m, int n, const double* A, int lda, double* B, int ldb,
                  double beta) {
  if (!ctx || m < 0 || n < 0) return SMG_ERR_ARG;
  if (m == 0 || n == 0) return SMG_OK;
  if (!A || !B || lda < m || ldb < n) return SMG_ERR_ARG;
  hipLaunchKernelGGL(k_transpose, dim3(smg_ceil_div(m, TT), smg_ceil_div(n, TT)), dim3(256), 0,
                     ctx->stream, m, n, A, lda, B, ldb, beta);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_sym_from_lower(smg_ctx* ctx, int n, double* A, int lda) {
  if (!ctx || n < 0) return SMG_ERR_ARG;
  if (n <= 1) return SMG_OK;
  if (!A || lda < n) return SMG_ERR_ARG;
  const int t = smg_ceil_div(n, TT);
  hipLaunchKernelGGL(k_sym_from_lower, dim3(t, t), dim3(256), 0, ctx->stream, n, A, lda);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_add_sym_from_upper(smg_ctx* ctx, int n, const double* S, int lds, double* B, int ldb) {
  if (n <= 0) return SMG_OK;
  const int t = smg_ceil_div(n, TT);
  hipLaunchKernelGGL(k_add_sym_from_upper, dim3(t, t), dim3(256), 0, ctx->stream, n, S, lds, B, ldb);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_pack_tril_cols(smg_ctx* ctx, int n, const double* A, int lda, int j0, int j1, double* dst) {
  if (j1 <= j0) return SMG_OK;
  hipLaunchKernelGGL(k_pack_tril_cols, dim3(j1 - j0 < 1024 ? j1 - j0 : 1024), dim3(256), 0, ctx->stream, n, A, lda,
                     j0, j1, dst);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_pack_tril(smg_ctx* ctx, int mode, int n, const double* A, int lda, double* dst) {
  if (!ctx || n < 0 || mode < 0 || mode > 2) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  if (!A || !dst || lda < n) return SMG_ERR_ARG;
  if (mode == 2) {
    hipLaunchKernelGGL(k_pack_diag, dim3(smg_ceil_div(n, 256) < 1024 ? smg_ceil_div(n, 256) : 1024), dim3(256), 0,
                       ctx->stream, n, A, lda, dst);
  } else {
    const int t = smg_ceil_div(n, TT);
    hipLaunchKernelGGL(k_pack_tril, dim3(t, t), dim3(256), 0, ctx->stream, mode, n, A, lda, dst);
  }
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_sum_strict_upper(smg_ctx* ctx, int n, const double* A, int lda, double* out) {
  if (!ctx || n < 0 || !out || (n > 0 && (!A || lda < n))) return SMG_ERR_ARG;
  const int g = n < 1024 ? (n > 0 ? n : 1) : 1024;
  double* part = smg_ws(ctx, SMG_WS_RED, g);
  if (!part) return SMG_ERR_OOM;
  hipLaunchKernelGGL(k_upper_sums, dim3(g), dim3(256), 0, ctx->stream, n, A, lda, part);
  smg_reduce_partials(ctx, part, g, 1, out, 0);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_unpack_tril_add(smg_ctx* ctx, int mode, int n, const double* src, double* A, int lda) {
  if (!ctx || n < 0 || mode < 0 || mode > 2) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  if (!A || !src || lda < n) return SMG_ERR_ARG;
  const int g = mode == 2 ? (smg_ceil_div(n, 256) < 1024 ? smg_ceil_div(n, 256) : 1024) : (n < 4096 ? n : 4096);
  hipLaunchKernelGGL(k_unpack_tril_add, dim3(g), dim3(256), 0, ctx->stream, mode, n, src, A, lda);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_shift(smg_ctx* ctx, int m, int n, double c, double* Y, int ldy, int uplo) {
  if (!ctx || m < 0 || n < 0) return SMG_ERR_ARG;
  if (m == 0 || n == 0 || c == 0.0) return SMG_OK;
  if (!Y || ldy < m) return SMG_ERR_ARG;
  hipLaunchKernelGGL(k_shift, dim3(grid_for((long long)m * n)), dim3(256), 0, ctx->stream, m, n,
                     c, Y, ldy, uplo);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_dot(smg_ctx* ctx, const double* x, const double* y, long long n, double* out) {
  if (!ctx || n < 0 || !out) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  if (!x || !y) return SMG_ERR_ARG;
  const int nb = grid_for(n, 1024);
  double* part = smg_ws(ctx, SMG_WS_RED, (size_t)nb);
  if (!part) return SMG_ERR_OOM;
  hipLaunchKernelGGL(k_dot_part, dim3(nb), dim3(256), 0, ctx->stream, x, y, n, part);
  smg_reduce_partials(ctx, part, nb, 1, out, 1);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_phi(smg_ctx* ctx, int n, const double* X, int ldx, double* Y, int ldy, int accumulate) {
  if (!ctx || n < 0) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  if (!X || !Y || ldx < n || ldy < n) return SMG_ERR_ARG;
  hipLaunchKernelGGL(k_phi, dim3(grid_for((long long)n * n)), dim3(256), 0, ctx->stream, n, X, ldx,
                     Y, ldy, accumulate);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_diag_ratio_fwd(smg_ctx* ctx, int n, const double* A, int lda, const double* B, int ldb,
                       double* out) {
  if (!ctx || n < 0 || !out) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  if (!A || !B) return SMG_ERR_ARG;
  hipLaunchKernelGGL(k_diag_ratio, dim3(1), dim3(1024), 0, ctx->stream, n, A, lda, B, ldb, out);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_diag_ratio_rev(smg_ctx* ctx, int n, const double* A, int lda, const double* B, int ldb,
                       double adj, double* Aadj, int ldaa, double* Badj, int ldba) {
  if (!ctx || n < 0) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  if (!A || !B) return SMG_ERR_ARG;
  hipLaunchKernelGGL(k_diag_ratio_rev, dim3(smg_ceil_div(n, 256)), dim3(256), 0, ctx->stream, n, A,
                     lda, B, ldb, adj, Aadj, ldaa, Badj, ldba);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_check_domain(smg_ctx* ctx, const double* x, long long n, int kind, double* flag) {
  if (!ctx || n < 0 || !flag || kind < 0 || kind > 3) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  if (!x) return SMG_ERR_ARG;
  hipLaunchKernelGGL(k_check_domain, dim3(grid_for(n, 1024)), dim3(256), 0, ctx->stream, x, n,
                     kind, flag);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_check_bounded_int(smg_ctx* ctx, const int* y, long long n, int lo, int hi, double* flag) {
  if (!ctx || n < 0 || !flag) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  if (!y) return SMG_ERR_ARG;
  hipLaunchKernelGGL(k_check_bounded_int, dim3(grid_for(n, 1024)), dim3(256), 0, ctx->stream, y,
                     n, lo, hi, flag);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

}  // extern "C"
