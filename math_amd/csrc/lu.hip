// log_determinant of a general square matrix on MI355X.
//
// Reference: stan/math/rev/mat/fun/log_determinant.hpp:14-37 (value
// log|det m| from a full-pivoting Householder QR, gradient = m^{-T} from the
// same factorisation, one precomputed-gradients vari) and
// prim/mat/fun/log_determinant.hpp:20-27 (size 0 -> 0).
//
// Here the factorisation is a blocked LU with partial (row) pivoting,
// P A = L U, stored LAPACK-style in one n x n buffer (unit L below the
// diagonal, U on and above) with the row-swap sequence in piv:
//   * panel of SMG_NB columns: one 1024-thread workgroup walks its columns
//     (pivot = first row of largest |a| in the column, the swap and the
//     rank-1 update restricted to the panel);
//   * the panel's swaps applied to every other column (k_lu_swaps);
//   * U12 = L11^{-1} A12 with L11's explicit unit-lower inverse (LDS) on the
//     MFMA GEMM, then the trailing A22 -= L21 U12 (MFMA GEMM).
// log|det| = sum_i log|u_ii| (fixed-order reduction).  The reverse forms
// A^{-1} = U^{-1} L^{-1} P with the blocked triangular solves and adds
// adj * A^{-T}.  |det| does not depend on the factorisation, so the value and
// the gradient agree with the reference's QR to round-off.
#include "smg_internal.h"
#include "tri_small.h"

namespace {

constexpr int LU_THREADS = 1024;

// one panel: columns [j, j + b) of rows [j, n); piv[j + c] = the pivot row
// of column j + c (absolute index); a zero pivot column is left unscaled
// (LAPACK getf2 semantics: U singular, the factorisation completes)
__global__ __launch_bounds__(LU_THREADS) void k_lu_panel(double* __restrict__ A, int ld, int n, int j, int b,
                                                         int* __restrict__ piv) {
  __shared__ double smax[LU_THREADS / 64];
  __shared__ int sidx[LU_THREADS / 64];
  __shared__ int sp;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  for (int c = 0; c < b; ++c) {
    const int col = j + c;
    double* Ac = A + (size_t)col * ld;
    // pivot search: largest |a| in rows col.., first index on ties
    double best = -1.0;
    int bi = n;
    for (int i = col + t; i < n; i += LU_THREADS) {
      const double v = fabs(Ac[i]);
      if (v > best) {
        best = v;
        bi = i;
      }
    }
    for (int off = 32; off > 0; off >>= 1) {
      const double ob = __shfl_down(best, off);
      const int oi = __shfl_down(bi, off);
      if (ob > best || (ob == best && oi < bi)) {
        best = ob;
        bi = oi;
      }
    }
    if (lane == 0) {
      smax[w] = best;
      sidx[w] = bi;
    }
    __syncthreads();
    if (t == 0) {
      double bb = smax[0];
      int ii = sidx[0];
      for (int q = 1; q < LU_THREADS / 64; ++q)
        if (smax[q] > bb || (smax[q] == bb && sidx[q] < ii)) {
          bb = smax[q];
          ii = sidx[q];
        }
      if (ii >= n) ii = col;  // empty / all-NaN column: no swap
      sp = ii;
      piv[col] = ii;
    }
    __syncthreads();
    const int p = sp;
    // swap rows col and p across the panel's columns
    if (p != col && t < b) {
      double* x = A + (size_t)(j + t) * ld;
      const double tmp = x[col];
      x[col] = x[p];
      x[p] = tmp;
    }
    __syncthreads();
    const double d = Ac[col];
    // scale the column below the pivot, then the rank-1 update of the
    // panel's later columns, one row per thread
    const double rd = 1.0 / d;
    for (int i = col + 1 + t; i < n; i += LU_THREADS) {
      const double l = d != 0.0 ? Ac[i] * rd : Ac[i];
      Ac[i] = l;
      if (d != 0.0)
        for (int cc = c + 1; cc < b; ++cc) {
          double* x = A + (size_t)(j + cc) * ld;
          x[i] -= l * x[col];
        }
    }
    __syncthreads();
  }
}

// the swaps piv[j .. j + b) applied, in order, to every column outside [j, j + b)
__global__ void k_lu_swaps(double* __restrict__ A, int ld, int n, int j, int b, const int* __restrict__ piv) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n || (c >= j && c < j + b)) return;
  double* x = A + (size_t)c * ld;
  for (int k = j; k < j + b; ++k) {
    const int p = piv[k];
    if (p != k) {
      const double tmp = x[k];
      x[k] = x[p];
      x[p] = tmp;
    }
  }
}

// W (b x b, ld ldw, upper zeros) = inverse of the unit-lower b x b block of A
__global__ __launch_bounds__(SMG_DIAG_THREADS) void k_lu_unit_inv(const double* __restrict__ A, int ld, int b,
                                                                  double* __restrict__ W, int ldw) {
  __shared__ double D[SMG_NB * SMG_NBP];
  __shared__ double X[SMG_NB * SMG_NBP];
  for (int e = threadIdx.x; e < SMG_NB * SMG_NB; e += blockDim.x) {
    const int c = e / SMG_NB, r = e % SMG_NB;
    double v = r == c ? 1.0 : 0.0;
    if (r < b && c < b && r > c) v = A[r + (size_t)c * ld];
    D[r * SMG_NBP + c] = v;
  }
  __syncthreads();
  lds_potrf_inv64_blk(D, X, b, nullptr, 0, W, ldw, nullptr, false);
}

// out[0] = sum_i log|A_ii| in index order (one workgroup, fixed order)
__global__ __launch_bounds__(256) void k_lu_logabsdet(const double* __restrict__ A, int ld, int n,
                                                      double* __restrict__ out) {
  __shared__ double part[256];
  double s = 0.0;
  const int per = (n + 255) / 256;
  const int i0 = threadIdx.x * per, i1 = min(n, i0 + per);
  for (int i = i0; i < i1; ++i) s += log(fabs(A[i + (size_t)i * ld]));
  part[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double tot = 0.0;
    for (int q = 0; q < 256; ++q) tot += part[q];
    out[0] = tot;
  }
}

// unit lower L (diagonal 1, upper 0) and U (upper incl. diagonal, lower 0) from LU
__global__ void k_lu_split(const double* __restrict__ LU, int n, double* __restrict__ L, double* __restrict__ U) {
  for (smg_mn it(n, n); it.ok(); it.next()) {
    const int i = it.i, j = it.j;
    const double v = LU[it.e];
    L[it.e] = i > j ? v : (i == j ? 1.0 : 0.0);
    U[it.e] = i <= j ? v : 0.0;
  }
}

// r = the swap sequence applied to 0..n-1 (one thread: the swaps are ordered)
__global__ void k_lu_perm(const int* __restrict__ piv, int n, int* __restrict__ r) {
  for (int i = 0; i < n; ++i) r[i] = i;
  for (int k = 0; k < n; ++k) {
    const int p = piv[k];
    const int tmp = r[k];
    r[k] = r[p];
    r[p] = tmp;
  }
}

// X = P I: row i of X is row r(i) of I
__global__ void k_lu_perm_identity(const int* __restrict__ r, int n, double* __restrict__ X) {
  for (smg_mn it(n, n); it.ok(); it.next()) X[it.e] = it.j == r[it.i] ? 1.0 : 0.0;
}

// Aadj(i, j) += adj * X(j, i)
__global__ void k_add_transpose(int n, double adj, const double* __restrict__ X, double* __restrict__ Aadj, int ld) {
  for (smg_mn it(n, n); it.ok(); it.next()) {
    const int i = it.i, j = it.j;
    Aadj[i + (size_t)j * ld] += adj * X[j + (size_t)i * n];
  }
}

inline int grid_for(long long tot) {
  long long g = (tot + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

extern "C" {

int smg_log_determinant_fwd(smg_ctx* ctx, const double* A, int lda, int n, double* LU, int* piv, double* ws,
                            double* out) {
  if (!ctx || n < 0 || !out) return SMG_ERR_ARG;
  if (n == 0) return smg_memset(ctx, out, 0, sizeof(double));
  if (!A || !LU || !piv || !ws || lda < n) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_CHOL_FWD);
  int rc = smg_copy_impl(ctx, n, n, A, lda, LU, n, 1.0, 0);
  if (rc) return rc;
  double* W = ws;  // SMG_NB x SMG_NB inverse of the panel's unit-lower block
  for (int j = 0; j < n; j += SMG_NB) {
    const int b = min(SMG_NB, n - j);
    hipLaunchKernelGGL(k_lu_panel, dim3(1), dim3(LU_THREADS), 0, ctx->stream, LU, n, n, j, b, piv);
    hipLaunchKernelGGL(k_lu_swaps, dim3(smg_ceil_div(n, 256)), dim3(256), 0, ctx->stream, LU, n, n, j, b, piv);
    const int k = j + b, m = n - k;
    if (m == 0) continue;
    hipLaunchKernelGGL(k_lu_unit_inv, dim3(1), dim3(SMG_DIAG_THREADS), 0, ctx->stream, LU + j + (size_t)j * n, n,
                       b, W, SMG_NB);
    // U12 = L11^{-1} A12 (in place: every workgroup owns whole columns)
    rc = smg_gemm_impl(ctx, 0, 0, 0, b, m, b, 1.0, W, SMG_NB, LU + j + (size_t)k * n, n, 0.0,
                       LU + j + (size_t)k * n, n, SMG_TRI_A_LOWER);
    if (rc) return rc;
    // A22 -= L21 U12
    rc = smg_gemm_impl(ctx, 0, 0, 0, m, m, b, -1.0, LU + k + (size_t)j * n, n, LU + j + (size_t)k * n, n, 1.0,
                       LU + k + (size_t)k * n, n);
    if (rc) return rc;
  }
  hipLaunchKernelGGL(k_lu_logabsdet, dim3(1), dim3(256), 0, ctx->stream, LU, n, n, out);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_log_determinant_rev(smg_ctx* ctx, const double* LU, const int* piv, int n, double adj, double* Aadj,
                            int ldaa, double* ws, int* iws) {
  if (!ctx || n < 0) return SMG_ERR_ARG;
  if (n == 0 || adj == 0.0) return SMG_OK;
  if (!LU || !piv || !Aadj || !ws || !iws || ldaa < n) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_TRSV);
  const size_t nn = (size_t)n * n;
  double* L = ws;
  double* U = ws + nn;
  double* X = ws + 2 * nn;
  hipLaunchKernelGGL(k_lu_split, dim3(grid_for((long long)nn)), dim3(256), 0, ctx->stream, LU, n, L, U);
  hipLaunchKernelGGL(k_lu_perm, dim3(1), dim3(1), 0, ctx->stream, piv, n, iws);
  hipLaunchKernelGGL(k_lu_perm_identity, dim3(grid_for((long long)nn)), dim3(256), 0, ctx->stream, iws, n, X);
  SMG_LAUNCH_CHECK();
  // X = U^{-1} L^{-1} P = A^{-1}
  int rc = smg_trsm_impl(ctx, 1, 0, L, n, nullptr, 0, X, n, n, n);
  if (rc) return rc;
  rc = smg_trsm_impl(ctx, 0, 0, U, n, nullptr, 0, X, n, n, n);
  if (rc) return rc;
  hipLaunchKernelGGL(k_add_transpose, dim3(grid_for((long long)nn)), dim3(256), 0, ctx->stream, n, adj, X, Aadj,
                     ldaa);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

}  // extern "C"
