// Blocked triangular solves and the multiply / mdivide_left_tri functors.
//
//   trsm: B <- op(tri(A))^{-1} B in place, op = identity or transpose,
//         SMG_NB diagonal blocks inverted in LDS (k_trtri_blocks) and applied
//         with the MFMA GEMM; off-diagonal updates are GEMMs as well.
//   mdivide_left_tri<TriView>  rev/mat/fun/mdivide_left_tri.hpp:16-373
//   multiply                   rev/mat/fun/multiply.hpp:65-135
#include "smg_internal.h"
#include "tri_small.h"

namespace {

// W_p = inverse of the lower-triangular form of diagonal block p:
//   lower: W_p = D_p^{-1};  upper: W_p = (U_p^T)^{-1} = (U_p^{-1})^T.
// W is m x SMG_NB (block p in rows p*NB.., ld m).
__global__ __launch_bounds__(512) void k_trtri_blocks(const double* __restrict__ A, int lda,
                                                      int m, int upper, double* __restrict__ W) {
  __shared__ double D[SMG_NB * SMG_NBP];
  __shared__ double X[SMG_NB * SMG_NBP];
  const int j = blockIdx.x * SMG_NB;
  const int b = min(SMG_NB, m - j);
  const double* Ab = A + j + (size_t)j * lda;
  for (int e = threadIdx.x; e < SMG_NB * SMG_NB; e += blockDim.x) {
    const int c = e / SMG_NB, r = e % SMG_NB;
    double v = (r == c) ? 1.0 : 0.0;  // identity padding beyond b
    if (r < b && c < b) v = r >= c ? (upper ? Ab[c + (size_t)r * lda] : Ab[r + (size_t)c * lda]) : 0.0;
    D[r * SMG_NBP + c] = v;
  }
  __syncthreads();
  lds_potrf_inv64_blk(D, X, b, nullptr, 0, W + j, m, nullptr, false);
}

__global__ void k_copy(int m, int n, const double* __restrict__ A, int lda,
                       double* __restrict__ B, int ldb, double alpha, int accumulate) {
  for (smg_mn it(m, n); it.ok(); it.next()) {
    const long long e = it.e;
    const int i = it.i, j = it.j;
    const double v = alpha * A[i + (size_t)j * lda];
    double* d = B + i + (size_t)j * ldb;
    *d = accumulate ? *d + v : v;
  }
}

__global__ void k_scale(int m, int n, double beta, double* C, int ldc, int tri) {
  for (smg_mn it(m, n); it.ok(); it.next()) {
    const long long e = it.e;
    const int i = it.i, j = it.j;
    if (tri == 1 && i < j) continue;
    if (tri == 2 && i > j) continue;
    if (tri == 3 && i >= j) continue;
    double* c = C + i + (size_t)j * ldc;
    *c = beta == 0.0 ? 0.0 : beta * *c;
  }
}

inline int grid_for(long long tot) {
  long long g = (tot + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

int smg_scale_impl(smg_ctx* ctx, int m, int n, double beta, double* C, int ldc, int tri) {
  hipLaunchKernelGGL(k_scale, dim3(grid_for((long long)m * n)), dim3(256), 0, ctx->stream, m, n,
                     beta, C, ldc, tri);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_copy_impl(smg_ctx* ctx, int m, int n, const double* A, int lda, double* B, int ldb,
                  double alpha, int accumulate) {
  if (m <= 0 || n <= 0) return SMG_OK;
  hipLaunchKernelGGL(k_copy, dim3(grid_for((long long)m * n)), dim3(256), 0, ctx->stream, m, n,
                     A, lda, B, ldb, alpha, accumulate);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_trtri_blocks_impl(smg_ctx* ctx, const double* L, int ldl, int n, double* W) {
  if (n <= 0) return SMG_OK;
  hipLaunchKernelGGL(k_trtri_blocks, dim3((n + SMG_NB - 1) / SMG_NB), dim3(SMG_DIAG_THREADS), 0, ctx->stream, L,
                     ldl, n, 0, W);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

// W: inverse diagonal blocks (m x SMG_NB, ld m) or NULL (computed here, or
// taken from aux: smg_cholesky_fwd's block inverses of a lower A, ld m)
int smg_trsm_impl(smg_ctx* ctx, int lower, int trans, const double* A, int lda, const double* W,
                  int ldw, double* B, int ldb, int m, int n, double* X, int ldx, const double* aux) {
  if (!lower || W) aux = nullptr;
  if (m <= 0 || n <= 0) return SMG_OK;
  if (X == B) X = nullptr;
  int BSZ = SMG_NB;  // diagonal-block size of the solve
  if (X && !(!W && n == 1 && lower && ldb >= m && m >= 512 && m % 256 == 0 && m / 64 <= 256)) {
    // out of place below; (the one-right-hand-side path copies into place first)
  } else if (X) {
    int rc = smg_copy_impl(ctx, m, n, B, ldb, X, ldx, 1.0, 0);
    if (rc) return rc;
    B = X;
    ldb = ldx;
    X = nullptr;
  }
  if (!W && n == 1 && lower && ldb >= m && m >= 512 && m % 256 == 0 && m / 64 <= 256) {
    // one right-hand side: the persistent solve (trsv.hip) on the 256- / 512-
    // row inverses, one launch instead of 2 m / 64 small GEMMs
    const double* w = aux;
    double* xr = smg_ws(ctx, SMG_WS_CW, 2 * (size_t)m);
    if (!xr) return SMG_ERR_OOM;
    int rc;
    if (!w) {
      double* wn = smg_ws(ctx, SMG_WS_TMP2, (size_t)m * SMG_AUX_COLS);
      if (!wn) return SMG_ERR_OOM;
      hipLaunchKernelGGL(k_trtri_blocks, dim3(m / SMG_NB), dim3(SMG_DIAG_THREADS), 0, ctx->stream, A, lda,
                         m, 0, wn);
      if ((rc = smg_block_inverses_impl(ctx, A, lda, wn, m))) return rc;
      w = wn;
    }
    rc = smg_copy_impl(ctx, m, 1, B, ldb, xr, m, 1.0, 0);
    if (rc) return rc;
    return smg_trsv_lower_impl(ctx, trans, A, lda, w, w + (size_t)m * SMG_AUX_W256,
                               m % SMG_NBR == 0 ? w + (size_t)m * SMG_AUX_W512 : nullptr, m, xr, B,
                               xr + m, m);
  }
  if (!W) {
    // a large lower solve without given inverses: 512-row blocks (inverses
    // doubled up from the 64-row ones, as the Cholesky aux), so the updates
    // are rank-512 GEMMs instead of rank-64 ones and the step count is m / 512
    const bool big = lower && m >= 4 * SMG_NBR && m % SMG_NBR == 0 && n >= SMG_NBR;
    const double* w = aux;
    if (!w) {
      const size_t wd = big ? (size_t)m * SMG_AUX_COLS : (size_t)m * SMG_NB;
      double* wn = smg_ws(ctx, SMG_WS_TMP2, wd);
      if (!wn) return SMG_ERR_OOM;
      hipLaunchKernelGGL(k_trtri_blocks, dim3((m + SMG_NB - 1) / SMG_NB), dim3(SMG_DIAG_THREADS), 0,
                         ctx->stream, A, lda, m, lower ? 0 : 1, wn);
      if (big) {
        const int rc = smg_block_inverses_impl(ctx, A, lda, wn, m);
        if (rc) return rc;
      }
      w = wn;
    }
    W = w;
    ldw = m;
    if (big) {
      W = w + (size_t)m * SMG_AUX_W512;
      BSZ = SMG_NBR;
    }
  }
  const int nblk = (m + BSZ - 1) / BSZ;
  const bool forward = (lower && !trans) || (!lower && trans);
  const bool wt = (trans != 0) != (lower == 0);  // X_p = W_p^T B_p
  int rc;
  if (lower && BSZ == SMG_NBR && m % SMG_NBR == 0) {
    // Recursive halving: solve the first half, ONE update of the second half
    // by the whole first half (a rank-m/2 GEMM), solve the second half (for
    // the transposed solve the halves swap roles).  The same flops as the
    // block loop, in fewer, larger GEMMs (m/2, m/4, ... ranks instead of
    // m/512 rank-512 updates); leaves are the 512-row blocks' W_p B_p.
    struct rec_t {
      smg_ctx* ctx;
      const double* A;
      int lda;
      const double* W;
      int ldw;
      double* B;
      int ldb;
      double* X;
      int ldx;
      int n, trans;
      int solve(int lo, int hi) {
        if (hi - lo == SMG_NBR) {
          double* Bp = X ? X + lo : B + lo;
          const int ldp = X ? ldx : ldb;
          return smg_gemm_impl(ctx, trans ? 1 : 0, 0, 0, SMG_NBR, n, SMG_NBR, 1.0, W + lo, ldw, B + lo, ldb, 0.0,
                               Bp, ldp, trans ? SMG_TRI_A_UPPER : SMG_TRI_A_LOWER);
        }
        const int mid = lo + ((hi - lo) / SMG_NBR / 2) * SMG_NBR;
        const double* Xs = X ? X : B;
        const int lds = X ? ldx : ldb;
        int rc;
        if (!trans) {  // X[lo:mid], then B[mid:hi] -= L[mid:hi, lo:mid] X[lo:mid], then X[mid:hi]
          if ((rc = solve(lo, mid))) return rc;
          rc = smg_gemm_impl(ctx, 0, 0, 0, hi - mid, n, mid - lo, -1.0, A + mid + (size_t)lo * lda, lda, Xs + lo,
                             lds, 1.0, B + mid, ldb);
          if (rc) return rc;
          return solve(mid, hi);
        }
        // L^T X = B: X[mid:hi], then B[lo:mid] -= L[mid:hi, lo:mid]^T X[mid:hi], then X[lo:mid]
        if ((rc = solve(mid, hi))) return rc;
        rc = smg_gemm_impl(ctx, 1, 0, 0, mid - lo, n, hi - mid, -1.0, A + mid + (size_t)lo * lda, lda, Xs + mid,
                           lds, 1.0, B + lo, ldb);
        if (rc) return rc;
        return solve(lo, mid);
      }
    };
    rec_t r{ctx, A, lda, W, ldw, B, ldb, X, ldx, n, trans};
    return r.solve(0, m);
  }
  for (int q = 0; q < nblk; ++q) {
    const int p = forward ? q : nblk - 1 - q;
    const int j = p * BSZ, b = min(BSZ, m - j), k = j + b;
    // X_p = W_p (or W_p^T) B_p: in place through the GEMM's aliasing path, or
    // straight into X; W_p is lower triangular with stored zeros: each
    // tile's K loop skips them.  Bp / ldp: where X_p lives afterwards.
    double* Bp = X ? X + j : B + j;
    const int ldp = X ? ldx : ldb;
    rc = smg_gemm_impl(ctx, wt ? 1 : 0, 0, 0, b, n, b, 1.0, W + j, ldw, B + j, ldb, 0.0, Bp, ldp,
                       wt ? SMG_TRI_A_UPPER : SMG_TRI_A_LOWER);
    if (rc) return rc;
    if (forward && k < m) {
      if (lower)  // B[k:] -= L[k:, j:k] X_p
        rc = smg_gemm_impl(ctx, 0, 0, 0, m - k, n, b, -1.0, A + k + (size_t)j * lda, lda, Bp, ldp,
                           1.0, B + k, ldb);
      else  // B[k:] -= (U[j:k, k:])^T X_p
        rc = smg_gemm_impl(ctx, 1, 0, 0, m - k, n, b, -1.0, A + j + (size_t)k * lda, lda, Bp, ldp,
                           1.0, B + k, ldb);
      if (rc) return rc;
    }
    if (!forward && j > 0) {
      if (!lower)  // B[0:j] -= U[0:j, j:k] X_p
        rc = smg_gemm_impl(ctx, 0, 0, 0, j, n, b, -1.0, A + (size_t)j * lda, lda, Bp, ldp, 1.0, B,
                           ldb);
      else  // B[0:j] -= (L[j:k, 0:j])^T X_p
        rc = smg_gemm_impl(ctx, 1, 0, 0, j, n, b, -1.0, A + j, lda, Bp, ldp, 1.0, B, ldb);
      if (rc) return rc;
    }
  }
  return SMG_OK;
}

extern "C" {

int smg_copy_matrix(smg_ctx* ctx, int m, int n, const double* A, int lda, double* B, int ldb,
                    int trans, int zero_upper) {
  if (!ctx || trans) return SMG_ERR_ARG;  // transposed copies are not needed by the host layer
  int rc = smg_copy_impl(ctx, m, n, A, lda, B, ldb, 1.0, 0);
  if (rc || !zero_upper) return rc;
  return smg_scale_impl(ctx, m, n, 0.0, B, ldb, 3);
}

int smg_mdivide_left_tri_fwd(smg_ctx* ctx, int lower, const double* A, int lda, const double* B,
                             int ldb, int m, int n, double* C, int ldc) {
  return smg_mdivide_left_tri_aux_fwd(ctx, lower, A, lda, nullptr, B, ldb, m, n, C, ldc);
}

int smg_mdivide_left_tri_aux_fwd(smg_ctx* ctx, int lower, const double* A, int lda, const double* aux,
                                 const double* B, int ldb, int m, int n, double* C, int ldc) {
  if (!ctx || m < 0 || n < 0) return SMG_ERR_ARG;
  if (m == 0 || n == 0) return SMG_OK;
  if (!A || !B || !C || lda < m || ldb < m || ldc < m) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_TRSV);
  if (m >= 512 && n >= 64) {  // the right-hand side in a workspace, blocks written straight to C
    double* R = smg_ws(ctx, SMG_WS_RHS, (size_t)m * n);
    if (!R) return SMG_ERR_OOM;
    int rc = smg_copy_impl(ctx, m, n, B, ldb, R, m, 1.0, 0);
    if (rc) return rc;
    return smg_trsm_impl(ctx, lower, 0, A, lda, nullptr, 0, R, m, m, n, C, ldc, aux);
  }
  int rc = smg_copy_impl(ctx, m, n, B, ldb, C, ldc, 1.0, 0);
  if (rc) return rc;
  return smg_trsm_impl(ctx, lower, 0, A, lda, nullptr, 0, C, ldc, m, n, nullptr, 0, aux);
}

int smg_mdivide_left_tri_rev(smg_ctx* ctx, int lower, const double* A, int lda, const double* C,
                             int ldc, const double* Cadj, int ldca, int m, int n, double* Aadj,
                             int ldaa, double* Badj, int ldba, double* ws) {
  return smg_mdivide_left_tri_aux_rev(ctx, lower, A, lda, nullptr, C, ldc, Cadj, ldca, m, n, Aadj, ldaa, Badj, ldba,
                                      ws);
}

int smg_mdivide_left_tri_aux_rev(smg_ctx* ctx, int lower, const double* A, int lda, const double* aux,
                                 const double* C, int ldc, const double* Cadj, int ldca, int m, int n, double* Aadj,
                                 int ldaa, double* Badj, int ldba, double* ws) {
  if (!ctx || m < 0 || n < 0) return SMG_ERR_ARG;
  if (m == 0 || n == 0) return SMG_OK;
  if (!A || !C || !Cadj || !ws) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_TRSV);
  // adjB = tri(A)^{-T} Cadj   (mdivide_left_tri.hpp:104-107)
  int rc;
  if (m >= 512 && n >= 64) {  // out of place: Cadj's copy in a workspace, the solve into ws
    double* R = smg_ws(ctx, SMG_WS_RHS, (size_t)m * n);
    if (!R) return SMG_ERR_OOM;
    rc = smg_copy_impl(ctx, m, n, Cadj, ldca, R, m, 1.0, 0);
    if (rc) return rc;
    rc = smg_trsm_impl(ctx, lower, 1, A, lda, nullptr, 0, R, m, m, n, ws, m, aux);
  } else {
    rc = smg_copy_impl(ctx, m, n, Cadj, ldca, ws, m, 1.0, 0);
    if (rc) return rc;
    rc = smg_trsm_impl(ctx, lower, 1, A, lda, nullptr, 0, ws, m, m, n, nullptr, 0, aux);
  }
  if (rc) return rc;
  if (Aadj) {  // adjA = -adjB C^T on the triangle only (:108, :111-123)
    rc = smg_gemm_impl(ctx, 0, 1, lower ? 1 : 2, m, m, n, -1.0, ws, m, C, ldc, 1.0, Aadj, ldaa);
    if (rc) return rc;
  }
  if (Badj) return smg_copy_impl(ctx, m, n, ws, m, Badj, ldba, 1.0, 1);
  return SMG_OK;
}

int smg_multiply_lower_fwd(smg_ctx* ctx, const double* L, int ldl, const double* P, int ldp, int n, double* C,
                           int ldc) {
  if (!ctx || n < 0) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  if (!L || !P || !C || ldl < n || ldp < n || ldc < n) return SMG_ERR_ARG;
  // C = L P is lower: the lower tiles only, each over k in [j, i]
  int rc = smg_scale_impl(ctx, n, n, 0.0, C, ldc, 3);
  if (rc) return rc;
  return smg_gemm_impl(ctx, 0, 0, 1, n, n, n, 1.0, L, ldl, P, ldp, 0.0, C, ldc,
                       SMG_TRI_A_LOWER | SMG_TRI_B_LOWER);
}

int smg_multiply_lower_rev(smg_ctx* ctx, const double* L, int ldl, const double* P, int ldp, const double* Cadj,
                           int ldca, int n, double* Ladj, int ldla, double* Padj, int ldpa, double* ws) {
  if (!ctx || n < 0) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  if (!L || !P || !Cadj || !ws || ldl < n || ldp < n || ldca < n) return SMG_ERR_ARG;
  // only C's lower triangle depends on (L, P); only the lower triangles of
  // Ladj and Padj are read downstream (both operands are lower-structured):
  //   T = tril(Cadj);  tril(Ladj) += tril(T P^T);  tril(Padj) += tril(L^T T)
  int rc = smg_copy_impl(ctx, n, n, Cadj, ldca, ws, n, 1.0, 0);
  if (rc) return rc;
  rc = smg_scale_impl(ctx, n, n, 0.0, ws, n, 3);
  if (rc) return rc;
  if (Ladj) {  // (T P^T)(i, j) = sum_{k <= j} T(i, k) P(j, k)
    rc = smg_gemm_impl(ctx, 0, 1, 1, n, n, n, 1.0, ws, n, P, ldp, 1.0, Ladj, ldla,
                       SMG_TRI_A_LOWER | SMG_TRI_B_UPPER);
    if (rc) return rc;
  }
  if (Padj)  // (L^T T)(i, j) = sum_{k >= i} L(k, i) T(k, j)
    rc = smg_gemm_impl(ctx, 1, 0, 1, n, n, n, 1.0, L, ldl, ws, n, 1.0, Padj, ldpa,
                       SMG_TRI_A_UPPER | SMG_TRI_B_LOWER);
  return rc;
}

int smg_multiply_fwd(smg_ctx* ctx, const double* A, int lda, const double* B, int ldb, int m, int k,
                     int n, double* C, int ldc) {
  if (!ctx) return SMG_ERR_ARG;
  return smg_gemm(ctx, 0, 0, 0, m, n, k, 1.0, A, lda, B, ldb, 0.0, C, ldc);
}

int smg_multiply_rev(smg_ctx* ctx, const double* A, int lda, const double* B, int ldb,
                     const double* Cadj, int ldca, int m, int k, int n, double* Aadj, int ldaa,
                     double* Badj, int ldba) {
  if (!ctx) return SMG_ERR_ARG;
  int rc = SMG_OK;
  if (Aadj) rc = smg_gemm(ctx, 0, 1, 0, m, k, n, 1.0, Cadj, ldca, B, ldb, 1.0, Aadj, ldaa);
  if (rc) return rc;
  if (Badj) rc = smg_gemm(ctx, 1, 0, 0, k, n, m, 1.0, A, lda, Cadj, ldca, 1.0, Badj, ldba);
  return rc;
}

}  // extern "C"
