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
#include "smg_internal.h"
#include "tri_small.h"

namespace {

__global__ void k_check_symmetric(const double* __restrict__ A, int lda, int n, int* status) {
  // CONSTRAINT_TOLERANCE = 1e-8 absolute (prim/mat/err/constraint_tolerance.hpp:12)
  const long long tot = (long long)n * n;
  bool bad = false;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < tot;
       e += (long long)gridDim.x * blockDim.x) {
    const int j = (int)(e / n), i = (int)(e % n);
    if (i <= j) continue;
    // !(|d| <= tol) so that NaN entries fail too (check_symmetric.hpp:45-46)
    if (!(fabs(A[i + (size_t)j * lda] - A[j + (size_t)i * lda]) <= 1e-8)) bad = true;
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(status, (int)SMG_ERR_NOT_SYMMETRIC);
}

__global__ void k_copy_lower(const double* __restrict__ A, int lda, int n,
                             double* __restrict__ L, int ldl) {
  const long long tot = (long long)n * n;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < tot;
       e += (long long)gridDim.x * blockDim.x) {
    const int j = (int)(e / n), i = (int)(e % n);
    L[i + (size_t)j * ldl] = (i >= j) ? A[i + (size_t)j * lda] : 0.0;
  }
}

__global__ void k_add_lower(const double* __restrict__ X, int ldx, int n,
                            double* __restrict__ Y, int ldy) {
  const long long tot = (long long)n * n;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < tot;
       e += (long long)gridDim.x * blockDim.x) {
    const int j = (int)(e / n), i = (int)(e % n);
    if (i >= j) Y[i + (size_t)j * ldy] += X[i + (size_t)j * ldx];
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

inline int grid_for(long long tot) {
  long long g = (tot + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

extern "C" {

int smg_cholesky_block_size(int n) { return SMG_NB; }

int smg_check_symmetric(smg_ctx* ctx, const double* A, int lda, int n) {
  if (!ctx || n < 0 || (n > 0 && (!A || lda < n))) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  hipLaunchKernelGGL(k_check_symmetric, dim3(grid_for((long long)n * n)), dim3(256), 0,
                     ctx->stream, A, lda, n, ctx->status_d);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_cholesky_fwd(smg_ctx* ctx, const double* A, int lda, int n, double* L, int ldl,
                     double* Dinv) {
  if (!ctx || n < 0 || (n > 0 && (!A || !L || lda < n || ldl < n))) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  smg_prof_scope prof(ctx, SMG_FAM_CHOL_FWD);
  if (!Dinv) {
    Dinv = smg_ws(ctx, SMG_WS_TMP2, (size_t)n * SMG_NB);
    if (!Dinv) return SMG_ERR_OOM;
  }
  if (A != L || lda != ldl)
    hipLaunchKernelGGL(k_copy_lower, dim3(grid_for((long long)n * n)), dim3(256), 0, ctx->stream,
                       A, lda, n, L, ldl);
  for (int j = 0; j < n; j += SMG_NB) {
    const int b = min(SMG_NB, n - j);
    const int m = n - j - b;
    double* L11 = L + j + (size_t)j * ldl;
    double* Di = Dinv + j;  // rows j..j+b, columns 0..b, ld n
    hipLaunchKernelGGL(k_potrf_diag, dim3(1), dim3(SMG_DIAG_THREADS), 0, ctx->stream, L11, ldl, b, Di, n,
                       ctx->status_d);
    if (m > 0) {
      double* L21 = L + (j + b) + (size_t)j * ldl;
      // L21 = A21 * Dinv^T  (in place: one column tile, reads finish before writes)
      int rc = smg_gemm_impl(ctx, 0, 1, 0, m, b, b, 1.0, L21, ldl, Di, n, 0.0, L21, ldl);
      if (rc) return rc;
      double* L22 = L + (j + b) + (size_t)(j + b) * ldl;
      rc = smg_gemm_impl(ctx, 0, 1, 1, m, m, b, -1.0, L21, ldl, L21, ldl, 1.0, L22, ldl);
      if (rc) return rc;
    }
  }
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_cholesky_rev(smg_ctx* ctx, const double* L, int ldl, const double* Dinv, double* La,
                     int ldla, int n, double* Aadj, int ldaa) {
  if (!ctx || n < 0 || (n > 0 && (!L || !La || !Aadj || ldl < n || ldla < n || ldaa < n)))
    return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  smg_prof_scope prof(ctx, SMG_FAM_CHOL_REV);
  double* Dv = const_cast<double*>(Dinv);
  if (!Dv) {
    Dv = smg_ws(ctx, SMG_WS_TMP2, (size_t)n * SMG_NB);
    if (!Dv) return SMG_ERR_OOM;
    for (int j = 0; j < n; j += SMG_NB) {
      const int b = min(SMG_NB, n - j);
      hipLaunchKernelGGL(k_trtri_diag, dim3(1), dim3(SMG_DIAG_THREADS), 0, ctx->stream,
                         L + j + (size_t)j * ldl, ldl, b, Dv + j, n);
    }
  }
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
      rc = smg_gemm_impl(ctx, 0, 0, 0, m, b, b, 1.0, Cadj, ldla, Di, n, 0.0, Cadj, ldla);
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
                       L + j + (size_t)j * ldl, ldl, Di, n, Dadj, ldla, b, Ssym);
    if (j > 0) {
      // R_adj -= sym(D_adj) R
      rc = smg_gemm_impl(ctx, 0, 0, 0, b, j, b, -1.0, Ssym, b, R, ldl, 1.0, Radj, ldla);
      if (rc) return rc;
    }
  }
  hipLaunchKernelGGL(k_add_lower, dim3(grid_for((long long)n * n)), dim3(256), 0, ctx->stream,
                     La, ldla, n, Aadj, ldaa);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

}  // extern "C"
