// The tangent of a Cholesky factor as ONE node of the fvar<var> tape:
//   L' = L Phi(Y),  Y = L^{-1} A' L^{-T}
// (the derivative of L = chol(A) along A'; Phi = strict lower triangle plus
// half the diagonal).  The reference (Stan Math 3.0.0) has no fvar
// specialisation of cholesky_decompose: fvar<var> runs Eigen's LLT
// (prim/mat/fun/cholesky_decompose.hpp) on fvar<var> scalars, which forms
// the same L' entry by entry at O(N^3) scalar tape nodes.  Composed from
// device functors, L' costs two triangular solves with N right-hand sides
// (2 N^3), their reverses (4 N^3) and L Phi with its reverse (N^3): 7 N^3.
// Here the node keeps W = L^{-1} (N^3 / 3 from the 512-row block inverses by
// recursive doubling) and Y, and its reverse is written out:
//   forward   T = tril(W A') (2 N^3 / 3),  Y = T W^T lower-computed and mirrored (N^3/3),
//             P = Phi(Y),  L' = L P (N^3/3)
//   reverse   Ladj += tril(tril(Ld_adj) P^T),  Padj = tril(L^T tril(Ld_adj))  (2 N^3/3)
//             S = Phi(Padj) + Phi(Padj)^T   (Padj's lower mirrored, by its product's store)
//             M = W^T S (N^3; W^T stored by the forward: an NN product)
//             Ladj -= tril(M Y) (N^3)
//             A'adj += (1/2) W^T S W = (1/2) M W, symmetric: its upper triangle (N^3 / 3)
// from dY = W dA' W^T - W dL Y - Y dL^T W^T: <Ybar, dY> = <W^T Ybar W, dA'>
// - <W^T (Ybar + Ybar^T) Y, dL>, Ybar = Phi(Padj) (Phi is its own adjoint).
// A' enters symmetrically (the tangent of a symmetric matrix), so its
// adjoint is the symmetric half (1/2) W^T S W; the parameters' gradients
// are the same sums.  Total ~5.3 N^3 instead of 7 N^3, in GEMMs whose K
// ranges are cut to the triangles.
#include "smg_internal.h"
#include "tri_small.h"

namespace {

// W[lo:hi, lo:hi] = L[lo:hi, lo:hi]^{-1} from the 512-row block inverses
// (aux level SMG_AUX_W512, ld n): halves combined by
//   W21 = -W22 (L21 W11)      (T: a (hi-mid) x (mid-lo) workspace, ld n)
int inv_rec(smg_ctx* ctx, const double* L, int ldl, const double* w512, int n, double* W, int ldw, double* T, int lo,
            int hi) {
  if (hi - lo == SMG_NBR)
    return smg_copy_impl(ctx, SMG_NBR, SMG_NBR, w512 + lo, n, W + lo + (size_t)lo * ldw, ldw, 1.0, 0);
  const int mid = lo + ((hi - lo) / SMG_NBR / 2) * SMG_NBR;
  int rc = inv_rec(ctx, L, ldl, w512, n, W, ldw, T, lo, mid);
  if (!rc) rc = inv_rec(ctx, L, ldl, w512, n, W, ldw, T, mid, hi);
  if (rc) return rc;
  const int a = hi - mid, b = mid - lo;
  rc = smg_gemm_impl(ctx, 0, 0, 0, a, b, b, 1.0, L + mid + (size_t)lo * ldl, ldl, W + lo + (size_t)lo * ldw, ldw,
                     0.0, T, n, SMG_TRI_B_LOWER);
  if (rc) return rc;
  return smg_gemm_impl(ctx, 0, 0, 0, a, b, a, -1.0, W + mid + (size_t)mid * ldw, ldw, T, n, 0.0,
                       W + mid + (size_t)lo * ldw, ldw, SMG_TRI_A_LOWER);
}

// fork: `side` follows everything queued on the main stream so far; join:
// the main stream follows everything queued on `side` (pooled events i)
int fork_side(smg_ctx* ctx, int i) {
  hipEvent_t e = smg_fork_event(ctx, i);
  if (!e) return SMG_ERR_HIP;
  SMG_HIP_TRY(hipEventRecord(e, ctx->stream));
  SMG_HIP_TRY(hipStreamWaitEvent(ctx->side, e, 0));
  return SMG_OK;
}
int join_side(smg_ctx* ctx, int i) {
  hipEvent_t e = smg_fork_event(ctx, i);
  if (!e) return SMG_ERR_HIP;
  SMG_HIP_TRY(hipEventRecord(e, ctx->side));
  SMG_HIP_TRY(hipStreamWaitEvent(ctx->stream, e, 0));
  return SMG_OK;
}

}  // namespace

extern "C" {

int smg_chol_tangent_fwd(smg_ctx* ctx, const double* L, int ldl, const double* aux, const double* Ad, int ldad, int n,
                         double* W, double* Wt, double* Y, double* P, double* Ld, int ld) {
  if (!ctx || n < 0) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  if (!L || !Ad || !W || !Wt || !Y || !P || !Ld || ldl < n || ldad < n || ld < n) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_TRSV);
  // W = L^{-1} (lower, stored zeros above)
  int rc = smg_memset(ctx, W, 0, sizeof(double) * (size_t)ld * n);
  if (rc) return rc;
  if (n % SMG_NBR == 0 && n >= 2 * SMG_NBR) {
    const double* w = aux;  // the factorisation's block inverses, or rebuilt here
    if (!w) {
      double* wn = smg_ws(ctx, SMG_WS_TMP2, (size_t)n * SMG_AUX_COLS);
      if (!wn) return SMG_ERR_OOM;
      if ((rc = smg_trtri_blocks_impl(ctx, L, ldl, n, wn))) return rc;
      if ((rc = smg_block_inverses_impl(ctx, L, ldl, wn, n))) return rc;
      w = wn;
    }
    if ((rc = inv_rec(ctx, L, ldl, w + (size_t)n * SMG_AUX_W512, n, W, ld, Y, 0, n))) return rc;
  } else {  // W = L^{-1} I by the blocked solve
    if ((rc = smg_add_diag_fwd(ctx, W, ld, n, 1.0, nullptr, W, ld))) return rc;  // W = I
    if ((rc = smg_trsm_impl(ctx, 1, 0, L, ldl, nullptr, 0, W, ld, n, n, nullptr, 0, aux))) return rc;
  }
  return smg_chol_tangent_fwd_w(ctx, L, ldl, W, Ad, ldad, n, Wt, Y, P, Ld, ld);
}

int smg_chol_tangent_fwd_w(smg_ctx* ctx, const double* L, int ldl, const double* W, const double* Ad, int ldad, int n,
                           double* Wt, double* Y, double* P, double* Ld, int ld) {
  if (!ctx || n < 0) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  if (!L || !W || !Ad || !Wt || !Y || !P || !Ld || ldl < n || ldad < n || ld < n) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_TRSV);
  int rc;
  // W^T stored for the reverse's M = W^T S (an NN product on the matrix
  // cores: the TN form ran at 34 TF/s against 75 for NN at N = 4096).  W's
  // strict upper may hold anything outside its 512-row diagonal blocks (the
  // progressive factorisation's W): every product below cuts K to the
  // triangles in bands of at most 128 rows / columns, so those entries (and
  // their transposes in Wt) are never read.  Only the reverse reads Wt: the
  // transpose runs on `side` beside T's product, joined at the end
  const bool fork = smg_side_begin(ctx) == SMG_OK;
  if (fork) {
    if ((rc = fork_side(ctx, 0))) return rc;
    smg_on_side on(ctx);
    if ((rc = smg_transpose(ctx, n, n, W, ld, Wt, ld, 0.0))) return rc;
  } else if ((rc = smg_transpose(ctx, n, n, W, ld, Wt, ld, 0.0))) {
    return rc;
  }
  // T = tril(W A') (in Ld's storage), Y = T W^T (lower computed, mirrored):
  // Y_ij, i >= j, sums T_ik W_jk over k <= j <= i, so only T's lower triangle
  // is read (its upper meets only the discarded upper outputs of the
  // diagonal tiles): N^3 / 3 instead of N^3 / 2 multiply-adds for T
  // (A' is symmetric -- the tangent of the factorised symmetric matrix -- so
  // it enters as op(B) = A'^T: the B tile then loads n-contiguous runs; the
  // NN form with a k-contiguous B ran 30-50 % slower in the HVP's trace)
  if ((rc = smg_gemm_impl(ctx, 0, 1, 1, n, n, n, 1.0, W, ld, Ad, ldad, 0.0, Ld, ld, SMG_TRI_A_LOWER))) return rc;
  // (P = Phi(Y) from the same epilogue: its strict upper is zeroed inside the
  // diagonal 64-blocks only -- L P cuts K to k >= j, T P^T to k <= j, in whole
  // blocks, so no other upper entry is read)
  if ((rc = smg_gemm_sym_phi_impl(ctx, 0, 1, n, n, 1.0, Ld, ld, W, ld, 0.0, Y, ld, P, ld, SMG_TRI_B_UPPER))) return rc;
  if ((rc = smg_multiply_lower_fwd(ctx, L, ldl, P, ld, n, Ld, ld))) return rc;
  return fork ? join_side(ctx, 1) : SMG_OK;
}

int smg_chol_tangent_rev(smg_ctx* ctx, const double* L, int ldl, const double* W, const double* Wt, const double* Y,
                         const double* P, int ld, const double* Ldadj, int ldla, int n, double* Ladj, int ldladj,
                         double* Adadj, int ldaa, double* ws) {
  if (!ctx || n < 0) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  if (!L || !W || !Wt || !Y || !P || !Ldadj || !ws || ldl < n || ld < n || ldla < n) return SMG_ERR_ARG;
  if ((Ladj && ldladj < n) || (Adadj && ldaa < n)) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_TRSV);
  const size_t nn = (size_t)n * n;
  double* S = ws;       // Padj, then S, then (1/2) M W
  double* M = ws + nn;  // tril(Ld_adj), then M
  // smg_multiply_lower_rev's two products on T = tril(Ld_adj) (one copy
  // pass zeroing the upper), Padj written (beta 0: its upper is never read,
  // sym_from_lower forms it from the lower) instead of accumulated into a
  // cleared S
  int rc = smg_copy_tril(ctx, n, n, Ldadj, ldla, M, n);
  if (rc) return rc;
  if (!Ladj && !Adadj) return SMG_OK;
  // The two pairs of independent products run at once, one on `side`: the
  // grids' last partial waves leave CUs to the other launch
  //   Ladj += tril(T P^T)  (main)  ||  Padj = tril(L^T T), S  (side)
  //   Ladj -= tril(M Y)    (main)  ||  (1/2) M W, A'adj      (side)
  const bool fork = Ladj && smg_side_begin(ctx) == SMG_OK;
  if (fork && (rc = fork_side(ctx, 2))) return rc;
  {
    smg_on_side on(ctx);
    if (!fork) ctx->stream = ctx->main_stream;
    // (S = Padj's lower triangle mirrored: the product's symmetric store, uplo 3)
    if ((rc = smg_gemm_impl(ctx, 1, 0, 3, n, n, n, 1.0, L, ldl, M, n, 0.0, S, n, SMG_TRI_A_UPPER | SMG_TRI_B_LOWER)))
      return rc;
  }
  if (Ladj && (rc = smg_gemm_impl(ctx, 0, 1, 1, n, n, n, 1.0, M, n, P, ld, 1.0, Ladj, ldladj,
                                  SMG_TRI_A_LOWER | SMG_TRI_B_UPPER)))
    return rc;
  if (fork && (rc = join_side(ctx, 3))) return rc;  // S formed, T no longer read: M may be overwritten
  if ((rc = smg_gemm_impl(ctx, 0, 0, 0, n, n, n, 1.0, Wt, ld, S, n, 0.0, M, n, SMG_TRI_A_UPPER))) return rc;
  if (Adadj) {
    if (fork && (rc = fork_side(ctx, 4))) return rc;
    smg_on_side on(ctx);
    if (!fork) ctx->stream = ctx->main_stream;
    // (1/2) M W = (1/2) W^T S W is symmetric: its UPPER triangle is computed
    // (with op(B) = W lower, tile column j takes K = n - j over j + 1 tiles:
    // half the lower triangle's multiply-adds, N^3 / 6 instead of N^3 / 3) and
    // added into A'adj symmetrically
    if ((rc = smg_gemm_impl(ctx, 0, 1, 2, n, n, n, 0.5, M, n, Wt, ld, 0.0, S, n, SMG_TRI_B_LOWER))) return rc;
    if ((rc = smg_add_sym_from_upper(ctx, n, S, n, Adadj, ldaa))) return rc;
  }
  // (Y is stored mirrored, so Y^T = Y bit for bit, and W = (W^T)^T: both
  // right operands enter transposed, as n-contiguous B tiles: in the HVP's
  // trace the NN forms ran tril(M Y) at 42 and (1/2) M W at 23 TF/s)
  if (Ladj && (rc = smg_gemm_impl(ctx, 0, 1, 1, n, n, n, -1.0, M, n, Y, ld, 1.0, Ladj, ldladj))) return rc;
  return fork && Adadj ? join_side(ctx, 5) : SMG_OK;
}

}  // extern "C"
