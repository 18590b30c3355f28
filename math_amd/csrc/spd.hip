// The SPD / quadratic-form functors of SURVEY.md §8(f) row 3, composed from
// the Cholesky, blocked TRSM and GEMM kernels (no explicit inverse in the
// forward of mdivide_left_spd, none anywhere except the gradient of
// log_determinant_spd, which IS the inverse):
//
//   mdivide_left_spd(A, B)      rev/mat/fun/mdivide_left_spd.hpp:20-150
//     fwd C = A^{-1} B through L = chol(lower(A)) (Eigen's LLT reads the lower
//     triangle only); rev W = A^{-1} Cadj, Aadj -= W C^T (every entry),
//     Badj += W (:57-63, :95-99, :131-135)
//   log_determinant_spd(A)      rev/mat/fun/log_determinant_spd.hpp:16-57
//     fwd 2 sum log L_ii; rev Aadj += adj A^{-1} (every entry, :48-53)
//   multiply_lower_tri_self_transpose(L)
//                               rev/mat/fun/multiply_lower_tri_self_transpose.hpp:14-44
//     fwd C = T T^T with T the lower trapezoid of L; the (m, n) and (n, m)
//     entries share one vari, so rev T_adj += (Cadj + Cadj^T) T on the
//     trapezoid
//   quad_form_sym(A, B)         rev/mat/fun/quad_form_sym.hpp:15-40, quad_form.hpp:17-100
//     fwd Cd = B^T A B, C = (Cd + Cd^T)/2; rev Aadj += B Cadj B^T,
//     Badj += A B Cadj^T + A^T B Cadj (the reference's chainA / chainB).
//     With A and B both var the reference resolves to the prim template
//     (prim/mat/fun/quad_form_sym.hpp:11-18) and autodiffs 0.5 (Cd + Cd^T):
//     sym_adj = 1 replaces Cadj by sym(Cadj) = (Cadj + Cadj^T)/2
#include "smg_internal.h"
#include "tri_small.h"

namespace {

// out[0] = 2 sum_i log L_ii (one workgroup, fixed order: deterministic)
__global__ __launch_bounds__(256) void k_logdet_chol(const double* __restrict__ L, int ldl, int n,
                                                     double* out) {
  __shared__ double lds[16];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += log(L[i + (size_t)i * ldl]);
  s = block_sum(s, lds);
  if (threadIdx.x == 0) out[0] = 2.0 * s;
}

// Y (m x n, ld ldy) = X + X^T scaled: Y = a (X + X^T) (X square n x n, ld ldx)
__global__ void k_sym_sum(int n, double a, const double* __restrict__ X, int ldx,
                          double* __restrict__ Y, int ldy) {
  for (smg_mn it(n, n); it.ok(); it.next()) {
    const int i = it.i, j = it.j;
    Y[i + (size_t)j * ldy] = a * (X[i + (size_t)j * ldx] + X[j + (size_t)i * ldx]);
  }
}

// T (K x J, ld K) = lower trapezoid of L (zeros above the diagonal)
__global__ void k_lower_trapezoid(int K, int J, const double* __restrict__ L, int ldl,
                                  double* __restrict__ T) {
  for (smg_mn it(K, J); it.ok(); it.next()) {
    const int i = it.i, j = it.j;
    T[i + (size_t)j * K] = i >= j ? L[i + (size_t)j * ldl] : 0.0;
  }
}

// Ladj (lower trapezoid, ld ldla) += G (K x J, ld K)
__global__ void k_add_lower_trapezoid(int K, int J, const double* __restrict__ G,
                                      double* __restrict__ Ladj, int ldla) {
  for (smg_mn it(K, J); it.ok(); it.next()) {
    const int i = it.i, j = it.j;
    if (i >= j) Ladj[i + (size_t)j * ldla] += G[i + (size_t)j * K];
  }
}

inline int grid_for(long long tot) {
  long long g = (tot + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (int)g;
}

// B (m x n, ld ldb) <- A^{-1} B given L = chol(A) and its 64-block inverses
int spd_solve(smg_ctx* ctx, const double* L, const double* aux, int m, double* B, int ldb, int n) {
  int rc = smg_trsm_impl(ctx, 1, 0, L, m, aux, m, B, ldb, m, n);  // L^{-1} B
  if (rc) return rc;
  return smg_trsm_impl(ctx, 1, 1, L, m, aux, m, B, ldb, m, n);    // L^{-T} (.)
}

}  // namespace

extern "C" {

int smg_mdivide_left_spd_fwd(smg_ctx* ctx, const double* A, int lda, const double* B, int ldb,
                             int m, int n, double* L, double* aux, double* C, int ldc) {
  if (!ctx || m < 0 || n < 0) return SMG_ERR_ARG;
  if (m == 0) return SMG_OK;
  if (!A || !L || !aux || lda < m || (n > 0 && (!B || !C || ldb < m || ldc < m)))
    return SMG_ERR_ARG;
  int rc = smg_cholesky_fwd(ctx, A, lda, m, L, m, aux);
  if (rc || n == 0) return rc;
  smg_prof_scope prof(ctx, SMG_FAM_TRSV);
  rc = smg_copy_impl(ctx, m, n, B, ldb, C, ldc, 1.0, 0);
  if (rc) return rc;
  return spd_solve(ctx, L, aux, m, C, ldc, n);
}

int smg_mdivide_left_spd_rev(smg_ctx* ctx, const double* L, const double* aux, int m, int n,
                             const double* C, int ldc, const double* Cadj, int ldca, double* Aadj,
                             int ldaa, double* Badj, int ldba, double* ws) {
  if (!ctx || m < 0 || n < 0) return SMG_ERR_ARG;
  if (m == 0 || n == 0) return SMG_OK;
  if (!L || !aux || !C || !Cadj || !ws) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_TRSV);
  int rc = smg_copy_impl(ctx, m, n, Cadj, ldca, ws, m, 1.0, 0);  // W = A^{-1} Cadj
  if (rc) return rc;
  rc = spd_solve(ctx, L, aux, m, ws, m, n);
  if (rc) return rc;
  if (Aadj) {  // Aadj -= W C^T
    rc = smg_gemm_impl(ctx, 0, 1, 0, m, m, n, -1.0, ws, m, C, ldc, 1.0, Aadj, ldaa);
    if (rc) return rc;
  }
  if (Badj) return smg_copy_impl(ctx, m, n, ws, m, Badj, ldba, 1.0, 1);
  return SMG_OK;
}

int smg_log_determinant_spd_fwd(smg_ctx* ctx, const double* A, int lda, int n, double* L,
                                double* aux, double* out) {
  if (!ctx || n < 0 || !out) return SMG_ERR_ARG;
  if (n == 0) return smg_memset(ctx, out, 0, sizeof(double));
  if (!A || !L || !aux || lda < n) return SMG_ERR_ARG;
  int rc = smg_cholesky_fwd(ctx, A, lda, n, L, n, aux);
  if (rc) return rc;
  hipLaunchKernelGGL(k_logdet_chol, dim3(1), dim3(256), 0, ctx->stream, L, n, n, out);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_log_determinant_spd_rev(smg_ctx* ctx, const double* L, const double* aux, int n,
                                double adj, double* Aadj, int ldaa, double* ws) {
  if (!ctx || n < 0) return SMG_ERR_ARG;
  if (n == 0 || adj == 0.0) return SMG_OK;
  if (!L || !aux || !Aadj || !ws) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_TRSV);
  // ws = A^{-1} = L^{-T} L^{-1} I
  int rc = smg_memset(ctx, ws, 0, sizeof(double) * (size_t)n * n);
  if (rc) return rc;
  rc = smg_add_diag_fwd(ctx, ws, n, n, 1.0, nullptr, ws, n);
  if (rc) return rc;
  rc = spd_solve(ctx, L, aux, n, ws, n, n);
  if (rc) return rc;
  return smg_copy_impl(ctx, n, n, ws, n, Aadj, ldaa, adj, 1);
}

int smg_multiply_lower_tri_self_transpose_fwd(smg_ctx* ctx, const double* L, int ldl, int K, int J,
                                              double* C, int ldc, double* ws) {
  if (!ctx || K < 0 || J < 0) return SMG_ERR_ARG;
  if (K == 0) return SMG_OK;
  if (!C || ldc < K || (J > 0 && (!L || !ws || ldl < K))) return SMG_ERR_ARG;
  if (J == 0) return smg_scale_impl(ctx, K, K, 0.0, C, ldc, 0);
  smg_prof_scope prof(ctx, SMG_FAM_GEMM);
  double* T = ws;  // K x J
  hipLaunchKernelGGL(k_lower_trapezoid, dim3(grid_for((long long)K * J)), dim3(256), 0, ctx->stream,
                     K, J, L, ldl, T);
  SMG_LAUNCH_CHECK();
  return smg_gemm_impl(ctx, 0, 1, 0, K, K, J, 1.0, T, K, T, K, 0.0, C, ldc);
}

int smg_multiply_lower_tri_self_transpose_rev(smg_ctx* ctx, const double* L, int ldl, int K, int J,
                                              const double* Cadj, int ldca, double* Ladj, int ldla,
                                              double* ws) {
  if (!ctx || K < 0 || J < 0) return SMG_ERR_ARG;
  if (K == 0 || J == 0) return SMG_OK;
  if (!L || !Cadj || !Ladj || !ws) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_GEMM);
  double* T = ws;                       // K x J
  double* S = ws + (size_t)K * J;       // K x K = Cadj + Cadj^T
  double* G = S + (size_t)K * K;        // K x J = S T
  hipLaunchKernelGGL(k_lower_trapezoid, dim3(grid_for((long long)K * J)), dim3(256), 0, ctx->stream,
                     K, J, L, ldl, T);
  hipLaunchKernelGGL(k_sym_sum, dim3(grid_for((long long)K * K)), dim3(256), 0, ctx->stream, K, 1.0,
                     Cadj, ldca, S, K);
  int rc = smg_gemm_impl(ctx, 0, 0, 0, K, J, K, 1.0, S, K, T, K, 0.0, G, K);
  if (rc) return rc;
  hipLaunchKernelGGL(k_add_lower_trapezoid, dim3(grid_for((long long)K * J)), dim3(256), 0,
                     ctx->stream, K, J, G, Ladj, ldla);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_quad_form_sym_fwd(smg_ctx* ctx, const double* A, int lda, const double* B, int ldb, int M,
                          int N, double* C, int ldc, double* ws) {
  if (!ctx || M < 0 || N < 0) return SMG_ERR_ARG;
  if (N == 0) return SMG_OK;
  if (!C || ldc < N || (M > 0 && (!A || !B || !ws || lda < M || ldb < M))) return SMG_ERR_ARG;
  if (M == 0) return smg_scale_impl(ctx, N, N, 0.0, C, ldc, 0);
  smg_prof_scope prof(ctx, SMG_FAM_GEMM);
  double* AB = ws;                      // M x N
  double* Cd = ws + (size_t)M * N;      // N x N
  int rc = smg_gemm_impl(ctx, 0, 0, 0, M, N, M, 1.0, A, lda, B, ldb, 0.0, AB, M);
  if (rc) return rc;
  rc = smg_gemm_impl(ctx, 1, 0, 0, N, N, M, 1.0, B, ldb, AB, M, 0.0, Cd, N);
  if (rc) return rc;
  hipLaunchKernelGGL(k_sym_sum, dim3(grid_for((long long)N * N)), dim3(256), 0, ctx->stream, N, 0.5,
                     Cd, N, C, ldc);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_quad_form_sym_rev(smg_ctx* ctx, const double* A, int lda, const double* B, int ldb, int M,
                          int N, const double* Cadj, int ldca, int sym_adj, double* Aadj, int ldaa,
                          double* Badj, int ldba, double* ws) {
  if (!ctx || M < 0 || N < 0) return SMG_ERR_ARG;
  if (M == 0 || N == 0) return SMG_OK;
  if (!A || !B || !Cadj || !ws) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_GEMM);
  double* BC = ws;  // M x N
  int rc;
  if (sym_adj) {  // the prim template's autodiff of 0.5 (Cd + Cd^T): Cd_adj = sym(Cadj)
    double* S = ws + (size_t)M * N;
    hipLaunchKernelGGL(k_sym_sum, dim3(grid_for((long long)N * N)), dim3(256), 0, ctx->stream, N, 0.5,
                       Cadj, ldca, S, N);
    SMG_LAUNCH_CHECK();
    Cadj = S;
    ldca = N;
  }
  if (Aadj) {  // Aadj += (B Cadj) B^T
    rc = smg_gemm_impl(ctx, 0, 0, 0, M, N, N, 1.0, B, ldb, Cadj, ldca, 0.0, BC, M);
    if (rc) return rc;
    rc = smg_gemm_impl(ctx, 0, 1, 0, M, M, N, 1.0, BC, M, B, ldb, 1.0, Aadj, ldaa);
    if (rc) return rc;
  }
  if (Badj) {  // Badj += A (B Cadj^T) + A^T (B Cadj)
    rc = smg_gemm_impl(ctx, 0, 1, 0, M, N, N, 1.0, B, ldb, Cadj, ldca, 0.0, BC, M);
    if (rc) return rc;
    rc = smg_gemm_impl(ctx, 0, 0, 0, M, N, M, 1.0, A, lda, BC, M, 1.0, Badj, ldba);
    if (rc) return rc;
    rc = smg_gemm_impl(ctx, 0, 0, 0, M, N, N, 1.0, B, ldb, Cadj, ldca, 0.0, BC, M);
    if (rc) return rc;
    rc = smg_gemm_impl(ctx, 1, 0, 0, M, N, M, 1.0, A, lda, BC, M, 1.0, Badj, ldba);
    if (rc) return rc;
  }
  return SMG_OK;
}

}  // extern "C"
