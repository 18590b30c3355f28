/*
 * oracle/cpu_ref.h — CPU restatement of the reference's algorithms on the
 * hot path (TEST INFRASTRUCTURE: the parity checker and the "port" CPU
 * baseline; never linked into math_amd/).  Every entry point cites the
 * reference code it restates.  All matrices are column-major fp64 with
 * leading dimension = rows.  Pinned against tests/golden/*.json (generated
 * from the real reference by oracle/ref_harness.cpp) in tests/test_oracle.py.
 */
#ifndef SMG_ORACLE_CPU_REF_H
#define SMG_ORACLE_CPU_REF_H

#ifdef __cplusplus
extern "C" {
#endif

/* gp_exp_quad_cov fwd: K_ij = s^2 exp(-(x_i-x_j)^2 / (2 l^2)), full n x n.
 * rev/mat/fun/gp_exp_quad_cov.hpp:64-94 */
void oracle_gp_cov(const double* x, int n, double sigma, double l, double* K);
/* gp_exp_quad_cov rev: Kadj is the full n x n adjoint of the returned matrix.
 * Entries (i,j) and (j,i) alias one vari in the reference (:233-238), so
 * their adjoints are summed.  rev/mat/fun/gp_exp_quad_cov.hpp:96-112 */
void oracle_gp_cov_rev(const double* x, int n, double sigma, double l,
                       const double* Kadj, double* adj_sigma, double* adj_l);

/* Cholesky factor (lower, upper zeroed).  Returns 0, or 1 when not PD.
 * rev/mat/fun/cholesky_decompose.hpp:378-392 (Eigen LLT, check_pos_definite) */
int oracle_cholesky(const double* A, int n, double* L);
/* Murray's blocked adjoint (n > 35) / Giles' scalar adjoint (n <= 35).
 * Ladj: lower-triangular adjoint of L (read only).  Aadj += adjoint of the
 * LOWER triangle of A (the upper triangle is never touched).
 * rev/mat/fun/cholesky_decompose.hpp:118-165 and :233-254 */
void oracle_cholesky_rev(const double* L, const double* Ladj, int n,
                         double* Aadj);

/* multi_normal_cholesky_lpdf(y | mu, L), propto = false.
 * Writes lp and the partials the reference's operands_and_partials holds:
 * gy = -sd, gmu = +sd, gL = sd*half - inv(L)^T over ALL n*n entries.
 * prim/mat/prob/multi_normal_cholesky_lpdf.hpp:117-157 */
void oracle_mvn_cholesky(const double* y, const double* mu, const double* L,
                         int n, double* lp, double* gy, double* gmu,
                         double* gL);

/* C = A B (m x k times k x n); rev: Aadj += Cadj B^T, Badj += A^T Cadj.
 * rev/mat/fun/multiply.hpp:65-135 */
void oracle_multiply(const double* A, const double* B, int m, int k, int n,
                     double* C);
void oracle_multiply_rev(const double* A, const double* B, const double* Cadj,
                         int m, int k, int n, double* Aadj, double* Badj);

/* C = tri(A)^-1 B; rev: Badj += tri(A)^-T Cadj, Aadj += tri(-Badj C^T).
 * rev/mat/fun/mdivide_left_tri.hpp:16-128 */
void oracle_mdivide_left_tri(int lower, const double* A, const double* B,
                             int m, int n, double* C);
void oracle_mdivide_left_tri_rev(int lower, const double* A, const double* C,
                                 const double* Cadj, int m, int n,
                                 double* Aadj, double* Badj);

/* log_sum_exp over a vector; rev: xadj_i += adj * exp(x_i - lse).
 * rev/mat/fun/log_sum_exp.hpp:20-53, prim/scal/fun/log_sum_exp.hpp:47-59 */
double oracle_log_sum_exp(const double* x, int n);
void oracle_log_sum_exp_rev(const double* x, int n, double lse, double adj,
                            double* xadj);

/* special functions: lgamma = libm lgamma_r (prim/scal/fun/lgamma.hpp:62-71),
 * digamma = boost::math::digamma 53-bit path restated
 * (boost/math/special_functions/digamma.hpp:108-128,300-347,381-449),
 * trigamma = prim/scal/fun/trigamma.hpp:33-80 */
double oracle_lgamma(double x);
double oracle_digamma(double x);
double oracle_trigamma(double x);

/* normal_lpdf<false>(y | mu, sigma) over n elements (each argument is either
 * a length-n vector or a scalar when its stride is 0).  Partials per element.
 * prim/scal/prob/normal_lpdf.hpp:36-119 */
double oracle_normal_lpdf(const double* y, int sy, const double* mu, int smu,
                          const double* sigma, int ssig, int n, double* gy,
                          double* gmu, double* gsigma);

/* bernoulli_logit_glm_lpmf<false>(y | x, alpha, beta), scalar alpha.
 * x is R x M column-major.  prim/mat/prob/bernoulli_logit_glm_lpmf.hpp:92-135 */
double oracle_glm(const int* y, const double* x, long long R, int M,
                  double alpha, const double* beta, double* galpha,
                  double* gbeta);

/* normal_id_glm_lpdf<false>(y | x, alpha, beta, sigma), scalar alpha and
 * sigma.  prim/mat/prob/normal_id_glm_lpdf.hpp:84-150.  Returns logp; the
 * gradient wrt (alpha, beta, sigma) into g (M + 2). */
double oracle_normal_id_glm(const double* y, const double* x, long long R, int M,
                            double alpha, const double* beta, double sigma, double* g);

/* categorical_logit_glm_lpmf<false>(y | x, alpha, beta)
 * prim/mat/prob/categorical_logit_glm_lpmf.hpp:84-183.  x R x M col-major,
 * alpha C, beta M x C col-major, y in 1..C.  g (optional): [alpha'(C),
 * beta'(M x C)]. */
double oracle_categorical_logit_glm(const int* y, const double* x, long long R, int M, int C,
                                    const double* alpha, const double* beta, double* g);

/* poisson_log_glm_lpmf<false>(y | x, alpha, beta), scalar alpha.
 * prim/mat/prob/poisson_log_glm_lpmf.hpp:81-123.  Returns logp (lgamma terms
 * included); the gradient wrt (alpha, beta) into g (M + 1). */
double oracle_poisson_log_glm(const int* y, const double* x, long long R, int M,
                              double alpha, const double* beta, double* g);

/* SURVEY.md 8(f) row 3, value of f = sum(W .* F(args)) and the gradients
 * wrt every argument entry (all col-major).
 *   mdivide_left_spd       rev/mat/fun/mdivide_left_spd.hpp:57-63 (A n x n, B n x k)
 *   log_determinant_spd    rev/mat/fun/log_determinant_spd.hpp:16-57 (f = the value)
 *   mlt_self_transpose     rev/mat/fun/multiply_lower_tri_self_transpose.hpp:14-44 (L K x J)
 *   quad_form_sym          rev/mat/fun/quad_form.hpp:17-100 (A M x M, B M x N);
 *                          sym = 1: both operands var (prim/mat/fun/quad_form_sym.hpp:11-18)
 * Returns 0, or -1 when the Cholesky factorisation fails. */
int oracle_mdivide_left_spd(const double* A, const double* B, int n, int k, const double* W,
                            double* fx, double* gA, double* gB);
int oracle_log_determinant_spd(const double* A, int n, double* fx, double* gA);
void oracle_mlt_self_transpose(const double* L, int K, int J, const double* W, double* fx,
                               double* gL);
void oracle_quad_form_sym(const double* A, const double* B, int M, int N, const double* W,
                          int sym, double* fx, double* gA, double* gB);

/* GP marginal gradient (config 3) through the restated functors. */
void oracle_gp_marginal(const double* x, const double* y, int n,
                        const double* theta, double* fx, double* grad);
/* config 2: f(A) = sum(chol(add_diag(A A^T, n))) and its gradient. */
void oracle_mulchol(const double* A, int n, double* fx, double* grad);

#ifdef __cplusplus
}
#endif
#endif
