#ifndef STAN_MATH_MIX_FVAR_FUNCTORS_HPP
#define STAN_MATH_MIX_FVAR_FUNCTORS_HPP

// The GP path's functors at T = fvar<var> (fwd-over-rev), as used by
// hessian_times_vector (mix/mat/functor/hessian_times_vector.hpp:13-40).
//
// The reference instantiates its prim templates with fvar<var> scalars and
// runs O(N^3) scalar fvar<var> operations (an LLT over fvar, SURVEY.md §8 a21:
// infeasible at N=4096).  Here a matrix of fvar<var> is a DUAL device matrix:
// value and tangent are each a device matrix of vars, and the tangent rules
// are written with the device var functors, so the tangent is itself on the
// tape and the reverse sweep differentiates it:
//   K'  = gp_exp_quad_cov tangent along (sigma', l')          (one kernel)
//   (A + diag d)' = A' + diag d'
//   L'  = L Phi(L^{-1} A' L^{-T})                               (2 TRSM + 1 GEMM)
//   lp' = w^T L^{-1} L' w - sum_i L'_ii / L_ii,  w = L^{-1}(y - mu)
// (the derivative of -|w|^2/2 - sum log L_ii, prim/mat/prob/
// multi_normal_cholesky_lpdf.hpp:117-131).
// Beyond the GP set, with the reference's tangent
// rules:
//   (A B)'            = A' B + A B'                (fwd/mat/fun/multiply.hpp)
//   (A^{-1} B)'       = A^{-1} (B' - tril(A') C)   (fwd/mat/fun/mdivide_left_tri_low.hpp:40-44)
//   log_sum_exp(x)'   = softmax(x) . x'            (fwd/mat/fun/log_sum_exp.hpp)
//   bernoulli_logit_glm_lpmf' = sum_i d_i (x_i beta' + alpha')
//                     (fwd operands_and_partials over the prim GLM's
//                      theta_derivative d, prim/mat/prob/bernoulli_logit_glm_lpmf.hpp:117-141)
// plus transpose, sum, add_diag and the Eigen Matrix<fvar<var>> bridge, so
// hessian() (mix/mat/functor/hessian.hpp:39-72) runs on models built from
// multiply / cholesky_decompose / mdivide_left_tri / log_sum_exp / the GLM.

#include <stan/math/amd/matrix.hpp>
#include <stan/math/fwd/core/fvar.hpp>
#include <stan/math/rev/core.hpp>
#include <stan/math/rev/fun/cholesky_decompose.hpp>
#include <cstdlib>
#include <stan/math/rev/fun/gp_exp_quad_cov.hpp>
#include <stan/math/rev/fun/mdivide_left_tri.hpp>
#include <stan/math/rev/fun/multi_normal_cholesky_lpdf.hpp>
#include <stan/math/rev/fun/multiply.hpp>
#include <stan/math/rev/fun/tangent_ops.hpp>
#include <stan/math/rev/fun/log_sum_exp.hpp>
#include <stan/math/rev/fun/bernoulli_logit_glm_lpmf.hpp>

#include <vector>

namespace stan {
namespace math {

/** A matrix of fvar<var>: value and tangent as device matrices of vars. */
struct dev_fvar_matrix {
  dev_var_matrix val_;
  dev_var_matrix d_;
  int rows() const { return val_.rows(); }
  int cols() const { return val_.cols(); }
};

inline dev_fvar_matrix gp_exp_quad_cov(const dev_data<double>& x, const fvar<var>& sigma,
                                       const fvar<var>& length_scale) {
  dev_fvar_matrix K;
  K.val_ = gp_exp_quad_cov(x, sigma.val_, length_scale.val_);
  K.d_ = gp_exp_quad_cov_tangent(x, sigma.val_, length_scale.val_, sigma.d_, length_scale.d_);
  return K;
}
inline dev_fvar_matrix gp_exp_quad_cov(const std::vector<double>& x, const fvar<var>& sigma,
                                       const fvar<var>& length_scale) {
  return gp_exp_quad_cov(internal::gp_x_to_device(x), sigma, length_scale);
}

inline dev_fvar_matrix add_diag(const dev_fvar_matrix& A, const fvar<var>& d) {
  return dev_fvar_matrix{add_diag(A.val_, d.val_), add_diag(A.d_, d.d_)};
}
inline dev_fvar_matrix add_diag(const dev_fvar_matrix& A, double d) {
  return dev_fvar_matrix{add_diag(A.val_, d), A.d_};
}

namespace internal {
// C = L Phi for lower-triangular L and Phi (smg_multiply_lower_fwd: lower
// tiles, K ranges cut to the triangles, N^3/3 flops); the reverse reads only
// the lower triangle of C's adjoint and writes only the lower triangles of
// L's and Phi's (both lower-structured: their upper adjoints are never read).
class multiply_lower_dev_vari : public device_vari {
 public:
  dev_matrix_vari* A_;
  dev_matrix_vari* B_;
  dev_matrix_vari* C_;
  multiply_lower_dev_vari(dev_matrix_vari* A, dev_matrix_vari* B)
      : device_vari(0.0), A_(A), B_(B), C_(new dev_matrix_vari(A->rows_, B->cols_, dev_structure::lower)) {
    const int n = A->rows_;
    amd::check(smg_multiply_lower_fwd(amd::ctx(), A_->val_, n, B_->val_, n, n, C_->val_, n), "multiply");
  }
  void chain() override {
    const int n = A_->rows_;
    double* ws = amd::alloc_doubles(size_t(n) * n);
    amd::check(smg_multiply_lower_rev(amd::ctx(), A_->val_, n, B_->val_, n, C_->adj_, n, n, A_->adj_, n,
                                      B_->adj_, n, ws),
               "multiply");
  }
};
}  // namespace internal

namespace internal {
// C = A + B (same shape)
class add_dev_vari : public device_vari {
 public:
  dev_matrix_vari* A_;
  dev_matrix_vari* B_;
  dev_matrix_vari* C_;
  add_dev_vari(dev_matrix_vari* A, dev_matrix_vari* B)
      : device_vari(0.0), A_(A), B_(B), C_(new dev_matrix_vari(A->rows_, A->cols_)) {
    smg_ctx* c = amd::ctx();
    amd::check(smg_copy_matrix(c, A->rows_, A->cols_, A->val_, A->rows_, C_->val_, C_->rows_, 0, 0), "add");
    amd::check(smg_axpy(c, (long long)C_->size(), 1.0, B->val_, 1, C_->val_, 1), "add");
  }
  void chain() override {
    smg_ctx* c = amd::ctx();
    amd::check(smg_axpy(c, (long long)C_->size(), 1.0, C_->adj_, 1, A_->adj_, 1), "add");
    amd::check(smg_axpy(c, (long long)C_->size(), 1.0, C_->adj_, 1, B_->adj_, 1), "add");
  }
};

// C = tril(A): the lower triangle (diagonal included), zeros above
class tril_dev_vari : public device_vari {
 public:
  dev_matrix_vari* A_;
  dev_matrix_vari* C_;
  explicit tril_dev_vari(dev_matrix_vari* A)
      : device_vari(0.0), A_(A), C_(new dev_matrix_vari(A->rows_, A->cols_, dev_structure::lower)) {
    smg_ctx* c = amd::ctx();
    amd::zero(C_->val_, C_->size());
    amd::check(smg_add_tril(c, A->rows_, A->cols_, 1.0, A->val_, A->rows_, C_->val_, C_->rows_), "tril");
  }
  void chain() override {
    amd::check(smg_add_tril(amd::ctx(), A_->rows_, A_->cols_, 1.0, C_->adj_, C_->rows_, A_->adj_, A_->rows_),
               "tril");
  }
};

// t = softmax(x) . x' (a var of x and x')
class lse_tangent_dev_vari : public device_vari {
 public:
  dev_matrix_vari* x_;
  dev_matrix_vari* xd_;
  double lse_;
  lse_tangent_dev_vari(double t, double lse, dev_matrix_vari* x, dev_matrix_vari* xd)
      : device_vari(t), x_(x), xd_(xd), lse_(lse) {}
  void chain() override {
    amd::check(smg_lse_tangent_rev(amd::ctx(), x_->val_, xd_->val_, (long long)x_->size(), lse_, val_, adj_,
                                   x_->adj_, xd_->adj_),
               "log_sum_exp");
  }
};

// t = sum_i d(eta_i + alpha) (eta'_i + alpha') of the bernoulli logit GLM
class glm_tangent_dev_vari : public device_vari {
 public:
  dev_matrix_vari* eta_;
  dev_matrix_vari* etad_;
  vari* alpha_;   // null: data
  vari* alphad_;  // null: data
  double a_, ad_;
  const int* y_;
  double* out2_;
  glm_tangent_dev_vari(double t, dev_matrix_vari* eta, dev_matrix_vari* etad, vari* alpha, vari* alphad, double a,
                       double ad, const int* y)
      : device_vari(t), eta_(eta), etad_(etad), alpha_(alpha), alphad_(alphad), a_(a), ad_(ad), y_(y),
        out2_(amd::alloc_doubles(2)) {}
  void chain() override {
    amd::check(smg_glm_tangent_rev(amd::ctx(), eta_->val_, a_, etad_->val_, ad_, y_, (long long)eta_->size(), adj_,
                                   eta_->adj_, etad_->adj_, out2_),
               "bernoulli_logit_glm_lpmf");
    if (alpha_) add_pending_adjoint(alpha_, out2_);
    if (alphad_) add_pending_adjoint(alphad_, out2_ + 1);
  }
};
}  // namespace internal

/** A + B of two device matrices of vars (same shape). */
inline dev_var_matrix add(const dev_var_matrix& A, const dev_var_matrix& B) {
  if (A.rows() != B.rows() || A.cols() != B.cols()) throw std::invalid_argument("add: size mismatch");
  return dev_var_matrix((new internal::add_dev_vari(A.vi_, B.vi_))->C_);
}
/** tril(A) of a device matrix of vars. */
inline dev_var_matrix tril(const dev_var_matrix& A) {
  return dev_var_matrix((new internal::tril_dev_vari(A.vi_))->C_);
}

/** Eigen Matrix<fvar<var>> (host) -> dual device matrix (both parts bridged). */
#ifdef STAN_MATH_AMD_HAS_EIGEN
template <int R, int C>
inline dev_fvar_matrix to_dev(const Eigen::Matrix<fvar<var>, R, C>& m, int rows = -1, int cols = -1) {
  const size_t n = size_t(m.size());
  std::vector<var> v(n), d(n);
  for (size_t i = 0; i < n; ++i) {
    v[i] = m(Eigen::Index(i)).val_;
    d[i] = m(Eigen::Index(i)).d_;
  }
  if (rows < 0) {  // the matrix's own shape; rows x cols reshapes (column-major)
    rows = int(m.rows());
    cols = int(m.cols());
  }
  return dev_fvar_matrix{to_dev(v, rows, cols), to_dev(d, rows, cols)};
}
#endif
inline dev_fvar_matrix to_dev(const std::vector<fvar<var>>& x, int rows = -1, int cols = 1) {
  std::vector<var> v(x.size()), d(x.size());
  for (size_t i = 0; i < x.size(); ++i) {
    v[i] = x[i].val_;
    d[i] = x[i].d_;
  }
  return dev_fvar_matrix{to_dev(v, rows, cols), to_dev(d, rows, cols)};
}

inline dev_fvar_matrix transpose(const dev_fvar_matrix& A) {
  return dev_fvar_matrix{transpose(A.val_), transpose(A.d_)};
}
inline fvar<var> sum(const dev_fvar_matrix& A) {
  fvar<var> s;
  s.val_ = sum(A.val_);
  s.d_ = sum(A.d_);
  return s;
}

/** (A B)' = A' B + A B' (fwd/mat/fun/multiply.hpp). */
inline dev_fvar_matrix multiply(const dev_fvar_matrix& A, const dev_fvar_matrix& B) {
  dev_fvar_matrix C;
  C.val_ = multiply(A.val_, B.val_);
  C.d_ = add(multiply(A.d_, B.val_), multiply(A.val_, B.d_));
  return C;
}
inline dev_fvar_matrix multiply(const dev_fvar_matrix& A, const dev_data<double>& B) {
  return dev_fvar_matrix{multiply(A.val_, B), multiply(A.d_, B)};
}
inline dev_fvar_matrix multiply(const dev_data<double>& A, const dev_fvar_matrix& B) {
  return dev_fvar_matrix{multiply(A, B.val_), multiply(A, B.d_)};
}

/** C = A^{-1} B for lower-triangular A: C' = A^{-1} (B' - tril(A') C)
 * (fwd/mat/fun/mdivide_left_tri_low.hpp:40-44). */
template <int TriView>
inline dev_fvar_matrix mdivide_left_tri(const dev_fvar_matrix& A, const dev_fvar_matrix& B) {
  static_assert(TriView == 1, "mdivide_left_tri<fvar<var>>: lower-triangular view (Eigen::Lower)");
  dev_fvar_matrix C;
  C.val_ = mdivide_left_tri<TriView>(A.val_, B.val_);
  C.d_ = mdivide_left_tri<TriView>(A.val_, add(B.d_, multiply(-1.0, multiply(tril(A.d_), C.val_))));
  return C;
}
template <int TriView>
inline dev_fvar_matrix mdivide_left_tri(const dev_data<double>& A, const dev_fvar_matrix& B) {
  static_assert(TriView == 1, "mdivide_left_tri<fvar<var>>: lower-triangular view (Eigen::Lower)");
  return dev_fvar_matrix{mdivide_left_tri<TriView>(A, B.val_), mdivide_left_tri<TriView>(A, B.d_)};
}
template <int TriView>
inline dev_fvar_matrix mdivide_left_tri(const dev_fvar_matrix& A, const dev_data<double>& B) {
  static_assert(TriView == 1, "mdivide_left_tri<fvar<var>>: lower-triangular view (Eigen::Lower)");
  dev_fvar_matrix C;
  C.val_ = mdivide_left_tri<TriView>(A.val_, B);
  C.d_ = mdivide_left_tri<TriView>(A.val_, multiply(-1.0, multiply(tril(A.d_), C.val_)));
  return C;
}

/** log_sum_exp' = softmax(x) . x' (fwd/mat/fun/log_sum_exp.hpp). */
inline fvar<var> log_sum_exp(const dev_fvar_matrix& x) {
  fvar<var> r;
  r.val_ = log_sum_exp(x.val_);
  if (x.val_.size() == 0) {
    r.d_ = var(0.0);
    return r;
  }
  smg_ctx* c = amd::ctx();
  double* out = amd::alloc_doubles(2);
  amd::check(smg_lse_tangent_fwd(c, x.val_.val_ptr(), x.d_.val_ptr(), (long long)x.val_.size(), out),
             "log_sum_exp");
  double h[2];
  amd::to_host(h, out, 2);
  r.d_ = var(new internal::lse_tangent_dev_vari(h[1], h[0], x.val_.vi_, x.d_.vi_));
  return r;
}
inline fvar<var> log_sum_exp(const std::vector<fvar<var>>& x) { return log_sum_exp(to_dev(x)); }

/** bernoulli_logit_glm_lpmf(y | x, alpha, beta) at fvar<var> alpha / beta,
 * x and y data on the device: the value by the var GLM, the tangent
 * sum_i d_i (x_i beta' + alpha') by the reference's theta_derivative. */
template <bool propto = false>
inline fvar<var> bernoulli_logit_glm_lpmf(const dev_data<int>& y, const dev_data<double>& x, const fvar<var>& alpha,
                                          const dev_fvar_matrix& beta) {
  fvar<var> lp;
  lp.val_ = bernoulli_logit_glm_lpmf<propto>(y, x, alpha.val_, beta.val_);
  const long long R = x.rows();
  if (R == 0) {
    lp.d_ = var(0.0);
    return lp;
  }
  dev_var_matrix eta = multiply(x, beta.val_);
  dev_var_matrix etad = multiply(x, beta.d_);
  smg_ctx* c = amd::ctx();
  double* out = amd::alloc_doubles(1);
  amd::check(smg_glm_tangent_fwd(c, eta.val_ptr(), alpha.val_.val(), etad.val_ptr(), alpha.d_.val(), y.data(), R, out),
             "bernoulli_logit_glm_lpmf");
  double t = 0.0;
  amd::to_host(&t, out, 1);
  lp.d_ = var(new internal::glm_tangent_dev_vari(t, eta.vi_, etad.vi_, alpha.val_.vi_, alpha.d_.vi_,
                                                 alpha.val_.val(), alpha.d_.val(), y.data()));
  return lp;
}
template <bool propto = false>
inline fvar<var> bernoulli_logit_glm_lpmf(const dev_data<int>& y, const dev_data<double>& x, const fvar<var>& alpha,
                                          const std::vector<fvar<var>>& beta) {
  return bernoulli_logit_glm_lpmf<propto>(y, x, alpha, to_dev(beta));
}

namespace internal {
// L' = L Phi(L^{-1} A' L^{-T}) as one node with a written-out reverse
// (smg_chol_tangent_fwd / _rev, csrc/chol_tangent.hip): W = L^{-1}, Y and
// Phi(Y) are kept for the reverse.  SMG_CHOL_TANGENT_COMPOSED=1 composes it
// from the device functors instead (two triangular solves with N right-hand
// sides, their reverses, L Phi).
class chol_tangent_dev_vari : public device_vari {
 public:
  dev_matrix_vari* L_;
  dev_matrix_vari* Ad_;
  dev_matrix_vari* Ld_;
  double* W_;
  double* Wt_;
  double* Y_;
  double* P_;
  chol_tangent_dev_vari(dev_matrix_vari* L, dev_matrix_vari* Ad)
      : device_vari(0.0), L_(L), Ad_(Ad), Ld_(new dev_matrix_vari(L->rows_, L->cols_, dev_structure::lower)) {
    const int n = L->rows_;
    const size_t nn = size_t(n) * n;
    Wt_ = amd::alloc_doubles(nn);
    Y_ = amd::alloc_doubles(nn);
    P_ = amd::alloc_doubles(nn);
    // W = L^{-1} from the factorisation when it formed it beside its panels
    // (cholesky_decompose_with_inverse), else here after it
    const double* Wf = L_->sink_ ? L_->sink_->inverse_factor() : nullptr;
    if (Wf) {
      W_ = const_cast<double*>(Wf);  // (read only)
      amd::check(smg_chol_tangent_fwd_w(amd::ctx(), L_->val_, n, W_, Ad_->val_, n, n, Wt_, Y_, P_, Ld_->val_, n),
                 "cholesky_decompose");
      return;
    }
    W_ = amd::alloc_doubles(nn);
    amd::check(smg_chol_tangent_fwd(amd::ctx(), L_->val_, n, L_->aux_, Ad_->val_, n, n, W_, Wt_, Y_, P_, Ld_->val_, n),
               "cholesky_decompose");
  }
  void chain() override {
    const int n = L_->rows_;
    double* ws = amd::alloc_doubles(2 * size_t(n) * n);
    amd::check(smg_chol_tangent_rev(amd::ctx(), L_->val_, n, W_, Wt_, Y_, P_, n, Ld_->adj_, n, n, L_->adj_, n,
                                    Ad_->adj_, n, ws),
               "cholesky_decompose");
  }
};
inline bool chol_tangent_composed() {
  static const bool c = [] {
    const char* e = std::getenv("SMG_CHOL_TANGENT_COMPOSED");
    return e && std::atoi(e) != 0;
  }();
  return c;
}
}  // namespace internal

inline dev_fvar_matrix cholesky_decompose(const dev_fvar_matrix& A) {
  dev_fvar_matrix L;
  if (!internal::chol_tangent_composed()) {
    L.val_ = internal::cholesky_decompose_with_inverse(A.val_);  // checks + L (structurally lower), W = L^{-1}
    L.d_ = dev_var_matrix((new internal::chol_tangent_dev_vari(L.val_.vi_, A.d_.vi_))->Ld_);
    return L;
  }
  L.val_ = cholesky_decompose(A.val_);
  dev_var_matrix X = mdivide_left_tri<1>(L.val_, A.d_);   // L^{-1} A'
  dev_var_matrix Y = mdivide_left_tri<1>(L.val_, transpose(X));  // L^{-1} A' L^{-T}
  // L' = L Phi(Y): lower times lower
  dev_var_matrix P = phi_lower(Y);
  L.d_ = dev_var_matrix((new internal::multiply_lower_dev_vari(L.val_.vi_, P.vi_))->C_);
  return L;
}

namespace internal {
// lp' given w = L^{-1}(y - mu) as a device var vector
inline var mvn_cholesky_tangent(const dev_fvar_matrix& L, const dev_data<double>& r) {
  dev_var_matrix w = mdivide_left_tri<1>(L.val_, r);
  dev_var_matrix z = mdivide_left_tri<1>(L.val_, multiply(L.d_, w));
  return dot_product(w, z) - diag_ratio_sum(L.d_, L.val_);
}
template <bool propto>
inline fvar<var> mvn_cholesky_fvar(const std::vector<double>& y, const std::vector<double>& mu,
                                   const dev_fvar_matrix& L) {
  fvar<var> lp;
  lp.val_ = multi_normal_cholesky_lpdf<propto>(y, mu, L.val_);
  if (y.empty()) return lp;
  std::vector<double> r(y.size());
  for (size_t i = 0; i < y.size(); ++i) r[i] = y[i] - mu[i];
  lp.d_ = mvn_cholesky_tangent(L, to_dev_data(r));
  return lp;
}
}  // namespace internal

/** Zero mean, y device-resident. */
template <bool propto = false>
inline fvar<var> multi_normal_cholesky_lpdf(const dev_data<double>& y, const dev_fvar_matrix& L) {
  internal::mvn_check_sizes(int(y.size()), int(y.size()), L.val_);
  fvar<var> lp;
  lp.val_ = multi_normal_cholesky_lpdf<propto>(y, L.val_);
  if (y.size() == 0) return lp;
  lp.d_ = internal::mvn_cholesky_tangent(L, dev_data<double>(y.data(), y.size(), int(y.size()), 1));
  return lp;
}

/** y and mu device-resident (the residual y - mu formed on the device). */
template <bool propto = false>
inline fvar<var> multi_normal_cholesky_lpdf(const dev_data<double>& y, const dev_data<double>& mu,
                                            const dev_fvar_matrix& L) {
  internal::mvn_check_sizes(int(y.size()), int(mu.size()), L.val_);
  fvar<var> lp;
  lp.val_ = multi_normal_cholesky_lpdf<propto>(y, mu, L.val_);
  const size_t n = y.size();
  if (n == 0) return lp;
  smg_ctx* c = amd::ctx();
  double* r = amd::alloc_doubles(n);
  amd::check(smg_memcpy_d2d(c, r, y.data(), n * sizeof(double)), "multi_normal_cholesky_lpdf");
  amd::check(smg_axpy(c, (long long)n, -1.0, mu.data(), 1, r, 1), "multi_normal_cholesky_lpdf");
  lp.d_ = internal::mvn_cholesky_tangent(L, dev_data<double>(r, n, int(n), 1));
  return lp;
}

template <bool propto = false>
inline fvar<var> multi_normal_cholesky_lpdf(const std::vector<double>& y,
                                            const std::vector<double>& mu,
                                            const dev_fvar_matrix& L) {
  internal::mvn_check_sizes(int(y.size()), int(mu.size()), L.val_);
  return internal::mvn_cholesky_fvar<propto>(y, mu, L);
}

}  // namespace math
}  // namespace stan
#endif
