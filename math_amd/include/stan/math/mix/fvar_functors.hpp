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

#include <stan/math/amd/matrix.hpp>
#include <stan/math/fwd/core/fvar.hpp>
#include <stan/math/rev/core.hpp>
#include <stan/math/rev/fun/cholesky_decompose.hpp>
#include <stan/math/rev/fun/gp_exp_quad_cov.hpp>
#include <stan/math/rev/fun/mdivide_left_tri.hpp>
#include <stan/math/rev/fun/multi_normal_cholesky_lpdf.hpp>
#include <stan/math/rev/fun/multiply.hpp>
#include <stan/math/rev/fun/tangent_ops.hpp>

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
class multiply_lower_dev_vari : public vari {
 public:
  dev_matrix_vari* A_;
  dev_matrix_vari* B_;
  dev_matrix_vari* C_;
  multiply_lower_dev_vari(dev_matrix_vari* A, dev_matrix_vari* B)
      : vari(0.0), A_(A), B_(B), C_(new dev_matrix_vari(A->rows_, B->cols_, dev_structure::lower)) {
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

inline dev_fvar_matrix cholesky_decompose(const dev_fvar_matrix& A) {
  dev_fvar_matrix L;
  L.val_ = cholesky_decompose(A.val_);                    // checks + L (structurally lower)
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
