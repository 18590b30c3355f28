#ifndef STAN_MATH_REV_FUN_TANGENT_OPS_HPP
#define STAN_MATH_REV_FUN_TANGENT_OPS_HPP

// Device var functors that the fvar<var> (fwd-over-rev) instantiations of the
// hot-path functors are built from (stan/math/mix/fvar_functors.hpp):
//   gp_exp_quad_cov_tangent  K' along (sigma', l'), reverse into all four
//   phi_lower                Phi(X): strict lower, halved diagonal
//   dot_product              <x, y> of two device vectors of vars
//   diag_ratio_sum           sum_i A_ii / B_ii
// Each is one node whose forward / reverse are C-ABI kernels.

#include <stan/math/amd/matrix.hpp>
#include <stan/math/rev/core.hpp>

namespace stan {
namespace math {

namespace internal {

class gp_tangent_dev_vari : public device_vari {
 public:
  const double* x_;
  int n_;
  double s_, l_, ds_, dl_;
  vari* vis_[4];  // sigma, l, sigma', l' (null: data)
  dev_matrix_vari* K_;
  double* out4_;
  gp_tangent_dev_vari(const double* x, int n, const var& s, const var& l, const var& ds,
                      const var& dl)
      : device_vari(0.0), x_(x), n_(n), s_(s.val()), l_(l.val()), ds_(ds.val()), dl_(dl.val()),
        vis_{s.vi_, l.vi_, ds.vi_, dl.vi_}, K_(new dev_matrix_vari(n, n)),
        out4_(amd::alloc_doubles(4)) {
    amd::check(smg_gp_exp_quad_cov_tangent_fwd(amd::ctx(), x_, n_, s_, l_, ds_, dl_, K_->val_, n_),
               "gp_exp_quad_cov");
  }
  void chain() override {
    smg_ctx* c = amd::ctx();
    amd::check(smg_memset(c, out4_, 0, 4 * sizeof(double)), "gp_exp_quad_cov");
    amd::check(smg_gp_exp_quad_cov_tangent_rev(c, x_, n_, s_, l_, ds_, dl_, K_->adj_, n_, out4_),
               "gp_exp_quad_cov");
    for (int i = 0; i < 4; ++i)
      if (vis_[i]) add_pending_adjoint(vis_[i], out4_ + i);
  }
};

class phi_dev_vari : public device_vari {
 public:
  dev_matrix_vari* X_;
  dev_matrix_vari* Y_;
  explicit phi_dev_vari(dev_matrix_vari* X)
      : device_vari(0.0), X_(X), Y_(new dev_matrix_vari(X->rows_, X->cols_, dev_structure::lower)) {
    amd::check(smg_phi(amd::ctx(), X_->rows_, X_->val_, X_->rows_, Y_->val_, Y_->rows_, 0), "phi");
  }
  void chain() override {
    amd::check(smg_phi(amd::ctx(), X_->rows_, Y_->adj_, Y_->rows_, X_->adj_, X_->rows_, 1), "phi");
  }
};

class dot_dev_vari : public device_vari {
 public:
  dev_matrix_vari* x_;
  dev_matrix_vari* y_;
  dot_dev_vari(double v, dev_matrix_vari* x, dev_matrix_vari* y) : device_vari(v), x_(x), y_(y) {}
  void chain() override {
    smg_ctx* c = amd::ctx();
    const long long n = (long long)x_->size();
    amd::check(smg_axpy(c, n, adj_, y_->val_, 1, x_->adj_, 1), "dot_product");
    amd::check(smg_axpy(c, n, adj_, x_->val_, 1, y_->adj_, 1), "dot_product");
  }
};

class diag_ratio_dev_vari : public device_vari {
 public:
  dev_matrix_vari* A_;
  dev_matrix_vari* B_;
  diag_ratio_dev_vari(double v, dev_matrix_vari* A, dev_matrix_vari* B) : device_vari(v), A_(A), B_(B) {}
  void chain() override {
    amd::check(smg_diag_ratio_rev(amd::ctx(), A_->rows_, A_->val_, A_->rows_, B_->val_, B_->rows_,
                                  adj_, A_->adj_, A_->rows_, B_->adj_, B_->rows_),
               "diag_ratio_sum");
  }
};

}  // namespace internal

inline dev_var_matrix gp_exp_quad_cov_tangent(const dev_data<double>& x, const var& sigma,
                                              const var& l, const var& dsigma, const var& dl) {
  auto* node = new internal::gp_tangent_dev_vari(x.data(), int(x.size()), sigma, l, dsigma, dl);
  return dev_var_matrix(node->K_);
}

inline dev_var_matrix phi_lower(const dev_var_matrix& X) {
  auto* node = new internal::phi_dev_vari(X.vi_);
  return dev_var_matrix(node->Y_);
}

inline var dot_product(const dev_var_matrix& x, const dev_var_matrix& y) {
  if (x.size() != y.size()) throw std::invalid_argument("dot_product: size mismatch");
  smg_ctx* c = amd::ctx();
  double* out = amd::alloc_doubles(1);
  amd::check(smg_memset(c, out, 0, sizeof(double)), "dot_product");
  amd::check(smg_dot(c, x.val_ptr(), y.val_ptr(), (long long)x.size(), out), "dot_product");
  double v = 0;
  amd::to_host(&v, out, 1);
  return var(new internal::dot_dev_vari(v, x.vi_, y.vi_));
}

inline var diag_ratio_sum(const dev_var_matrix& A, const dev_var_matrix& B) {
  smg_ctx* c = amd::ctx();
  double* out = amd::alloc_doubles(1);
  amd::check(smg_memset(c, out, 0, sizeof(double)), "diag_ratio_sum");
  amd::check(smg_diag_ratio_fwd(c, A.rows(), A.val_ptr(), A.rows(), B.val_ptr(), B.rows(), out),
             "diag_ratio_sum");
  double v = 0;
  amd::to_host(&v, out, 1);
  return var(new internal::diag_ratio_dev_vari(v, A.vi_, B.vi_));
}

}  // namespace math
}  // namespace stan
#endif
