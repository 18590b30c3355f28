#ifndef STAN_MATH_REV_FUN_LGAMMA_HPP
#define STAN_MATH_REV_FUN_LGAMMA_HPP

// lgamma / digamma of vars.
//   scalar  lgamma(var)   rev/scal/fun/lgamma.hpp:13-32   y = lgamma_r(x), x' += y' digamma(x)
//           digamma(var)  rev/scal/fun/digamma.hpp:13-22  y = digamma(x),  x' += y' trigamma(x)
//   vectorised over a device matrix (apply_scalar_unary,
//   rev/mat/vectorize/apply_scalar_unary.hpp:18-32, prim/mat/fun/lgamma.hpp:17-35):
//   one node, value and adjoint by element-wise kernels (smg_lgamma_* /
//   smg_digamma_*) evaluating the same formulas (math_amd/csrc/elementwise.hip).
// Scalar vars are host tape operations (one scalar, like operators.hpp).

#include <stan/math/amd/matrix.hpp>
#include <stan/math/prim/special.hpp>
#include <stan/math/rev/core.hpp>

#include <vector>

namespace stan {
namespace math {

namespace internal {
class lgamma_vari : public op_v_vari {
 public:
  lgamma_vari(double val, vari* avi) : op_v_vari(val, avi) {}
  void chain() override { avi_->adj_ += adj_ * digamma(avi_->val_); }
};
class digamma_vari : public op_v_vari {
 public:
  digamma_vari(double val, vari* avi) : op_v_vari(val, avi) {}
  void chain() override { avi_->adj_ += adj_ * trigamma(avi_->val_); }
};

template <int OP>  // 0 = lgamma, 1 = digamma
class unary_special_dev_vari : public device_vari {
 public:
  dev_matrix_vari* x_;
  dev_matrix_vari* y_;
  explicit unary_special_dev_vari(dev_matrix_vari* x)
      : device_vari(0.0), x_(x), y_(new dev_matrix_vari(x->rows_, x->cols_)) {
    const long long n = (long long)x_->size();
    amd::check(OP == 0 ? smg_lgamma_fwd(amd::ctx(), x_->val_, n, y_->val_)
                       : smg_digamma_fwd(amd::ctx(), x_->val_, n, y_->val_),
               OP == 0 ? "lgamma" : "digamma");
  }
  void chain() override {
    const long long n = (long long)x_->size();
    amd::check(OP == 0 ? smg_lgamma_rev(amd::ctx(), x_->val_, n, y_->adj_, x_->adj_)
                       : smg_digamma_rev(amd::ctx(), x_->val_, n, y_->adj_, x_->adj_),
               OP == 0 ? "lgamma" : "digamma");
  }
};
}  // namespace internal

inline var lgamma(const var& a) {
  return var(new internal::lgamma_vari(lgamma(a.val()), a.vi_));
}
inline var digamma(const var& a) {
  return var(new internal::digamma_vari(digamma(a.val()), a.vi_));
}

inline dev_var_matrix lgamma(const dev_var_matrix& x) {
  auto* node = new internal::unary_special_dev_vari<0>(x.vi_);
  return dev_var_matrix(node->y_);
}
inline dev_var_matrix digamma(const dev_var_matrix& x) {
  auto* node = new internal::unary_special_dev_vari<1>(x.vi_);
  return dev_var_matrix(node->y_);
}
inline std::vector<var> lgamma(const std::vector<var>& x) { return to_var_vector(lgamma(to_dev(x))); }
inline std::vector<var> digamma(const std::vector<var>& x) {
  return to_var_vector(digamma(to_dev(x)));
}

}  // namespace math
}  // namespace stan
#endif
