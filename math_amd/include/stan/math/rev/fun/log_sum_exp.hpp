#ifndef STAN_MATH_REV_FUN_LOG_SUM_EXP_HPP
#define STAN_MATH_REV_FUN_LOG_SUM_EXP_HPP

// log_sum_exp over a container of vars (rev/mat/fun/log_sum_exp.hpp:20-53,
// rev/arr/fun/log_sum_exp.hpp:14-50): max-shifted value computed by a
// deterministic two-pass device reduction; empty -> -inf; a non-finite max
// short-circuits to the max (prim/scal/fun/log_sum_exp.hpp:47-59).
// Reverse: x_i' += adj exp(x_i - lse).  The pair form log_sum_exp(var, var)
// is a scalar op (stan/math/rev/core/operators.hpp).

#include <stan/math/amd/matrix.hpp>
#include <stan/math/rev/core.hpp>

#include <vector>

namespace stan {
namespace math {

namespace internal {
class log_sum_exp_dev_vari : public device_vari {
 public:
  dev_matrix_vari* x_;
  log_sum_exp_dev_vari(double v, dev_matrix_vari* x) : device_vari(v), x_(x) {}
  void chain() override {
    amd::check(smg_log_sum_exp_rev(amd::ctx(), x_->val_, (long long)x_->size(), val_, adj_,
                                   x_->adj_),
               "log_sum_exp");
  }
};
}  // namespace internal

inline var log_sum_exp(const dev_var_matrix& x) {
  smg_ctx* c = amd::ctx();
  double* out = amd::alloc_doubles(1);
  amd::check(smg_log_sum_exp_fwd(c, x.val_ptr(), (long long)x.size(), out), "log_sum_exp");
  double v = 0;
  amd::to_host(&v, out, 1);
  return var(new internal::log_sum_exp_dev_vari(v, x.vi_));
}

inline var log_sum_exp(const std::vector<var>& x) { return log_sum_exp(to_dev(x)); }

}  // namespace math
}  // namespace stan
#endif
