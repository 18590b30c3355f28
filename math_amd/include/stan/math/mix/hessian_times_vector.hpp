#ifndef STAN_MATH_MIX_HESSIAN_TIMES_VECTOR_HPP
#define STAN_MATH_MIX_HESSIAN_TIMES_VECTOR_HPP

// gradient_dot_vector (mix/mat/functor/gradient_dot_vector.hpp:12-25) and
// hessian_times_vector (mix/mat/functor/hessian_times_vector.hpp:13-40):
// fwd-over-rev.  x becomes vars, each seeded as fvar<var>(x_i, v_i); f runs at
// fvar<var>; grad() of the tangent (= grad f . v, a var) leaves H v in the
// adjoints of x.  Nested tape, recovered also when f throws.

#include <stan/math/fwd/core/fvar.hpp>
#include <stan/math/rev/core.hpp>

#include <vector>

namespace stan {
namespace math {

template <typename F, typename VecV, typename VecF>
void gradient_dot_vector(const F& f, const VecV& x, const std::vector<double>& v, var& fx,
                         var& grad_fx_dot_v) {
  VecF x_fvar(x.size());
  for (size_t i = 0; i < size_t(x.size()); ++i) x_fvar[i] = fvar<var>(x[i], var(v[i]));
  fvar<var> fx_fvar = f(x_fvar);
  fx = fx_fvar.val_;
  grad_fx_dot_v = fx_fvar.d_;
}

template <typename F>
void hessian_times_vector(const F& f, const std::vector<double>& x, const std::vector<double>& v,
                          double& fx, std::vector<double>& Hv) {
  start_nested();
  try {
    std::vector<var> x_var(x.begin(), x.end());
    std::vector<fvar<var>> x_fvar(x.size());
    for (size_t i = 0; i < x.size(); ++i) x_fvar[i] = fvar<var>(x_var[i], var(v[i]));
    fvar<var> fx_fvar = f(x_fvar);
    fx = fx_fvar.val_.val();
    grad(fx_fvar.d_.vi_);
    Hv.resize(x.size());
    for (size_t i = 0; i < x.size(); ++i) Hv[i] = x_var[i].adj();
  } catch (const std::exception&) {
    recover_memory_nested();
    throw;
  }
  recover_memory_nested();
}

#ifdef STAN_MATH_AMD_HAS_EIGEN
/** hessian_times_vector.hpp:13-40 signature: Eigen x, v, Hv; f takes Matrix<fvar<var>,-1,1>. */
template <typename F>
void hessian_times_vector(const F& f, const Eigen::Matrix<double, Eigen::Dynamic, 1>& x,
                          const Eigen::Matrix<double, Eigen::Dynamic, 1>& v, double& fx,
                          Eigen::Matrix<double, Eigen::Dynamic, 1>& Hv) {
  start_nested();
  try {
    const Eigen::Index n = x.size();
    Eigen::Matrix<var, Eigen::Dynamic, 1> x_var(n);
    Eigen::Matrix<fvar<var>, Eigen::Dynamic, 1> x_fvar(n);
    for (Eigen::Index i = 0; i < n; ++i) {
      x_var(i) = x(i);
      x_fvar(i) = fvar<var>(x_var(i), var(v(i)));
    }
    fvar<var> fx_fvar = f(x_fvar);
    fx = fx_fvar.val_.val();
    grad(fx_fvar.d_.vi_);
    Hv.resize(n);
    for (Eigen::Index i = 0; i < n; ++i) Hv(i) = x_var(i).adj();
  } catch (const std::exception&) {
    recover_memory_nested();
    throw;
  }
  recover_memory_nested();
}
#endif

}  // namespace math
}  // namespace stan
#endif
