#ifndef STAN_MATH_MIX_HESSIAN_TIMES_VECTOR_HPP
#define STAN_MATH_MIX_HESSIAN_TIMES_VECTOR_HPP

// gradient_dot_vector (mix/mat/functor/gradient_dot_vector.hpp:12-25) and
// hessian_times_vector (mix/mat/functor/hessian_times_vector.hpp:13-40) and
// hessian (mix/mat/functor/hessian.hpp:39-72):
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
  no_publish_scope quiet;
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
  no_publish_scope quiet;
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

/**
 * hessian(f, x, fx, grad, H) (mix/mat/functor/hessian.hpp:39-72): one
 * fwd-over-rev sweep per coordinate i -- x_j seeded as fvar<var>(x_j, i == j),
 * grad(i) = the tangent's value, H(i, :) = the adjoints of x after grad() of
 * the tangent; each sweep on its own nested tape (recovered also on throw).
 * With device functors underneath, every sweep is one forward + one reverse
 * of the tangent network on the GPU.
 */
template <typename F>
void hessian(const F& f, const Eigen::Matrix<double, Eigen::Dynamic, 1>& x, double& fx,
             Eigen::Matrix<double, Eigen::Dynamic, 1>& grad_out,
             Eigen::Matrix<double, Eigen::Dynamic, Eigen::Dynamic>& H) {
  const Eigen::Index n = x.size();
  H.resize(n, n);
  grad_out.resize(n);
  if (n == 0) {  // (:45-48): the value at the empty input (evaluated at fvar<var>,
                 // so functors need not instantiate at double)
    start_nested();
    no_publish_scope quiet;
    try {
      fx = f(Eigen::Matrix<fvar<var>, Eigen::Dynamic, 1>(0)).val_.val();
    } catch (const std::exception&) {
      recover_memory_nested();
      throw;
    }
    recover_memory_nested();
    return;
  }
  for (Eigen::Index i = 0; i < n; ++i) {
    start_nested();
    no_publish_scope quiet;
    try {
      Eigen::Matrix<var, Eigen::Dynamic, 1> x_var(n);
      Eigen::Matrix<fvar<var>, Eigen::Dynamic, 1> x_fvar(n);
      for (Eigen::Index j = 0; j < n; ++j) {
        x_var(j) = x(j);
        x_fvar(j) = fvar<var>(x_var(j), var(i == j ? 1.0 : 0.0));
      }
      fvar<var> fx_fvar = f(x_fvar);
      grad_out(i) = fx_fvar.d_.val();
      if (i == 0) fx = fx_fvar.val_.val();
      grad(fx_fvar.d_.vi_);
      for (Eigen::Index j = 0; j < n; ++j) H(i, j) = x_var(j).adj();
    } catch (const std::exception&) {
      recover_memory_nested();
      throw;
    }
    recover_memory_nested();
  }
}
#endif

}  // namespace math
}  // namespace stan
#endif
