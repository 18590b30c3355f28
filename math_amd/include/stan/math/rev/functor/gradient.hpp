#ifndef STAN_MATH_REV_FUNCTOR_GRADIENT_HPP
#define STAN_MATH_REV_FUNCTOR_GRADIENT_HPP

// stan::math::gradient(f, x, fx, grad_fx)
// (stan/math/rev/mat/functor/gradient.hpp:41-57): nested tape, independent
// vars for x, forward f, reverse sweep, read adjoints, recover the nested
// memory (host arena AND device arena) -- also when f throws.
//
// Vec is any vector type with size(), operator[] / operator() and resize()
// (Eigen::VectorXd as in the reference, or std::vector<double>); f receives
// the same container type over var.

#include <stan/math/rev/core.hpp>

#include <type_traits>
#include <vector>

namespace stan {
namespace math {

namespace internal {
template <typename Vec>
struct var_vector_of;
template <>
struct var_vector_of<std::vector<double>> {
  using type = std::vector<var>;
};
}  // namespace internal

template <typename F, typename Vec>
void gradient(const F& f, const Vec& x, double& fx, Vec& grad_fx) {
  using VarVec = typename internal::var_vector_of<Vec>::type;
  start_nested();
  try {
    VarVec x_var(x.size());
    for (size_t i = 0; i < size_t(x.size()); ++i) x_var[i] = x[i];
    var fx_var = f(x_var);
    fx = fx_var.val();
    grad(fx_var.vi_);
    grad_fx.resize(x.size());
    for (size_t i = 0; i < size_t(x.size()); ++i) grad_fx[i] = x_var[i].adj();
  } catch (const std::exception& e) {
    recover_memory_nested();
    throw;
  }
  recover_memory_nested();
}

}  // namespace math
}  // namespace stan
#endif
