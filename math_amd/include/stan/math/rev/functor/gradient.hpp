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

#include <stan/math/amd/matrix.hpp>
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
  no_publish_scope quiet;  // (the tape is recovered before anyone could read a block)
  try {
    // the independent variables are leaves (their chain() is a no-op): they
    // go on the no-chain stack, so the reverse sweep makes no call for them;
    // set_zero_all_adjoints and the nested recovery cover both stacks
    VarVec x_var(x.size());
    for (size_t i = 0; i < size_t(x.size()); ++i) x_var[i] = var(new vari(x[i], false));
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

/**
 * gradient() with a device-resident independent matrix: x (rows x cols,
 * column-major, device) becomes ONE dev_matrix_vari leaf, f receives it as a
 * dev_var_matrix, and the gradient is copied device-to-device into grad_dev
 * (rows * cols doubles).  Same nesting / recovery contract as above; this is
 * the form for functions of N^2 parameters (config 2: A -> sum(chol(A A^T + N I)))
 * where the reference materialises N^2 host varis.
 */
template <typename F>
void gradient(const F& f, const dev_data<double>& x, double& fx, double* grad_dev) {
  start_nested();
  no_publish_scope quiet;  // (the tape is recovered before anyone could read a block)
  try {
    smg_ctx* c = amd::ctx();
    auto* leaf = new dev_matrix_vari(x.rows(), x.cols());
    const size_t n = leaf->size();
    amd::check(smg_memcpy_d2d(c, leaf->val_, x.data(), n * sizeof(double)), "gradient");
    var fx_var = f(dev_var_matrix(leaf));
    fx = fx_var.val();
    grad(fx_var.vi_);
    amd::check(smg_memcpy_d2d(c, grad_dev, leaf->adj_, n * sizeof(double)), "gradient");
  } catch (const std::exception& e) {
    recover_memory_nested();
    throw;
  }
  recover_memory_nested();
}

}  // namespace math
}  // namespace stan
#endif
