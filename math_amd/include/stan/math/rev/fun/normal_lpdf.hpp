#ifndef STAN_MATH_REV_FUN_NORMAL_LPDF_HPP
#define STAN_MATH_REV_FUN_NORMAL_LPDF_HPP

// normal_lpdf<propto>(y | mu, sigma) (prim/scal/prob/normal_lpdf.hpp:36-119)
// as one device reduction: value sum_i [-1/2 z_i^2 - log sigma_i - log sqrt(2 pi)]
// and the partials dy = -z/sigma, dmu = z/sigma, dsigma = -1/sigma + z^2/sigma
// (:92-104) written by the same kernel (smg_normal_lpdf).
//
// Operands: double, var, std::vector<double>, std::vector<var>, dev_data<double>
// and dev_var_matrix (a vector of vars kept on the device).  Semantics kept:
//   size_zero -> 0 (:45-47); checks in the reference order (:51-55)
//   check_not_nan(y), check_finite(mu), check_positive(sigma) -- evaluated on
//   the device, one flag per argument, read back with the value -- then
//   check_consistent_sizes; include_summand<propto, ...> drops constant terms
//   (:56-58, :86-91).  One node per call; its chain() scatters adj * partial
//   into device adjoints (axpy) or host varis.

#include <stan/math/amd/matrix.hpp>
#include <stan/math/rev/core.hpp>

#include <sstream>
#include <stdexcept>
#include <type_traits>
#include <vector>

namespace stan {
namespace math {

namespace internal {

/** An argument of a device lpdf reducer. */
struct lpdf_operand {
  const double* val = nullptr;  // device values (null: host scalar, uploaded by the caller)
  double host = 0.0;            // host scalar value
  size_t n = 1;
  bool vec = false;
  vari* svi = nullptr;              // scalar var
  dev_matrix_vari* dvi = nullptr;   // device vector of vars
  bool is_var() const { return svi || dvi; }
};

inline lpdf_operand lpdf_arg(double x) {
  lpdf_operand o;
  o.host = x;
  return o;
}
inline lpdf_operand lpdf_arg(const var& x) {
  lpdf_operand o;
  o.host = x.val();
  o.svi = x.vi_;
  return o;
}
inline lpdf_operand lpdf_arg(const dev_data<double>& x) {
  lpdf_operand o;
  o.val = x.data();
  o.n = x.size();
  o.vec = true;
  return o;
}
inline lpdf_operand lpdf_arg(const dev_var_matrix& x) {
  lpdf_operand o;
  o.val = x.val_ptr();
  o.n = x.size();
  o.vec = true;
  o.dvi = x.vi_;
  return o;
}
inline lpdf_operand lpdf_arg(const std::vector<double>& x) {
  if (x.empty()) {
    lpdf_operand o;
    o.n = 0;
    o.vec = true;
    return o;
  }
  return lpdf_arg(to_dev_data(x));
}
inline lpdf_operand lpdf_arg(const std::vector<var>& x) {
  if (x.empty()) {
    lpdf_operand o;
    o.n = 0;
    o.vec = true;
    return o;
  }
  return lpdf_arg(to_dev(x));
}

#ifdef STAN_MATH_AMD_HAS_EIGEN
template <int R, int C>
inline lpdf_operand lpdf_arg(const Eigen::Matrix<var, R, C>& x) {
  std::vector<var> v(x.data(), x.data() + x.size());
  return lpdf_arg(v);
}
template <int R, int C>
inline lpdf_operand lpdf_arg(const Eigen::Matrix<double, R, C>& x) {
  std::vector<double> v(x.data(), x.data() + x.size());
  return lpdf_arg(v);
}
template <typename T>
struct is_eigen_double : std::false_type {};
template <int R, int C>
struct is_eigen_double<Eigen::Matrix<double, R, C>> : std::true_type {};
#else
template <typename T>
struct is_eigen_double : std::false_type {};
#endif

template <typename T>
struct is_var_arg : std::integral_constant<bool, !std::is_same<T, double>::value &&
                                                     !std::is_same<T, std::vector<double>>::value &&
                                                     !std::is_same<T, dev_data<double>>::value &&
                                                     !is_eigen_double<T>::value> {};

inline void lpdf_check_sizes(const char* fn, const char* const names[], const lpdf_operand* ops,
                             int k) {
  size_t expect = 0;
  int first = -1;
  for (int i = 0; i < k; ++i)
    if (ops[i].vec) {
      if (first < 0) {
        first = i;
        expect = ops[i].n;
      } else if (ops[i].n != expect) {
        std::ostringstream m;
        m << fn << ": " << names[i] << " has dimension = " << ops[i].n
          << ", expecting dimension = " << expect
          << "; a function was called with arguments of different scalar, array, vector, or "
             "matrix types, and they were not consistently sized;  all arguments must be "
             "scalars or multidimensional values of the same shape.";
        throw std::invalid_argument(m.str());
      }
    }
}

class lpdf_dev_vari : public vari {
 public:
  static constexpr int K = 3;
  lpdf_operand ops_[K];
  double* g_[K];  // device partials (vector operands) -- null when constant
  double gs_[K];  // host partials of scalar var operands
  lpdf_dev_vari(double v, const lpdf_operand* ops, double* const* g, const double* gs)
      : vari(v) {
    for (int i = 0; i < K; ++i) {
      ops_[i] = ops[i];
      g_[i] = g[i];
      gs_[i] = gs[i];
    }
  }
  void chain() override {
    for (int i = 0; i < K; ++i) {
      if (ops_[i].dvi)
        amd::check(smg_axpy(amd::ctx(), (long long)ops_[i].n, adj_, g_[i], 1, ops_[i].dvi->adj_, 1),
                   "lpdf");
      else if (ops_[i].svi)
        ops_[i].svi->adj_ += adj_ * gs_[i];
    }
  }
};

}  // namespace internal

template <bool propto, typename T_y, typename T_loc, typename T_scale>
inline typename std::conditional<internal::is_var_arg<T_y>::value ||
                                     internal::is_var_arg<T_loc>::value ||
                                     internal::is_var_arg<T_scale>::value,
                                 var, double>::type
normal_lpdf(const T_y& y, const T_loc& mu, const T_scale& sigma) {
  using internal::lpdf_operand;
  static const char* fn = "normal_lpdf";
  constexpr bool vy = internal::is_var_arg<T_y>::value, vmu = internal::is_var_arg<T_loc>::value,
                 vs = internal::is_var_arg<T_scale>::value;
  lpdf_operand ops[3] = {internal::lpdf_arg(y), internal::lpdf_arg(mu), internal::lpdf_arg(sigma)};
  if ((ops[0].vec && ops[0].n == 0) || (ops[1].vec && ops[1].n == 0) ||
      (ops[2].vec && ops[2].n == 0))
    return 0.0;
  // include_summand<propto, ...>
  const bool inc_const = !propto;
  const bool inc_logsig = !propto || vs;
  const bool inc_quad = !propto || vy || vmu || vs;
  size_t N = 1;
  for (auto& o : ops)
    if (o.vec && o.n > N) N = o.n;

  smg_ctx* c = amd::ctx();
  // res = [lp, flag_y, flag_mu, flag_sigma, g_y, g_mu, g_sigma (scalar partials), host scalars y, mu, sigma]
  double* res = amd::alloc_doubles(10);
  std::vector<double> init(10, 0.0);
  for (int i = 0; i < 3; ++i)
    if (!ops[i].vec) init[7 + i] = ops[i].host;
  amd::to_device(res, init.data(), 10);
  for (int i = 0; i < 3; ++i)
    if (!ops[i].vec) ops[i].val = res + 7 + i;
  amd::check(smg_check_domain(c, ops[0].val, (long long)ops[0].n, 0, res + 1), fn);
  amd::check(smg_check_domain(c, ops[1].val, (long long)ops[1].n, 1, res + 2), fn);
  amd::check(smg_check_domain(c, ops[2].val, (long long)ops[2].n, 2, res + 3), fn);
  double* g[3] = {nullptr, nullptr, nullptr};
  for (int i = 0; i < 3; ++i) {
    if (!ops[i].is_var()) continue;
    if (ops[i].vec) {
      g[i] = amd::alloc_doubles(ops[i].n);
      amd::zero(g[i], ops[i].n);
    } else {
      g[i] = res + 4 + i;
    }
  }
  // sizes are checked after the domain checks (reference order) but before
  // the reduction reads N elements of every vector operand
  bool sizes_ok = true;
  for (auto& o : ops)
    if (o.vec && o.n != N) sizes_ok = false;
  double h[10];
  const int include = (inc_const ? 1 : 0) | (inc_logsig ? 2 : 0) | (inc_quad ? 4 : 0);
  const bool any_var = vy || vmu || vs;
  if (sizes_ok && (any_var || !propto))
    amd::check(smg_normal_lpdf(c, ops[0].val, ops[0].vec ? 1 : 0, ops[1].val, ops[1].vec ? 1 : 0,
                               ops[2].val, ops[2].vec ? 1 : 0, (long long)N, include, res, g[0],
                               g[1], g[2]),
               fn);
  amd::to_host(h, res, 10);
  static const char* const names[3] = {"Random variable", "Location parameter", "Scale parameter"};
  if (h[1] != 0.0) throw std::domain_error(std::string(fn) + ": Random variable is nan, but must not be nan!");
  if (h[2] != 0.0) throw std::domain_error(std::string(fn) + ": Location parameter is not finite, but must be finite!");
  if (h[3] != 0.0) throw std::domain_error(std::string(fn) + ": Scale parameter is not positive, but must be > 0!");
  internal::lpdf_check_sizes(fn, names, ops, 3);
  if constexpr (vy || vmu || vs) {
    return var(new internal::lpdf_dev_vari(h[0], ops, g, h + 4));
  } else {
    return propto ? 0.0 : h[0];
  }
}

template <typename T_y, typename T_loc, typename T_scale>
inline auto normal_lpdf(const T_y& y, const T_loc& mu, const T_scale& sigma) {
  return normal_lpdf<false>(y, mu, sigma);
}

}  // namespace math
}  // namespace stan
#endif
