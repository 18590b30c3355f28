#ifndef STAN_MATH_REV_FUN_POISSON_LOG_GLM_LPMF_HPP
#define STAN_MATH_REV_FUN_POISSON_LOG_GLM_LPMF_HPP

// poisson_log_glm_lpmf<propto>(y | x, alpha, beta), scalar intercept
// (prim/mat/prob/poisson_log_glm_lpmf.hpp:37-123), with y and x resident on
// the device: ONE fused pass over x (smg_poisson_log_glm) yields
// [sum(y theta - exp theta), sum theta', x^T theta', sum lgamma(y + 1)],
// theta = x beta + alpha, theta' = y - exp(theta).  Semantics kept:
//   * consistent sizes of y and beta (:55-56), check_nonnegative(y) (:61);
//   * size_zero(y) -> 0 (:63-65); every operand data with propto -> 0 (:67-69);
//   * a non-finite sum of theta' runs check_finite on beta, alpha, then the
//     linear predictor under the name of x (:87-91);
//   * logp (:92-100): -sum lgamma(y + 1) unless propto, and
//     + sum(y theta - exp theta) only when include_summand<propto,
//     T_partials_return> -- T_partials_return is double, so with propto the
//     reference returns 0 while its partials are kept; so does this layer;
//   * partials (:102-116): alpha' = sum theta', beta' = x^T theta'.
// Row shards all-reduce the M + 3 sums over RCCL like bernoulli_logit_glm_lpmf.

#include <stan/math/rev/fun/bernoulli_logit_glm_lpmf.hpp>

#include <climits>
#include <algorithm>
#include <cmath>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

namespace stan {
namespace math {
namespace internal {

// index (global: row0 = the shard's first row) and value of the first
// negative y (host copy: error path only); a rank whose own rows are all
// non-negative (the flag came from another rank) names no element
inline void glm_throw_negative_y(const char* fn, const int* y, long long n, long long row0 = 0) {
  smg_ctx* c = amd::ctx();
  const long long chunk = 1 << 20;
  std::vector<int> h(size_t(n > chunk ? chunk : (n > 0 ? n : 0)));
  for (long long i0 = 0; i0 < n; i0 += chunk) {
    const long long k = std::min(chunk, n - i0);
    void* stage = smg_host_scratch(c, size_t(k) * sizeof(int));
    if (!stage) throw std::bad_alloc();
    amd::check(smg_memcpy_d2h(c, stage, y + i0, size_t(k) * sizeof(int)), fn);
    amd::check(smg_sync(c), fn);
    __builtin_memcpy(h.data(), stage, size_t(k) * sizeof(int));
    for (long long i = 0; i < k; ++i)
      if (h[size_t(i)] < 0) {
        std::ostringstream m;
        m << fn << ": Vector of dependent variables[" << row0 + i0 + i + 1 << "] is " << h[size_t(i)]
          << ", but must be >= 0!";
        throw std::domain_error(m.str());
      }
  }
  throw std::domain_error(std::string(fn) +
                          ": Vector of dependent variables is negative (on another rank's rows), but must be >= 0!");
}

template <bool propto>
inline glm_result poisson_glm_eval(const glm_shard& s, const glm_params& p) {
  static const char* fn = "poisson_log_glm_lpmf";
  const int M = s.M;
  if (int(p.beta.size()) != M) {
    std::ostringstream m;
    m << fn << ": Weight vector has dimension = " << p.beta.size() << ", expecting dimension = " << M
      << "; a function was called with arguments of different scalar, array, vector, or matrix "
         "types, and they were not consistently sized;  all arguments must be scalars or "
         "multidimensional values of the same shape.";
    throw std::invalid_argument(m.str());
  }
  smg_ctx* c = amd::ctx();
  // [alpha, beta(M) | out: s, alpha', beta'(M), lgamma sum | flag]
  double* buf = amd::alloc_doubles(size_t(2 * M + 5));
  double* ab = buf;
  double* out = buf + M + 1;
  double* flag = buf + 2 * M + 4;
  std::vector<double> h(size_t(2 * M + 5), 0.0);
  h[0] = p.alpha;
  for (int j = 0; j < M; ++j) h[1 + j] = p.beta[j];
  amd::to_device(buf, h.data(), h.size());
  amd::check(smg_check_bounded_int(c, s.y, s.rows, 0, INT_MAX, flag), fn);  // check_nonnegative (:61)
  const bool run = s.total_rows > 0 && (p.any_var() || !propto);
  if (run) {
    if (s.rows > 0) {
      double* ws = amd::alloc_doubles(size_t(smg_glm_ws_doubles(s.rows, M)));
      amd::check(smg_poisson_log_glm(c, s.y, s.x, s.rows, M, s.ldx, ab, ws, out), fn);
    }
  }
  // [s, alpha', beta'(M), lgamma sum | flag] are contiguous (zeros when not
  // run): the y flag is summed with them, so every rank throws together
  if (s.distributed) amd::allreduce_sum(out, M + 4, fn);
  amd::to_host(h.data(), buf, h.size());
  if (h[2 * M + 4] != 0.0) glm_throw_negative_y(fn, s.y, s.rows, s.row0);
  if (!run) return glm_result{};
  const double sd = h[M + 2];
  if (!std::isfinite(sd)) {  // (:87-91)
    for (int j = 0; j < M; ++j)
      if (!std::isfinite(p.beta[j])) {
        std::ostringstream m;
        m << fn << ": Weight vector[" << j + 1 << "] is " << p.beta[j] << ", but must be finite!";
        throw std::domain_error(m.str());
      }
    if (!std::isfinite(p.alpha)) {
      std::ostringstream m;
      m << fn << ": Intercept is " << p.alpha << ", but must be finite!";
      throw std::domain_error(m.str());
    }
    throw std::domain_error(std::string(fn) +
                            ": Matrix of independent variables is not finite, but must be finite!");
  }
  const double lp = propto ? 0.0 : h[M + 1] - h[2 * M + 3];
  if (!p.any_var()) return glm_result{lp, nullptr};
  double* g = ChainableStack::instance_->memalloc_.alloc_array<double>(size_t(M + 1));
  for (int j = 0; j <= M; ++j) g[j] = h[M + 2 + j];
  return glm_result{lp, new glm_dev_vari(lp, p.alpha_vi, p.beta_vi, p.beta_dev, g, out + 2, M)};
}

}  // namespace internal

/** Device-resident (y, x) row block. */
template <bool propto, typename T_alpha, typename T_beta>
inline typename std::conditional<internal::glm_is_var<T_alpha>::value ||
                                     internal::glm_is_var<T_beta>::value,
                                 var, double>::type
poisson_log_glm_lpmf(const glm_shard& s, const T_alpha& alpha, const T_beta& beta) {
  internal::glm_params p;
  internal::glm_alpha(p, alpha);
  internal::glm_beta(p, beta);
  const internal::glm_result r = internal::poisson_glm_eval<propto>(s, p);
  if constexpr (internal::glm_is_var<T_alpha>::value || internal::glm_is_var<T_beta>::value) {
    if (r.node) return var(r.node);
    return var(r.lp);
  } else {
    return r.lp;
  }
}

template <bool propto, typename T_alpha, typename T_beta>
inline auto poisson_log_glm_lpmf(const dev_data<int>& y, const dev_data<double>& x,
                                 const T_alpha& alpha, const T_beta& beta) {
  static const char* fn = "poisson_log_glm_lpmf";
  if ((long long)y.size() != (long long)x.rows()) {
    std::ostringstream m;
    m << fn << ": Vector of dependent variables has dimension = " << y.size()
      << ", expecting dimension = " << x.rows()
      << "; a function was called with arguments of different scalar, array, vector, or matrix "
         "types, and they were not consistently sized;  all arguments must be scalars or "
         "multidimensional values of the same shape.";
    throw std::invalid_argument(m.str());
  }
  glm_shard s;
  s.y = y.data();
  s.x = x.data();
  s.rows = x.rows();
  s.M = x.cols();
  s.ldx = x.rows();
  s.total_rows = s.rows;
  return poisson_log_glm_lpmf<propto>(s, alpha, beta);
}

template <typename T_alpha, typename T_beta>
inline auto poisson_log_glm_lpmf(const dev_data<int>& y, const dev_data<double>& x,
                                 const T_alpha& alpha, const T_beta& beta) {
  return poisson_log_glm_lpmf<false>(y, x, alpha, beta);
}

/** Host data (uploaded per call, like the reference reading host memory). */
template <bool propto, typename T_alpha, typename T_beta>
inline auto poisson_log_glm_lpmf(const std::vector<int>& y, const std::vector<double>& x_colmajor,
                                 int M, const T_alpha& alpha, const T_beta& beta) {
  const int R = int(y.size());
  if ((long long)x_colmajor.size() != (long long)R * M)
    throw std::invalid_argument("poisson_log_glm_lpmf: x must hold y.size() * M values");
  dev_data<int> yd = to_dev_data(y);
  dev_data<double> xd = to_dev_data(x_colmajor.data(), x_colmajor.size(), R, M);
  return poisson_log_glm_lpmf<propto>(yd, xd, alpha, beta);
}

template <typename T_alpha, typename T_beta>
inline auto poisson_log_glm_lpmf(const std::vector<int>& y, const std::vector<double>& x_colmajor,
                                 int M, const T_alpha& alpha, const T_beta& beta) {
  return poisson_log_glm_lpmf<false>(y, x_colmajor, M, alpha, beta);
}

}  // namespace math
}  // namespace stan
#endif
