#ifndef STAN_MATH_REV_FUN_NORMAL_ID_GLM_LPDF_HPP
#define STAN_MATH_REV_FUN_NORMAL_ID_GLM_LPDF_HPP

// normal_id_glm_lpdf<propto>(y | x, alpha, beta, sigma), scalar intercept and
// scale (prim/mat/prob/normal_id_glm_lpdf.hpp:40-150), with y and x resident
// on the device: ONE fused pass over x (smg_normal_id_glm) yields
// [sum y_scaled^2, sum mu', x^T mu'], y_scaled = (y - x beta - alpha)/sigma,
// mu' = y_scaled / sigma.  Semantics kept:
//   * check_positive_finite(sigma) first (:58), then the consistent sizes of
//     y and beta (:59-60);
//   * size_zero(y, sigma) -> 0 (:68-70); include_summand<propto, ...> -> 0
//     when every operand is data (:72-74);
//   * partials (:90-128): alpha' = sum mu', beta' = x^T mu',
//     sigma' = (sum y_scaled^2 - N) / sigma;
//   * a non-finite sum of squares runs check_finite on y, beta, alpha, then
//     on the sum itself under the name of x (:130-136);
//   * logp (:139-150): -N log sqrt(2 pi) unless propto; -N log sigma when
//     !propto or sigma is a var; -sum y_scaled^2 / 2.
// Row shards (glm_shard with yd set) all-reduce the M + 2 sums over RCCL like
// bernoulli_logit_glm_lpmf; N is then the global row count.

#include <stan/math/rev/fun/bernoulli_logit_glm_lpmf.hpp>

#include <algorithm>
#include <cmath>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

namespace stan {
namespace math {
namespace internal {

/** One node over (alpha, beta, sigma): partials g = [alpha', beta'(M), sigma']
 * on the host (arena), beta' also on the device for device-resident beta. */
class glm_sigma_dev_vari : public local_adjoint_vari {
 public:
  vari* alpha_vi_;
  vari** beta_vi_;
  dev_matrix_vari* beta_dev_;
  vari* sigma_vi_;
  double* g_;
  const double* g_dev_;
  int M_;
  glm_sigma_dev_vari(double lp, vari* a, vari** b, dev_matrix_vari* bd, vari* s, double* g,
                     const double* gd, int M)
      : local_adjoint_vari(lp), alpha_vi_(a), beta_vi_(b), beta_dev_(bd), sigma_vi_(s), g_(g), g_dev_(gd), M_(M) {}
  bool touches_adjoints_in(const vari* lo, const vari* hi) const override {
    auto in = [&](const vari* v) { return v && v >= lo && v < hi; };
    if (in(alpha_vi_) || in(sigma_vi_)) return true;
    if (beta_vi_)
      for (int j = 0; j < M_; ++j)
        if (in(beta_vi_[j])) return true;
    return false;
  }
  void chain() override {
    if (alpha_vi_) alpha_vi_->adj_ += adj_ * g_[0];
    if (beta_vi_)
      for (int j = 0; j < M_; ++j) beta_vi_[j]->adj_ += adj_ * g_[1 + j];
    if (beta_dev_)
      amd::check(smg_axpy(amd::ctx(), M_, adj_, g_dev_, 1, beta_dev_->adj_, 1), "normal_id_glm_lpdf");
    if (sigma_vi_) sigma_vi_->adj_ += adj_ * g_[M_ + 1];
  }
};

// first non-finite y (host copy: error path only) -> check_finite's message
inline void glm_throw_nonfinite_y(const char* fn, const double* y, long long n, long long row0 = 0) {
  std::vector<double> h(size_t(n > 0 ? n : 0));
  for (long long i0 = 0; i0 < n; i0 += 1 << 20) {
    const long long c = std::min<long long>(1 << 20, n - i0);
    amd::to_host(h.data() + i0, y + i0, size_t(c));
  }
  for (long long i = 0; i < n; ++i)
    if (!std::isfinite(h[size_t(i)])) {
      std::ostringstream m;
      m << fn << ": Vector of dependent variables[" << row0 + i + 1 << "] is " << h[size_t(i)]
        << ", but must be finite!";
      throw std::domain_error(m.str());
    }
}

// check_positive_finite(function, "Scale vector", sigma) (:58)
inline void normal_glm_check_scale(double sigma) {
  static const char* fn = "normal_id_glm_lpdf";
  if (!(sigma > 0)) {
    std::ostringstream m;
    m << fn << ": Scale vector is " << sigma << ", but must be > 0!";
    throw std::domain_error(m.str());
  }
  if (!std::isfinite(sigma)) {
    std::ostringstream m;
    m << fn << ": Scale vector is " << sigma << ", but must be finite!";
    throw std::domain_error(m.str());
  }
}

template <bool propto>
inline glm_result normal_glm_eval(const glm_shard& s, const glm_params& p, double sigma,
                                  vari* sigma_vi) {
  static const char* fn = "normal_id_glm_lpdf";
  normal_glm_check_scale(sigma);
  const int M = s.M;
  if (int(p.beta.size()) != M) {
    std::ostringstream m;
    m << fn << ": Weight vector has dimension = " << p.beta.size() << ", expecting dimension = " << M
      << "; a function was called with arguments of different scalar, array, vector, or matrix "
         "types, and they were not consistently sized;  all arguments must be scalars or "
         "multidimensional values of the same shape.";
    throw std::invalid_argument(m.str());
  }
  const bool any_var = p.any_var() || sigma_vi;
  if (s.total_rows == 0 || (propto && !any_var)) return glm_result{};
  smg_ctx* c = amd::ctx();
  // [alpha, beta(M), sigma | out: sq, alpha', beta'(M)]
  double* buf = amd::alloc_doubles(size_t(2 * M + 4));
  double* abs = buf;
  double* out = buf + M + 2;
  std::vector<double> h(size_t(2 * M + 4), 0.0);
  h[0] = p.alpha;
  for (int j = 0; j < M; ++j) h[1 + j] = p.beta[j];
  h[M + 1] = sigma;
  amd::to_device(buf, h.data(), h.size());
  if (s.rows > 0) {
    double* ws = amd::alloc_doubles(size_t(smg_glm_ws_doubles(s.rows, M)));
    amd::check(smg_normal_id_glm(c, s.yd, s.x, s.rows, M, s.ldx, abs, ws, out), fn);
  } else {
    amd::zero(out, size_t(M + 2));
  }
  if (s.distributed) amd::allreduce_sum(out, M + 2, fn);
  amd::to_host(h.data(), buf, h.size());
  const double sq = h[M + 2];
  if (!std::isfinite(sq)) {  // (:130-136)
    glm_throw_nonfinite_y(fn, s.yd, s.rows, s.row0);
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
    std::ostringstream m;
    m << fn << ": Matrix of independent variables is " << sq << ", but must be finite!";
    throw std::domain_error(m.str());
  }
  const double N = double(s.total_rows);
  double lp = 0.0;
  if (!propto) lp += -0.91893853320467274178 * N;           // NEG_LOG_SQRT_TWO_PI * N
  if (!propto || sigma_vi) lp -= N * std::log(sigma);
  lp -= 0.5 * sq;
  if (!any_var) return glm_result{lp, nullptr};
  double* g = ChainableStack::instance_->memalloc_.alloc_array<double>(size_t(M + 2));
  for (int j = 0; j <= M; ++j) g[j] = h[M + 3 + j];
  g[M + 1] = (sq - N) / sigma;
  return glm_result{lp, new glm_sigma_dev_vari(lp, p.alpha_vi, p.beta_vi, p.beta_dev, sigma_vi, g,
                                               out + 2, M)};
}

inline double glm_sigma_val(double s) { return s; }
inline double glm_sigma_val(const var& s) { return s.val(); }
inline vari* glm_sigma_vi(double) { return nullptr; }
inline vari* glm_sigma_vi(const var& s) { return s.vi_; }

}  // namespace internal

/** Device-resident (y, x) row block: shard.yd (double y), shard.x. */
template <bool propto, typename T_alpha, typename T_beta, typename T_scale>
inline typename std::conditional<internal::glm_is_var<T_alpha>::value ||
                                     internal::glm_is_var<T_beta>::value ||
                                     std::is_same<T_scale, var>::value,
                                 var, double>::type
normal_id_glm_lpdf(const glm_shard& s, const T_alpha& alpha, const T_beta& beta, const T_scale& sigma) {
  internal::glm_params p;
  internal::glm_alpha(p, alpha);
  internal::glm_beta(p, beta);
  const internal::glm_result r = internal::normal_glm_eval<propto>(
      s, p, internal::glm_sigma_val(sigma), internal::glm_sigma_vi(sigma));
  if constexpr (internal::glm_is_var<T_alpha>::value || internal::glm_is_var<T_beta>::value ||
                std::is_same<T_scale, var>::value) {
    if (r.node) return var(r.node);
    return var(r.lp);
  } else {
    return r.lp;
  }
}

template <bool propto, typename T_alpha, typename T_beta, typename T_scale>
inline auto normal_id_glm_lpdf(const dev_data<double>& y, const dev_data<double>& x,
                               const T_alpha& alpha, const T_beta& beta, const T_scale& sigma) {
  static const char* fn = "normal_id_glm_lpdf";
  internal::normal_glm_check_scale(internal::glm_sigma_val(sigma));  // first (:58)
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
  s.yd = y.data();
  s.x = x.data();
  s.rows = x.rows();
  s.M = x.cols();
  s.ldx = x.rows();
  s.total_rows = s.rows;
  return normal_id_glm_lpdf<propto>(s, alpha, beta, sigma);
}

template <typename T_alpha, typename T_beta, typename T_scale>
inline auto normal_id_glm_lpdf(const dev_data<double>& y, const dev_data<double>& x,
                               const T_alpha& alpha, const T_beta& beta, const T_scale& sigma) {
  return normal_id_glm_lpdf<false>(y, x, alpha, beta, sigma);
}

/** Host data (uploaded per call, like the reference reading host memory). */
template <bool propto, typename T_alpha, typename T_beta, typename T_scale>
inline auto normal_id_glm_lpdf(const std::vector<double>& y, const std::vector<double>& x_colmajor,
                               int M, const T_alpha& alpha, const T_beta& beta, const T_scale& sigma) {
  const int R = int(y.size());
  if ((long long)x_colmajor.size() != (long long)R * M)
    throw std::invalid_argument("normal_id_glm_lpdf: x must hold y.size() * M values");
  dev_data<double> yd = to_dev_data(y);
  dev_data<double> xd = to_dev_data(x_colmajor.data(), x_colmajor.size(), R, M);
  return normal_id_glm_lpdf<propto>(yd, xd, alpha, beta, sigma);
}

template <typename T_alpha, typename T_beta, typename T_scale>
inline auto normal_id_glm_lpdf(const std::vector<double>& y, const std::vector<double>& x_colmajor,
                               int M, const T_alpha& alpha, const T_beta& beta, const T_scale& sigma) {
  return normal_id_glm_lpdf<false>(y, x_colmajor, M, alpha, beta, sigma);
}

}  // namespace math
}  // namespace stan
#endif
