#ifndef STAN_MATH_REV_FUN_CATEGORICAL_LOGIT_GLM_LPMF_HPP
#define STAN_MATH_REV_FUN_CATEGORICAL_LOGIT_GLM_LPMF_HPP

// categorical_logit_glm_lpmf<propto>(y | x, alpha, beta)
// (prim/mat/prob/categorical_logit_glm_lpmf.hpp:38-183), y in 1..C, x an
// R x M design matrix, alpha C intercepts, beta M x C weights, all on the
// device: ONE fused pass over x (smg_categorical_logit_glm) yields
// [logp, alpha'(C), beta'(M x C)], with lin = x beta + alpha and
//   logp = sum_i lin(i, y_i) - max_c lin(i, c) - log sum_c exp(lin(i, c) - max)
//   alpha' = sum_i (onehot(y_i) - softmax(lin_i)),  beta' = x^T (onehot - softmax).
// The partials stay on the device; the node's chain() is two axpys into the
// adjoints of alpha and beta.  Semantics kept, in the reference's order:
//   * consistent sizes: y vs x.rows() ("Vector of dependent variables",
//     :57-60), alpha vs beta.cols() ("Intercept vector", :61);
//     check_size_match("x.cols()", M, "beta.rows()") (:62-63);
//   * check_bounded(y, 1, C) as "categorical outcome out of support" (:64-65);
//   * size_zero(y) or C == 1 -> 0 (:67-69); propto with every operand data
//     -> 0 (:71-74) -- with a var operand every term is kept;
//   * a non-finite logp runs check_finite on beta ("Weight vector"), alpha
//     ("Intercept"), then x ("Matrix of independent variables") (:105-109).
// x is data (the device design matrix); the reference's var-x edge and its
// broadcast row-vector x (T_x_rows == 1) are not on this path.  A scalar y is
// broadcast like the reference's int overload (host overload below).
// Row shards (glm_shard) all-reduce the 1 + C + M C sums over RCCL like the
// other GLM reducers.

#include <stan/math/rev/fun/bernoulli_logit_glm_lpmf.hpp>
#include <stan/math/rev/fun/multiply.hpp>

#include <algorithm>
#include <cmath>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

namespace stan {
namespace math {
namespace internal {

inline void glm_size_mismatch(const char* fn, const char* name, long long got, long long want) {
  std::ostringstream m;
  m << fn << ": " << name << " has dimension = " << got << ", expecting dimension = " << want
    << "; a function was called with arguments of different scalar, array, vector, or matrix "
       "types, and they were not consistently sized;  all arguments must be scalars or "
       "multidimensional values of the same shape.";
  throw std::invalid_argument(m.str());
}

// check_finite on a device matrix (column-major, ld): the first non-finite
// entry by linear index (error path only: host copy column by column)
inline void glm_check_finite_dev(const char* fn, const char* name, const double* d, long long rows,
                                 long long cols, long long ld) {
  std::vector<double> h(size_t(rows > 0 ? rows : 0));
  for (long long j = 0; j < cols; ++j) {
    if (rows > 0) amd::to_host(h.data(), d + j * ld, size_t(rows));
    for (long long i = 0; i < rows; ++i)
      if (!std::isfinite(h[size_t(i)])) {
        std::ostringstream m;
        m << fn << ": " << name << "[" << j * rows + i + 1 << "] is " << h[size_t(i)] << ", but must be finite!";
        throw std::domain_error(m.str());
      }
  }
}

// check_bounded's message for the first y outside [lo, hi]; row0: the shard's
// first global row (indices are global).  A rank whose own rows are all in
// support (the flag came from another rank's shard) throws a message naming
// no element.
inline void glm_throw_out_of_support(const char* fn, const int* y, long long n, int lo, int hi,
                                     long long row0 = 0) {
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
      if (h[size_t(i)] < lo || h[size_t(i)] > hi) {
        std::ostringstream m;
        m << fn << ": categorical outcome out of support[" << row0 + i0 + i + 1 << "] is " << h[size_t(i)]
          << ", but must be in the interval [" << lo << ", " << hi << "]";
        throw std::domain_error(m.str());
      }
  }
  std::ostringstream m;
  m << fn << ": categorical outcome out of support (on another rank's rows), but must be in the interval ["
    << lo << ", " << hi << "]";
  throw std::domain_error(m.str());
}

/** One node over device alpha (C) and beta (M x C); out = [lp, alpha', beta']
 * on the device. */
class glm_cat_dev_vari : public device_vari {
 public:
  dev_operand alpha_, beta_;
  const double* g_dev_;
  int C_, M_;
  glm_cat_dev_vari(double lp, const dev_operand& a, const dev_operand& b, const double* g, int C, int M)
      : device_vari(lp), alpha_(a), beta_(b), g_dev_(g), C_(C), M_(M) {}
  void chain() override {
    smg_ctx* c = amd::ctx();
    if (alpha_.adj()) amd::check(smg_axpy(c, C_, adj_, g_dev_ + 1, 1, alpha_.adj(), 1), "categorical_logit_glm_lpmf");
    if (beta_.adj() && M_ > 0)
      amd::check(smg_axpy(c, (long long)M_ * C_, adj_, g_dev_ + 1 + C_, 1, beta_.adj(), 1),
                 "categorical_logit_glm_lpmf");
  }
};

template <bool propto>
inline glm_result categorical_glm_eval(const glm_shard& s, const dev_operand& alpha, const dev_operand& beta) {
  static const char* fn = "categorical_logit_glm_lpmf";
  const int C = beta.cols;
  const int M = s.M;
  if ((long long)alpha.rows * alpha.cols != C) glm_size_mismatch(fn, "Intercept vector", (long long)alpha.rows * alpha.cols, C);
  if (M != beta.rows) {
    std::ostringstream m;
    m << fn << ": x.cols() (" << M << ") and beta.rows() (" << beta.rows << ") must match in size";
    throw std::invalid_argument(m.str());
  }
  smg_ctx* c = amd::ctx();
  const long long W = 1 + C + (long long)M * C;
  // [alpha(C), beta(M x C) | out (W) | flag]
  double* buf = amd::alloc_doubles(size_t(C + (long long)M * C + W + 1));
  double* ab = buf;
  double* out = buf + C + (long long)M * C;
  double* flag = out + W;
  amd::zero(flag, 1);
  amd::check(smg_check_bounded_int(c, s.y, s.rows, 1, C, flag), fn);  // (:64-65)
  const bool any_var = alpha.vi || beta.vi;
  const bool run = s.total_rows > 0 && C > 1 && (any_var || !propto);
  if (run) {
    if (C > 0) amd::check(smg_memcpy_d2d(c, ab, alpha.val(), sizeof(double) * C), fn);
    if ((long long)M * C > 0) amd::check(smg_memcpy_d2d(c, ab + C, beta.val(), sizeof(double) * M * C), fn);
    if (s.rows > 0) {
      double* ws = amd::alloc_doubles(size_t(smg_glm_categorical_ws_doubles(s.rows, M, C)));
      amd::check(smg_categorical_logit_glm(c, s.y, s.x, s.rows, M, s.ldx, C, ab, ws, out), fn);
    } else {
      amd::zero(out, size_t(W));
    }
  }
  // out (W) and the y flag are contiguous: summed together, so every rank
  // throws together (only the flag when the pass did not run)
  if (s.distributed) amd::allreduce_sum(run ? out : flag, run ? W + 1 : 1, fn);
  double h[2] = {0.0, 0.0};  // [lp, flag]
  amd::to_host(&h[1], flag, 1);
  if (h[1] != 0.0) glm_throw_out_of_support(fn, s.y, s.rows, 1, C, s.row0);
  if (!run) return glm_result{};
  amd::to_host(&h[0], out, 1);
  const double lp = h[0];
  if (!std::isfinite(lp)) {  // (:105-109)
    glm_check_finite_dev(fn, "Weight vector", beta.val(), beta.rows, beta.cols, beta.rows);
    glm_check_finite_dev(fn, "Intercept", alpha.val(), (long long)alpha.rows * alpha.cols, 1, C);
    glm_check_finite_dev(fn, "Matrix of independent variables", s.x, s.rows, M, s.ldx);
  }
  if (!any_var) return glm_result{lp, nullptr};
  return glm_result{lp, new glm_cat_dev_vari(lp, alpha, beta, out, C, M)};
}

template <typename T>
struct glm_cat_is_var : std::is_same<T, dev_var_matrix> {};

}  // namespace internal

/** Device-resident (y, x) row block; alpha (C) and beta (M x C) device
 * operands (dev_var_matrix or dev_data<double>). */
template <bool propto, typename T_alpha, typename T_beta>
inline typename std::conditional<internal::glm_cat_is_var<T_alpha>::value ||
                                     internal::glm_cat_is_var<T_beta>::value,
                                 var, double>::type
categorical_logit_glm_lpmf(const glm_shard& s, const T_alpha& alpha, const T_beta& beta) {
  const internal::glm_result r =
      internal::categorical_glm_eval<propto>(s, internal::operand(alpha), internal::operand(beta));
  if constexpr (internal::glm_cat_is_var<T_alpha>::value || internal::glm_cat_is_var<T_beta>::value) {
    if (r.node) return var(r.node);
    return var(r.lp);
  } else {
    return r.lp;
  }
}

template <bool propto, typename T_alpha, typename T_beta>
inline auto categorical_logit_glm_lpmf(const dev_data<int>& y, const dev_data<double>& x, const T_alpha& alpha,
                                       const T_beta& beta) {
  static const char* fn = "categorical_logit_glm_lpmf";
  if ((long long)y.size() != (long long)x.rows())  // (:57-60)
    internal::glm_size_mismatch(fn, "Vector of dependent variables", (long long)y.size(), x.rows());
  glm_shard s;
  s.y = y.data();
  s.x = x.data();
  s.rows = x.rows();
  s.M = x.cols();
  s.ldx = x.rows() > 0 ? x.rows() : 1;
  s.total_rows = s.rows;
  return categorical_logit_glm_lpmf<propto>(s, alpha, beta);
}

template <typename T_alpha, typename T_beta>
inline auto categorical_logit_glm_lpmf(const dev_data<int>& y, const dev_data<double>& x, const T_alpha& alpha,
                                       const T_beta& beta) {
  return categorical_logit_glm_lpmf<false>(y, x, alpha, beta);
}

}  // namespace math
}  // namespace stan
#endif
