#ifndef STAN_MATH_REV_FUN_BERNOULLI_LOGIT_GLM_LPMF_HPP
#define STAN_MATH_REV_FUN_BERNOULLI_LOGIT_GLM_LPMF_HPP

// bernoulli_logit_glm_lpmf<propto>(y | x, alpha, beta), scalar intercept
// (prim/mat/prob/bernoulli_logit_glm_lpmf.hpp:46-144), with x and y resident
// on the device: ONE fused pass over x yields [logp, sum theta', x^T theta',
// y-bounds count] (smg_bernoulli_logit_glm_io: parameters in the kernel
// arguments, results written to pinned host memory by the pass's last
// workgroup).
// Semantics kept: check_consistent_size of y / beta (:63-64), check_bounded(y,
// 0, 1) (:69), size_zero -> 0 (:71-73), include_summand<propto, x, alpha,
// beta> (:75-77), the non-finite logp checks of beta, alpha, then the linear
// predictor (:106-110), partials beta' = x^T theta', alpha' = sum theta'
// (:113-135) in one precomputed-gradients node.
//
// Row sharding (the reduce_sum / map_rect path): each rank
// holds a contiguous row block of (y, x) on its own GPU (glm_shard); every
// rank computes its local [logp, alpha', beta'] and ONE RCCL all-reduce sums
// the M + 2 doubles and the y-bounds flag across ranks (amd::allreduce_sum);
// every rank then builds the same node (or throws the same error).  Replaces map_rect's MPI/TBB gather
// (prim/mat/functor/map_rect.hpp:120-177, map_rect_combine.hpp:36-92).

#include <stan/math/amd/comm.hpp>
#include <stan/math/amd/matrix.hpp>
#include <stan/math/rev/core.hpp>
#include <stan/math/rev/fun/normal_lpdf.hpp>

#include <cmath>
#include <sstream>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

namespace stan {
namespace math {

/** Device-resident GLM data: a row block [row0, row0 + rows) of y and x.
 * x: rows x M column-major with leading dimension ldx (ldx >= rows). */
struct glm_shard {
  const int* y = nullptr;
  const double* yd = nullptr;  // real-valued y (normal_id_glm_lpdf)
  const double* x = nullptr;
  long long rows = 0;
  int M = 0;
  long long ldx = 0;
  long long row0 = 0;      // first global row (bookkeeping)
  long long total_rows = 0;
  bool distributed = false;  // all-reduce across the communicator
};

/** Contiguous row partition used by every sharded reducer: rank r of W owns
 * rows [r*R/W, (r+1)*R/W) (integer division), so the blocks tile [0, R). */
inline void row_partition(long long R, int world, int rank, long long* begin, long long* end) {
  *begin = R * rank / world;
  *end = R * (rank + 1) / world;
}

namespace internal {

class glm_dev_vari : public local_adjoint_vari {
 public:
  vari* alpha_vi_;
  vari** beta_vi_;           // host varis of beta (null when beta is data / on device)
  dev_matrix_vari* beta_dev_;  // device beta vars
  double* g_;                // [alpha', beta'(M)] on host (arena)
  const double* g_dev_;      // beta' on device
  int M_;
  glm_dev_vari(double lp, vari* a, vari** b, dev_matrix_vari* bd, double* g, const double* gd, int M)
      : local_adjoint_vari(lp), alpha_vi_(a), beta_vi_(b), beta_dev_(bd), g_(g), g_dev_(gd), M_(M) {}
  bool touches_adjoints_in(const vari* lo, const vari* hi) const override {
    auto in = [&](const vari* v) { return v && v >= lo && v < hi; };
    if (in(alpha_vi_)) return true;
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
      amd::check(smg_axpy(amd::ctx(), M_, adj_, g_dev_, 1, beta_dev_->adj_, 1),
                 "bernoulli_logit_glm_lpmf");
  }
};

// check_bounded(fn, "Vector of dependent variables", y, 0, 1)'s message
// (prim/scal/err/check_bounded.hpp:40-50) for the first y outside [lo, hi],
// with the global index (row0 = the shard's first row); error path only.  A
// rank whose own rows are all in bounds (the flag came from another rank's
// shard) names no element.
inline void glm_throw_y_bounds(const char* fn, const int* y, long long n, int lo, int hi, long long row0) {
  smg_ctx* c = amd::ctx();
  const long long chunk = 1 << 20;
  for (long long i0 = 0; i0 < n; i0 += chunk) {
    const long long k = n - i0 < chunk ? n - i0 : chunk;
    int* stage = static_cast<int*>(smg_host_scratch(c, size_t(k) * sizeof(int)));
    if (!stage) throw std::bad_alloc();
    amd::check(smg_memcpy_d2h(c, stage, y + i0, size_t(k) * sizeof(int)), fn);
    amd::check(smg_sync(c), fn);
    for (long long i = 0; i < k; ++i)
      if (stage[i] < lo || stage[i] > hi) {
        std::ostringstream m;
        m << fn << ": Vector of dependent variables[" << row0 + i0 + i + 1 << "] is " << stage[i]
          << ", but must be in the interval [" << lo << ", " << hi << "]";
        throw std::domain_error(m.str());
      }
  }
  std::ostringstream m;
  m << fn << ": Vector of dependent variables is out of bounds (on another rank's rows), but must be in "
          "the interval [" << lo << ", " << hi << "]";
  throw std::domain_error(m.str());
}

struct glm_params {
  double alpha = 0;
  vari* alpha_vi = nullptr;
  std::vector<double> beta;       // host values (for upload and the finite check)
  vari** beta_vi = nullptr;       // host beta varis
  dev_matrix_vari* beta_dev = nullptr;
  bool any_var() const { return alpha_vi || beta_vi || beta_dev; }
};

inline void glm_alpha(glm_params& p, double a) { p.alpha = a; }
inline void glm_alpha(glm_params& p, const var& a) {
  p.alpha = a.val();
  p.alpha_vi = a.vi_;
}
inline void glm_beta(glm_params& p, const std::vector<double>& b) { p.beta = b; }
inline void glm_beta(glm_params& p, const std::vector<var>& b) {
  p.beta.resize(b.size());
  p.beta_vi = ChainableStack::instance_->memalloc_.alloc_array<vari*>(b.size() ? b.size() : 1);
  for (size_t j = 0; j < b.size(); ++j) {
    p.beta[j] = b[j].val();
    p.beta_vi[j] = b[j].vi_;
  }
}
inline void glm_beta(glm_params& p, const dev_var_matrix& b) {
  p.beta = b.val();
  p.beta_dev = b.vi_;
}

struct glm_result {
  double lp = 0.0;
  vari* node = nullptr;  // null: constant result
};

template <bool propto>
inline glm_result glm_eval(const glm_shard& s, const glm_params& p) {
  static const char* fn = "bernoulli_logit_glm_lpmf";
  const int M = s.M;
  if (int(p.beta.size()) != M) {
    std::ostringstream m;
    m << fn << ": Weight vector has dimension = " << p.beta.size()
      << ", expecting dimension = " << M
      << "; a function was called with arguments of different scalar, array, vector, or matrix "
         "types, and they were not consistently sized;  all arguments must be scalars or "
         "multidimensional values of the same shape.";
    throw std::invalid_argument(m.str());
  }
  smg_ctx* c = amd::ctx();
  // (alpha, beta) travel in the launch's kernel arguments; the fused pass also
  // counts y outside {0, 1}, and its last workgroup writes [logp, alpha',
  // beta'(M), bad-y count] to `out` (device) and -- on one GPU with no
  // latched-status launch outstanding -- straight to pinned host memory,
  // publishing a completion word the host spins on (no copy, no stream sync)
  double* out = amd::alloc_doubles(size_t(M + 3));
  double* ws = amd::alloc_doubles(size_t(smg_glm_ws_doubles(s.rows > 0 ? s.rows : 1, M)));
  int armed = 0;
  amd::check(smg_status_armed(c, &armed), fn);
  const double* h;
  if (!s.distributed && !armed) {
    double* o = static_cast<double*>(smg_pinned_result(c, size_t(M + 3) * sizeof(double)));
    if (!o) throw std::bad_alloc();
    amd::check(smg_bernoulli_logit_glm_io(c, s.y, s.x, s.rows, M, s.ldx, p.alpha, p.beta.data(), ws, out, o), fn);
    h = o;
  } else if (!armed) {
    // sharded: the local results, ONE all-reduce of the M + 3 doubles (the
    // y-support count is summed with the rest, so a bad y on any rank makes
    // every rank throw), then the same zero-copy read of the sums
    amd::check(smg_bernoulli_logit_glm_io(c, s.y, s.x, s.rows, M, s.ldx, p.alpha, p.beta.data(), ws, out,
                                          nullptr), fn);
    amd::allreduce_sum(out, M + 3, fn);
    double* o = static_cast<double*>(smg_pinned_result(c, size_t(M + 3) * sizeof(double)));
    if (!o) throw std::bad_alloc();
    amd::check(smg_publish_to_host(c, out, M + 3, o), fn);
    h = o;
  } else {
    amd::check(smg_bernoulli_logit_glm_io(c, s.y, s.x, s.rows, M, s.ldx, p.alpha, p.beta.data(), ws, out,
                                          nullptr), fn);
    if (s.distributed) amd::allreduce_sum(out, M + 3, fn);
    double* o = static_cast<double*>(smg_host_scratch(c, size_t(M + 4) * sizeof(double)));
    if (!o) throw std::bad_alloc();
    amd::check(smg_memcpy_d2h(c, o, out, size_t(M + 3) * sizeof(double)), fn);
    if (armed) amd::check(smg_status_enqueue(c, reinterpret_cast<int*>(o + M + 3)), fn);
    amd::check(smg_sync(c), fn);
    if (armed) amd::throw_if_sync(*reinterpret_cast<int*>(o + M + 3), fn, "a persistent solve");
    h = o;
  }
  if (h[M + 2] != 0.0) glm_throw_y_bounds(fn, s.y, s.rows, 0, 1, s.row0);
  if (s.total_rows == 0 || !(p.any_var() || !propto)) return glm_result{};
  const double lp = h[0];
  if (!std::isfinite(lp)) {
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
  if (!p.any_var()) return glm_result{lp, nullptr};
  double* g = ChainableStack::instance_->memalloc_.alloc_array<double>(size_t(M + 1));
  for (int j = 0; j <= M; ++j) g[j] = h[1 + j];
  return glm_result{lp, new glm_dev_vari(lp, p.alpha_vi, p.beta_vi, p.beta_dev, g, out + 2, M)};
}

template <typename T>
struct glm_is_var
    : std::integral_constant<bool, !std::is_same<T, double>::value &&
                                       !std::is_same<T, std::vector<double>>::value> {};

}  // namespace internal

/** Device-resident (y, x) -- the config-4 layout; one GPU or one shard. */
template <bool propto, typename T_alpha, typename T_beta>
inline typename std::conditional<internal::glm_is_var<T_alpha>::value ||
                                     internal::glm_is_var<T_beta>::value,
                                 var, double>::type
bernoulli_logit_glm_lpmf(const glm_shard& s, const T_alpha& alpha, const T_beta& beta) {
  internal::glm_params p;
  internal::glm_alpha(p, alpha);
  internal::glm_beta(p, beta);
  const internal::glm_result r = internal::glm_eval<propto>(s, p);
  if constexpr (internal::glm_is_var<T_alpha>::value || internal::glm_is_var<T_beta>::value) {
    if (r.node) return var(r.node);
    return var(r.lp);
  } else {
    return r.lp;
  }
}

template <bool propto, typename T_alpha, typename T_beta>
inline auto bernoulli_logit_glm_lpmf(const dev_data<int>& y, const dev_data<double>& x,
                                     const T_alpha& alpha, const T_beta& beta) {
  static const char* fn = "bernoulli_logit_glm_lpmf";
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
  return bernoulli_logit_glm_lpmf<propto>(s, alpha, beta);
}

template <typename T_alpha, typename T_beta>
inline auto bernoulli_logit_glm_lpmf(const dev_data<int>& y, const dev_data<double>& x,
                                     const T_alpha& alpha, const T_beta& beta) {
  return bernoulli_logit_glm_lpmf<false>(y, x, alpha, beta);
}

/** Host data (uploaded per call, like the reference reading host memory). */
template <bool propto, typename T_alpha, typename T_beta>
inline auto bernoulli_logit_glm_lpmf(const std::vector<int>& y, const std::vector<double>& x_colmajor,
                                     int M, const T_alpha& alpha, const T_beta& beta) {
  const int R = int(y.size());
  if ((long long)x_colmajor.size() != (long long)R * M)
    throw std::invalid_argument("bernoulli_logit_glm_lpmf: x must hold y.size() * M values");
  dev_data<int> yd = to_dev_data(y);
  dev_data<double> xd = to_dev_data(x_colmajor.data(), x_colmajor.size(), R, M);
  return bernoulli_logit_glm_lpmf<propto>(yd, xd, alpha, beta);
}

template <typename T_alpha, typename T_beta>
inline auto bernoulli_logit_glm_lpmf(const std::vector<int>& y, const std::vector<double>& x_colmajor,
                                     int M, const T_alpha& alpha, const T_beta& beta) {
  return bernoulli_logit_glm_lpmf<false>(y, x_colmajor, M, alpha, beta);
}

/**
 * Row-sharded reducer (reduce_sum-style entry point): `shard` holds this
 * rank's rows with shard.distributed = true and the communicator joined via
 * amd::comm_init; every rank calls it with the same (alpha, beta) and gets the
 * full-data log density and gradient.
 */
template <bool propto = false, typename T_alpha, typename T_beta>
inline auto reduce_sum_bernoulli_logit_glm(const glm_shard& shard, const T_alpha& alpha,
                                           const T_beta& beta) {
  return bernoulli_logit_glm_lpmf<propto>(shard, alpha, beta);
}

}  // namespace math
}  // namespace stan
#endif
