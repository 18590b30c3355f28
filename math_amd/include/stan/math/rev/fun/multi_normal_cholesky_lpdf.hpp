#ifndef STAN_MATH_REV_FUN_MULTI_NORMAL_CHOLESKY_LPDF_HPP
#define STAN_MATH_REV_FUN_MULTI_NORMAL_CHOLESKY_LPDF_HPP

// multi_normal_cholesky_lpdf<propto>(y | mu, L) with a device Cholesky factor.
// Reference: prim/mat/prob/multi_normal_cholesky_lpdf.hpp:40-160 (single
// vector y).  Value: -n log(sqrt(2 pi)) - |L^{-1}(y-mu)|^2/2 - sum log L_ii;
// partials for L: sd half^T - inv_L^T (:147,155) applied by chain() on the
// device; when L is a cholesky_decompose output (structurally lower) the
// upper-triangle partials land on the reference's dummy vari and are skipped,
// which removes the explicit O(n^3) inverse (see math_amd/csrc/mvn.hip).
// y and mu may be data (double / dev_data) or device vectors of vars: the
// reverse adds -adj sd into y' and +adj sd into mu' (:139-146).
// With L a var, propto = true drops only the constant NEG_LOG_SQRT_TWO_PI
// term (include_summand<propto>, :107-109).

#include <stan/math/amd/matrix.hpp>
#include <stan/math/rev/core.hpp>
#include <stan/math/rev/fun/multiply.hpp>

#include <cmath>
#include <sstream>
#include <stdexcept>
#include <vector>

namespace stan {
namespace math {

namespace internal {

class mvn_cholesky_dev_vari : public device_vari {
 public:
  dev_matrix_vari* L_;
  const double* ws_;  // [w, sd] on device
  int n_;
  dev_matrix_vari* y_;   // null when y is data
  dev_matrix_vari* mu_;  // null when mu is data

  bool deposited_ = false;  // the last chain() handed L's partials to its producer

  mvn_cholesky_dev_vari(double lp, dev_matrix_vari* L, const double* ws,
                        dev_matrix_vari* y = nullptr, dev_matrix_vari* mu = nullptr)
      : device_vari(lp), L_(L), ws_(ws), n_(L->rows_), y_(y), mu_(mu) {}

  bool may_write_device_adjoint(const void* node) const override {
    return (node == L_ && !deposited_) || (y_ && node == y_) || (mu_ && node == mu_);
  }

  void chain() override {
    const int lower_only = L_->structure_ == dev_structure::lower ? 1 : 0;
    // a cholesky_decompose factor takes the lower-only partials unexpanded
    // (rev/fun/cholesky_decompose.hpp: its reverse then has a closed form)
    deposited_ = lower_only && L_->sink_ && L_->sink_->take_mvn_adjoint(this, ws_, adj_);
    amd::check(smg_mvn_cholesky_rev(amd::ctx(), L_->val_, n_, L_->aux_, n_, ws_, adj_, lower_only,
                                    y_ ? y_->adj_ : nullptr, mu_ ? mu_->adj_ : nullptr,
                                    deposited_ ? nullptr : L_->adj_, n_),
               "multi_normal_cholesky_lpdf");
  }
};

inline void mvn_check_sizes(int ny, int nmu, const dev_var_matrix& L) {
  const char* fn = "multi_normal_cholesky_lpdf";
  auto mismatch = [&](const char* a, int x, const char* b, int y) {
    std::ostringstream m;
    m << fn << ": " << a << " (" << x << ") and " << b << " (" << y << ") must match in size";
    throw std::invalid_argument(m.str());
  };
  if (ny != nmu) mismatch("Size of random variable", ny, "size of location parameter", nmu);
  if (ny != L.rows()) mismatch("Size of random variable", ny, "rows of covariance parameter", L.rows());
  if (ny != L.cols()) mismatch("Size of random variable", ny, "columns of covariance parameter", L.cols());
}

inline void mvn_check_data(const std::vector<double>& y, const std::vector<double>* mu) {
  // (prim/mat/prob/multi_normal_cholesky_lpdf.hpp:100-103: check_finite of
  // the location vector, then check_not_nan of the random variable; the
  // whole vectors are checked, so the message carries the 1-based index)
  const char* fn = "multi_normal_cholesky_lpdf";
  if (mu)
    for (size_t i = 0; i < mu->size(); ++i)
      if (!std::isfinite((*mu)[i])) {
        std::ostringstream m;
        m << fn << ": Location parameter[" << i + 1 << "] is " << (*mu)[i] << ", but must be finite!";
        throw std::domain_error(m.str());
      }
  for (size_t i = 0; i < y.size(); ++i)
    if (std::isnan(y[i])) {
      std::ostringstream m;
      m << fn << ": Random variable[" << i + 1 << "] is nan, but must not be nan!";
      throw std::domain_error(m.str());
    }
}

template <bool propto>
inline var mvn_cholesky_dev(const double* y_d, const double* mu_d, int n, const dev_var_matrix& L,
                            dev_matrix_vari* y_vi = nullptr, dev_matrix_vari* mu_vi = nullptr) {
  const char* fn = "multi_normal_cholesky_lpdf";
  if (n == 0) return var(0.0);
  smg_ctx* c = amd::ctx();
  double* ws = amd::alloc_doubles(2 * size_t(n) + 3);
  double* lp_d = ws + 2 * size_t(n);  // [lp, mu not finite, y nan]: read back together
  // check_finite(mu), check_not_nan(y) (prim/mat/prob/multi_normal_cholesky_lpdf.hpp:100-103)
  // on the device values, their flags landing with the value (one sync)
  amd::check(smg_memset(c, lp_d + 1, 0, 2 * sizeof(double)), fn);
  if (mu_d) amd::check(smg_check_domain(c, mu_d, n, 1, lp_d + 1), fn);
  amd::check(smg_check_domain(c, y_d, n, 0, lp_d + 2), fn);
  // with the factor's explicit inverse at hand, the reference's own products
  // (half = inv_L (y - mu), scaled_diff = half inv_L, :117-131)
  const double* W = L.vi_->sink_ ? L.vi_->sink_->inverse_factor() : nullptr;
  if (W)
    amd::check(smg_mvn_cholesky_fwd_inv(c, y_d, mu_d, L.val_ptr(), n, W, n, n, ws, lp_d), fn);
  else
    amd::check(smg_mvn_cholesky_fwd(c, y_d, mu_d, L.val_ptr(), n, L.vi_->aux_, n, ws, lp_d), fn);
  if (L.vi_->sink_) L.vi_->sink_->prepare_mvn_adjoint();  // (behind the solves: overlaps their tail and the host)
  double out[3] = {0, 0, 0};
  amd::to_host(out, lp_d, 3);
  if (out[1] != 0.0 || out[2] != 0.0) {  // error path: the values on the host, the reference's message
    std::vector<double> yh(static_cast<size_t>(n)), mh;
    amd::to_host(yh.data(), y_d, yh.size());
    if (mu_d) {
      mh.resize(size_t(n));
      amd::to_host(mh.data(), mu_d, mh.size());
    }
    mvn_check_data(yh, mu_d ? &mh : nullptr);
  }
  double lp = out[0];
  if (propto) lp -= -std::log(std::sqrt(2.0 * 3.14159265358979323846)) * n;
  return var(new mvn_cholesky_dev_vari(lp, L.vi_, ws, y_vi, mu_vi));
}


/** One observation of the multi-observation form: device pointers of y_i and
 * mu_i (mu null: zero mean) and their adjoints (null: data). */
struct mvn_obs {
  const double* y;
  double* yadj;
  const double* mu;
  double* muadj;
};

// The array forms (prim/mat/prob/multi_normal_cholesky_lpdf.hpp:59-80,
// vector_seq_view): the observations share L; each contributes its own
// quadratic term and the -log|L| term, so the partials of L sum over them
// (:139-155: size_vec * inv_L^T).  L may be a var node or data.
class mvn_multi_dev_vari : public device_vari {
 public:
  dev_operand L_;
  const double* aux_;
  int n_, k_, lower_only_;
  const double* ws_;  // k blocks of 2n doubles: [w_i, sd_i]
  mvn_obs* obs_;
  bool deposited_ = false;  // the last chain() handed L's partials to its producer
  mvn_multi_dev_vari(double lp, const dev_operand& L, const double* aux, int lower_only, const double* ws,
                     mvn_obs* obs, int k)
      : device_vari(lp), L_(L), aux_(aux), n_(L.rows), k_(k), lower_only_(lower_only), ws_(ws), obs_(obs) {}
  bool may_write_device_adjoint(const void* node) const override {
    if (L_.vi && node == L_.vi) return !deposited_;
    for (int i = 0; i < k_; ++i)  // (an observation's y / mu nodes)
      if (node && (obs_[i].yadj || obs_[i].muadj)) return true;
    return false;
  }
  void chain() override {
    smg_ctx* c = amd::ctx();
    // a cholesky_decompose factor: the lower-only partials of all the
    // observations go to the factor's node unexpanded (rev/fun/cholesky_decompose.hpp)
    deposited_ = lower_only_ && L_.vi && L_.vi->sink_ && L_.vi->sink_->take_mvn_adjoint(this, ws_, adj_, k_);
    for (int i = 0; i < k_; ++i)
      amd::check(smg_mvn_cholesky_rev(c, L_.val(), n_, aux_, n_, ws_ + 2 * size_t(n_) * i, adj_, lower_only_,
                                      obs_[i].yadj, obs_[i].muadj, deposited_ ? nullptr : L_.adj(), n_),
                 "multi_normal_cholesky_lpdf");
  }
};

/**
 * Sum over k observations of log N(y_i | mu_i, L L^T) on the device, as one
 * node.  Value terms: include_const (-n log sqrt(2 pi)), include_logdet
 * (-log|L|, from the device lp minus host_logdet when dropped); the
 * quadratic term is always there (the caller returns early when all of y,
 * mu, L are data under propto).  Returns the node (null when nothing is a
 * var) and the value in *lp_out.
 */
inline vari* mvn_cholesky_multi(const dev_operand& L, const double* aux, bool lower_only, mvn_obs* obs, int k,
                                bool include_const, bool include_logdet, double host_logdet, double* lp_out) {
  const char* fn = "multi_normal_cholesky_lpdf";
  const int n = L.rows;
  smg_ctx* c = amd::ctx();
  double* ws = amd::alloc_doubles(2 * size_t(n) * size_t(k) + size_t(k));
  double* lp_d = ws + 2 * size_t(n) * size_t(k);
  const double* W = lower_only && L.vi && L.vi->sink_ ? L.vi->sink_->inverse_factor() : nullptr;
  for (int i = 0; i < k; ++i)
    amd::check(W ? smg_mvn_cholesky_fwd_inv(c, obs[i].y, obs[i].mu, L.val(), n, W, n, n, ws + 2 * size_t(n) * i,
                                            lp_d + i)
                 : smg_mvn_cholesky_fwd(c, obs[i].y, obs[i].mu, L.val(), n, aux, n, ws + 2 * size_t(n) * i, lp_d + i),
               fn);
  if (lower_only && L.vi && L.vi->sink_) L.vi->sink_->prepare_mvn_adjoint();  // (behind the solves)
  std::vector<double> lps(static_cast<size_t>(k));
  amd::to_host(lps.data(), lp_d, lps.size());
  double lp = 0.0;
  for (double v : lps) lp += v;
  if (!include_const) lp -= -std::log(std::sqrt(2.0 * 3.14159265358979323846)) * n * k;
  if (!include_logdet) lp -= host_logdet * k;
  *lp_out = lp;
  bool any_adj = L.adj() != nullptr;
  for (int i = 0; i < k; ++i) any_adj = any_adj || obs[i].yadj || obs[i].muadj;
  if (!any_adj) return nullptr;
  return new mvn_multi_dev_vari(lp, L, aux, lower_only ? 1 : 0, ws, obs, k);
}

}  // namespace internal

template <bool propto = false>
inline var multi_normal_cholesky_lpdf(const std::vector<double>& y, const std::vector<double>& mu,
                                      const dev_var_matrix& L) {
  internal::mvn_check_sizes(int(y.size()), int(mu.size()), L);
  internal::mvn_check_data(y, &mu);
  if (y.empty()) return var(0.0);
  dev_data<double> yd = to_dev_data(y), md = to_dev_data(mu);
  return internal::mvn_cholesky_dev<propto>(yd.data(), md.data(), int(y.size()), L);
}

/** Zero mean (mu == 0), y device-resident. */
template <bool propto = false>
inline var multi_normal_cholesky_lpdf(const dev_data<double>& y, const dev_var_matrix& L) {
  internal::mvn_check_sizes(int(y.size()), int(y.size()), L);
  return internal::mvn_cholesky_dev<propto>(y.data(), nullptr, int(y.size()), L);
}
template <bool propto = false>
inline var multi_normal_cholesky_lpdf(const dev_data<double>& y, const dev_data<double>& mu,
                                      const dev_var_matrix& L) {
  internal::mvn_check_sizes(int(y.size()), int(mu.size()), L);
  return internal::mvn_cholesky_dev<propto>(y.data(), mu.data(), int(y.size()), L);
}

/** y and mu as device vectors of vars. */
template <bool propto = false>
inline var multi_normal_cholesky_lpdf(const dev_var_matrix& y, const dev_var_matrix& mu,
                                      const dev_var_matrix& L) {
  internal::mvn_check_sizes(int(y.size()), int(mu.size()), L);
  return internal::mvn_cholesky_dev<propto>(y.val_ptr(), mu.val_ptr(), int(y.size()), L, y.vi_,
                                            mu.vi_);
}
template <bool propto = false>
inline var multi_normal_cholesky_lpdf(const dev_var_matrix& y, const dev_data<double>& mu,
                                      const dev_var_matrix& L) {
  internal::mvn_check_sizes(int(y.size()), int(mu.size()), L);
  return internal::mvn_cholesky_dev<propto>(y.val_ptr(), mu.data(), int(y.size()), L, y.vi_,
                                            nullptr);
}

}  // namespace math
}  // namespace stan
#endif
