#ifndef STAN_MATH_REV_FUN_GP_EXP_QUAD_COV_HPP
#define STAN_MATH_REV_FUN_GP_EXP_QUAD_COV_HPP

// gp_exp_quad_cov(x, sigma, length_scale) for scalar inputs x (the
// D-dimensional std::vector<Eigen vector> forms are in eigen/interop.hpp and
// share this node: x on the device as D x n).
// Reference: rev/mat/fun/gp_exp_quad_cov.hpp:32-286.  Same checks
// (check_positive sigma / length_scale, check_not_nan x, :216-221), same
// value K_ij = sigma^2 exp(-(x_i - x_j)^2 / (2 l^2)) and adjoint
//   l' += sum_lower Kadj K d^2 / l^3,  sigma' += 2 (sum_lower Kadj K + sum_diag Kadj K) / sigma
// (:96-112), with the whole matrix on the device (kernels: smg_gp_exp_quad_cov_*).

#include <stan/math/amd/matrix.hpp>
#include <stan/math/rev/core.hpp>

#include <cmath>
#include <sstream>
#include <stdexcept>
#include <vector>

namespace stan {
namespace math {

namespace internal {
inline void gp_check_positive(const char* fn, const char* name, double v) {
  if (!(v > 0)) {
    std::ostringstream m;
    m << fn << ": " << name << " is " << v << ", but must be > 0!";
    throw std::domain_error(m.str());
  }
}

class gp_exp_quad_cov_dev_vari : public device_vari, public structured_adjoint_sink {
 public:
  const double* x_;  // D x n column-major (point i at x_ + i D)
  const int n_;
  const int D_;
  const double sigma_d_, l_d_;
  vari* sigma_vi_;  // null when sigma is data
  vari* l_vi_;      // null when l is data
  dev_matrix_vari* K_;
  double* out2_;
  size_t pos_;  // this node's index in var_stack_
  // K's adjoint in inverse form (the GP marginal's closed form through
  // add_diag, rev/fun/cholesky_decompose.hpp): its reduction was queued when
  // it was deposited (dep_); exp_: consumed without forming K's dense adjoint
  inverse_adjoint dep_, exp_;

  gp_exp_quad_cov_dev_vari(const double* x, int n, int D, double sigma, vari* sigma_vi, double l, vari* l_vi)
      : device_vari(0.0),
        x_(x),
        n_(n),
        D_(D),
        sigma_d_(sigma),
        l_d_(l),
        sigma_vi_(sigma_vi),
        l_vi_(l_vi),
        K_(new dev_matrix_vari(n, n, dev_structure::symmetric)),
        out2_(amd::alloc_doubles(2)),
        pos_(ChainableStack::instance_->var_stack_.size() - 1) {
    K_->sink_ = this;
    amd::check(smg_gp_exp_quad_cov_nd_fwd(amd::ctx(), x_, D_, n_, sigma_d_, l_d_, K_->val_, n_), "gp_exp_quad_cov");
  }

  bool may_write_device_adjoint(const void*) const override { return false; }  // (host scalars only)

  // The inverse form's reduction (this node's sigma', l' and the depositing
  // add_diag's d') is queued right away, so that the d' a host node reads
  // before this node's chain() is complete; chain() keeps sigma', l' only if
  // no other node wrote K's adjoint, else it recomputes them from the dense sum.
  // One deposit per sweep: a second producer (K shared by two add_diag /
  // cholesky chains, or passed to cholesky and add_diag) is refused and
  // writes its G densely, and chain() expands the kept deposit on top of it.
  bool take_inverse_adjoint(const inverse_adjoint& d, double* dadj) override {
    if (d.n != n_) return false;
    if (dep_.C && dep_.sweep == ChainableStack::instance_->sweep_) return false;
    amd::check(smg_gp_inverse_adjoint(amd::ctx(), d.C, n_, n_, d.s, d.k, d.ss, d.adj, K_->val_, n_, x_, D_, sigma_d_,
                                      l_d_, dadj, (sigma_vi_ || l_vi_) ? out2_ : nullptr),
               "gp_exp_quad_cov");
    dep_ = d;
    return true;
  }
  // K's adjoint read: the deposit of this sweep is written densely whether
  // chain() consumed it (exp_) or has not run (dep_: a nested sweep whose
  // window holds the depositing factor but not this node, or a read before
  // this node's turn -- chain() then takes the dense path on the sum)
  void expand_adjoint() override {
    const size_t sw = ChainableStack::instance_->sweep_;
    if (exp_.C && exp_.sweep == sw) exp_.expand_into(K_->adj_);
    exp_ = inverse_adjoint{};
    if (dep_.C && dep_.sweep == sw) dep_.expand_into(K_->adj_);
    dep_ = inverse_adjoint{};
  }

  void chain() override {
    auto* st = ChainableStack::instance_;
    if (dep_.C && dep_.sweep == st->sweep_) {
      const inverse_adjoint d = dep_;
      dep_ = inverse_adjoint{};
      if (!others_write_device_adjoint(pos_, K_, d.owner)) {
        if (sigma_vi_) add_pending_adjoint(sigma_vi_, out2_);
        if (l_vi_) add_pending_adjoint(l_vi_, out2_ + 1);
        exp_ = d;
        return;
      }
      d.expand_into(K_->adj_);  // another node wrote K's adjoint too: the dense sum
    }
    if (!sigma_vi_ && !l_vi_) return;
    smg_ctx* c = amd::ctx();
    amd::check(smg_memset(c, out2_, 0, 2 * sizeof(double)), "gp_exp_quad_cov");
    amd::check(smg_gp_exp_quad_cov_nd_rev(c, x_, D_, n_, sigma_d_, l_d_, K_->adj_, n_, out2_), "gp_exp_quad_cov");
    if (sigma_vi_) add_pending_adjoint(sigma_vi_, out2_);
    if (l_vi_) add_pending_adjoint(l_vi_, out2_ + 1);
  }
};

/** names: the checked argument names of the overload (rev: "sigma" /
 * "length_scale" for (var, var), "marginal variance" / "length-scale" for
 * (double, var), :216-221,254-259; prim: "magnitude" / "length scale",
 * prim/mat/fun/gp_exp_quad_cov.hpp:180-181). */
inline dev_var_matrix gp_exp_quad_cov_dev(const dev_data<double>& x, int D, double sigma, vari* sigma_vi, double l,
                                          vari* l_vi, const char* sigma_name = nullptr,
                                          const char* l_name = nullptr) {
  const char* fn = "gp_exp_quad_cov";
  gp_check_positive(fn, sigma_name ? sigma_name : sigma_vi ? "sigma" : "marginal variance", sigma);
  gp_check_positive(fn, l_name ? l_name : l_vi ? "length_scale" : "length-scale", l);
  const int n = D > 0 ? int(x.size() / size_t(D)) : 0;
  auto* node = new gp_exp_quad_cov_dev_vari(x.data(), n, D, sigma, sigma_vi, l, l_vi);
  return dev_var_matrix(node->K_);
}
inline dev_var_matrix gp_exp_quad_cov_dev(const dev_data<double>& x, double sigma, vari* sigma_vi, double l,
                                          vari* l_vi) {
  return gp_exp_quad_cov_dev(x, 1, sigma, sigma_vi, l, l_vi);
}

inline dev_data<double> gp_x_to_device(const std::vector<double>& x) {
  for (size_t i = 0; i < x.size(); ++i)
    if (std::isnan(x[i])) {
      std::ostringstream m;
      // check_not_nan("gp_exp_quad_cov", "x", x[i]) on the element (:220): no index in the message
      m << "gp_exp_quad_cov: x is nan, but must not be nan!";
      throw std::domain_error(m.str());
    }
  return to_dev_data(x);
}
}  // namespace internal

inline dev_var_matrix gp_exp_quad_cov(const std::vector<double>& x, const var& sigma,
                                      const var& length_scale) {
  return internal::gp_exp_quad_cov_dev(internal::gp_x_to_device(x), sigma.val(), sigma.vi_,
                                       length_scale.val(), length_scale.vi_);
}
inline dev_var_matrix gp_exp_quad_cov(const std::vector<double>& x, double sigma,
                                      const var& length_scale) {
  return internal::gp_exp_quad_cov_dev(internal::gp_x_to_device(x), sigma, nullptr,
                                       length_scale.val(), length_scale.vi_);
}
/** Device-resident x (kept across gradient evaluations by the caller). */
inline dev_var_matrix gp_exp_quad_cov(const dev_data<double>& x, const var& sigma,
                                      const var& length_scale) {
  return internal::gp_exp_quad_cov_dev(x, sigma.val(), sigma.vi_, length_scale.val(),
                                       length_scale.vi_);
}
inline dev_var_matrix gp_exp_quad_cov(const dev_data<double>& x, double sigma,
                                      const var& length_scale) {
  return internal::gp_exp_quad_cov_dev(x, sigma, nullptr, length_scale.val(), length_scale.vi_);
}
/** (var sigma, double length_scale): the reference's prim template
 * (prim/mat/fun/gp_exp_quad_cov.hpp:175-198, names "magnitude" / "length scale"). */
inline dev_var_matrix gp_exp_quad_cov(const std::vector<double>& x, const var& sigma, double length_scale) {
  return internal::gp_exp_quad_cov_dev(internal::gp_x_to_device(x), 1, sigma.val(), sigma.vi_, length_scale,
                                       nullptr, "magnitude", "length scale");
}

}  // namespace math
}  // namespace stan
#endif
