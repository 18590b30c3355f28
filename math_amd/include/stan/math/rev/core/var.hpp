#ifndef STAN_MATH_REV_CORE_VAR_HPP
#define STAN_MATH_REV_CORE_VAR_HPP

// stan::math::var — an 8-byte handle to a vari, same interface as the
// reference (stan/math/rev/core/var.hpp): vi_, val(), adj(), grad(),
// grad(x, g), implicit construction from arithmetic types (each creates a
// vari pushed on var_stack_, as in var.hpp:81-164), compound assignment.

#include <stan/math/rev/core/grad.hpp>
#include <stan/math/rev/core/vari.hpp>

#include <ostream>
#include <type_traits>
#include <vector>

namespace stan {
namespace math {

class var {
 public:
  vari* vi_;

  var() : vi_(nullptr) {}
  var(vari* vi) : vi_(vi) {}  // NOLINT
  template <typename T, typename = std::enable_if_t<std::is_arithmetic<T>::value>>
  var(T x) : vi_(new vari(static_cast<double>(x))) {}  // NOLINT

  bool is_uninitialized() const { return vi_ == nullptr; }
  inline double val() const { return vi_->val_; }
  inline double adj() const { return vi_->adj_; }

  /** Reverse sweep from this variable; fills g with the adjoints of x
   * (var.hpp:318-324; does not recover memory).  This is the reference's
   * log_prob_grad path, which reads only x and recovers the tape next: the
   * host blocks of an Eigen boundary are not published (grad() publishes
   * them, grad.hpp). */
  void grad(std::vector<var>& x, std::vector<double>& g) {
    no_publish_scope quiet;
    stan::math::grad(vi_);
    g.resize(x.size());
    for (size_t i = 0; i < x.size(); ++i) g[i] = x[i].vi_->adj_;
  }

  void grad() { stan::math::grad(vi_); }

  inline vari& operator*() { return *vi_; }
  inline vari* operator->() { return vi_; }

  inline var& operator+=(const var& b);
  inline var& operator+=(double b);
  inline var& operator-=(const var& b);
  inline var& operator-=(double b);
  inline var& operator*=(const var& b);
  inline var& operator*=(double b);
  inline var& operator/=(const var& b);
  inline var& operator/=(double b);

  friend std::ostream& operator<<(std::ostream& os, const var& v) {
    if (v.vi_ == nullptr) return os << "uninitialized";
    return os << v.val();
  }
};

}  // namespace math
}  // namespace stan
#endif
