#ifndef STAN_MATH_FWD_CORE_FVAR_HPP
#define STAN_MATH_FWD_CORE_FVAR_HPP

// fvar<T>: forward-mode dual number (value, tangent) over T -- the reference's
// fwd/core/fvar.hpp:40-49 -- with the scalar arithmetic the hot-path functors
// need.  Instantiated as fvar<var> by hessian_times_vector (fwd-over-rev): the
// tangent is then itself a var on the tape, and the matrix functors take dual
// device matrices (stan/math/mix/fvar_functors.hpp).

#include <cmath>
#include <ostream>
#include <type_traits>

namespace stan {
namespace math {

template <typename T>
class fvar {
 public:
  using value_type = T;
  T val_;  // value
  T d_;    // tangent

  fvar() : val_(0.0), d_(0.0) {}
  fvar(const T& v) : val_(v), d_(0.0) {}  // NOLINT
  fvar(const T& v, const T& d) : val_(v), d_(d) {}
  template <typename A, typename = std::enable_if_t<std::is_arithmetic<A>::value &&
                                                    !std::is_same<A, T>::value>>
  fvar(A v) : val_(static_cast<double>(v)), d_(0.0) {}  // NOLINT

  const T& val() const { return val_; }
  const T& tangent() const { return d_; }

  fvar& operator+=(const fvar& b) { return *this = *this + b; }
  fvar& operator-=(const fvar& b) { return *this = *this - b; }
  fvar& operator*=(const fvar& b) { return *this = *this * b; }
  fvar& operator/=(const fvar& b) { return *this = *this / b; }

  friend fvar operator+(const fvar& a, const fvar& b) { return fvar(a.val_ + b.val_, a.d_ + b.d_); }
  friend fvar operator+(const fvar& a, double b) { return fvar(a.val_ + b, a.d_); }
  friend fvar operator+(double a, const fvar& b) { return fvar(a + b.val_, b.d_); }
  friend fvar operator-(const fvar& a, const fvar& b) { return fvar(a.val_ - b.val_, a.d_ - b.d_); }
  friend fvar operator-(const fvar& a, double b) { return fvar(a.val_ - b, a.d_); }
  friend fvar operator-(double a, const fvar& b) { return fvar(a - b.val_, -b.d_); }
  friend fvar operator-(const fvar& a) { return fvar(-a.val_, -a.d_); }
  friend fvar operator*(const fvar& a, const fvar& b) {
    return fvar(a.val_ * b.val_, a.d_ * b.val_ + a.val_ * b.d_);
  }
  friend fvar operator*(const fvar& a, double b) { return fvar(a.val_ * b, a.d_ * b); }
  friend fvar operator*(double a, const fvar& b) { return fvar(a * b.val_, a * b.d_); }
  friend fvar operator/(const fvar& a, const fvar& b) {
    return fvar(a.val_ / b.val_, (a.d_ * b.val_ - a.val_ * b.d_) / (b.val_ * b.val_));
  }
  friend fvar operator/(const fvar& a, double b) { return fvar(a.val_ / b, a.d_ / b); }
  friend fvar operator/(double a, const fvar& b) {
    return fvar(a / b.val_, -a * b.d_ / (b.val_ * b.val_));
  }
  friend std::ostream& operator<<(std::ostream& os, const fvar& v) { return os << v.val_; }
};

// fwd/scal/fun/{square,exp,log,sqrt}.hpp
template <typename T>
inline fvar<T> square(const fvar<T>& x) {
  return fvar<T>(square(x.val_), x.d_ * (2.0 * x.val_));
}
template <typename T>
inline fvar<T> exp(const fvar<T>& x) {
  using std::exp;
  T e = exp(x.val_);
  return fvar<T>(e, x.d_ * e);
}
template <typename T>
inline fvar<T> log(const fvar<T>& x) {
  using std::log;
  return fvar<T>(log(x.val_), x.d_ / x.val_);
}
template <typename T>
inline fvar<T> sqrt(const fvar<T>& x) {
  using std::sqrt;
  T s = sqrt(x.val_);
  return fvar<T>(s, x.d_ / (2.0 * s));
}

template <typename T>
inline T value_of(const fvar<T>& v) {
  return v.val_;
}

}  // namespace math
}  // namespace stan
#endif
