#ifndef STAN_MATH_REV_CORE_OPERATORS_HPP
#define STAN_MATH_REV_CORE_OPERATORS_HPP

// Scalar var arithmetic and the scalar functions the hot-path functors and
// their callers use.  Each result is one vari on var_stack_ whose chain()
// applies the local partials, as in the reference's op_*_vari classes
// (rev/core/operator_*.hpp, rev/scal/fun/*.hpp).  NaN rule of
// rev/core/operator_multiplication.hpp:19-26: a NaN operand value makes the
// operand adjoints NaN.

#include <stan/math/rev/core/var.hpp>

#include <cmath>
#include <limits>

namespace stan {
namespace math {

namespace internal {
constexpr double NaN = std::numeric_limits<double>::quiet_NaN();

class op_v_vari : public host_local_vari {
 protected:
  vari* avi_;

 public:
  op_v_vari(double f, vari* a) : host_local_vari(f), avi_(a) {}
  bool touches_adjoints_in(const vari* lo, const vari* hi) const override { return avi_ >= lo && avi_ < hi; }
};
class op_vv_vari : public host_local_vari {
 protected:
  vari* avi_;
  vari* bvi_;

 public:
  op_vv_vari(double f, vari* a, vari* b) : host_local_vari(f), avi_(a), bvi_(b) {}
  bool touches_adjoints_in(const vari* lo, const vari* hi) const override {
    return (avi_ >= lo && avi_ < hi) || (bvi_ >= lo && bvi_ < hi);
  }
};

// z = a op b with precomputed local partials (da, db); NaN rule applied
class binary_vv_vari : public op_vv_vari {
  double da_, db_;

 public:
  binary_vv_vari(double f, vari* a, vari* b, double da, double db)
      : op_vv_vari(f, a, b), da_(da), db_(db) {}
  void chain() override {
    if (__builtin_expect(std::isnan(avi_->val_) || std::isnan(bvi_->val_), 0)) {
      avi_->adj_ = NaN;
      bvi_->adj_ = NaN;
    } else {
      avi_->adj_ += adj_ * da_;
      bvi_->adj_ += adj_ * db_;
    }
  }
};
class unary_vari : public op_v_vari {
  double da_;

 public:
  unary_vari(double f, vari* a, double da) : op_v_vari(f, a), da_(da) {}
  void chain() override {
    if (__builtin_expect(std::isnan(avi_->val_), 0))
      avi_->adj_ = NaN;
    else
      avi_->adj_ += adj_ * da_;
  }
};
}  // namespace internal

// ------------------------------------------------------------- arithmetic
inline var operator+(const var& a, const var& b) {
  return var(new internal::binary_vv_vari(a.val() + b.val(), a.vi_, b.vi_, 1.0, 1.0));
}
inline var operator+(const var& a, double b) {
  if (b == 0.0) return a;
  return var(new internal::unary_vari(a.val() + b, a.vi_, 1.0));
}
inline var operator+(double a, const var& b) { return b + a; }

inline var operator-(const var& a, const var& b) {
  return var(new internal::binary_vv_vari(a.val() - b.val(), a.vi_, b.vi_, 1.0, -1.0));
}
inline var operator-(const var& a, double b) {
  if (b == 0.0) return a;
  return var(new internal::unary_vari(a.val() - b, a.vi_, 1.0));
}
inline var operator-(double a, const var& b) {
  return var(new internal::unary_vari(a - b.val(), b.vi_, -1.0));
}

inline var operator*(const var& a, const var& b) {
  return var(new internal::binary_vv_vari(a.val() * b.val(), a.vi_, b.vi_, b.val(), a.val()));
}
inline var operator*(const var& a, double b) {
  if (b == 1.0) return a;
  return var(new internal::unary_vari(a.val() * b, a.vi_, b));
}
inline var operator*(double a, const var& b) { return b * a; }

inline var operator/(const var& a, const var& b) {
  const double bv = b.val();
  return var(new internal::binary_vv_vari(a.val() / bv, a.vi_, b.vi_, 1.0 / bv,
                                          -a.val() / (bv * bv)));
}
inline var operator/(const var& a, double b) {
  if (b == 1.0) return a;
  return var(new internal::unary_vari(a.val() / b, a.vi_, 1.0 / b));
}
inline var operator/(double a, const var& b) {
  const double bv = b.val();
  return var(new internal::unary_vari(a / bv, b.vi_, -a / (bv * bv)));
}

inline var operator-(const var& a) { return var(new internal::unary_vari(-a.val(), a.vi_, -1.0)); }
inline var operator+(const var& a) { return a; }

inline var& var::operator+=(const var& b) { return *this = *this + b; }
inline var& var::operator+=(double b) { return *this = *this + b; }
inline var& var::operator-=(const var& b) { return *this = *this - b; }
inline var& var::operator-=(double b) { return *this = *this - b; }
inline var& var::operator*=(const var& b) { return *this = *this * b; }
inline var& var::operator*=(double b) { return *this = *this * b; }
inline var& var::operator/=(const var& b) { return *this = *this / b; }
inline var& var::operator/=(double b) { return *this = *this / b; }

// ----------------------------------------------------------- comparisons
#define SMG_VAR_CMP(OP)                                                          \
  inline bool operator OP(const var& a, const var& b) { return a.val() OP b.val(); } \
  inline bool operator OP(const var& a, double b) { return a.val() OP b; }           \
  inline bool operator OP(double a, const var& b) { return a OP b.val(); }
SMG_VAR_CMP(==)
SMG_VAR_CMP(!=)
SMG_VAR_CMP(<)
SMG_VAR_CMP(<=)
SMG_VAR_CMP(>)
SMG_VAR_CMP(>=)
#undef SMG_VAR_CMP

// ------------------------------------------------------ scalar functions
inline double value_of(double x) { return x; }
inline double value_of(const var& v) { return v.val(); }
inline double value_of_rec(double x) { return x; }
inline double value_of_rec(const var& v) { return v.val(); }

inline var exp(const var& a) {
  const double e = std::exp(a.val());
  return var(new internal::unary_vari(e, a.vi_, e));
}
inline var log(const var& a) {
  return var(new internal::unary_vari(std::log(a.val()), a.vi_, 1.0 / a.val()));
}
inline var sqrt(const var& a) {
  const double s = std::sqrt(a.val());
  return var(new internal::unary_vari(s, a.vi_, 0.5 / s));
}
inline var square(const var& a) {
  return var(new internal::unary_vari(a.val() * a.val(), a.vi_, 2.0 * a.val()));
}
inline double square(double a) { return a * a; }
inline var log1p(const var& a) {
  return var(new internal::unary_vari(std::log1p(a.val()), a.vi_, 1.0 / (1.0 + a.val())));
}
inline var fabs(const var& a) {
  const double v = a.val();
  if (v > 0) return a;
  if (v < 0) return -a;
  if (v == 0) return var(new vari(0.0));
  return var(new internal::unary_vari(internal::NaN, a.vi_, internal::NaN));
}
inline var pow(const var& a, double e) {
  if (e == 1.0) return a;
  if (e == 2.0) return square(a);
  return var(new internal::unary_vari(std::pow(a.val(), e), a.vi_,
                                      e * std::pow(a.val(), e - 1.0)));
}

/** log1p_exp (prim/scal/fun/log1p_exp.hpp:43-50) */
inline double log1p_exp(double a) {
  if (a > 0.0) return a + std::log1p(std::exp(-a));
  return std::log1p(std::exp(a));
}

/** log_sum_exp(double, double) (prim/scal/fun/log_sum_exp.hpp:47-59) */
inline double log_sum_exp(double a, double b) {
  const double inf = std::numeric_limits<double>::infinity();
  if (a == -inf) return b;
  if (a == inf && b == inf) return inf;
  if (a > b) return a + log1p_exp(b - a);
  return b + log1p_exp(a - b);
}

namespace internal {
// rev/scal/fun/log_sum_exp.hpp:15-68
class lse_vv_vari : public op_vv_vari {
 public:
  lse_vv_vari(vari* a, vari* b) : op_vv_vari(log_sum_exp(a->val_, b->val_), a, b) {}
  void chain() override {
    avi_->adj_ += adj_ * std::exp(avi_->val_ - val_);
    bvi_->adj_ += adj_ * std::exp(bvi_->val_ - val_);
  }
};
class lse_vd_vari : public op_v_vari {
 public:
  lse_vd_vari(vari* a, double b) : op_v_vari(log_sum_exp(a->val_, b), a) {}
  void chain() override {
    if (val_ == -std::numeric_limits<double>::infinity())
      avi_->adj_ += adj_;
    else
      avi_->adj_ += adj_ * std::exp(avi_->val_ - val_);
  }
};
}  // namespace internal

inline var log_sum_exp(const var& a, const var& b) {
  return var(new internal::lse_vv_vari(a.vi_, b.vi_));
}
inline var log_sum_exp(const var& a, double b) { return var(new internal::lse_vd_vari(a.vi_, b)); }
inline var log_sum_exp(double a, const var& b) { return var(new internal::lse_vd_vari(b.vi_, a)); }

}  // namespace math
}  // namespace stan
#endif
