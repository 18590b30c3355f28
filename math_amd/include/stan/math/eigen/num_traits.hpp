#ifndef STAN_MATH_EIGEN_NUM_TRAITS_HPP
#define STAN_MATH_EIGEN_NUM_TRAITS_HPP

// Eigen::NumTraits<var> (reference: rev/mat/fun/Eigen_NumTraits.hpp:20-60).
// Included right after var is defined, before any header whose var
// arithmetic could make Eigen instantiate the primary template.
#include <Eigen/Core>
#include <stan/math/fwd/core/fvar.hpp>
#include <stan/math/rev/core/var.hpp>

#include <limits>

namespace Eigen {
// NumTraits for var (reference: rev/mat/fun/Eigen_NumTraits.hpp:20-60)
template <>
struct NumTraits<stan::math::var> : GenericNumTraits<stan::math::var> {
  using Real = stan::math::var;
  using NonInteger = stan::math::var;
  using Nested = stan::math::var;
  using Literal = stan::math::var;
  static inline Real epsilon() { return std::numeric_limits<double>::epsilon(); }
  static inline Real dummy_precision() { return 1e-12; }
  static inline Real highest() { return std::numeric_limits<double>::max(); }
  static inline Real lowest() { return -std::numeric_limits<double>::max(); }
  enum {
    IsComplex = 0,
    IsInteger = 0,
    IsSigned = 1,
    RequireInitialization = 0,
    ReadCost = 1,
    AddCost = 1,
    MulCost = 1
  };
  static inline int digits10() { return std::numeric_limits<double>::digits10; }
};
// NumTraits for fvar<var> (fwd/mat/fun/Eigen_NumTraits.hpp)
template <>
struct NumTraits<stan::math::fvar<stan::math::var>>
    : GenericNumTraits<stan::math::fvar<stan::math::var>> {
  using Real = stan::math::fvar<stan::math::var>;
  using NonInteger = Real;
  using Nested = Real;
  using Literal = Real;
  enum {
    IsComplex = 0,
    IsInteger = 0,
    IsSigned = 1,
    RequireInitialization = 1,
    ReadCost = 1,
    AddCost = 1,
    MulCost = 1
  };
  static inline int digits10() { return std::numeric_limits<double>::digits10; }
};
}  // namespace Eigen

#endif
