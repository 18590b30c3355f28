#ifndef STAN_MATH_PRIM_SPECIAL_HPP
#define STAN_MATH_PRIM_SPECIAL_HPP

// Host-side double special functions with the reference's definitions:
//   lgamma   : libm lgamma_r            (prim/scal/fun/lgamma.hpp:62-71)
//   digamma  : boost::math::digamma, 53-bit path, errno_on_error policy ->
//              NaN at poles             (prim/scal/fun/digamma.hpp:46-48)
//   trigamma : AS121-style recurrence    (prim/scal/fun/trigamma.hpp:33-80)
// The device kernels (math_amd/csrc/elementwise.hip) evaluate the same
// formulas; these host versions serve scalar var overloads.

#include <cmath>
#include <limits>

namespace stan {
namespace math {

inline double lgamma(double x) {
  int sign;
  return ::lgamma_r(x, &sign);
}

namespace internal {
inline double digamma_large(double x) {
  static const double P[] = {0.083333333333333333333333333333333333333333333333333,
                             -0.0083333333333333333333333333333333333333333333333333,
                             0.003968253968253968253968253968253968253968253968254,
                             -0.0041666666666666666666666666666666666666666666666667,
                             0.0075757575757575757575757575757575757575757575757576,
                             -0.021092796092796092796092796092796092796092796092796,
                             0.083333333333333333333333333333333333333333333333333,
                             -0.44325980392156862745098039215686274509803921568627};
  x -= 1;
  double r = std::log(x) + 1 / (2 * x);
  const double z = 1 / (x * x);
  double p = P[7];
  for (int i = 6; i >= 0; --i) p = p * z + P[i];
  return r - z * p;
}
inline double digamma_1_2(double x) {
  const double Y = static_cast<double>(0.99558162689208984F);
  const double root1 = 1569415565.0 / 1073741824.0;
  const double root2 = (381566830.0 / 1073741824.0) / 1073741824.0;
  const double root3 = 0.9016312093258695918615325266959189453125e-19;
  static const double P[] = {0.25479851061131551,   -0.32555031186804491, -0.65031853770896507,
                             -0.28919126444774784, -0.045251321448739056, -0.0020713321167745952};
  static const double Q[] = {1.0,
                             2.0767117023730469,
                             1.4606242909763515,
                             0.43593529692665969,
                             0.054151797245674225,
                             0.0021284987017821144,
                             -0.55789841321675513e-6};
  double g = x - root1;
  g -= root2;
  g -= root3;
  const double t = x - 1;
  double p = P[5], q = Q[6];
  for (int i = 4; i >= 0; --i) p = p * t + P[i];
  for (int i = 5; i >= 0; --i) q = q * t + Q[i];
  return g * Y + g * (p / q);
}
inline double trigamma_pos(double x) {
  const double b2 = 1.0 / 6.0, b4 = -1.0 / 30.0, b6 = 1.0 / 42.0, b8 = -1.0 / 30.0;
  if (x <= 0.0001) return 1.0 / (x * x);
  double z = x, value = 0.0;
  while (z < 5.0) {
    value += 1.0 / (z * z);
    z += 1.0;
  }
  const double y = 1.0 / (z * z);
  return value + 0.5 * y + (1.0 + y * (b2 + y * (b4 + y * (b6 + y * b8)))) / z;
}
}  // namespace internal

inline double digamma(double x) {
  const double pi = 3.14159265358979323846;
  double result = 0;
  if (std::isnan(x)) return x;
  if (x <= -1) {
    x = 1 - x;
    double rem = x - std::floor(x);
    if (rem > 0.5) rem -= 1;
    if (rem == 0) return std::numeric_limits<double>::quiet_NaN();
    result = pi / std::tan(pi * rem);
  }
  if (x == 0) return std::numeric_limits<double>::quiet_NaN();
  if (x >= 10) return result + internal::digamma_large(x);
  while (x > 2) {
    x -= 1;
    result += 1 / x;
  }
  while (x < 1) {
    result -= 1 / x;
    x += 1;
  }
  return result + internal::digamma_1_2(x);
}

inline double trigamma(double x) {
  const double pi = 3.14159265358979323846;
  if (std::isnan(x)) return x;
  if (x <= 0.0 && std::floor(x) == x) return std::numeric_limits<double>::infinity();
  if (x <= 0) {
    const double s = pi / std::sin(-pi * x);
    return -internal::trigamma_pos(-x + 1.0) + s * s;
  }
  return internal::trigamma_pos(x);
}

}  // namespace math
}  // namespace stan
#endif
