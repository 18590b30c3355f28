#ifndef STAN_MATH_EIGEN_INTEROP_HPP
#define STAN_MATH_EIGEN_INTEROP_HPP

// Eigen-typed boundary: the reference's signatures take and return
// Eigen::Matrix<var, R, C>.  A device matrix converts to one by
// materialising its N^2 host varis (nochain, like the reference's output
// varis) plus one bridge vari on var_stack_ that, in the reverse sweep,
// gathers their adjoints into the device adjoint; the other direction
// gathers host values to the device and scatters device adjoints back.
//
// Requires Eigen (the user's Eigen, as for the reference; tests compile
// against the Eigen 3.3.3 vendored with the reference, read-only).

#include <Eigen/Dense>

#if defined(STAN_MATH_AMD_MATRIX_HPP) && !defined(STAN_MATH_AMD_HAS_EIGEN)
#error "include <stan/math.hpp> (or define STAN_MATH_AMD_HAS_EIGEN) before stan/math/amd/matrix.hpp"
#endif
#ifndef STAN_MATH_AMD_HAS_EIGEN
#define STAN_MATH_AMD_HAS_EIGEN 1
#endif

#include <stan/math/amd/matrix.hpp>
#include <stan/math/rev/core.hpp>
#include <stan/math/rev/fun/cholesky_decompose.hpp>
#include <stan/math/rev/fun/multi_normal_cholesky_lpdf.hpp>
#include <stan/math/rev/functor/gradient.hpp>

#include <limits>
#include <vector>

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
}  // namespace Eigen

namespace stan {
namespace math {

using matrix_v = Eigen::Matrix<var, Eigen::Dynamic, Eigen::Dynamic>;
using vector_v = Eigen::Matrix<var, Eigen::Dynamic, 1>;
using row_vector_v = Eigen::Matrix<var, 1, Eigen::Dynamic>;
using matrix_d = Eigen::Matrix<double, Eigen::Dynamic, Eigen::Dynamic>;
using vector_d = Eigen::Matrix<double, Eigen::Dynamic, 1>;

namespace internal {
template <>
struct var_vector_of<Eigen::Matrix<double, Eigen::Dynamic, 1>> {
  using type = Eigen::Matrix<var, Eigen::Dynamic, 1>;
};

// device -> host varis (reverse: host adjoints -> device adjoint)
class dev_to_host_vari : public vari {
 public:
  dev_matrix_vari* src_;
  vari** elems_;
  double* stage_;  // device scratch for the gathered adjoints
  dev_to_host_vari(dev_matrix_vari* src, vari** elems)
      : vari(0.0), src_(src), elems_(elems), stage_(amd::alloc_doubles(src->size())) {}
  void chain() override {
    const size_t n = src_->size();
    std::vector<double> h(n);
    for (size_t i = 0; i < n; ++i) h[i] = elems_[i]->adj_;
    amd::to_device(stage_, h.data(), n);
    amd::check(smg_axpy(amd::ctx(), (long long)n, 1.0, stage_, 1, src_->adj_, 1), "to_host");
  }
};

// host varis -> device (reverse: device adjoint -> host adjoints)
class host_to_dev_vari : public vari {
 public:
  dev_matrix_vari* dst_;
  vari** elems_;
  host_to_dev_vari(dev_matrix_vari* dst, vari** elems) : vari(0.0), dst_(dst), elems_(elems) {}
  void chain() override {
    const size_t n = dst_->size();
    std::vector<double> h(n);
    amd::to_host(h.data(), dst_->adj_, n);
    for (size_t i = 0; i < n; ++i) elems_[i]->adj_ += h[i];
  }
};
}  // namespace internal

/** Materialise a device matrix of vars as host varis. */
inline matrix_v to_host_matrix(const dev_var_matrix& m) {
  const size_t n = m.size();
  std::vector<double> vals = m.val();
  vari** elems = ChainableStack::instance_->memalloc_.alloc_array<vari*>(n ? n : 1);
  for (size_t i = 0; i < n; ++i) elems[i] = new vari(vals[i], false);
  new internal::dev_to_host_vari(m.vi_, elems);
  matrix_v out(m.rows(), m.cols());
  for (size_t i = 0; i < n; ++i) out(i) = var(elems[i]);
  if (m.vi_->structure_ == dev_structure::lower) {
    // upper entries alias one dummy vari like cholesky_decompose.hpp:34-48
    vari* dummy = new vari(0.0, false);
    for (int j = 0; j < m.cols(); ++j)
      for (int i = 0; i < j; ++i) out(i, j) = var(dummy);
  }
  return out;
}

/** Copy host vars to a device matrix node (bridged in the reverse sweep). */
template <int R, int C>
inline dev_var_matrix to_dev(const Eigen::Matrix<var, R, C>& m) {
  const size_t n = size_t(m.size());
  auto* d = new dev_matrix_vari(int(m.rows()), int(m.cols()));
  std::vector<double> vals(n);
  vari** elems = ChainableStack::instance_->memalloc_.alloc_array<vari*>(n ? n : 1);
  for (size_t i = 0; i < n; ++i) {
    vals[i] = m(i).val();
    elems[i] = m(i).vi_;
  }
  amd::to_device(d->val_, vals.data(), n);
  new internal::host_to_dev_vari(d, elems);
  return dev_var_matrix(d);
}

inline dev_var_matrix::operator Eigen::Matrix<var, Eigen::Dynamic, Eigen::Dynamic>() const {
  return to_host_matrix(*this);
}
inline dev_var_matrix::operator Eigen::Matrix<var, Eigen::Dynamic, 1>() const {
  matrix_v m = to_host_matrix(*this);
  return Eigen::Map<vector_v>(m.data(), m.size());
}

inline matrix_d value_of(const dev_var_matrix& m) {
  std::vector<double> v = m.val();
  return Eigen::Map<matrix_d>(v.data(), m.rows(), m.cols());
}
inline matrix_d adjoint_of(const dev_var_matrix& m) {
  std::vector<double> v = m.adj();
  return Eigen::Map<matrix_d>(v.data(), m.rows(), m.cols());
}
template <int R, int C>
inline Eigen::Matrix<double, R, C> value_of(const Eigen::Matrix<var, R, C>& m) {
  Eigen::Matrix<double, R, C> out(m.rows(), m.cols());
  for (Eigen::Index i = 0; i < m.size(); ++i) out(i) = m(i).val();
  return out;
}

// ------------------------------------------------ Eigen-typed functors

/** rev/mat/fun/cholesky_decompose.hpp:378 signature: Matrix<var> -> Matrix<var>. */
inline matrix_v cholesky_decompose(const matrix_v& A) {
  internal::check_square("cholesky_decompose", "A", int(A.rows()), int(A.cols()));
  return to_host_matrix(cholesky_decompose(to_dev(A)));
}

template <bool propto = false>
inline var multi_normal_cholesky_lpdf(const vector_d& y, const vector_d& mu, const dev_var_matrix& L) {
  std::vector<double> yv(y.data(), y.data() + y.size()), mv(mu.data(), mu.data() + mu.size());
  return multi_normal_cholesky_lpdf<propto>(yv, mv, L);
}
template <bool propto = false>
inline var multi_normal_cholesky_lpdf(const vector_d& y, const vector_d& mu, const matrix_v& L) {
  return multi_normal_cholesky_lpdf<propto>(y, mu, to_dev(L));
}

}  // namespace math
}  // namespace stan
#endif
