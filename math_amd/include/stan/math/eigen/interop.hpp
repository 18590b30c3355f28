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
#include <stan/math/rev/fun/bernoulli_logit_glm_lpmf.hpp>
#include <stan/math/rev/fun/categorical_logit_glm_lpmf.hpp>
#include <stan/math/rev/fun/spd_functors.hpp>
#include <stan/math/rev/fun/lgamma.hpp>
#include <stan/math/rev/fun/log_sum_exp.hpp>
#include <stan/math/rev/fun/mdivide_left_tri.hpp>
#include <stan/math/rev/fun/multiply.hpp>
#include <stan/math/rev/fun/normal_lpdf.hpp>
#include <stan/math/rev/functor/gradient.hpp>

#include <limits>
#include <vector>

#include <stan/math/eigen/num_traits.hpp>

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

inline dev_data<double> to_dev_data(const matrix_d& m) {
  return to_dev_data(m.data(), size_t(m.size()), int(m.rows()), int(m.cols()));
}

/** multiply.hpp:619-661 signatures (Matrix<var> / Matrix<double> operands). */
inline matrix_v multiply(const matrix_v& A, const matrix_v& B) {
  internal::check_multiplicable("multiply", int(A.rows()), int(A.cols()), int(B.rows()), int(B.cols()));
  return to_host_matrix(multiply(to_dev(A), to_dev(B)));
}
inline matrix_v multiply(const matrix_v& A, const matrix_d& B) {
  internal::check_multiplicable("multiply", int(A.rows()), int(A.cols()), int(B.rows()), int(B.cols()));
  return to_host_matrix(multiply(to_dev(A), to_dev_data(B)));
}
inline matrix_v multiply(const matrix_d& A, const matrix_v& B) {
  internal::check_multiplicable("multiply", int(A.rows()), int(A.cols()), int(B.rows()), int(B.cols()));
  return to_host_matrix(multiply(to_dev_data(A), to_dev(B)));
}
inline matrix_v multiply(const var& c, const matrix_v& A) { return to_host_matrix(multiply(c, to_dev(A))); }
inline matrix_v multiply(const matrix_v& A, const var& c) { return multiply(c, A); }
inline matrix_v multiply(double c, const matrix_v& A) { return to_host_matrix(multiply(c, to_dev(A))); }
inline matrix_v multiply(const matrix_v& A, double c) { return multiply(c, A); }

/** prim/mat/fun/transpose.hpp: a plain Eigen transpose (shares the varis). */
template <typename T, int R, int C>
inline Eigen::Matrix<T, C, R> transpose(const Eigen::Matrix<T, R, C>& m) {
  return m.transpose();
}

template <int R, int C>
inline var sum(const Eigen::Matrix<var, R, C>& m) {
  return sum(to_dev(m));
}
inline matrix_v add_diag(const matrix_v& A, double d) { return to_host_matrix(add_diag(to_dev(A), d)); }
inline matrix_v add_diag(const matrix_v& A, const var& d) {
  return to_host_matrix(add_diag(to_dev(A), d));
}

template <int R, int C>
inline var log_sum_exp(const Eigen::Matrix<var, R, C>& x) {
  return log_sum_exp(to_dev(x));
}
template <int R, int C>
inline Eigen::Matrix<var, R, C> lgamma(const Eigen::Matrix<var, R, C>& x) {
  matrix_v m = to_host_matrix(lgamma(to_dev(x)));
  return Eigen::Map<Eigen::Matrix<var, R, C>>(m.data(), x.rows(), x.cols());
}
template <int R, int C>
inline Eigen::Matrix<var, R, C> digamma(const Eigen::Matrix<var, R, C>& x) {
  matrix_v m = to_host_matrix(digamma(to_dev(x)));
  return Eigen::Map<Eigen::Matrix<var, R, C>>(m.data(), x.rows(), x.cols());
}

/** mdivide_left_tri<TriView>(A, b), rev/mat/fun/mdivide_left_tri.hpp:322-373. */
template <int TriView, int R2, int C2>
inline Eigen::Matrix<var, Eigen::Dynamic, C2> mdivide_left_tri(const matrix_v& A,
                                                               const Eigen::Matrix<var, R2, C2>& b) {
  matrix_v m = to_host_matrix(mdivide_left_tri<TriView>(to_dev(A), to_dev(b)));
  return Eigen::Map<Eigen::Matrix<var, Eigen::Dynamic, C2>>(m.data(), m.rows(), m.cols());
}
template <int TriView, int R2, int C2>
inline Eigen::Matrix<var, Eigen::Dynamic, C2> mdivide_left_tri(
    const matrix_d& A, const Eigen::Matrix<var, R2, C2>& b) {
  matrix_v m = to_host_matrix(mdivide_left_tri<TriView>(to_dev_data(A), to_dev(b)));
  return Eigen::Map<Eigen::Matrix<var, Eigen::Dynamic, C2>>(m.data(), m.rows(), m.cols());
}
template <int TriView, int R2, int C2>
inline Eigen::Matrix<var, Eigen::Dynamic, C2> mdivide_left_tri(
    const matrix_v& A, const Eigen::Matrix<double, R2, C2>& b) {
  const matrix_d bd = b;
  matrix_v m = to_host_matrix(mdivide_left_tri<TriView>(to_dev(A), to_dev_data(bd)));
  return Eigen::Map<Eigen::Matrix<var, Eigen::Dynamic, C2>>(m.data(), m.rows(), m.cols());
}
template <int TriView>
inline matrix_v mdivide_left_tri(const matrix_v& A) {
  return to_host_matrix(mdivide_left_tri<TriView>(to_dev(A)));
}

// ------------------------------------------------ §8(f) row 3 (spd_functors.hpp)
/** rev/mat/fun/mdivide_left_spd.hpp:232-260 signatures. */
template <int R1, int C1, int R2, int C2>
inline matrix_v mdivide_left_spd(const Eigen::Matrix<var, R1, C1>& A, const Eigen::Matrix<var, R2, C2>& b) {
  internal::check_square("mdivide_left_spd", "A", int(A.rows()), int(A.cols()));
  internal::check_multiplicable_named("mdivide_left_spd", "A", int(A.cols()), "b", int(b.rows()));
  return to_host_matrix(mdivide_left_spd(to_dev(A), to_dev(b)));
}
template <int R1, int C1, int R2, int C2>
inline matrix_v mdivide_left_spd(const Eigen::Matrix<double, R1, C1>& A, const Eigen::Matrix<var, R2, C2>& b) {
  internal::check_square("mdivide_left_spd", "A", int(A.rows()), int(A.cols()));
  internal::check_multiplicable_named("mdivide_left_spd", "A", int(A.cols()), "b", int(b.rows()));
  const matrix_d Ad = A;
  return to_host_matrix(mdivide_left_spd(to_dev_data(Ad.data(), size_t(Ad.size()), int(Ad.rows()), int(Ad.cols())),
                                         to_dev(b)));
}
template <int R1, int C1, int R2, int C2>
inline matrix_v mdivide_left_spd(const Eigen::Matrix<var, R1, C1>& A, const Eigen::Matrix<double, R2, C2>& b) {
  internal::check_square("mdivide_left_spd", "A", int(A.rows()), int(A.cols()));
  internal::check_multiplicable_named("mdivide_left_spd", "A", int(A.cols()), "b", int(b.rows()));
  const matrix_d bd = b;
  return to_host_matrix(mdivide_left_spd(to_dev(A), to_dev_data(bd.data(), size_t(bd.size()), int(bd.rows()),
                                                               int(bd.cols()))));
}
/** rev/mat/fun/log_determinant_spd.hpp:16 signature. */
template <int R, int C>
inline var log_determinant_spd(const Eigen::Matrix<var, R, C>& m) {
  internal::check_square("log_determinant_spd", "m", int(m.rows()), int(m.cols()));
  return log_determinant_spd(to_dev(m));
}
/** rev/mat/fun/log_determinant.hpp:14 signature. */
template <int R, int C>
inline var log_determinant(const Eigen::Matrix<var, R, C>& m) {
  internal::check_square("log_determinant", "m", int(m.rows()), int(m.cols()));
  if (m.size() == 0) return var(0.0);
  return log_determinant(to_dev(m));
}
/** prim/mat/fun/log_determinant.hpp:20 signature (double matrix -> double). */
template <int R, int C>
inline double log_determinant(const Eigen::Matrix<double, R, C>& m) {
  internal::check_square("log_determinant", "m", int(m.rows()), int(m.cols()));
  if (m.size() == 0) return 0.0;
  const Eigen::Matrix<double, -1, -1> md = m;
  return log_determinant(to_dev_data(md.data(), size_t(md.size()), int(md.rows()), int(md.cols())));
}
/** rev/mat/fun/multiply_lower_tri_self_transpose.hpp:14 signature. */
inline matrix_v multiply_lower_tri_self_transpose(const matrix_v& L) {
  if (L.rows() == 0) return matrix_v(0, 0);
  return to_host_matrix(multiply_lower_tri_self_transpose(to_dev(L)));
}
/** rev/mat/fun/quad_form_sym.hpp:15-40 signatures (matrix B -> matrix, vector b -> var). */
template <int Ra, int Ca, int Rb, int Cb>
inline matrix_v quad_form_sym(const Eigen::Matrix<var, Ra, Ca>& A, const Eigen::Matrix<var, Rb, Cb>& B) {
  return to_host_matrix(quad_form_sym(to_dev(A), to_dev(B)));
}
template <int Ra, int Ca, int Rb, int Cb>
inline matrix_v quad_form_sym(const Eigen::Matrix<double, Ra, Ca>& A, const Eigen::Matrix<var, Rb, Cb>& B) {
  const matrix_d Ad = A;
  return to_host_matrix(quad_form_sym(to_dev_data(Ad.data(), size_t(Ad.size()), int(Ad.rows()), int(Ad.cols())),
                                      to_dev(B)));
}
template <int Ra, int Ca, int Rb>
inline var quad_form_sym(const Eigen::Matrix<var, Ra, Ca>& A, const Eigen::Matrix<var, Rb, 1>& b) {
  matrix_v B = b;
  return quad_form_sym(A, B)(0, 0);
}

/** bernoulli_logit_glm_lpmf(y, x, alpha, beta) with Eigen x / beta (:46-144). */
template <bool propto = false, typename T_alpha, int RB>
inline var bernoulli_logit_glm_lpmf(const std::vector<int>& y, const matrix_d& x,
                                    const T_alpha& alpha, const Eigen::Matrix<var, RB, 1>& beta) {
  std::vector<var> b(beta.data(), beta.data() + beta.size());
  std::vector<double> xv(x.data(), x.data() + x.size());
  if (y.size() != size_t(x.rows()))
    throw std::invalid_argument(
        "bernoulli_logit_glm_lpmf: Vector of dependent variables has dimension = " +
        std::to_string(y.size()) + ", expecting dimension = " + std::to_string(x.rows()));
  return bernoulli_logit_glm_lpmf<propto>(y, xv, int(x.cols()), alpha, b);
}

namespace internal {
template <int R, int C>
inline dev_var_matrix glm_cat_operand(const Eigen::Matrix<var, R, C>& m) { return to_dev(m); }
template <int R, int C>
inline dev_data<double> glm_cat_operand(const Eigen::Matrix<double, R, C>& m) {
  const matrix_d d = m;
  return to_dev_data(d);
}
}  // namespace internal

/** categorical_logit_glm_lpmf(y, x, alpha, beta) with Eigen x / alpha / beta
 * (prim/mat/prob/categorical_logit_glm_lpmf.hpp:38-43); var or double alpha
 * and beta in any combination. */
template <bool propto = false, typename T_a, typename T_b>
inline typename std::conditional<std::is_same<T_a, var>::value || std::is_same<T_b, var>::value, var,
                                 double>::type
categorical_logit_glm_lpmf(const std::vector<int>& y, const matrix_d& x,
                           const Eigen::Matrix<T_a, Eigen::Dynamic, 1>& alpha,
                           const Eigen::Matrix<T_b, Eigen::Dynamic, Eigen::Dynamic>& beta) {
  if (y.size() != size_t(x.rows()))
    internal::glm_size_mismatch("categorical_logit_glm_lpmf", "Vector of dependent variables",
                                (long long)y.size(), x.rows());
  return categorical_logit_glm_lpmf<propto>(to_dev_data(y), to_dev_data(x), internal::glm_cat_operand(alpha),
                                            internal::glm_cat_operand(beta));
}

/** The reference's scalar-y overload: y broadcast to every row. */
template <bool propto = false, typename T_a, typename T_b>
inline auto categorical_logit_glm_lpmf(int y, const matrix_d& x, const Eigen::Matrix<T_a, Eigen::Dynamic, 1>& alpha,
                                       const Eigen::Matrix<T_b, Eigen::Dynamic, Eigen::Dynamic>& beta) {
  static const char* fn = "categorical_logit_glm_lpmf";
  if (alpha.size() != beta.cols())
    internal::glm_size_mismatch(fn, "Intercept vector", (long long)alpha.size(), beta.cols());
  if (x.cols() != beta.rows()) {
    std::ostringstream m;
    m << fn << ": x.cols() (" << x.cols() << ") and beta.rows() (" << beta.rows() << ") must match in size";
    throw std::invalid_argument(m.str());
  }
  if (y < 1 || y > beta.cols()) {
    std::ostringstream m;
    m << fn << ": categorical outcome out of support is " << y << ", but must be in the interval [1, "
      << beta.cols() << "]";
    throw std::domain_error(m.str());
  }
  return categorical_logit_glm_lpmf<propto>(std::vector<int>(size_t(x.rows()), y), x, alpha, beta);
}

template <bool propto = false>
inline var multi_normal_cholesky_lpdf(const vector_d& y, const vector_d& mu, const dev_var_matrix& L) {
  std::vector<double> yv(y.data(), y.data() + y.size()), mv(mu.data(), mu.data() + mu.size());
  return multi_normal_cholesky_lpdf<propto>(yv, mv, L);
}
template <bool propto = false, int RB>
inline double bernoulli_logit_glm_lpmf(const std::vector<int>& y, const matrix_d& x, double alpha,
                                       const Eigen::Matrix<double, RB, 1>& beta) {
  std::vector<double> b(beta.data(), beta.data() + beta.size());
  std::vector<double> xv(x.data(), x.data() + x.size());
  if (y.size() != size_t(x.rows()))
    throw std::invalid_argument(
        "bernoulli_logit_glm_lpmf: Vector of dependent variables has dimension = " +
        std::to_string(y.size()) + ", expecting dimension = " + std::to_string(x.rows()));
  return bernoulli_logit_glm_lpmf<propto>(y, xv, int(x.cols()), alpha, b);
}

template <bool propto = false>
inline var multi_normal_cholesky_lpdf(const vector_v& y, const vector_v& mu, const matrix_v& L) {
  return multi_normal_cholesky_lpdf<propto>(to_dev(y), to_dev(mu), to_dev(L));
}
template <bool propto = false>
inline var multi_normal_cholesky_lpdf(const vector_d& y, const vector_d& mu, const matrix_v& L) {
  return multi_normal_cholesky_lpdf<propto>(y, mu, to_dev(L));
}

}  // namespace math
}  // namespace stan
#endif
