#ifndef STAN_MATH_EIGEN_INTEROP_HPP
#define STAN_MATH_EIGEN_INTEROP_HPP

// Eigen-typed boundary: the reference's signatures take and return
// Eigen::Matrix<T, R, C> with T = var or double, and its overload sets are
// templates on <T, R, C> constrained by require_* traits (e.g.
// rev/mat/fun/multiply.hpp:562-661, prim/mat/prob/multi_normal_cholesky_lpdf.hpp:40-41).
// The same here: every Eigen overload is a template over the scalar types and
// static shapes of its operands, constrained with enable_if, so mixed
// var / double calls and vector / row-vector / matrix shapes resolve exactly
// as they do against the reference.
//
// Crossing the boundary:
//   device node -> Eigen::Matrix<var>: to_host_matrix materialises the node
//     as n contiguous host varis (one arena block, one value copy, a parallel
//     construction; stan/math/amd/matrix.hpp materialise) plus one bridge vari;
//   Eigen::Matrix<var> -> device: to_dev recognises a matrix that is exactly
//     such a block (pointer identity of every element) and hands back the
//     node itself -- no gather, no upload; otherwise it gathers the values
//     (bridged by host_to_dev_vari in the reverse sweep).
// In the reverse sweep a block's bridge gathers its N^2 host adjoints only
// when a node chained after it touched them (dev_to_host_vari::chain).
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
#include <stan/math/rev/fun/gp_exp_quad_cov.hpp>
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

#include <cmath>
#include <limits>
#include <sstream>
#include <type_traits>
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

// ------------------------------------------------------------ type traits
template <typename T>
struct is_var : std::is_same<std::decay_t<T>, var> {};
template <typename T>
struct is_ad_scalar : std::integral_constant<bool, std::is_arithmetic<std::decay_t<T>>::value || is_var<T>::value> {};

/** scalar type of a (nested) container: var / double / int ... */
template <typename T>
struct scalar_of {
  using type = std::decay_t<T>;
};
template <typename S, int R, int C, int O, int MR, int MC>
struct scalar_of<Eigen::Matrix<S, R, C, O, MR, MC>> {
  using type = typename scalar_of<S>::type;
};
template <typename T, typename A>
struct scalar_of<std::vector<T, A>> {
  using type = typename scalar_of<T>::type;
};
template <>
struct scalar_of<dev_var_matrix> {
  using type = var;
};
template <typename... T>
struct any_var : std::integral_constant<bool, (is_var<typename scalar_of<T>::type>::value || ...)> {};

/** an Eigen column or row vector of var / double */
template <typename T>
struct is_eigen_vec : std::false_type {};
template <typename S, int R, int C, int O, int MR, int MC>
struct is_eigen_vec<Eigen::Matrix<S, R, C, O, MR, MC>>
    : std::integral_constant<bool, (R == 1 || C == 1) && is_ad_scalar<S>::value> {};
/** a multivariate argument of the mvn: an Eigen vector or a std::vector of them */
template <typename T>
struct is_mvt_arg : is_eigen_vec<T> {};
template <typename T, typename A>
struct is_mvt_arg<std::vector<T, A>> : is_eigen_vec<T> {};

// ------------------------------------------------------------ conversions
/** A var or double Eigen operand prepared for a device functor without
 * touching the tape: a recognised host block (its node), or host values to
 * gather / upload when committed. */
struct eig_in {
  const var* vd = nullptr;
  const double* dd = nullptr;
  size_t n = 0;
  int rows = 0, cols = 0;
  dev_matrix_vari* node = nullptr;
  long block = -1;  // its host block's index
};
template <int R, int C, int O, int MR, int MC>
inline eig_in prepare(const Eigen::Matrix<var, R, C, O, MR, MC>& m, const char* nan_fn = nullptr,
                      const char* nan_name = nullptr) {
  eig_in e;
  e.vd = m.data();
  e.n = size_t(m.size());
  e.rows = int(m.rows());
  e.cols = int(m.cols());
  e.block = recognise_block_index(e.vd, e.n, e.rows, e.cols);
  if (e.block >= 0) e.node = static_cast<dev_matrix_vari*>(ChainableStack::instance_->host_blocks_[size_t(e.block)].node);
  if (nan_fn) {
    if (e.node) {
      smg_ctx* c = amd::ctx();
      double* flag = amd::alloc_doubles(1);
      amd::check(smg_memset(c, flag, 0, sizeof(double)), nan_fn);
      amd::check(smg_check_domain(c, e.node->val_, (long long)e.n, 0, flag), nan_fn);
      double f = 0;
      amd::to_host(&f, flag, 1);
      if (f == 0.0) return e;
    }
    for (size_t i = 0; i < e.n; ++i)
      if (std::isnan(e.vd[i].vi_->val_)) throw_not_nan(nan_fn, nan_name, i);
  }
  return e;
}
template <int R, int C, int O, int MR, int MC>
inline eig_in prepare(const Eigen::Matrix<double, R, C, O, MR, MC>& m, const char* nan_fn = nullptr,
                      const char* nan_name = nullptr) {
  eig_in e;
  e.dd = m.data();
  e.n = size_t(m.size());
  e.rows = int(m.rows());
  e.cols = int(m.cols());
  if (nan_fn)
    for (size_t i = 0; i < e.n; ++i)
      if (std::isnan(e.dd[i])) throw_not_nan(nan_fn, nan_name, i);
  return e;
}
/** The device operand of a prepared input (this may push the bridge vari). */
inline dev_operand commit(const eig_in& e) {
  if (e.node) return operand(dev_var_matrix(e.node));
  if (e.vd) return operand(to_dev_vars(e.vd, e.n, e.rows, e.cols));
  return operand(to_dev_data(e.dd, e.n, e.rows, e.cols));
}
}  // namespace internal

/** Materialise a device matrix of vars as an Eigen matrix of host varis. */
template <int R = Eigen::Dynamic, int C = Eigen::Dynamic>
inline Eigen::Matrix<var, R, C> to_host_matrix(const dev_var_matrix& m) {
  Eigen::Matrix<var, R, C> out(m.rows(), m.cols());
  var* d = out.data();
  // the pointer array needs only the block's addresses: filled while the
  // values are in flight
  internal::materialise(m.vi_, [&](const host_block& b) { internal::fill_block_pointers(b, d); });
  return out;
}

/** Eigen vars -> device node (the materialised node itself when m is exactly
 * a host block, else a gathered copy bridged in the reverse sweep). */
template <int R, int C, int O, int MR, int MC>
inline dev_var_matrix to_dev(const Eigen::Matrix<var, R, C, O, MR, MC>& m) {
  return internal::to_dev_vars(m.data(), size_t(m.size()), int(m.rows()), int(m.cols()));
}

inline dev_var_matrix::operator Eigen::Matrix<var, Eigen::Dynamic, Eigen::Dynamic>() const {
  return to_host_matrix<Eigen::Dynamic, Eigen::Dynamic>(*this);
}
inline dev_var_matrix::operator Eigen::Matrix<var, Eigen::Dynamic, 1>() const {
  return to_host_matrix<Eigen::Dynamic, 1>(*this);
}

template <int R, int C, int O, int MR, int MC>
inline dev_data<double> to_dev_data(const Eigen::Matrix<double, R, C, O, MR, MC>& m) {
  return to_dev_data(m.data(), size_t(m.size()), int(m.rows()), int(m.cols()));
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
  matrix_v out(A.rows(), A.cols());
  amd::phase_mark(18);
  // the factor's varis are built as its panels finish (cholesky_decompose_impl).
  // A materialised node (the usual case) is factorised speculatively: the
  // full pointer check runs on the host while the first panels factor, and a
  // mismatch (an element replaced) discards that factorisation for the
  // gathered copy's
  const long k = internal::candidate_block_index(A.data(), size_t(A.size()), int(A.rows()), int(A.cols()));
  amd::phase_mark(19);
  if (k >= 0) {
    auto* node = static_cast<dev_matrix_vari*>(ChainableStack::instance_->host_blocks_[size_t(k)].node);
    const std::function<bool()> verify = [&] { return internal::block_matches(A.data(), size_t(k)); };
    if (internal::cholesky_decompose_impl(dev_var_matrix(node), out.data(), &verify).vi_) return out;
  }
  internal::cholesky_decompose_impl(to_dev(A), out.data());
  return out;
}

/**
 * multiply (rev/mat/fun/multiply.hpp:562-661), every var / double mix:
 *   matrix x matrix / vector, row vector x matrix -> Matrix<var, Ra, Cb> (:619-645);
 *   row vector x vector -> var (:647-661);
 *   scalar x matrix, matrix x scalar (:574-600) and scalar x scalar (:561-565).
 * Same checks first: check_multiplicable, then check_not_nan of A and B.
 */
template <typename Ta, int Ra, int Ca, typename Tb, int Cb,
          typename = std::enable_if_t<internal::is_ad_scalar<Ta>::value && internal::is_ad_scalar<Tb>::value &&
                                      internal::any_var<Ta, Tb>::value>>
inline Eigen::Matrix<var, Ra, Cb> multiply(const Eigen::Matrix<Ta, Ra, Ca>& A, const Eigen::Matrix<Tb, Ca, Cb>& B) {
  internal::check_multiplicable("multiply", int(A.rows()), int(A.cols()), int(B.rows()), int(B.cols()));
  const internal::eig_in a = internal::prepare(A, "multiply", "A");
  const internal::eig_in b = internal::prepare(B, "multiply", "B");
  const internal::dev_operand da = internal::commit(a);
  const internal::dev_operand db = internal::commit(b);
  return to_host_matrix<Ra, Cb>(internal::multiply_dev(da, db));
}
template <typename Ta, int Ca, typename Tb,
          typename = std::enable_if_t<internal::is_ad_scalar<Ta>::value && internal::is_ad_scalar<Tb>::value &&
                                      internal::any_var<Ta, Tb>::value>>
inline var multiply(const Eigen::Matrix<Ta, 1, Ca>& A, const Eigen::Matrix<Tb, Ca, 1>& B) {
  internal::check_multiplicable("multiply", int(A.rows()), int(A.cols()), int(B.rows()), int(B.cols()));
  const internal::eig_in a = internal::prepare(A, "multiply", "A");
  const internal::eig_in b = internal::prepare(B, "multiply", "B");
  const internal::dev_operand da = internal::commit(a);
  const internal::dev_operand db = internal::commit(b);
  return to_host_matrix<1, 1>(internal::multiply_dev(da, db))(0);
}
template <typename T1, typename T2, int R, int C,
          typename = std::enable_if_t<internal::is_ad_scalar<T1>::value && internal::is_ad_scalar<T2>::value &&
                                      internal::any_var<T1, T2>::value>>
inline Eigen::Matrix<var, R, C> multiply(const T1& c, const Eigen::Matrix<T2, R, C>& m) {
  const internal::dev_operand dm = internal::commit(internal::prepare(m));
  const bool cv = internal::is_var<T1>::value;
  vari* c_vi = nullptr;
  double c_val = 0;
  if constexpr (internal::is_var<T1>::value) {
    c_vi = c.vi_;
    c_val = c.val();
  } else {
    c_val = double(c);
  }
  (void)cv;
  auto* node = new internal::scale_dev_vari(dm, c_val, c_vi);
  return to_host_matrix<R, C>(dev_var_matrix(node->B_));
}
template <typename T1, int R, int C, typename T2,
          typename = std::enable_if_t<internal::is_ad_scalar<T1>::value && internal::is_ad_scalar<T2>::value &&
                                      internal::any_var<T1, T2>::value>>
inline Eigen::Matrix<var, R, C> multiply(const Eigen::Matrix<T1, R, C>& m, const T2& c) {
  return multiply(c, m);
}
template <typename T1, typename T2,
          typename = std::enable_if_t<internal::is_ad_scalar<T1>::value && internal::is_ad_scalar<T2>::value &&
                                      internal::any_var<T1, T2>::value>>
inline var multiply(const T1& a, const T2& b) {
  return a * b;
}

/** prim/mat/fun/transpose.hpp: a plain Eigen transpose (shares the varis). */
template <typename T, int R, int C>
inline Eigen::Matrix<T, C, R> transpose(const Eigen::Matrix<T, R, C>& m) {
  return m.transpose();
}

template <int R, int C>
inline var sum(const Eigen::Matrix<var, R, C>& m) {
  return sum(to_dev(m));
}

/**
 * add_diag(mat, to_add) (prim/mat/fun/add_diag.hpp:20-55): to_add a scalar
 * (:20-29) or a vector of min(rows, cols) entries (:42-55), mat and to_add
 * var or double in any combination, mat rectangular or square.
 */
namespace internal {
/** add_diag's Eigen output: mat's own varis off the diagonal, new ones on it
 * (prim/mat/fun/add_diag.hpp:25-27: mat_out(mat), then diagonal() +=);
 * B is the device node of mat + diag(to_add).  A double mat has no varis to
 * share: every element is new, as the reference's var(double) conversions. */
template <typename T_m>
inline matrix_v add_diag_output(const Eigen::Matrix<T_m, Eigen::Dynamic, Eigen::Dynamic>& mat, const eig_in& em,
                                const dev_var_matrix& B) {
  if constexpr (!is_var<T_m>::value) {
    return to_host_matrix(B);
  } else {
    matrix_v out(mat.rows(), mat.cols());
    const long base = em.block;
    vari** elems = nullptr;
    if (base < 0 && em.n) {  // mat is no block: its pointers, for recognising the output later
      elems = ChainableStack::instance_->memalloc_.alloc_array<vari*>(em.n);
      host_parallel_for(em.n, [&](size_t s, size_t e) {
        for (size_t i = s; i < e; ++i) elems[i] = em.vd[i].vi_;
      });
    }
    const size_t k = materialise_diag(B.vi_, base, elems);
    fill_block_pointers(ChainableStack::instance_->host_blocks_[k], out.data());
    return out;
  }
}
}  // namespace internal

template <typename T_m, typename T_a,
          typename = std::enable_if_t<internal::is_ad_scalar<T_m>::value && internal::is_ad_scalar<T_a>::value &&
                                      internal::any_var<T_m, T_a>::value>>
inline matrix_v add_diag(const Eigen::Matrix<T_m, Eigen::Dynamic, Eigen::Dynamic>& mat, const T_a& to_add) {
  const internal::eig_in em = internal::prepare(mat);
  const internal::dev_operand a = internal::commit(em);
  if constexpr (internal::is_var<T_a>::value)
    return internal::add_diag_output(mat, em, internal::add_diag_dev(a, to_add.val(), to_add.vi_, {}));
  else
    return internal::add_diag_output(mat, em, internal::add_diag_dev(a, double(to_add), nullptr, {}));
}
template <typename T_m, typename T_a, int R, int C,
          typename = std::enable_if_t<internal::is_ad_scalar<T_m>::value && internal::is_ad_scalar<T_a>::value &&
                                      internal::any_var<T_m, T_a>::value>>
inline matrix_v add_diag(const Eigen::Matrix<T_m, Eigen::Dynamic, Eigen::Dynamic>& mat,
                         const Eigen::Matrix<T_a, R, C>& to_add) {
  const size_t k = size_t(std::min(mat.rows(), mat.cols()));
  if (size_t(to_add.size()) != k) {  // check_consistent_size before anything is built
    std::ostringstream m;
    m << "add_diag: number of elements of to_add has dimension = " << to_add.size() << ", expecting dimension = " << k
      << "; a function was called with arguments of different scalar, array, vector, or matrix types, and they "
         "were not consistently sized;  all arguments must be scalars or multidimensional values of the same shape.";
    throw std::invalid_argument(m.str());
  }
  const internal::eig_in em = internal::prepare(mat);
  const internal::eig_in ed = internal::prepare(to_add);
  const internal::dev_operand a = internal::commit(em);
  internal::dev_operand d = internal::commit(ed);
  d.rows = int(d.size());
  d.cols = 1;
  return internal::add_diag_output(mat, em, internal::add_diag_dev(a, 0.0, nullptr, d));
}

template <int R, int C>
inline var log_sum_exp(const Eigen::Matrix<var, R, C>& x) {
  return log_sum_exp(to_dev(x));
}
template <int R, int C>
inline Eigen::Matrix<var, R, C> lgamma(const Eigen::Matrix<var, R, C>& x) {
  return to_host_matrix<R, C>(lgamma(to_dev(x)));
}
template <int R, int C>
inline Eigen::Matrix<var, R, C> digamma(const Eigen::Matrix<var, R, C>& x) {
  return to_host_matrix<R, C>(digamma(to_dev(x)));
}

/** mdivide_left_tri<TriView>(A, b), rev/mat/fun/mdivide_left_tri.hpp:311-373
 * (vv, dv, vd): C = tri(A)^{-1} b with b's static column count. */
template <int TriView, typename T1, int R1, int C1, typename T2, int R2, int C2,
          typename = std::enable_if_t<internal::is_ad_scalar<T1>::value && internal::is_ad_scalar<T2>::value &&
                                      internal::any_var<T1, T2>::value>>
inline Eigen::Matrix<var, R1, C2> mdivide_left_tri(const Eigen::Matrix<T1, R1, C1>& A,
                                                   const Eigen::Matrix<T2, R2, C2>& b) {
  internal::check_square("mdivide_left_tri", "A", int(A.rows()), int(A.cols()));
  internal::check_multiplicable("mdivide_left_tri", int(A.rows()), int(A.cols()), int(b.rows()), int(b.cols()), "A",
                                "b");
  const internal::dev_operand a = internal::commit(internal::prepare(A));
  const internal::dev_operand bb = internal::commit(internal::prepare(b));
  return to_host_matrix<R1, C2>(internal::mdivide_left_tri_dev<TriView>(a, bb));
}
template <int TriView, int R, int C>
inline Eigen::Matrix<var, R, C> mdivide_left_tri(const Eigen::Matrix<var, R, C>& A) {
  return to_host_matrix<R, C>(mdivide_left_tri<TriView>(to_dev(A)));
}
/** prim/mat/fun/mdivide_left_tri.hpp:25-44 on data (host, Eigen's triangular solve) */
template <int TriView, int R1, int C1, int R2, int C2>
inline Eigen::Matrix<double, R1, C2> mdivide_left_tri(const Eigen::Matrix<double, R1, C1>& A,
                                                      const Eigen::Matrix<double, R2, C2>& b) {
  internal::check_square("mdivide_left_tri", "A", int(A.rows()), int(A.cols()));
  internal::check_multiplicable("mdivide_left_tri", int(A.rows()), int(A.cols()), int(b.rows()), int(b.cols()), "A",
                                "b");
  return A.template triangularView<Eigen::UpLoType(TriView)>().solve(b);
}

/** mdivide_left_tri_low(A, b) = mdivide_left_tri<Lower>(A, b) after the
 * reference's own checks (prim/mat/fun/mdivide_left_tri_low.hpp:33-47), and
 * the one-argument form tril(A)^{-1} -- the name Stan-generated code emits. */
template <typename T1, int R1, int C1, typename T2, int R2, int C2,
          typename = std::enable_if_t<internal::is_ad_scalar<T1>::value && internal::is_ad_scalar<T2>::value>>
inline auto mdivide_left_tri_low(const Eigen::Matrix<T1, R1, C1>& A, const Eigen::Matrix<T2, R2, C2>& b) {
  internal::check_square("mdivide_left_tri_low", "A", int(A.rows()), int(A.cols()));
  internal::check_multiplicable("mdivide_left_tri_low", int(A.rows()), int(A.cols()), int(b.rows()), int(b.cols()),
                                "A", "b");
  return mdivide_left_tri<Eigen::Lower>(A, b);
}
template <typename T, int R1, int C1, typename = std::enable_if_t<internal::is_ad_scalar<T>::value>>
inline Eigen::Matrix<T, R1, C1> mdivide_left_tri_low(const Eigen::Matrix<T, R1, C1>& A) {
  internal::check_square("mdivide_left_tri_low", "A", int(A.rows()), int(A.cols()));
  if constexpr (internal::is_var<T>::value) {
    return mdivide_left_tri<Eigen::Lower>(A);
  } else {
    const Eigen::Matrix<double, R1, C1> I = Eigen::Matrix<double, R1, C1>::Identity(A.rows(), A.cols());
    return A.template triangularView<Eigen::Lower>().solve(I);
  }
}

/** mdivide_right_tri_low(b, A) = b tril(A)^{-1} (prim/mat/fun/
 * mdivide_right_tri_low.hpp:25-31 -> mdivide_right_tri<Lower>,
 * prim/mat/fun/mdivide_right_tri.hpp:28-48: check_square, then
 * check_multiplicable(b, A)).  On the device as (tril(A)^{-T} b^T)^T: the
 * transposes are Eigen pointer copies (they share the varis, as the
 * reference's transpose does), the solve is mdivide_left_tri<Upper>. */
template <typename T1, int R1, int C1, typename T2, int R2, int C2,
          typename = std::enable_if_t<internal::is_ad_scalar<T1>::value && internal::is_ad_scalar<T2>::value>>
inline auto mdivide_right_tri_low(const Eigen::Matrix<T1, R1, C1>& b, const Eigen::Matrix<T2, R2, C2>& A) {
  internal::check_square("mdivide_right_tri", "A", int(A.rows()), int(A.cols()));
  internal::check_multiplicable("mdivide_right_tri", int(b.rows()), int(b.cols()), int(A.rows()), int(A.cols()), "b",
                                "A");
  using R = std::conditional_t<internal::any_var<T1, T2>::value, var, double>;
  const Eigen::Matrix<T2, C2, R2> At = A.transpose();
  const Eigen::Matrix<T1, C1, R1> bt = b.transpose();
  const Eigen::Matrix<R, C2, R1> xt = mdivide_left_tri<Eigen::Upper>(At, bt);
  return Eigen::Matrix<R, R1, C2>(xt.transpose());
}

// ------------------------------------------------ §8(f) row 3 (spd_functors.hpp)
/** rev/mat/fun/mdivide_left_spd.hpp:232-260 signatures: Matrix<var, R1, C2>. */
template <typename T1, int R1, int C1, typename T2, int R2, int C2,
          typename = std::enable_if_t<internal::is_ad_scalar<T1>::value && internal::is_ad_scalar<T2>::value &&
                                      internal::any_var<T1, T2>::value>>
inline Eigen::Matrix<var, R1, C2> mdivide_left_spd(const Eigen::Matrix<T1, R1, C1>& A,
                                                   const Eigen::Matrix<T2, R2, C2>& b) {
  internal::check_square("mdivide_left_spd", "A", int(A.rows()), int(A.cols()));
  internal::check_multiplicable_named("mdivide_left_spd", "A", int(A.cols()), "b", int(b.rows()));
  const internal::dev_operand a = internal::commit(internal::prepare(A));
  const internal::dev_operand bb = internal::commit(internal::prepare(b));
  return to_host_matrix<R1, C2>(internal::mdivide_left_spd_dev(a, bb));
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
  return log_determinant(to_dev_data(md));
}
/** rev/mat/fun/multiply_lower_tri_self_transpose.hpp:14 signature. */
inline matrix_v multiply_lower_tri_self_transpose(const matrix_v& L) {
  if (L.rows() == 0) return matrix_v(0, 0);
  return to_host_matrix(multiply_lower_tri_self_transpose(to_dev(L)));
}
/** rev/mat/fun/quad_form_sym.hpp:15-40 signatures (matrix B -> Matrix<var, Cb, Cb>, vector b -> var). */
template <typename Ta, int Ra, int Ca, typename Tb, int Rb, int Cb,
          typename = std::enable_if_t<(Cb != 1) && internal::is_ad_scalar<Ta>::value &&
                                      internal::is_ad_scalar<Tb>::value && internal::any_var<Ta, Tb>::value>>
inline Eigen::Matrix<var, Cb, Cb> quad_form_sym(const Eigen::Matrix<Ta, Ra, Ca>& A,
                                                const Eigen::Matrix<Tb, Rb, Cb>& B) {
  const internal::dev_operand a = internal::commit(internal::prepare(A));
  const internal::dev_operand b = internal::commit(internal::prepare(B));
  return to_host_matrix<Cb, Cb>(internal::quad_form_sym_dev(a, b));
}
template <typename Ta, int Ra, int Ca, typename Tb, int Rb,
          typename = std::enable_if_t<internal::is_ad_scalar<Ta>::value && internal::is_ad_scalar<Tb>::value &&
                                      internal::any_var<Ta, Tb>::value>>
inline var quad_form_sym(const Eigen::Matrix<Ta, Ra, Ca>& A, const Eigen::Matrix<Tb, Rb, 1>& b) {
  const internal::dev_operand a = internal::commit(internal::prepare(A));
  const internal::dev_operand bb = internal::commit(internal::prepare(b));
  return to_host_matrix<1, 1>(internal::quad_form_sym_dev(a, bb))(0);
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

// ------------------------------------------------ multi_normal_cholesky_lpdf
namespace internal {

/** vector_seq_view (prim/mat/meta/vector_seq_view.hpp): one vector or a
 * std::vector of vectors, as a list of (data pointer, size). */
template <typename S, int R, int C>
inline void seq_of(const Eigen::Matrix<S, R, C>& v, std::vector<const S*>& p, std::vector<int>& n) {
  p.push_back(v.data());
  n.push_back(int(v.size()));
}
template <typename S, int R, int C, typename A>
inline void seq_of(const std::vector<Eigen::Matrix<S, R, C>, A>& v, std::vector<const S*>& p, std::vector<int>& n) {
  for (const auto& e : v) {
    p.push_back(e.data());
    n.push_back(int(e.size()));
  }
}
template <typename T>
struct is_array_mvt : std::false_type {};
template <typename T, typename A>
struct is_array_mvt<std::vector<T, A>> : std::true_type {};

inline double host_value(const double& x) { return x; }
inline double host_value(const var& x) { return x.vi_->val_; }

/** check_consistent_size_mvt (prim/mat/err/check_consistent_size_mvt.hpp),
 * including its reported size (the inner size_x shadows the outer one, so
 * the message says 0). */
template <typename T>
inline void check_consistent_size_mvt(const char* fn, const char* name, const T& x, size_t expected) {
  size_t len;
  if constexpr (is_array_mvt<T>::value)
    len = x.size();
  else
    len = size_t(x.size());
  if (len == 0) {
    if (expected == 0) return;
  } else {
    if (!is_array_mvt<T>::value) return;  // x[0] is a scalar: nothing to check
    if (expected == len) return;
  }
  std::ostringstream m;
  m << fn << ": " << name << " has dimension = 0, expecting dimension = " << expected
    << "; a function was called with arguments of different scalar, array, vector, or matrix types, and they "
       "were not consistently sized;  all arguments must be scalars or multidimensional values of the same shape.";
  throw std::invalid_argument(m.str());
}

inline void size_match(const char* fn, const char* n1, long long x1, const char* n2, long long x2) {
  if (x1 == x2) return;
  std::ostringstream m;
  m << fn << ": " << n1 << " (" << x1 << ") and " << n2 << " (" << x2 << ") must match in size";
  throw std::invalid_argument(m.str());
}

/** The observations of one mvn argument on the device: a single (n x k)
 * buffer (one gather / upload for every observation). */
template <typename S>
struct mvt_dev {
  std::vector<const double*> val;
  std::vector<double*> adj;
};
inline mvt_dev<double> mvt_to_dev(const std::vector<const double*>& p, int n) {
  std::vector<double> h;
  h.reserve(p.size() * size_t(n));
  for (const double* e : p) h.insert(h.end(), e, e + n);
  dev_data<double> d = to_dev_data(h.data(), h.size(), n, int(p.size()));
  mvt_dev<double> out;
  for (size_t i = 0; i < p.size(); ++i) {
    out.val.push_back(d.data() + i * size_t(n));
    out.adj.push_back(nullptr);
  }
  return out;
}
inline mvt_dev<var> mvt_to_dev(const std::vector<const var*>& p, int n) {
  dev_matrix_vari* node = nullptr;
  if (p.size() == 1) {
    node = to_dev_vars(p[0], size_t(n), n, 1).vi_;
  } else {
    std::vector<var> h;
    h.reserve(p.size() * size_t(n));
    for (const var* e : p) h.insert(h.end(), e, e + n);
    node = to_dev_vars(h.data(), h.size(), n, int(p.size())).vi_;
  }
  mvt_dev<var> out;
  for (size_t i = 0; i < p.size(); ++i) {
    out.val.push_back(node->val_ + i * size_t(n));
    out.adj.push_back(node->adj_ + i * size_t(n));
  }
  return out;
}

}  // namespace internal

/**
 * multi_normal_cholesky_lpdf<propto>(y | mu, L)
 * (prim/mat/prob/multi_normal_cholesky_lpdf.hpp:40-166), every combination
 * the reference accepts: y and mu each an Eigen column / row vector of var or
 * double or a std::vector of them (vector_seq_view, :59-80; a single vector
 * is broadcast over the other's observations), L an Eigen matrix of var or
 * double or a device matrix node.  The reference's checks in its order, the
 * same early returns, the same include_summand<propto, ...> terms; the value
 * and the partials are computed on the device per observation (two
 * triangular solves each, no explicit inverse) and summed into one node.
 * Returns var when any argument is var, else double.
 */
template <bool propto = false, typename T_y, typename T_loc, typename T_covar,
          typename = std::enable_if_t<internal::is_mvt_arg<T_y>::value && internal::is_mvt_arg<T_loc>::value &&
                                      (internal::is_ad_scalar<typename internal::scalar_of<T_covar>::type>::value)>>
inline std::conditional_t<internal::any_var<T_y, T_loc, T_covar>::value, var, double> multi_normal_cholesky_lpdf(
    const T_y& y, const T_loc& mu, const T_covar& L) {
  using S_y = typename internal::scalar_of<T_y>::type;
  using S_mu = typename internal::scalar_of<T_loc>::type;
  using S_L = typename internal::scalar_of<T_covar>::type;
  using ret_t = std::conditional_t<internal::any_var<T_y, T_loc, T_covar>::value, var, double>;
  constexpr bool L_var = internal::is_var<S_L>::value;
  constexpr bool any_v = internal::any_var<T_y, T_loc, T_covar>::value;
  const char* fn = "multi_normal_cholesky_lpdf";
  // check_consistent_sizes_mvt(function, "y", y, "mu", mu) (:52)
  const size_t len_y = internal::is_array_mvt<T_y>::value ? size_t(y.size()) : 1;
  const size_t len_mu = internal::is_array_mvt<T_loc>::value ? size_t(mu.size()) : 1;
  const size_t max_len = std::max(len_y, len_mu);
  internal::check_consistent_size_mvt(fn, "y", y, max_len);
  internal::check_consistent_size_mvt(fn, "mu", mu, max_len);
  if (len_y == 0 || len_mu == 0) return ret_t(0.0);
  std::vector<const S_y*> py;
  std::vector<const S_mu*> pm;
  std::vector<int> ny, nm;
  internal::seq_of(y, py, ny);
  internal::seq_of(mu, pm, nm);
  const size_t size_vec = max_len;
  const int size_y = ny[0], size_mu = nm[0];
  if (size_vec > 1) {  // :65-89
    for (size_t i = 1; i < ny.size(); ++i)
      internal::size_match(fn, "Size of one of the vectors of the random variable", ny[i],
                           "Size of another vector of the random variable", ny[i - 1]);
    for (size_t i = 1; i < nm.size(); ++i)
      internal::size_match(fn, "Size of one of the vectors of the location variable", nm[i],
                           "Size of another vector of the location variable", nm[i - 1]);
  }
  internal::size_match(fn, "Size of random variable", size_y, "size of location parameter", size_mu);
  internal::size_match(fn, "Size of random variable", size_y, "rows of covariance parameter", (long long)L.rows());
  internal::size_match(fn, "Size of random variable", size_y, "columns of covariance parameter",
                       (long long)L.cols());
  for (size_t i = 0; i < size_vec; ++i) {  // :100-103
    const S_mu* m = pm[len_mu > 1 ? i : 0];
    for (int j = 0; j < size_mu; ++j) {
      const double v = internal::host_value(m[j]);
      if (!std::isfinite(v)) {
        std::ostringstream o;
        o << fn << ": Location parameter[" << j + 1 << "] is " << v << ", but must be finite!";
        throw std::domain_error(o.str());
      }
    }
    const S_y* yy = py[len_y > 1 ? i : 0];
    for (int j = 0; j < size_y; ++j)
      if (std::isnan(internal::host_value(yy[j]))) {
        std::ostringstream o;
        o << fn << ": Random variable[" << j + 1 << "] is nan, but must not be nan!";
        throw std::domain_error(o.str());
      }
  }
  if (size_y == 0) return ret_t(0.0);
  if (propto && !any_v) return ret_t(0.0);  // every include_summand<propto, ...> is false
  // L on the device: a var node (recognised block / gathered) or data
  internal::dev_operand Ld;
  const double* aux = nullptr;
  bool lower_only = false;
  double host_logdet = 0.0;
  if constexpr (std::is_same<T_covar, dev_var_matrix>::value) {
    Ld = internal::operand(L);
    aux = L.vi_->aux_;
    lower_only = L.vi_->structure_ == dev_structure::lower;
  } else {
    const internal::eig_in eL = internal::prepare(L);
    Ld = internal::commit(eL);
    if (Ld.vi) {
      aux = Ld.vi->aux_;
      lower_only = Ld.vi->structure_ == dev_structure::lower;
    }
    if (!L_var && propto)  // the -log|L| term is dropped (include_summand<propto, T_covar_elem>)
      for (int i = 0; i < size_y; ++i) host_logdet += std::log(1.0 / internal::host_value(L(i, i)));
  }
  const internal::mvt_dev<S_y> dy = internal::mvt_to_dev(py, size_y);
  const internal::mvt_dev<S_mu> dm = internal::mvt_to_dev(pm, size_y);
  auto* obs = ChainableStack::instance_->memalloc_.alloc_array<internal::mvn_obs>(size_vec);
  for (size_t i = 0; i < size_vec; ++i) {
    const size_t iy = len_y > 1 ? i : 0, im = len_mu > 1 ? i : 0;
    obs[i] = internal::mvn_obs{dy.val[iy], dy.adj[iy], dm.val[im], dm.adj[im]};
  }
  double lp = 0.0;
  vari* node = internal::mvn_cholesky_multi(Ld, aux, lower_only, obs, int(size_vec), !propto, !propto || L_var,
                                            host_logdet, &lp);
  if constexpr (any_v)
    return node ? var(node) : var(lp);
  else
    return lp;
}

// ------------------------------------------------ D-dimensional gp_exp_quad_cov
namespace internal {
/** x (std::vector of D-vectors) -> device D x n, with the reference's checks:
 * check_not_nan(x[i]) per point (index within the point), then the first
 * size mismatch squared_distance(x[i], x[0]) meets (:158-170). */
template <typename T_x>
inline dev_data<double> gp_points_to_device(const std::vector<T_x>& x, int& D) {
  const size_t n = x.size();
  D = n ? int(x[0].size()) : 1;
  for (size_t i = 0; i < n; ++i)
    for (int d = 0; d < int(x[i].size()); ++d)
      if (std::isnan(x[i](d))) {
        std::ostringstream m;
        m << "gp_exp_quad_cov: x[" << d + 1 << "] is nan, but must not be nan!";
        throw std::domain_error(m.str());
      }
  for (size_t i = 1; i < n; ++i)
    if (int(x[i].size()) != D) {
      std::ostringstream m;
      m << "squared_distance: size of v1 (" << x[i].size() << ") and size of v2 (" << D << ") must match in size";
      throw std::invalid_argument(m.str());
    }
  std::vector<double> h(n * size_t(D));
  for (size_t i = 0; i < n; ++i)
    for (int d = 0; d < D; ++d) h[i * size_t(D) + size_t(d)] = x[i](d);
  return to_dev_data(h.data(), h.size(), D, int(n));
}
}  // namespace internal

/**
 * gp_exp_quad_cov(std::vector<T_x> x, sigma, length_scale) with T_x an Eigen
 * vector of doubles (rev/mat/fun/gp_exp_quad_cov.hpp:211-286): (var, var) and
 * (double, var) with the reference's argument names, and (var, double) as the
 * prim template (prim/mat/fun/gp_exp_quad_cov.hpp:175-198).  K on the device
 * (smg_gp_exp_quad_cov_nd_*), converting to Eigen::Matrix<var, -1, -1>.
 */
template <int R, int C, typename A>
inline dev_var_matrix gp_exp_quad_cov(const std::vector<Eigen::Matrix<double, R, C>, A>& x, const var& sigma,
                                      const var& length_scale) {
  internal::gp_check_positive("gp_exp_quad_cov", "sigma", sigma.val());
  internal::gp_check_positive("gp_exp_quad_cov", "length_scale", length_scale.val());
  int D = 1;
  const dev_data<double> xd = internal::gp_points_to_device(x, D);
  return internal::gp_exp_quad_cov_dev(xd, D, sigma.val(), sigma.vi_, length_scale.val(), length_scale.vi_);
}
template <int R, int C, typename A>
inline dev_var_matrix gp_exp_quad_cov(const std::vector<Eigen::Matrix<double, R, C>, A>& x, double sigma,
                                      const var& length_scale) {
  internal::gp_check_positive("gp_exp_quad_cov", "marginal variance", sigma);
  internal::gp_check_positive("gp_exp_quad_cov", "length-scale", length_scale.val());
  int D = 1;
  const dev_data<double> xd = internal::gp_points_to_device(x, D);
  return internal::gp_exp_quad_cov_dev(xd, D, sigma, nullptr, length_scale.val(), length_scale.vi_);
}
template <int R, int C, typename A>
inline dev_var_matrix gp_exp_quad_cov(const std::vector<Eigen::Matrix<double, R, C>, A>& x, const var& sigma,
                                      double length_scale) {
  internal::gp_check_positive("gp_exp_quad_cov", "magnitude", sigma.val());
  internal::gp_check_positive("gp_exp_quad_cov", "length scale", length_scale);
  int D = 1;
  const dev_data<double> xd = internal::gp_points_to_device(x, D);
  return internal::gp_exp_quad_cov_dev(xd, D, sigma.val(), sigma.vi_, length_scale, nullptr, "magnitude",
                                       "length scale");
}

}  // namespace math
}  // namespace stan
#endif
