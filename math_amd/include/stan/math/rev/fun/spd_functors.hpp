#ifndef STAN_MATH_REV_FUN_SPD_FUNCTORS_HPP
#define STAN_MATH_REV_FUN_SPD_FUNCTORS_HPP

// SURVEY.md §8(f) row 3 -- the GP toolbox beyond cholesky_decompose, on
// device matrices, without explicit inverses in the forward:
//   mdivide_left_spd(A, b)                rev/mat/fun/mdivide_left_spd.hpp:20-260
//   log_determinant_spd(m)                rev/mat/fun/log_determinant_spd.hpp:16-57
//   multiply_lower_tri_self_transpose(L)  rev/mat/fun/multiply_lower_tri_self_transpose.hpp:14-44
//   quad_form_sym(A, B)                   rev/mat/fun/quad_form_sym.hpp:15-40
// Each is one vari over device operands (smg_* entries in spd.hip).  Checks,
// in the reference's order, before the tape is touched:
//   * mdivide_left_spd: check_square(A), check_multiplicable(A, b)
//     (:237-238).  The rev reference factors A without a check (Eigen's LLT
//     of a non-SPD matrix yields garbage); here a failed factorisation throws
//     the prim overload's check_pos_definite error instead
//     (prim/mat/fun/mdivide_left_spd.hpp:29).
//   * log_determinant_spd: check_symmetric (:18), size 0 -> 0 (:19-20), a
//     failed factorisation -> "matrix argument matrix is negative definite"
//     (:35-39, the reference's domain_error formatting), check_finite of the
//     value (:43-44).
//   * quad_form_sym: with A and B both var the reference resolves to the prim
//     template (prim/mat/fun/quad_form_sym.hpp:11-18: check_multiplicable,
//     check_symmetric, autodiff of 0.5 (Cd + Cd^T), i.e. a symmetrised
//     adjoint); mixed operands take the rev vari (check_symmetric,
//     check_multiplicable, rev/mat/fun/quad_form_sym.hpp:19-20).

#include <stan/math/amd/matrix.hpp>
#include <stan/math/rev/core.hpp>
#include <stan/math/rev/fun/cholesky_decompose.hpp>
#include <stan/math/rev/fun/multiply.hpp>

#include <cmath>
#include <sstream>
#include <stdexcept>
#include <string>

namespace stan {
namespace math {
namespace internal {

inline void check_multiplicable_named(const char* fn, const char* n1, int c1, const char* n2, int r2) {
  if (c1 != r2) {
    std::ostringstream m;
    m << fn << ": Columns of " << n1 << " (" << c1 << ") and Rows of " << n2 << " (" << r2
      << ") must match in size";
    throw std::invalid_argument(m.str());
  }
}

inline void check_symmetric_dev(const char* fn, const char* name, const double* A, int n) {
  smg_ctx* c = amd::ctx();
  amd::check(smg_check_symmetric(c, A, n, n), fn);
  int st = 0;
  amd::check(smg_status(c, &st), fn);
  if (st & SMG_ERR_NOT_SYMMETRIC) throw_not_symmetric_dev(fn, name, A, n);
  if (st) amd::throw_status(st, fn, name);
}

// ---------------------------------------------------------------- mdivide_left_spd
class mdivide_left_spd_dev_vari : public device_vari {
 public:
  dev_operand A_, B_;
  double* L_;
  double* aux_;
  dev_matrix_vari* C_;
  mdivide_left_spd_dev_vari(const dev_operand& A, const dev_operand& B)
      : device_vari(0.0), A_(A), B_(B), C_(new dev_matrix_vari(B.rows, B.cols)) {
    static const char* fn = "mdivide_left_spd";
    const int m = A.rows;
    smg_ctx* c = amd::ctx();
    L_ = amd::alloc_doubles(size_t(m) * m);
    aux_ = amd::alloc_doubles(size_t(smg_cholesky_aux_doubles(m)));
    amd::check(smg_mdivide_left_spd_fwd(c, A_.val(), m, B_.val(), m, m, B_.cols, L_, aux_, C_->val_, m),
               fn);
    int st = 0;
    amd::check(smg_status(c, &st), fn);
    if (st & SMG_ERR_NOT_PD) {
      std::ostringstream msg;
      msg << fn << ": A is not positive definite.";
      throw std::domain_error(msg.str());
    }
    if (st) amd::throw_status(st, fn, "A");
  }
  void chain() override {
    const int m = B_.rows, n = B_.cols;
    if (!A_.adj() && !B_.adj()) return;
    double* ws = amd::alloc_doubles(size_t(m) * n);
    amd::check(smg_mdivide_left_spd_rev(amd::ctx(), L_, aux_, m, n, C_->val_, m, C_->adj_, m, A_.adj(), m,
                                        B_.adj(), m, ws),
               "mdivide_left_spd");
  }
};

inline dev_var_matrix mdivide_left_spd_dev(const dev_operand& A, const dev_operand& B) {
  check_square("mdivide_left_spd", "A", A.rows, A.cols);
  check_multiplicable_named("mdivide_left_spd", "A", A.cols, "b", B.rows);
  auto* node = new mdivide_left_spd_dev_vari(A, B);
  return dev_var_matrix(node->C_);
}

// ---------------------------------------------------------------- log_determinant_spd
class log_determinant_spd_dev_vari : public device_vari {
 public:
  dev_matrix_vari* A_;
  double* L_;
  double* aux_;
  log_determinant_spd_dev_vari(double v, dev_matrix_vari* A, double* L, double* aux)
      : device_vari(v), A_(A), L_(L), aux_(aux) {}
  void chain() override {
    const int n = A_->rows_;
    double* ws = amd::alloc_doubles(size_t(n) * n);
    amd::check(smg_log_determinant_spd_rev(amd::ctx(), L_, aux_, n, adj_, A_->adj_, n, ws),
               "log_determinant_spd");
  }
};

// ---------------------------------------------------------------- multiply_lower_tri_self_transpose
class mlt_self_transpose_dev_vari : public device_vari {
 public:
  dev_matrix_vari* L_;
  dev_matrix_vari* C_;
  explicit mlt_self_transpose_dev_vari(dev_matrix_vari* L)
      : device_vari(0.0), L_(L), C_(new dev_matrix_vari(L->rows_, L->rows_)) {
    const int K = L->rows_, J = L->cols_;
    double* ws = amd::alloc_doubles(size_t(K) * (J > 0 ? J : 1));
    amd::check(smg_multiply_lower_tri_self_transpose_fwd(amd::ctx(), L_->val_, K, K, J, C_->val_, K, ws),
               "multiply_lower_tri_self_transpose");
  }
  void chain() override {
    const int K = L_->rows_, J = L_->cols_;
    double* ws = amd::alloc_doubles(size_t(2) * K * J + size_t(K) * K);
    amd::check(smg_multiply_lower_tri_self_transpose_rev(amd::ctx(), L_->val_, K, K, J, C_->adj_, K,
                                                         L_->adj_, K, ws),
               "multiply_lower_tri_self_transpose");
  }
};

// ---------------------------------------------------------------- quad_form_sym
class quad_form_sym_dev_vari : public device_vari {
 public:
  dev_operand A_, B_;
  dev_matrix_vari* C_;
  const int sym_adj_;
  quad_form_sym_dev_vari(const dev_operand& A, const dev_operand& B)
      : device_vari(0.0), A_(A), B_(B), C_(new dev_matrix_vari(B.cols, B.cols)),
        sym_adj_(A.vi && B.vi ? 1 : 0) {
    const int M = B.rows, N = B.cols;
    double* ws = amd::alloc_doubles(size_t(M) * N + size_t(N) * N);
    amd::check(smg_quad_form_sym_fwd(amd::ctx(), A_.val(), M, B_.val(), M, M, N, C_->val_, N, ws),
               "quad_form_sym");
  }
  void chain() override {
    const int M = B_.rows, N = B_.cols;
    if (!A_.adj() && !B_.adj()) return;
    double* ws = amd::alloc_doubles(size_t(M) * N + size_t(N) * N);
    amd::check(smg_quad_form_sym_rev(amd::ctx(), A_.val(), M, B_.val(), M, M, N, C_->adj_, N, sym_adj_,
                                     A_.adj(), M, B_.adj(), M, ws),
               "quad_form_sym");
  }
};

// (var, var): the prim template -- check_multiplicable, then check_symmetric
// (prim/mat/fun/quad_form_sym.hpp:14-15); mixed: the rev overload --
// check_symmetric, then check_multiplicable (rev/mat/fun/quad_form_sym.hpp:19-20)
inline dev_var_matrix quad_form_sym_dev(const dev_operand& A, const dev_operand& B) {
  static const char* fn = "quad_form_sym";
  check_square(fn, "A", A.rows, A.cols);
  if (A.vi && B.vi) {
    check_multiplicable_named(fn, "A", A.cols, "B", B.rows);
    check_symmetric_dev(fn, "A", A.val(), A.rows);
  } else {
    check_symmetric_dev(fn, "A", A.val(), A.rows);
    check_multiplicable_named(fn, "A", A.cols, "B", B.rows);
  }
  auto* node = new quad_form_sym_dev_vari(A, B);
  return dev_var_matrix(node->C_);
}

}  // namespace internal

/** A^{-1} b for symmetric positive-definite A (lower triangle read). */
inline dev_var_matrix mdivide_left_spd(const dev_var_matrix& A, const dev_var_matrix& b) {
  return internal::mdivide_left_spd_dev(internal::operand(A), internal::operand(b));
}
inline dev_var_matrix mdivide_left_spd(const dev_data<double>& A, const dev_var_matrix& b) {
  return internal::mdivide_left_spd_dev(internal::operand(A), internal::operand(b));
}
inline dev_var_matrix mdivide_left_spd(const dev_var_matrix& A, const dev_data<double>& b) {
  return internal::mdivide_left_spd_dev(internal::operand(A), internal::operand(b));
}

/** log det(m) of a symmetric positive-definite m. */
inline var log_determinant_spd(const dev_var_matrix& m) {
  static const char* fn = "log_determinant_spd";
  internal::check_square(fn, "m", m.rows(), m.cols());
  const int n = m.rows();
  internal::check_symmetric_dev(fn, "m", m.val_ptr(), n);
  if (n == 0) return var(0.0);
  smg_ctx* c = amd::ctx();
  double* L = amd::alloc_doubles(size_t(n) * n);
  double* aux = amd::alloc_doubles(size_t(smg_cholesky_aux_doubles(n)));
  double* out = amd::alloc_doubles(1);
  amd::check(smg_log_determinant_spd_fwd(c, m.val_ptr(), n, n, L, aux, out), fn);
  double v = 0.0;
  amd::to_host(&v, out, 1);
  int st = 0;
  amd::check(smg_status(c, &st), fn);
  if (st & SMG_ERR_NOT_PD)  // domain_error(fn, "matrix argument", 0, "matrix is negative definite")
    throw std::domain_error(std::string(fn) + ": matrix argument matrix is negative definite0");
  if (st) amd::throw_status(st, fn, "m");
  if (!std::isfinite(v)) {
    std::ostringstream msg;
    msg << fn << ": log determininant of the matrix argument is " << v << ", but must be finite!";
    throw std::domain_error(msg.str());
  }
  return var(new internal::log_determinant_spd_dev_vari(v, m.vi_, L, aux));
}

/** L_lower L_lower^T for a K x J matrix L (entries above the diagonal ignored). */
inline dev_var_matrix multiply_lower_tri_self_transpose(const dev_var_matrix& L) {
  if (L.rows() == 0) return dev_var_matrix(new dev_matrix_vari(0, 0));
  auto* node = new internal::mlt_self_transpose_dev_vari(L.vi_);
  return dev_var_matrix(node->C_);
}

/** B^T A B, symmetrised, for symmetric A. */
inline dev_var_matrix quad_form_sym(const dev_var_matrix& A, const dev_var_matrix& B) {
  return internal::quad_form_sym_dev(internal::operand(A), internal::operand(B));
}
inline dev_var_matrix quad_form_sym(const dev_data<double>& A, const dev_var_matrix& B) {
  return internal::quad_form_sym_dev(internal::operand(A), internal::operand(B));
}
inline dev_var_matrix quad_form_sym(const dev_var_matrix& A, const dev_data<double>& B) {
  return internal::quad_form_sym_dev(internal::operand(A), internal::operand(B));
}

}  // namespace math
}  // namespace stan
#endif
