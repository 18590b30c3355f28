#ifndef STAN_MATH_REV_FUN_MULTIPLY_HPP
#define STAN_MATH_REV_FUN_MULTIPLY_HPP

// multiply / transpose / sum on device matrices of vars.
//
// multiply (rev/mat/fun/multiply.hpp:619-661, multiply_mat_vari :35-552):
//   C = A B;  reverse Aadj += Cadj B^T, Badj += A^T Cadj (MFMA fp64 GEMMs,
//   smg_multiply_*).  var*var, var*double and double*var operand kinds, and
//   scalar * matrix (:562-600): B = c A, Aadj += c Badj, c' += <Badj, A>.
// Same size check as :623-625 (check_multiplicable) before the tape is touched.
//
// transpose: the reference's transpose(Matrix<var>) shares the varis; here it
// is a node whose reverse adds Badj^T into Aadj (one tiled copy each way).
//
// sum (rev/mat/fun/sum.hpp:18-60): value = deterministic device reduction;
// reverse Aadj += adj.  On a structurally lower matrix (cholesky_decompose
// output) the upper entries are the reference's dummy vari and get nothing.

#include <stan/math/amd/matrix.hpp>
#include <stan/math/rev/core.hpp>

#include <sstream>
#include <stdexcept>

namespace stan {
namespace math {

namespace internal {

/** check_positive(function, name, expr, size) (prim/scal/err/check_positive.hpp:68-77) */
inline void check_positive_size(const char* fn, const char* name, const char* expr, int size) {
  if (size <= 0) {
    std::ostringstream m;
    m << fn << ": " << name << " must have a positive size, but is " << size << "; dimension size expression = "
      << expr;
    throw std::invalid_argument(m.str());
  }
}

/** check_multiplicable(function, name1, y1, name2, y2)
 * (prim/mat/err/check_multiplicable.hpp:30-38), in its order: positive
 * rows of y1 and columns of y2, the size match, positive columns of y1. */
inline void check_multiplicable(const char* fn, int a_rows, int a_cols, int b_rows, int b_cols,
                                const char* na = "A", const char* nb = "B") {
  check_positive_size(fn, na, "rows()", a_rows);
  check_positive_size(fn, nb, "cols()", b_cols);
  if (a_cols != b_rows) {
    std::ostringstream m;
    m << fn << ": Columns of " << na << " (" << a_cols << ") and Rows of " << nb << " (" << b_rows
      << ") must match in size";
    throw std::invalid_argument(m.str());
  }
  check_positive_size(fn, na, "cols()", a_cols);
}

class multiply_dev_vari : public device_vari {
 public:
  dev_operand A_, B_;
  dev_matrix_vari* C_;
  // B = transpose(A) of the same var node: C = A A^T is formed as its lower
  // half (one triangular GEMM on A itself) mirrored, and the reverse is ONE
  // GEMM, Aadj += (Cadj + Cadj^T) A, instead of Aadj += Cadj B^T plus
  // Badj += A^T Cadj folded back through the transpose node (whose own
  // reverse then adds this node's share of nothing).  Same derivative as the
  // reference's two products (rev/mat/fun/multiply.hpp:65-135).
  bool gram_;
  // A structurally lower (a Cholesky factor or its tangent) times a vector:
  // one pass over A's lower tiles each way (smg_trmv_inv), and A's adjoint
  // written on its lower triangle only (its upper entries are the
  // reference's dummy vari)
  bool lowvec_;
  multiply_dev_vari(const dev_operand& A, const dev_operand& B)
      : device_vari(0.0), A_(A), B_(B), C_(new dev_matrix_vari(A.rows, B.cols)),
        gram_(A.vi && B.vi && B.vi->transpose_of_ == A.vi),
        lowvec_(A.vi && A.vi->structure_ == dev_structure::lower && A.rows == A.cols && B.cols == 1 &&
                A.rows % 64 == 0) {
    smg_ctx* c = amd::ctx();
    if (lowvec_) {
      amd::check(smg_trmv_inv(c, 0, A_.val(), A_.rows, A_.rows, B_.val(), C_->val_), "multiply");
      return;
    }
    if (gram_) {
      amd::check(smg_gemm(c, 0, 1, 1, A_.rows, A_.rows, A_.cols, 1.0, A_.val(), A_.rows, A_.val(), A_.rows, 0.0,
                          C_->val_, C_->rows_),
                 "multiply");
      amd::check(smg_sym_from_lower(c, C_->rows_, C_->val_, C_->rows_), "multiply");
      return;
    }
    amd::check(smg_multiply_fwd(c, A_.val(), A_.rows, B_.val(), B_.rows, A_.rows, A_.cols, B_.cols, C_->val_,
                                C_->rows_),
               "multiply");
  }
  void chain() override {
    smg_ctx* c = amd::ctx();
    if (lowvec_) {  // Aadj (lower) += Cadj b^T;  badj += A^T Cadj
      const int m = A_.rows;
      if (A_.adj()) amd::check(smg_rank1_lower(c, m, 1.0, C_->adj_, B_.val(), A_.adj(), m), "multiply");
      if (B_.adj()) {
        double* t = amd::alloc_doubles(size_t(m));
        amd::check(smg_trmv_inv(c, 1, A_.val(), A_.rows, m, C_->adj_, t), "multiply");
        amd::check(smg_axpy(c, (long long)m, 1.0, t, 1, B_.adj(), 1), "multiply");
      }
      return;
    }
    if (gram_) {
      const int m = C_->rows_;
      double* S = amd::alloc_doubles(size_t(m) * m);  // Cadj + Cadj^T
      amd::check(smg_memcpy_d2d(c, S, C_->adj_, size_t(m) * m * sizeof(double)), "multiply");
      amd::check(smg_transpose(c, m, m, C_->adj_, m, S, m, 1.0), "multiply");
      amd::check(smg_gemm(c, 0, 0, 0, m, A_.cols, m, 1.0, S, m, A_.val(), A_.rows, 1.0, A_.adj(), A_.rows),
                 "multiply");
      return;
    }
    amd::check(smg_multiply_rev(c, A_.val(), A_.rows, B_.val(), B_.rows, C_->adj_, C_->rows_, A_.rows, A_.cols,
                                B_.cols, A_.adj(), A_.rows, B_.adj(), B_.rows),
               "multiply");
  }
};

class scale_dev_vari : public device_vari {
 public:
  dev_operand A_;
  double c_;
  vari* c_vi_;   // null when c is data
  double* cadj_;  // device scalar
  dev_matrix_vari* B_;
  scale_dev_vari(const dev_operand& A, double c, vari* c_vi)
      : device_vari(0.0), A_(A), c_(c), c_vi_(c_vi), cadj_(c_vi ? amd::alloc_doubles(1) : nullptr),
        B_(new dev_matrix_vari(A.rows, A.cols)) {
    smg_ctx* x = amd::ctx();
    const long long n = (long long)A.rows * A.cols;
    amd::check(smg_memset(x, B_->val_, 0, size_t(n) * sizeof(double)), "multiply");
    amd::check(smg_axpy(x, n, c_, A_.val(), 1, B_->val_, 1), "multiply");
  }
  void chain() override {
    smg_ctx* x = amd::ctx();
    const long long n = (long long)A_.rows * A_.cols;
    if (A_.adj()) amd::check(smg_axpy(x, n, c_, B_->adj_, 1, A_.adj(), 1), "multiply");
    if (c_vi_) {
      amd::check(smg_memset(x, cadj_, 0, sizeof(double)), "multiply");
      amd::check(smg_dot(x, B_->adj_, A_.val(), n, cadj_), "multiply");
      add_pending_adjoint(c_vi_, cadj_);
    }
  }
};

class transpose_dev_vari : public device_vari {
 public:
  dev_matrix_vari* A_;
  dev_matrix_vari* B_;
  explicit transpose_dev_vari(dev_matrix_vari* A)
      : device_vari(0.0), A_(A), B_(new dev_matrix_vari(A->cols_, A->rows_)) {
    B_->transpose_of_ = A;
    amd::check(smg_transpose(amd::ctx(), A_->rows_, A_->cols_, A_->val_, A_->rows_, B_->val_,
                             B_->rows_, 0.0),
               "transpose");
  }
  void chain() override {
    amd::check(smg_transpose(amd::ctx(), B_->rows_, B_->cols_, B_->adj_, B_->rows_, A_->adj_,
                             A_->rows_, 1.0),
               "transpose");
  }
};

class sum_dev_vari : public device_vari {
 public:
  dev_matrix_vari* A_;
  sum_dev_vari(double v, dev_matrix_vari* A) : device_vari(v), A_(A) {}
  void chain() override {
    const int uplo = A_->structure_ == dev_structure::lower ? 1 : 0;
    amd::check(smg_shift(amd::ctx(), A_->rows_, A_->cols_, adj_, A_->adj_, A_->rows_, uplo), "sum");
  }
};

// sum(std::vector<var>) (rev/arr/fun/sum.hpp:14-57): a host node, the
// values summed in order on the host like the reference's sum_of_val
class sum_v_vari : public host_local_vari {
 public:
  vari** v_;
  size_t n_;
  sum_v_vari(double s, vari** v, size_t n) : host_local_vari(s), v_(v), n_(n) {}
  void chain() override {
    for (size_t i = 0; i < n_; ++i) v_[i]->adj_ += adj_;
  }
  bool touches_adjoints_in(const vari* lo, const vari* hi) const override {
    for (size_t i = 0; i < n_; ++i)
      if (v_[i] >= lo && v_[i] < hi) return true;
    return false;
  }
};

inline dev_var_matrix multiply_dev(const dev_operand& A, const dev_operand& B) {
  check_multiplicable("multiply", A.rows, A.cols, B.rows, B.cols);
  auto* node = new multiply_dev_vari(A, B);
  return dev_var_matrix(node->C_);
}

}  // namespace internal

inline dev_var_matrix multiply(const dev_var_matrix& A, const dev_var_matrix& B) {
  return internal::multiply_dev(internal::operand(A), internal::operand(B));
}
inline dev_var_matrix multiply(const dev_var_matrix& A, const dev_data<double>& B) {
  return internal::multiply_dev(internal::operand(A), internal::operand(B));
}
inline dev_var_matrix multiply(const dev_data<double>& A, const dev_var_matrix& B) {
  return internal::multiply_dev(internal::operand(A), internal::operand(B));
}
inline dev_var_matrix multiply(const var& c, const dev_var_matrix& A) {
  auto* node = new internal::scale_dev_vari(internal::operand(A), c.val(), c.vi_);
  return dev_var_matrix(node->B_);
}
inline dev_var_matrix multiply(const dev_var_matrix& A, const var& c) { return multiply(c, A); }
inline dev_var_matrix multiply(double c, const dev_var_matrix& A) {
  auto* node = new internal::scale_dev_vari(internal::operand(A), c, nullptr);
  return dev_var_matrix(node->B_);
}
inline dev_var_matrix multiply(const dev_var_matrix& A, double c) { return multiply(c, A); }
inline dev_var_matrix multiply(const var& c, const dev_data<double>& A) {
  auto* node = new internal::scale_dev_vari(internal::operand(A), c.val(), c.vi_);
  return dev_var_matrix(node->B_);
}

inline dev_var_matrix transpose(const dev_var_matrix& A) {
  auto* node = new internal::transpose_dev_vari(A.vi_);
  return dev_var_matrix(node->B_);
}

inline var sum(const std::vector<var>& v) {
  if (v.empty()) return var(0.0);
  vari** p = ChainableStack::instance_->memalloc_.alloc_array<vari*>(v.size());
  double s = 0.0;
  for (size_t i = 0; i < v.size(); ++i) {
    p[i] = v[i].vi_;
    s += v[i].vi_->val_;
  }
  return var(new internal::sum_v_vari(s, p, v.size()));
}
inline double sum(const std::vector<double>& v) {
  double s = 0.0;
  for (double x : v) s += x;
  return s;
}

inline var sum(const dev_var_matrix& A) {
  if (A.size() == 0) return var(0.0);
  smg_ctx* c = amd::ctx();
  double* s = amd::alloc_doubles(1);
  amd::check(smg_memset(c, s, 0, sizeof(double)), "sum");
  amd::check(smg_sum(c, A.val_ptr(), (long long)A.size(), s), "sum");
  double v = 0;
  amd::to_host(&v, s, 1);
  return var(new internal::sum_dev_vari(v, A.vi_));
}

}  // namespace math
}  // namespace stan
#endif
