#ifndef STAN_MATH_REV_FUN_MDIVIDE_LEFT_TRI_HPP
#define STAN_MATH_REV_FUN_MDIVIDE_LEFT_TRI_HPP

// mdivide_left_tri<TriView>(A, B) = tri(A)^{-1} B on device matrices
// (rev/mat/fun/mdivide_left_tri.hpp:16-373; vv :16-130, dv :132-227,
// vd :229-320).  TriView uses Eigen's values (Eigen::Lower = 1,
// Eigen::Upper = 2); only that triangle of A is read.  Reverse:
//   Badj += tri(A)^{-T} Cadj,  Aadj(tri) -= (tri(A)^{-T} Cadj) C^T   (:104-123)
// Checks (:335-340): check_square(A), check_multiplicable(A, B), before the
// tape is touched.  The one-argument form is the explicit inverse
// (prim/mat/fun/mdivide_left_tri.hpp:68-83), B = I.

#include <stan/math/amd/matrix.hpp>
#include <stan/math/rev/core.hpp>
#include <stan/math/rev/fun/cholesky_decompose.hpp>
#include <stan/math/rev/fun/multiply.hpp>

namespace stan {
namespace math {

namespace internal {

class mdivide_left_tri_dev_vari : public device_vari {
 public:
  const int lower_;
  dev_operand A_, B_;
  dev_matrix_vari* C_;
  const double* W_ = nullptr;  // tri(A)^{-1} when A's factorisation formed it (one vector: products, not solves)
  mdivide_left_tri_dev_vari(int lower, const dev_operand& A, const dev_operand& B)
      : device_vari(0.0), lower_(lower), A_(A), B_(B), C_(new dev_matrix_vari(B.rows, B.cols)) {
    // a Cholesky factor whose W = L^{-1} exists (the HVP's value factor, a
    // GP's progressive K^{-1}): C = W b, one HBM pass instead of a
    // latency-bound persistent solve
    if (lower_ && B_.cols == 1 && B_.rows % 64 == 0 && A_.vi && A_.vi->sink_) W_ = A_.vi->sink_->inverse_factor();
    if (W_) {
      amd::check(smg_trmv_inv(amd::ctx(), 0, W_, A_.rows, B_.rows, B_.val(), C_->val_), "mdivide_left_tri");
      return;
    }
    amd::check(smg_mdivide_left_tri_aux_fwd(amd::ctx(), lower_, A_.val(), A_.rows, aux(), B_.val(), B_.rows,
                                            B_.rows, B_.cols, C_->val_, C_->rows_),
               "mdivide_left_tri");
  }
  // A Cholesky factor carries its diagonal-block inverses (aux_): the
  // solves reuse them
  const double* aux() const { return lower_ && A_.vi ? A_.vi->aux_ : nullptr; }
  void chain() override {
    const int m = B_.rows, n = B_.cols;
    double* ws = amd::alloc_doubles(size_t(m) * n);
    if (W_) {  // ws = W^T Cadj;  Aadj (lower) -= ws C^T;  Badj += ws  (:104-123)
      smg_ctx* c = amd::ctx();
      amd::check(smg_trmv_inv(c, 1, W_, A_.rows, m, C_->adj_, ws), "mdivide_left_tri");
      if (A_.adj()) amd::check(smg_rank1_lower(c, m, -1.0, ws, C_->val_, A_.adj(), A_.rows), "mdivide_left_tri");
      if (B_.adj()) amd::check(smg_axpy(c, (long long)m, 1.0, ws, 1, B_.adj(), 1), "mdivide_left_tri");
      return;
    }
    amd::check(smg_mdivide_left_tri_aux_rev(amd::ctx(), lower_, A_.val(), A_.rows, aux(), C_->val_, m,
                                            C_->adj_, m, m, n, A_.adj(), A_.rows, B_.adj(), m, ws),
               "mdivide_left_tri");
  }
};

template <int TriView>
inline dev_var_matrix mdivide_left_tri_dev(const dev_operand& A, const dev_operand& B) {
  static_assert(TriView == 1 || TriView == 2, "TriView must be Eigen::Lower or Eigen::Upper");
  check_square("mdivide_left_tri", "A", A.rows, A.cols);
  check_multiplicable("mdivide_left_tri", A.rows, A.cols, B.rows, B.cols, "A", "b");
  auto* node = new mdivide_left_tri_dev_vari(TriView == 1 ? 1 : 0, A, B);
  return dev_var_matrix(node->C_);
}

inline dev_data<double> dev_identity(int n) {
  double* I = amd::alloc_doubles(size_t(n) * n);
  smg_ctx* c = amd::ctx();
  amd::check(smg_memset(c, I, 0, size_t(n) * n * sizeof(double)), "mdivide_left_tri");
  amd::check(smg_add_diag_fwd(c, I, n, n, 1.0, nullptr, I, n), "mdivide_left_tri");
  return dev_data<double>(I, size_t(n) * n, n, n);
}

}  // namespace internal

template <int TriView>
inline dev_var_matrix mdivide_left_tri(const dev_var_matrix& A, const dev_var_matrix& B) {
  return internal::mdivide_left_tri_dev<TriView>(internal::operand(A), internal::operand(B));
}
template <int TriView>
inline dev_var_matrix mdivide_left_tri(const dev_data<double>& A, const dev_var_matrix& B) {
  return internal::mdivide_left_tri_dev<TriView>(internal::operand(A), internal::operand(B));
}
template <int TriView>
inline dev_var_matrix mdivide_left_tri(const dev_var_matrix& A, const dev_data<double>& B) {
  return internal::mdivide_left_tri_dev<TriView>(internal::operand(A), internal::operand(B));
}
/** tri(A)^{-1} */
template <int TriView>
inline dev_var_matrix mdivide_left_tri(const dev_var_matrix& A) {
  internal::check_square("mdivide_left_tri", "A", A.rows(), A.cols());
  return internal::mdivide_left_tri_dev<TriView>(internal::operand(A),
                                                 internal::operand(internal::dev_identity(A.rows())));
}

}  // namespace math
}  // namespace stan
#endif
