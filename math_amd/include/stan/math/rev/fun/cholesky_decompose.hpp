#ifndef STAN_MATH_REV_FUN_CHOLESKY_DECOMPOSE_HPP
#define STAN_MATH_REV_FUN_CHOLESKY_DECOMPOSE_HPP

// add_diag and cholesky_decompose on device matrices of vars.
//
// add_diag (prim/mat/fun/add_diag.hpp:20-55): the reference builds N scalar
// `+` varis for the diagonal and shares the off-diagonal varis; here the
// output node carries its own value/adjoint columns and chain() folds the
// adjoint back: Aadj += Badj, d' += diag(Badj).
//
// cholesky_decompose (rev/mat/fun/cholesky_decompose.hpp:378-427): the same
// checks in the same order (check_square, check_symmetric at absolute 1e-8,
// check_pos_definite -> std::domain_error) BEFORE the node is pushed; the
// output's strict upper triangle is structurally zero (the reference points
// those entries at a dummy vari, :34-48), which downstream nodes exploit.
// chain() runs Murray's blocked adjoint on the device (smg_cholesky_rev) and
// adds into the LOWER triangle of A's adjoint only, like :159-164.

#include <stan/math/amd/matrix.hpp>
#include <stan/math/rev/core.hpp>

#include <sstream>
#include <stdexcept>

namespace stan {
namespace math {

namespace internal {

class add_diag_dev_vari : public vari {
 public:
  dev_matrix_vari* A_;
  dev_matrix_vari* B_;
  vari* d_vi_;     // scalar var diagonal (null when data)
  double* dadj_;   // device scalar

  add_diag_dev_vari(dev_matrix_vari* A, double d, vari* d_vi)
      : vari(0.0), A_(A), B_(new dev_matrix_vari(A->rows_, A->cols_)), d_vi_(d_vi),
        dadj_(d_vi ? amd::alloc_doubles(1) : nullptr) {
    amd::check(smg_add_diag_fwd(amd::ctx(), A_->val_, A_->rows_, A_->rows_, d, nullptr, B_->val_,
                                B_->rows_),
               "add_diag");
  }
  void chain() override {
    smg_ctx* c = amd::ctx();
    if (dadj_) amd::check(smg_memset(c, dadj_, 0, sizeof(double)), "add_diag");
    amd::check(smg_add_diag_rev(c, B_->adj_, B_->rows_, B_->rows_, A_->adj_, A_->rows_, dadj_, 0),
               "add_diag");
    if (d_vi_) add_pending_adjoint(d_vi_, dadj_);
  }
};

class cholesky_dev_vari : public vari {
 public:
  dev_matrix_vari* A_;
  dev_matrix_vari* L_;
  int n_;

  cholesky_dev_vari(dev_matrix_vari* A, dev_matrix_vari* L) : vari(0.0), A_(A), L_(L), n_(A->rows_) {}

  void chain() override {
    smg_ctx* c = amd::ctx();
    const size_t nn = size_t(n_) * n_;
    // Murray's algorithm overwrites its input and reads only its lower triangle
    double* work = amd::alloc_doubles(nn);
    amd::check(smg_copy_tril(c, n_, n_, L_->adj_, n_, work, n_), "cholesky_decompose");
    amd::check(smg_cholesky_rev(c, L_->val_, n_, L_->aux_, work, n_, n_, A_->adj_, n_),
               "cholesky_decompose");
  }
};

inline void check_square(const char* fn, const char* name, int rows, int cols) {
  if (rows != cols) {
    std::ostringstream m;
    m << fn << ": Expecting a square matrix; rows of " << name << " (" << rows << ") and columns of "
      << name << " (" << cols << ") must match in size";
    throw std::invalid_argument(m.str());
  }
}

/** check_symmetric's message for a device matrix the device check flagged
 * (error path: one host copy of A). */
inline void throw_not_symmetric_dev(const char* fn, const char* name, const double* A, int n) {
  std::vector<double> h(size_t(n) * n);
  amd::to_host(h.data(), A, h.size());
  amd::throw_not_symmetric_host(fn, name, h.data(), n);
}

}  // namespace internal

inline dev_var_matrix add_diag(const dev_var_matrix& A, const var& d) {
  internal::check_square("add_diag", "mat", A.rows(), A.cols());
  auto* node = new internal::add_diag_dev_vari(A.vi_, d.val(), d.vi_);
  return dev_var_matrix(node->B_);
}
inline dev_var_matrix add_diag(const dev_var_matrix& A, double d) {
  internal::check_square("add_diag", "mat", A.rows(), A.cols());
  auto* node = new internal::add_diag_dev_vari(A.vi_, d, nullptr);
  return dev_var_matrix(node->B_);
}

inline dev_var_matrix cholesky_decompose(const dev_var_matrix& A) {
  const char* fn = "cholesky_decompose";
  internal::check_square(fn, "A", A.rows(), A.cols());
  const int n = A.rows();
  smg_ctx* c = amd::ctx();
  if (n == 0) return dev_var_matrix(new dev_matrix_vari(0, 0, dev_structure::lower));
  auto* L = new dev_matrix_vari(n, n, dev_structure::lower);
  L->aux_ = amd::alloc_doubles(size_t(smg_cholesky_aux_doubles(n)));
  // check_symmetric fused with the factorisation's copy of A (one pass); the
  // status is read at the mark after the panels, so the block inverses that
  // follow run while the host builds the next node
  amd::check(smg_cholesky_fwd_checked_mark(c, A.val_ptr(), n, n, L->val_, n, L->aux_), fn);
  int st = 0;
  amd::check(smg_status_mark_wait(c, &st), fn);
  if (st & SMG_ERR_NOT_SYMMETRIC) internal::throw_not_symmetric_dev(fn, "A", A.val_ptr(), n);
  if (st) amd::throw_status(st, fn, "m");
  new internal::cholesky_dev_vari(A.vi_, L);
  return dev_var_matrix(L);
}

}  // namespace math
}  // namespace stan
#endif
