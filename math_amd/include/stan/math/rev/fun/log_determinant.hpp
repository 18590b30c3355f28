#ifndef STAN_MATH_REV_FUN_LOG_DETERMINANT_HPP
#define STAN_MATH_REV_FUN_LOG_DETERMINANT_HPP

// log_determinant(m) of a general square matrix of vars
// (rev/mat/fun/log_determinant.hpp:14-37): check_square, value log|det m|,
// one node whose partials are m^{-T} (the reference's precomputed-gradients
// vari).  The factorisation is a device LU with partial pivoting
// (smg_log_determinant_fwd, csrc/lu.hip) kept for the reverse, which forms
// m^{-T} from it and adds adj * m^{-T} to m's device adjoint.  Size 0 -> 0
// (prim/mat/fun/log_determinant.hpp:22-23).  A singular m gives -inf, as the
// reference's logAbsDeterminant does.

#include <stan/math/amd/matrix.hpp>
#include <stan/math/rev/core.hpp>
#include <stan/math/rev/fun/cholesky_decompose.hpp>

namespace stan {
namespace math {
namespace internal {

class log_determinant_dev_vari : public device_vari {
 public:
  dev_matrix_vari* A_;
  double* LU_;
  int* piv_;
  log_determinant_dev_vari(double v, dev_matrix_vari* A, double* LU, int* piv)
      : device_vari(v), A_(A), LU_(LU), piv_(piv) {}
  void chain() override {
    const int n = A_->rows_;
    double* ws = amd::alloc_doubles(3 * size_t(n) * n);
    int* iws = amd::alloc_ints(size_t(n));
    amd::check(smg_log_determinant_rev(amd::ctx(), LU_, piv_, n, adj_, A_->adj_, n, ws, iws), "log_determinant");
  }
};

/** value of log|det A| and the factorisation (device) */
inline double log_determinant_value(const double* A, int n, double* LU, int* piv) {
  smg_ctx* c = amd::ctx();
  double* ws = amd::alloc_doubles(size_t(64) * 64);
  double* out = amd::alloc_doubles(1);
  amd::check(smg_log_determinant_fwd(c, A, n, n, LU, piv, ws, out), "log_determinant");
  double v = 0.0;
  amd::to_host(&v, out, 1);
  return v;
}

}  // namespace internal

/** log|det m| of a square device matrix of vars. */
inline var log_determinant(const dev_var_matrix& m) {
  internal::check_square("log_determinant", "m", m.rows(), m.cols());
  const int n = m.rows();
  if (n == 0) return var(0.0);
  double* LU = amd::alloc_doubles(size_t(n) * n);
  int* piv = amd::alloc_ints(size_t(n));
  const double v = internal::log_determinant_value(m.val_ptr(), n, LU, piv);
  return var(new internal::log_determinant_dev_vari(v, m.vi_, LU, piv));
}

/** log|det m| of a square device matrix of doubles (prim/mat/fun/log_determinant.hpp:20-27). */
inline double log_determinant(const dev_data<double>& m) {
  internal::check_square("log_determinant", "m", m.rows(), m.cols());
  const int n = m.rows();
  if (n == 0) return 0.0;
  double* LU = amd::alloc_doubles(size_t(n) * n);
  int* piv = amd::alloc_ints(size_t(n));
  return internal::log_determinant_value(m.data(), n, LU, piv);
}

}  // namespace math
}  // namespace stan
#endif
