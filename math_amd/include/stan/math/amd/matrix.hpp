#ifndef STAN_MATH_AMD_MATRIX_HPP
#define STAN_MATH_AMD_MATRIX_HPP

// Device-resident matrices of vars (struct-of-arrays).
//
// The reference represents an N x N matrix of vars as N^2 host varis
// (AoS, one `vari*` per element) and every matrix functor gathers/scatters
// through those pointers (e.g. rev/mat/fun/cholesky_decompose.hpp:74-92,
// 159-164).  Here a matrix node is ONE arena object holding a device column
// of values and a device column of adjoints; functor nodes (vari subclasses
// on var_stack_) read and write those columns with HIP kernels.  Host varis
// are materialised only at an Eigen boundary (stan/math/eigen/interop.hpp).
//
//   dev_matrix_vari  the node (arena object, never chained itself)
//   dev_var_matrix   the handle user code holds (like var for vari)
//   dev_data         a device copy of constant data (double or int)

#include <stan/math/amd/device.hpp>
#include <stan/math/rev/core/grad.hpp>
#include <stan/math/rev/core/vari.hpp>

#include <vector>

namespace stan {
namespace math {

/** Structural information carried by a matrix node. */
enum class dev_structure : int {
  general = 0,
  lower = 1  // strict upper triangle is constant zero (cholesky_decompose output)
};

class dev_matrix_vari {
 public:
  const int rows_;
  const int cols_;
  double* val_;  // device, column-major, ld = rows_
  double* adj_;  // device, column-major, registered with the tape
  dev_structure structure_;
  double* aux_;  // node-specific device side data (e.g. Cholesky diagonal-block inverses)

  dev_matrix_vari(int rows, int cols, dev_structure s = dev_structure::general)
      : rows_(rows),
        cols_(cols),
        val_(amd::alloc_doubles(size_t(rows) * cols)),
        adj_(amd::alloc_doubles(size_t(rows) * cols)),
        structure_(s),
        aux_(nullptr) {
    register_device_adjoint(adj_, size_t(rows) * cols);
  }

  size_t size() const { return size_t(rows_) * cols_; }

  static inline void* operator new(size_t nbytes) {
    return ChainableStack::instance_->memalloc_.alloc(nbytes);
  }
  static inline void operator delete(void*) {}
};

class dev_var_matrix {
 public:
  dev_matrix_vari* vi_;

  dev_var_matrix() : vi_(nullptr) {}
  explicit dev_var_matrix(dev_matrix_vari* vi) : vi_(vi) {}

  int rows() const { return vi_->rows_; }
  int cols() const { return vi_->cols_; }
  size_t size() const { return vi_->size(); }
  const double* val_ptr() const { return vi_->val_; }
  double* adj_ptr() const { return vi_->adj_; }

  /** Column-major host copy of the values (synchronising). */
  std::vector<double> val() const {
    std::vector<double> h(size());
    amd::to_host(h.data(), vi_->val_, size());
    return h;
  }
  /** Column-major host copy of the adjoints (synchronising). */
  std::vector<double> adj() const {
    std::vector<double> h(size());
    amd::to_host(h.data(), vi_->adj_, size());
    return h;
  }

#ifdef STAN_MATH_AMD_HAS_EIGEN
  // materialise as N^2 host varis (stan/math/eigen/interop.hpp)
  operator Eigen::Matrix<var, Eigen::Dynamic, Eigen::Dynamic>() const;
  operator Eigen::Matrix<var, Eigen::Dynamic, 1>() const;
#endif
};

/** Device copy of constant data (arena-owned, recovered with the tape). */
template <typename T>
class dev_data {
 public:
  const T* ptr_ = nullptr;
  size_t n_ = 0;
  int rows_ = 0, cols_ = 0;
  dev_data() = default;
  dev_data(const T* p, size_t n, int rows, int cols) : ptr_(p), n_(n), rows_(rows), cols_(cols) {}
  size_t size() const { return n_; }
  int rows() const { return rows_; }
  int cols() const { return cols_; }
  const T* data() const { return ptr_; }
};

inline dev_data<double> to_dev_data(const double* h, size_t n, int rows = -1, int cols = 1) {
  double* d = amd::alloc_doubles(n);
  amd::to_device(d, h, n);
  return dev_data<double>(d, n, rows < 0 ? int(n) : rows, cols);
}
inline dev_data<double> to_dev_data(const std::vector<double>& v) {
  return to_dev_data(v.data(), v.size());
}
inline dev_data<int> to_dev_data(const std::vector<int>& v) {
  int* d = amd::alloc_ints(v.size());
  amd::to_device_int(d, v.data(), v.size());
  return dev_data<int>(d, v.size(), int(v.size()), 1);
}

/** A fresh device matrix of vars initialised from host values (a leaf:
 * its adjoint is read back by the caller, like x_var in gradient()). */
inline dev_var_matrix to_dev_var_matrix(const double* host_colmajor, int rows, int cols) {
  auto* vi = new dev_matrix_vari(rows, cols);
  amd::to_device(vi->val_, host_colmajor, size_t(rows) * cols);
  return dev_var_matrix(vi);
}

}  // namespace math
}  // namespace stan
#endif
