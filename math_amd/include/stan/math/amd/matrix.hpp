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
#include <stan/math/rev/core/var.hpp>
#include <stan/math/rev/core/vari.hpp>

#include <stdexcept>
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
  // set on transpose(A)'s output: multiply(A, transpose(A)) recognises the
  // Gram product (one lower GEMM forward, one GEMM reverse)
  dev_matrix_vari* transpose_of_ = nullptr;

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
    join_device_adjoints();
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

namespace internal {
// device -> host varis (reverse: host adjoints -> device adjoint)
class dev_to_host_vari : public vari {
 public:
  dev_matrix_vari* src_;
  vari** elems_;
  double* stage_;  // device scratch for the gathered adjoints
  dev_to_host_vari(dev_matrix_vari* src, vari** elems)
      : vari(0.0), src_(src), elems_(elems), stage_(amd::alloc_doubles(src->size())) {}
  bool reads_other_adjoints() const override { return true; }
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

/** Host vars (column-major; a column vector by default) -> device node
 * (bridged in the reverse sweep). */
inline dev_var_matrix to_dev(const std::vector<var>& v, int rows = -1, int cols = 1) {
  const size_t n = v.size();
  if (rows < 0) rows = int(n);
  if (size_t(rows) * size_t(cols) != n) throw std::invalid_argument("to_dev: rows * cols != size");
  auto* d = new dev_matrix_vari(rows, cols);
  std::vector<double> vals(n);
  vari** elems = ChainableStack::instance_->memalloc_.alloc_array<vari*>(n ? n : 1);
  for (size_t i = 0; i < n; ++i) {
    vals[i] = v[i].val();
    elems[i] = v[i].vi_;
  }
  amd::to_device(d->val_, vals.data(), n);
  new internal::host_to_dev_vari(d, elems);
  return dev_var_matrix(d);
}

/** Device node -> host vars, column-major (bridged in the reverse sweep). */
inline std::vector<var> to_var_vector(const dev_var_matrix& m) {
  const size_t n = m.size();
  std::vector<double> vals = m.val();
  vari** elems = ChainableStack::instance_->memalloc_.alloc_array<vari*>(n ? n : 1);
  std::vector<var> out(n);
  for (size_t i = 0; i < n; ++i) {
    elems[i] = new vari(vals[i], false);
    out[i] = var(elems[i]);
  }
  new internal::dev_to_host_vari(m.vi_, elems);
  return out;
}

}  // namespace math
}  // namespace stan
#endif
