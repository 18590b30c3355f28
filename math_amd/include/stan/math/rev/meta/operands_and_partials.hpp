#ifndef STAN_MATH_REV_META_OPERANDS_AND_PARTIALS_HPP
#define STAN_MATH_REV_META_OPERANDS_AND_PARTIALS_HPP

// operands_and_partials<Op1, ..., Op5, T_return> -- the reference's
// "compressed node" builder behind every *_lpdf
// (prim/scal/meta/operands_and_partials.hpp:12-90,
//  rev/scal/meta/operands_and_partials.hpp:15-127,
//  rev/mat/meta/operands_and_partials.hpp:15-159):
// one edge per operand holds the partials of the result with respect to that
// operand (edgeK_.partials_, and partials_vec_ for multivariate use); build(v)
// puts ONE node on the tape whose chain() adds adj * partial into every
// operand.  Same member names and broadcast semantics: a scalar operand's
// partials_[i] all alias its one partial; a data operand's partials_ swallow
// writes.
//
// Device-capable edge (MI355X addition): an operand held on the device as a
// dev_var_matrix gets a DEVICE partials buffer (edgeK_.partials_ is a device
// pointer of size() doubles, zeroed, arena-owned), filled by the caller's
// kernels (or from the host with set_partials); the node's chain() applies it
// with one axpy into the operand's device adjoint -- no host varis, no
// per-element pointer chasing.

#include <stan/math/amd/matrix.hpp>
#include <stan/math/rev/core.hpp>

#include <type_traits>
#include <vector>

namespace stan {
namespace math {

namespace internal {

/** x[i] is the one scalar for every i (prim/scal/meta/broadcast_array.hpp). */
template <typename T>
class broadcast_array {
  T& prim_;

 public:
  explicit broadcast_array(T& prim) : prim_(prim) {}
  T& operator[](int) { return prim_; }
  /** assigns the first element of m (a container of length 1) */
  template <typename Y>
  void operator=(const Y& m) {
    prim_ = m[0];
  }
};

/** partials of a data operand: writes vanish, reads are 0. */
template <typename T>
class empty_broadcast_array {
 public:
  T& operator[](int) {
    static thread_local T sink;
    sink = T(0);
    return sink;
  }
  template <typename Y>
  void operator=(const Y&) {}
  template <typename Y>
  void operator+=(const Y&) {}
  template <typename Y>
  void operator-=(const Y&) {}
};

template <typename T>
struct op_is_var : std::false_type {};
template <>
struct op_is_var<var> : std::true_type {};
template <>
struct op_is_var<std::vector<var>> : std::true_type {};
template <>
struct op_is_var<std::vector<std::vector<var>>> : std::true_type {};
template <>
struct op_is_var<dev_var_matrix> : std::true_type {};
#ifdef STAN_MATH_AMD_HAS_EIGEN
template <int R, int C>
struct op_is_var<Eigen::Matrix<var, R, C>> : std::true_type {};
template <int R, int C>
struct op_is_var<std::vector<Eigen::Matrix<var, R, C>>> : std::true_type {};
#endif

/** One device edge of a node: adj(operand) += adj * partials (device). */
struct dev_edge {
  dev_matrix_vari* op = nullptr;
  const double* partials = nullptr;
};

/** Data operand (double, int, std::vector<double>, Eigen<double>, dev_data). */
template <typename ViewElt, typename Op>
class ops_partials_edge {
 public:
  empty_broadcast_array<ViewElt> partials_;
  empty_broadcast_array<ViewElt> partials_vec_;
  ops_partials_edge() {}
  explicit ops_partials_edge(const Op&) {}
  int size() const { return 0; }
  void dump_operands(vari**) const {}
  void dump_partials(double*) const {}
  dev_edge device() const { return dev_edge{}; }
};

/** A scalar var. */
template <>
class ops_partials_edge<double, var> {
 public:
  double partial_;
  broadcast_array<double> partials_;
  broadcast_array<double> partials_vec_;
  explicit ops_partials_edge(const var& op)
      : partial_(0), partials_(partial_), partials_vec_(partial_), operand_(op) {}
  int size() const { return 1; }
  void dump_operands(vari** v) const { *v = operand_.vi_; }
  void dump_partials(double* p) const { *p = partial_; }
  dev_edge device() const { return dev_edge{}; }

 private:
  const var& operand_;
};

#ifdef STAN_MATH_AMD_HAS_EIGEN
using vec_partials_t = Eigen::VectorXd;
#else
using vec_partials_t = std::vector<double>;
#endif

#ifdef STAN_MATH_AMD_HAS_EIGEN
// the partials of a std::vector<var> edge live in the tape's arena (no heap
// allocation per call); an Eigen vector view, indexed and assigned like the
// reference's Eigen::VectorXd
using vec_partials_view_t = Eigen::Map<Eigen::VectorXd>;
inline vec_partials_view_t arena_partials(size_t n) {
  double* p = ChainableStack::instance_->memalloc_.alloc_array<double>(n ? n : 1);
  vec_partials_view_t v(p, Eigen::Index(n));
  v.setZero();
  return v;
}
#else
using vec_partials_view_t = vec_partials_t;
inline vec_partials_view_t arena_partials(size_t n) { return vec_partials_t(n, 0.0); }
#endif

/** std::vector<var> (rev/mat/meta/operands_and_partials.hpp:15-43). */
template <>
class ops_partials_edge<double, std::vector<var>> {
 public:
  vec_partials_view_t partials_;
  broadcast_array<vec_partials_view_t> partials_vec_;
  explicit ops_partials_edge(const std::vector<var>& op)
      : partials_(arena_partials(op.size())), partials_vec_(partials_), operands_(op) {}
  int size() const { return int(operands_.size()); }
  void dump_operands(vari** v) const {
    for (size_t i = 0; i < operands_.size(); ++i) v[i] = operands_[i].vi_;
  }
  void dump_partials(double* p) const {
    for (size_t i = 0; i < operands_.size(); ++i) p[i] = partials_[i];
  }
  dev_edge device() const { return dev_edge{}; }

 private:
  const std::vector<var>& operands_;
};

/** std::vector<std::vector<var>> (rev/mat/meta/operands_and_partials.hpp:122-155). */
template <>
class ops_partials_edge<double, std::vector<std::vector<var>>> {
 public:
  std::vector<std::vector<double>> partials_vec_;
  explicit ops_partials_edge(const std::vector<std::vector<var>>& ops)
      : partials_vec_(ops.size()), operands_(ops) {
    for (size_t i = 0; i < ops.size(); ++i) partials_vec_[i].assign(ops[i].size(), 0.0);
  }
  int size() const {
    int s = 0;
    for (auto& o : operands_) s += int(o.size());
    return s;
  }
  void dump_operands(vari** v) const {
    for (auto& o : operands_)
      for (auto& x : o) *v++ = x.vi_;
  }
  void dump_partials(double* p) const {
    for (auto& o : partials_vec_)
      for (double x : o) *p++ = x;
  }
  dev_edge device() const { return dev_edge{}; }

 private:
  const std::vector<std::vector<var>>& operands_;
};

#ifdef STAN_MATH_AMD_HAS_EIGEN
/** Eigen::Matrix<var, R, C> (rev/mat/meta/operands_and_partials.hpp:45-75). */
template <int R, int C>
class ops_partials_edge<double, Eigen::Matrix<var, R, C>> {
 public:
  using partials_t = Eigen::Matrix<double, R, C>;
  partials_t partials_;
  broadcast_array<partials_t> partials_vec_;
  explicit ops_partials_edge(const Eigen::Matrix<var, R, C>& ops)
      : partials_(partials_t::Zero(ops.rows(), ops.cols())), partials_vec_(partials_), operands_(ops) {}
  int size() const { return int(operands_.size()); }
  void dump_operands(vari** v) const {
    for (Eigen::Index i = 0; i < operands_.size(); ++i) v[i] = operands_(i).vi_;
  }
  void dump_partials(double* p) const {
    for (Eigen::Index i = 0; i < partials_.size(); ++i) p[i] = partials_(i);
  }
  dev_edge device() const { return dev_edge{}; }

 private:
  const Eigen::Matrix<var, R, C>& operands_;
};

/** std::vector<Eigen::Matrix<var, R, C>> (rev/mat/meta/operands_and_partials.hpp:79-119). */
template <int R, int C>
class ops_partials_edge<double, std::vector<Eigen::Matrix<var, R, C>>> {
 public:
  std::vector<Eigen::MatrixXd> partials_vec_;
  explicit ops_partials_edge(const std::vector<Eigen::Matrix<var, R, C>>& ops)
      : partials_vec_(ops.size()), operands_(ops) {
    for (size_t i = 0; i < ops.size(); ++i) partials_vec_[i] = Eigen::MatrixXd::Zero(ops[i].rows(), ops[i].cols());
  }
  int size() const {
    int s = 0;
    for (auto& o : operands_) s += int(o.size());
    return s;
  }
  void dump_operands(vari** v) const {
    for (auto& o : operands_)
      for (Eigen::Index j = 0; j < o.size(); ++j) *v++ = o(j).vi_;
  }
  void dump_partials(double* p) const {
    for (auto& o : partials_vec_)
      for (Eigen::Index j = 0; j < o.size(); ++j) *p++ = o(j);
  }
  dev_edge device() const { return dev_edge{}; }

 private:
  const std::vector<Eigen::Matrix<var, R, C>>& operands_;
};
#endif

/** A matrix of vars resident on the device: device partials. */
template <>
class ops_partials_edge<double, dev_var_matrix> {
 public:
  double* partials_;  // device, operand's size, zeroed
  explicit ops_partials_edge(const dev_var_matrix& op)
      : partials_(amd::alloc_doubles(op.size())), operand_(op) {
    amd::zero(partials_, op.size());
  }
  /** copy host partials (operand's size, column-major) into the device edge */
  void set_partials(const double* host) { amd::to_device(partials_, host, operand_.size()); }
  int size() const { return 0; }  // no host varis
  void dump_operands(vari**) const {}
  void dump_partials(double*) const {}
  dev_edge device() const { return dev_edge{operand_.vi_, partials_}; }

 private:
  const dev_var_matrix& operand_;
};

/** The node build() puts on the tape: host operands (precomputed-gradients
 * form) plus up to five device edges (one axpy each). */
class ops_partials_vari : public local_adjoint_vari {
 public:
  size_t size_;
  vari** varis_;
  double* partials_;
  dev_edge dev_[5];
  int ndev_;
  ops_partials_vari(double v, size_t size, vari** varis, double* partials, const dev_edge* dev, int ndev)
      : local_adjoint_vari(v), size_(size), varis_(varis), partials_(partials), ndev_(ndev) {
    for (int i = 0; i < ndev; ++i) dev_[i] = dev[i];
  }
  bool touches_adjoints_in(const vari* lo, const vari* hi) const override {
    for (size_t i = 0; i < size_; ++i)
      if (varis_[i] >= lo && varis_[i] < hi) return true;
    return false;
  }
  void chain() override {
    for (size_t i = 0; i < size_; ++i) varis_[i]->adj_ += adj_ * partials_[i];
    for (int i = 0; i < ndev_; ++i)
      amd::check(smg_axpy(amd::ctx(), (long long)dev_[i].op->size(), adj_, dev_[i].partials, 1,
                          dev_[i].op->adj_, 1),
                 "operands_and_partials");
  }
};

template <typename... Ops>
struct ops_return {
  using type = typename std::conditional<(op_is_var<Ops>::value || ...), var, double>::type;
};

}  // namespace internal

template <typename Op1 = double, typename Op2 = double, typename Op3 = double, typename Op4 = double,
          typename Op5 = double,
          typename T_return_type = typename internal::ops_return<Op1, Op2, Op3, Op4, Op5>::type>
class operands_and_partials;

/** All operands data: build() returns the value (prim/scal/meta/operands_and_partials.hpp:60-90). */
template <typename Op1, typename Op2, typename Op3, typename Op4, typename Op5>
class operands_and_partials<Op1, Op2, Op3, Op4, Op5, double> {
 public:
  internal::ops_partials_edge<double, Op1> edge1_;
  internal::ops_partials_edge<double, Op2> edge2_;
  internal::ops_partials_edge<double, Op3> edge3_;
  internal::ops_partials_edge<double, Op4> edge4_;
  internal::ops_partials_edge<double, Op5> edge5_;
  explicit operands_and_partials(const Op1&) {}
  operands_and_partials(const Op1&, const Op2&) {}
  operands_and_partials(const Op1&, const Op2&, const Op3&) {}
  operands_and_partials(const Op1&, const Op2&, const Op3&, const Op4&) {}
  operands_and_partials(const Op1&, const Op2&, const Op3&, const Op4&, const Op5&) {}
  double build(double value) const { return value; }
};

/** Reverse mode (rev/scal/meta/operands_and_partials.hpp:72-127). */
template <typename Op1, typename Op2, typename Op3, typename Op4, typename Op5>
class operands_and_partials<Op1, Op2, Op3, Op4, Op5, var> {
 public:
  internal::ops_partials_edge<double, Op1> edge1_;
  internal::ops_partials_edge<double, Op2> edge2_;
  internal::ops_partials_edge<double, Op3> edge3_;
  internal::ops_partials_edge<double, Op4> edge4_;
  internal::ops_partials_edge<double, Op5> edge5_;

  explicit operands_and_partials(const Op1& o1) : edge1_(o1) {}
  operands_and_partials(const Op1& o1, const Op2& o2) : edge1_(o1), edge2_(o2) {}
  operands_and_partials(const Op1& o1, const Op2& o2, const Op3& o3) : edge1_(o1), edge2_(o2), edge3_(o3) {}
  operands_and_partials(const Op1& o1, const Op2& o2, const Op3& o3, const Op4& o4)
      : edge1_(o1), edge2_(o2), edge3_(o3), edge4_(o4) {}
  operands_and_partials(const Op1& o1, const Op2& o2, const Op3& o3, const Op4& o4, const Op5& o5)
      : edge1_(o1), edge2_(o2), edge3_(o3), edge4_(o4), edge5_(o5) {}

  /** One node holding every operand's partials (host edges gathered into
   * arena arrays, device edges by pointer). */
  var build(double value) {
    const size_t size = size_t(edge1_.size()) + edge2_.size() + edge3_.size() + edge4_.size() + edge5_.size();
    auto& mem = ChainableStack::instance_->memalloc_;
    vari** varis = mem.alloc_array<vari*>(size ? size : 1);
    double* partials = mem.alloc_array<double>(size ? size : 1);
    size_t idx = 0;
    edge1_.dump_operands(varis + idx);
    edge1_.dump_partials(partials + idx);
    idx += size_t(edge1_.size());
    edge2_.dump_operands(varis + idx);
    edge2_.dump_partials(partials + idx);
    idx += size_t(edge2_.size());
    edge3_.dump_operands(varis + idx);
    edge3_.dump_partials(partials + idx);
    idx += size_t(edge3_.size());
    edge4_.dump_operands(varis + idx);
    edge4_.dump_partials(partials + idx);
    idx += size_t(edge4_.size());
    edge5_.dump_operands(varis + idx);
    edge5_.dump_partials(partials + idx);
    internal::dev_edge dev[5] = {edge1_.device(), edge2_.device(), edge3_.device(), edge4_.device(),
                                 edge5_.device()};
    internal::dev_edge used[5];
    int nd = 0;
    for (auto& d : dev)
      if (d.op) used[nd++] = d;
    return var(new internal::ops_partials_vari(value, size, varis, partials, used, nd));
  }
};

}  // namespace math
}  // namespace stan
#endif
