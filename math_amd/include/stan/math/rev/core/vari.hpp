#ifndef STAN_MATH_REV_CORE_VARI_HPP
#define STAN_MATH_REV_CORE_VARI_HPP

// stan::math::vari — same public interface as the reference
// (stan/math/rev/core/vari.hpp:30-143): const val_, adj_, virtual chain(),
// init_dependent(), set_zero_adjoint(), arena operator new / no-op delete,
// and the (double, bool stacked) constructor that selects var_stack_ vs
// var_nochain_stack_.

#include <stan/math/rev/core/autodiffstackstorage.hpp>

#include <ostream>

namespace stan {
namespace math {

class vari {
 private:
  friend class var;

 public:
  const double val_;
  double adj_;

  explicit vari(double x) : val_(x), adj_(0.0) {
    ChainableStack::instance_->var_stack_.push_back(this);
  }

  vari(double x, bool stacked) : val_(x), adj_(0.0) {
    if (stacked)
      ChainableStack::instance_->var_stack_.push_back(this);
    else
      ChainableStack::instance_->var_nochain_stack_.push_back(this);
  }

  /** A vari on no stack: an element of a host block (the tape's
   * host_blocks_ holds the whole block; stan/math/eigen/bridge.hpp). */
  struct unstacked_tag {};
  vari(double x, unstacked_tag) : val_(x), adj_(0.0) {}

  virtual ~vari() {}

  virtual void chain() {}

  /** True for a node whose chain() may read the adjoints of OTHER varis
   * (not only its own adj_): the reverse sweep lands every pending
   * device->host contribution before such a node runs (grad.hpp).  The
   * default is true, so a user vari written in the reference's style (an
   * output-element vari read by a base vari's chain(), e.g.
   * rev/mat/fun/multiply.hpp:107-135) always sees complete adjoints; the
   * library's own nodes derive from local_adjoint_vari (audited: chain()
   * reads only this->adj_ and device buffers) and skip that synchronisation. */
  virtual bool reads_other_adjoints() const { return true; }

  /** False only when chain() provably adds nothing to the adj_ of any vari
   * in [lo, hi) directly (a device->host pending adjoint is tracked
   * separately).  A host block materialised from a device node
   * (stan/math/eigen/bridge.hpp) skips gathering its N^2 host adjoints when
   * no node chained after it touches them.  Conservative default: true. */
  virtual bool touches_adjoints_in(const vari* lo, const vari* hi) const {
    (void)lo;
    (void)hi;
    return true;
  }

  /** True when chain() may add into the DEVICE adjoint of the matrix node
   * `node` (a dev_matrix_vari; stan/math/amd/matrix.hpp), asked of the nodes
   * chained after a cholesky_decompose node once they have run: its factor's
   * adjoint may skip the dense form only when no node but the consuming
   * multi_normal_cholesky_lpdf wrote it (rev/fun/cholesky_decompose.hpp).  A
   * vari written in the reference's style sees host adjoints only: false.
   * The library's own nodes (local_adjoint_vari) answer true unless audited. */
  virtual bool may_write_device_adjoint(const void* node) const {
    (void)node;
    return false;
  }

  void init_dependent() { adj_ = 1.0; }

  void set_zero_adjoint() { adj_ = 0.0; }

  friend std::ostream& operator<<(std::ostream& os, const vari* v) {
    return os << v->val_ << ":" << v->adj_;
  }

  static inline void* operator new(size_t nbytes) {
    return ChainableStack::instance_->memalloc_.alloc(nbytes);
  }
  static inline void operator delete(void* /* ignored */) {}
};

/** Base of the library's own nodes: chain() reads no host adjoint but its
 * own adj_ (device adjoints are stream-ordered), so a pending device->host
 * contribution need only land before it when it targets this node. */
class local_adjoint_vari : public vari {
 public:
  explicit local_adjoint_vari(double x) : vari(x) { register_dev_writer(this); }
  local_adjoint_vari(double x, bool stacked) : vari(x, stacked) {
    if (stacked) register_dev_writer(this);
  }
  bool reads_other_adjoints() const override { return false; }
  bool may_write_device_adjoint(const void*) const override { return true; }
  /** v (just pushed on var_stack_) may write device adjoints: the structured
   * reverses' writer checks visit it (matrix.hpp others_write_device_adjoint) */
  static void register_dev_writer(vari* v) {
    auto* st = ChainableStack::instance_;
    st->dev_writers_.push_back({st->var_stack_.size() - 1, v});
  }
};

/** A library node whose chain() writes host adjoints only. */
class host_local_vari : public local_adjoint_vari {
 public:
  explicit host_local_vari(double x) : local_adjoint_vari(x) { ChainableStack::instance_->dev_writers_.pop_back(); }
  host_local_vari(double x, bool stacked) : local_adjoint_vari(x, stacked) {
    if (stacked) ChainableStack::instance_->dev_writers_.pop_back();
  }
  bool may_write_device_adjoint(const void*) const override { return false; }
};

/** Base of the library's device nodes: chain() reads only this->adj_ and
 * writes only device adjoint buffers (host scalars receive device results
 * through add_pending_adjoint), so it touches no host vari's adj_ directly. */
class device_vari : public local_adjoint_vari {
 public:
  using local_adjoint_vari::local_adjoint_vari;
  bool touches_adjoints_in(const vari*, const vari*) const override { return false; }
};

/** Objects with destructors living as long as the tape
 * (stan/math/rev/core/chainable_alloc.hpp:16-22). */
class chainable_alloc {
 public:
  chainable_alloc() { ChainableStack::instance_->var_alloc_stack_.push_back(this); }
  virtual ~chainable_alloc() {}
};

}  // namespace math
}  // namespace stan
#endif
