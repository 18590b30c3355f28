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

  virtual ~vari() {}

  virtual void chain() {}

  /** True for a node whose chain() reads the adjoints of OTHER varis (not
   * only its own adj_): the reverse sweep lands pending device->host
   * contributions before such a node runs (grad.hpp). */
  virtual bool reads_other_adjoints() const { return false; }

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
