#ifndef STAN_MATH_REV_CORE_PRECOMPUTED_GRADIENTS_HPP
#define STAN_MATH_REV_CORE_PRECOMPUTED_GRADIENTS_HPP

// precomputed_gradients_vari / precomputed_gradients
// (stan/math/rev/core/precomputed_gradients.hpp:20-93): one vari over K
// operands with K partials; chain() scatters adj * g[i] into the operands.

#include <stan/math/rev/core/var.hpp>

#include <stdexcept>
#include <vector>

namespace stan {
namespace math {

class precomputed_gradients_vari : public host_local_vari {
 protected:
  const size_t size_;
  vari** varis_;
  double* gradients_;

 public:
  precomputed_gradients_vari(double val, size_t size, vari** varis, double* gradients)
      : host_local_vari(val), size_(size), varis_(varis), gradients_(gradients) {}

  precomputed_gradients_vari(double val, const std::vector<var>& vars,
                             const std::vector<double>& gradients)
      : host_local_vari(val),
        size_(vars.size()),
        varis_(ChainableStack::instance_->memalloc_.alloc_array<vari*>(vars.size())),
        gradients_(ChainableStack::instance_->memalloc_.alloc_array<double>(vars.size())) {
    if (vars.size() != gradients.size())
      throw std::invalid_argument(
          "precomputed_gradients_vari: sizes of vars and gradients do not match");
    for (size_t i = 0; i < vars.size(); ++i) {
      varis_[i] = vars[i].vi_;
      gradients_[i] = gradients[i];
    }
  }

  void chain() override {
    for (size_t i = 0; i < size_; ++i) varis_[i]->adj_ += adj_ * gradients_[i];
  }
  bool touches_adjoints_in(const vari* lo, const vari* hi) const override {
    for (size_t i = 0; i < size_; ++i)
      if (varis_[i] >= lo && varis_[i] < hi) return true;
    return false;
  }
};

inline var precomputed_gradients(double value, const std::vector<var>& operands,
                                 const std::vector<double>& gradients) {
  return var(new precomputed_gradients_vari(value, operands, gradients));
}

}  // namespace math
}  // namespace stan
#endif
