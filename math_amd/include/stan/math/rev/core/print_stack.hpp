#ifndef STAN_MATH_REV_CORE_PRINT_STACK_HPP
#define STAN_MATH_REV_CORE_PRINT_STACK_HPP

// print_stack (stan/math/rev/core/print_stack.hpp:20-31): one line per
// var_stack_ entry, plus the device adjoint buffers this build adds.

#include <stan/math/rev/core/vari.hpp>

#include <ostream>

namespace stan {
namespace math {

inline void print_stack(std::ostream& o) {
  auto* st = ChainableStack::instance_;
  o << "STACK, size=" << st->var_stack_.size() << std::endl;
  for (size_t i = 0; i < st->var_stack_.size(); ++i)
    o << i << "  " << st->var_stack_[i] << "  " << st->var_stack_[i]->val_ << " : "
      << st->var_stack_[i]->adj_ << std::endl;
  o << "DEVICE ADJOINT BUFFERS, size=" << st->dev_adj_stack_.size() << std::endl;
}

}  // namespace math
}  // namespace stan
#endif
