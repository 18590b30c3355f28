#ifndef STAN_MATH_REV_CORE_HPP
#define STAN_MATH_REV_CORE_HPP

// Reverse-mode core: tape, vari/var, sweep, nesting, scalar operators.
#include <stan/math/rev/core/autodiffstackstorage.hpp>
#include <stan/math/rev/core/vari.hpp>
#include <stan/math/rev/core/grad.hpp>
#include <stan/math/rev/core/var.hpp>
#include <stan/math/rev/core/operators.hpp>
#include <stan/math/rev/core/precomputed_gradients.hpp>
#include <stan/math/rev/core/print_stack.hpp>
#include <stan/math/prim/special.hpp>

#endif
