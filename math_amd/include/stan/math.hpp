#ifndef STAN_MATH_HPP
#define STAN_MATH_HPP

// Public entry point, mirroring the reference's `#include <stan/math.hpp>`
// (stan/math.hpp:148).  Header-only host layer over libsmg_hip.so; needs
// Eigen on the include path and -lsmg_hip at link time.
#include <Eigen/Dense>
#define STAN_MATH_AMD_HAS_EIGEN 1

#include <stan/math/rev/core/var.hpp>
#include <stan/math/eigen/num_traits.hpp>
#include <stan/math/rev/core.hpp>
#include <stan/math/amd/matrix.hpp>
#include <stan/math/rev/meta/operands_and_partials.hpp>
#include <stan/math/rev/fun/gp_exp_quad_cov.hpp>
#include <stan/math/rev/fun/cholesky_decompose.hpp>
#include <stan/math/rev/fun/multi_normal_cholesky_lpdf.hpp>
#include <stan/math/rev/fun/multiply.hpp>
#include <stan/math/rev/fun/mdivide_left_tri.hpp>
#include <stan/math/rev/fun/log_sum_exp.hpp>
#include <stan/math/rev/fun/lgamma.hpp>
#include <stan/math/rev/fun/normal_lpdf.hpp>
#include <stan/math/rev/fun/bernoulli_logit_glm_lpmf.hpp>
#include <stan/math/rev/fun/normal_id_glm_lpdf.hpp>
#include <stan/math/rev/fun/poisson_log_glm_lpmf.hpp>
#include <stan/math/rev/fun/categorical_logit_glm_lpmf.hpp>
#include <stan/math/rev/fun/spd_functors.hpp>
#include <stan/math/rev/fun/log_determinant.hpp>
#include <stan/math/rev/functor/gradient.hpp>
#include <stan/math/eigen/interop.hpp>
#include <stan/math/mix/fvar_functors.hpp>
#include <stan/math/mix/hessian_times_vector.hpp>
#include <stan/math/rev/functor/map_rect.hpp>

#endif
