// libsmg_bench.so — BASELINE workloads written against the drop-in
// stan::math API (header-only layer + libsmg_hip.so), exported with a C ABI
// for bench.py / __graft_entry__.smoke().  One "step" = one
// stan::math::gradient() call (stan/math/rev/mat/functor/gradient.hpp:41-57).
#include <stan/math.hpp>

#include <cstdio>
#include <exception>
#include <vector>

namespace {

using stan::math::dev_data;
using stan::math::var;

// config 3: multi_normal_cholesky_lpdf(y | 0, cholesky_decompose(add_diag(
//           gp_exp_quad_cov(x, alpha, rho), sigma^2)))
struct gp_functor {
  const dev_data<double>& x;
  const dev_data<double>& y;
  template <typename T>
  var operator()(const T& th) const {
    using namespace stan::math;
    auto K = gp_exp_quad_cov(x, th[0], th[1]);
    auto Kd = add_diag(K, square(th[2]));
    auto L = cholesky_decompose(Kd);
    return multi_normal_cholesky_lpdf(y, L);
  }
};

dev_data<double> g_x, g_y;
int g_n = 0;
char g_err[512];

int fail(const std::exception& e) {
  std::snprintf(g_err, sizeof g_err, "%s", e.what());
  return -1;
}

}  // namespace

extern "C" {

const char* smg_bench_error() { return g_err; }

void* smg_bench_ctx() { return stan::math::amd::ctx(); }

int smg_bench_gp_init(int device, int n, const double* x, const double* y) {
  try {
    stan::math::amd::set_device(device);
    // data resident in HBM before the timed region (outer arena level, so the
    // nested gradient() scopes never rewind it)
    g_x = stan::math::to_dev_data(x, size_t(n));
    g_y = stan::math::to_dev_data(y, size_t(n));
    g_n = n;
    return 0;
  } catch (const std::exception& e) {
    return fail(e);
  }
}

int smg_bench_gp_step(const double* theta, double* fx, double* grad) {
  try {
    std::vector<double> th(theta, theta + 3), g;
    stan::math::gradient(gp_functor{g_x, g_y}, th, *fx, g);
    for (int i = 0; i < 3; ++i) grad[i] = g[i];
    return 0;
  } catch (const std::exception& e) {
    return fail(e);
  }
}

}  // extern "C"
