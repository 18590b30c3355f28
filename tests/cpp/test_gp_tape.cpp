// GP marginal gradient through the header-only stan::math layer (device path)
// vs the reference golden values (tests/golden/gp_N*.json read by the driver
// script and passed on stdin: N theta(3) x(N) y(N)); prints fx and gradient.
// argv[1] == "mixed": the factor gets a second consumer (+ 1e-3 sum(L)), so
// its adjoint is no longer the MVN's alone (the dense-adjoint fallback of
// rev/fun/cholesky_decompose.hpp).
#include <stan/math.hpp>
#include <cstdio>
#include <iostream>
#include <string>
#include <vector>

struct gp_functor {
  const std::vector<double>& x;
  const std::vector<double>& y;
  bool mixed;
  template <typename T>
  stan::math::var operator()(const T& th) const {
    using namespace stan::math;
    auto K = gp_exp_quad_cov(x, th[0], th[1]);
    auto Kd = add_diag(K, square(th[2]));
    auto L = cholesky_decompose(Kd);
    std::vector<double> mu(x.size(), 0.0);
    var lp = multi_normal_cholesky_lpdf(y, mu, L);
    if (mixed) lp += 1e-3 * sum(L);
    return lp;
  }
};

int main(int argc, char** argv) {
  const bool mixed = argc > 1 && std::string(argv[1]) == "mixed";
  int N;
  std::vector<double> th(3);
  if (!(std::cin >> N >> th[0] >> th[1] >> th[2])) return 2;
  std::vector<double> x(N), y(N);
  for (auto& v : x) std::cin >> v;
  for (auto& v : y) std::cin >> v;
  for (int rep = 0; rep < 2; ++rep) {
    double fx;
    std::vector<double> g;
    stan::math::gradient(gp_functor{x, y, mixed}, th, fx, g);
    std::printf("%.17g %.17g %.17g %.17g\n", fx, g[0], g[1], g[2]);
  }
  // Eigen signature: gradient(F, VectorXd, double&, VectorXd&)
  Eigen::VectorXd t(3), ge;
  t << th[0], th[1], th[2];
  double fx;
  stan::math::gradient(gp_functor{x, y, mixed}, t, fx, ge);
  std::printf("%.17g %.17g %.17g %.17g\n", fx, ge[0], ge[1], ge[2]);
  std::printf("stack %zu %zu\n", stan::math::ChainableStack::instance_->var_stack_.size(),
              stan::math::ChainableStack::instance_->dev_adj_stack_.size());
  return 0;
}
