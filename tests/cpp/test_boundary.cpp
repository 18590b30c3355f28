// The drop-in boundary's call forms (tests/cpp/boundary_cases.hpp, the same
// source the reference harness compiles to write the fixtures) against
// math_amd.  Compiling this file is the compile probe: every reference call
// form must resolve to a math_amd overload.  Commands (stdin):
//   forms <inputs of tests/golden/boundary_forms.json>   per case: "<name> f g..."
//   errors                                               "<name> <kind> <what()>"
//   gp_nd N D nobs x(N*D) ys(nobs*N) form P theta(P) reps
//                                                        the Stan-codegen-shaped GP
//                                                        (Eigen::Matrix<var> K / L) through gradient()
//   bridge N touch                                       host-block bookkeeping of the
//                                                        device <-> Eigen round trip
//   chol_nan_arena N                                     cholesky gradient after NaN-poisoned arena
//   gp_share N mode reps                                 one K with two inverse-form consumers / a
//                                                        nested window (closed form vs dense)
//   gp_inter_rep N variant reps x y theta                bnd::run_gp_intermediate, repeated
#include <stan/math.hpp>
#include <algorithm>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <string>
#include <vector>

#include "boundary_cases.hpp"

using namespace stan::math;

static std::vector<double> read_vec(size_t n) {
  std::vector<double> v(n);
  std::string t;
  for (auto& x : v) {
    std::cin >> t;
    x = std::strtod(t.c_str(), nullptr);
  }
  return v;
}
static void print(const std::string& tag, double f, const std::vector<double>& v) {
  std::printf("%s %.17g", tag.c_str(), f);
  for (double x : v) std::printf(" %.17g", x);
  std::printf("\n");
}

static void cmd_forms() {
  bnd::form_inputs in;
  std::cin >> in.m >> in.k >> in.n >> in.s >> in.nobs;
  in.A = read_vec(size_t(in.m) * in.k);
  in.B = read_vec(size_t(in.k) * in.n);
  in.v = read_vec(in.k);
  in.r = read_vec(in.k);
  in.r5 = read_vec(in.m);
  in.S = read_vec(size_t(in.s) * in.s);
  in.d = read_vec(in.s);
  in.L = read_vec(size_t(in.s) * in.s);
  in.ys = read_vec(size_t(in.s) * in.nobs);
  in.mu = read_vec(in.s);
  in.W = read_vec(64);
  in.c = read_vec(1)[0];
  bnd::run_form_cases(in, [](const std::string& name, double f, const std::vector<double>& g) { print(name, f, g); });
  std::printf("stack %zu %zu\n", ChainableStack::instance_->var_stack_.size(),
              ChainableStack::instance_->host_blocks_.size());
}

static void cmd_errors() {
  bnd::run_error_cases([](const std::string& name, const std::function<void()>& f) {
    std::string out;
    try {
      f();
      out = "nothrow";
    } catch (const std::domain_error& e) {
      out = std::string("domain_error ") + e.what();
    } catch (const std::invalid_argument& e) {
      out = std::string("invalid_argument ") + e.what();
    } catch (const std::exception& e) {
      out = std::string("other ") + e.what();
    }
    recover_memory();
    std::printf("%s %s\n", name.c_str(), out.c_str());
  });
}

static void cmd_gp_nd() {
  int N, D, nobs, form, P, reps;
  std::cin >> N >> D >> nobs;
  std::vector<double> xf = read_vec(size_t(N) * D), yf = read_vec(size_t(N) * nobs);
  std::cin >> form >> P;
  std::vector<double> th = read_vec(P);
  std::cin >> reps;
  std::vector<Eigen::VectorXd> x(N, Eigen::VectorXd(D)), ys(nobs, Eigen::VectorXd(N));
  for (int i = 0; i < N; ++i)
    for (int d = 0; d < D; ++d) x[i](d) = xf[size_t(i) * D + d];
  for (int j = 0; j < nobs; ++j)
    for (int i = 0; i < N; ++i) ys[j](i) = yf[size_t(j) * N + i];
  Eigen::VectorXd t = Eigen::Map<Eigen::VectorXd>(th.data(), P), g;
  double fx = 0;
  double best = 1e30;
  for (int r = 0; r < reps; ++r) {
    auto t0 = std::chrono::steady_clock::now();
    gradient(bnd::gp_marginal<Eigen::VectorXd>{x, ys, form}, t, fx, g);
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (dt < best) best = dt;
  }
  print("gp_nd", fx, std::vector<double>(g.data(), g.data() + g.size()));
  std::printf("seconds %.9g\n", best);
  std::printf("stack %zu %zu\n", ChainableStack::instance_->var_stack_.size(),
              ChainableStack::instance_->host_blocks_.size());
}

// The round trip device -> Eigen -> device: the second crossing hands back the
// same node (no gather, no upload), a copy with one element replaced does
// not, and the reverse sweep skips the N^2 host gather unless a host node
// touched the block.  Prints the facts; tests/test_boundary.py checks them.
static void cmd_bridge() {
  int N;
  std::cin >> N;
  std::vector<double> a(size_t(N) * N);
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < N; ++i) a[size_t(j) * N + i] = (i == j ? 2.0 : 0.0) + 1.0 / (1.0 + i + j);
  start_nested();
  dev_var_matrix A = to_dev_var_matrix(a.data(), N, N);
  matrix_v K = add_diag(A, 1.0);  // materialised: one host block
  const size_t h2d_stack = ChainableStack::instance_->var_stack_.size();
  dev_var_matrix back = to_dev(K);
  std::printf("same_node %d\n",
              int(static_cast<void*>(back.vi_) == ChainableStack::instance_->host_blocks_.back().node));
  std::printf("no_bridge_pushed %d\n", int(ChainableStack::instance_->var_stack_.size() == h2d_stack));
  matrix_v K2 = K;
  K2(0, 1) = var(5.0);
  dev_var_matrix other = to_dev(K2);
  std::printf("modified_copy_new_node %d\n",
              int(static_cast<void*>(other.vi_) != ChainableStack::instance_->host_blocks_.back().node));
  matrix_v L = cholesky_decompose(K);  // recognised K, lower block
  const host_block& lb = ChainableStack::instance_->host_blocks_.back();
  int dummy_ok = 1;
  for (int j = 1; j < N; ++j)
    for (int i = 0; i < j; ++i) dummy_ok &= int(L(i, j).vi_ == lb.dummy);
  std::printf("lower_dummy %d\n", dummy_ok);
  // touch == 0: only device consumers (the bridges skip their gathers);
  // touch == 1: a host node reads K(0,0) and L(1,0) too (the gathers run)
  int touch;
  std::cin >> touch;
  var f = sum(cholesky_decompose(K)) + 0.5 * sum(to_dev(L));
  if (touch) f += 2.0 * K(0, 0) + 3.0 * L(1, 0) + 7.0 * L(0, 1);  // L(0,1): the dummy (dropped)
  f.grad();
  print("grad_eigen", f.val(), A.adj());
  std::printf("blocks %zu\n", ChainableStack::instance_->host_blocks_.size());
  recover_memory_nested();
  std::printf("blocks_after %zu\n", ChainableStack::instance_->host_blocks_.size());
  // the same function on device nodes only, K = A + I, L = chol(K)
  start_nested();
  dev_var_matrix A2 = to_dev_var_matrix(a.data(), N, N);
  dev_var_matrix Kd = add_diag(A2, 1.0);
  dev_var_matrix Ld = cholesky_decompose(Kd);
  var g = 1.5 * sum(Ld);
  g.grad();
  print("grad_device", g.val(), A2.adj());
  std::vector<double> lv = Ld.val();
  std::printf("L10 %.17g\n", lv[1]);
  recover_memory_nested();
}

// the Murray reverse reads its work matrix's strict upper as
// stored zeros; recycled arena memory may hold NaN there.  Poison the arena,
// recover it, take the gradient again: it must equal the clean one.
static void cmd_chol_nan_arena() {
  int N;
  std::cin >> N;
  std::vector<double> a(size_t(N) * N);
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < N; ++i) a[size_t(j) * N + i] = (i == j ? double(N) : 0.0) + std::cos(0.37 * (i + j));
  auto run = [&]() {
    start_nested();
    dev_var_matrix A = to_dev_var_matrix(a.data(), N, N);
    var f = sum(cholesky_decompose(A));
    f.grad();
    std::vector<double> g = A.adj();
    recover_memory_nested();
    return g;
  };
  const size_t used0 = smg_arena_used(amd::ctx());
  std::vector<double> g1 = run();
  // poison everything the evaluation used (and more) with NaN bytes
  start_nested();
  const size_t span = size_t(64) * N * N + (size_t(1) << 20);
  double* p = amd::alloc_doubles(span);
  amd::check(smg_memset(amd::ctx(), p, 0xFF, span * sizeof(double)), "poison");
  amd::check(smg_sync(amd::ctx()), "poison");
  recover_memory_nested();
  std::vector<double> g2 = run();
  size_t nan2 = 0, diff = 0;
  for (size_t i = 0; i < g1.size(); ++i) {
    nan2 += std::isnan(g2[i]) ? 1 : 0;
    diff += g1[i] != g2[i] ? 1 : 0;
  }
  std::printf("arena_used0 %zu\n", used0);
  std::printf("nan_entries %zu\n", nan2);
  std::printf("diff_entries %zu\n", diff);
}

// The closed-form Cholesky reverse under an MVN across evaluations at one
// tape position (rev/fun/cholesky_decompose.hpp): evaluation 1 takes it
// unpredicted, 2 with K^{-1} formed alongside the factorisation (history),
// 3 fails in the factorisation (not positive definite) with that work queued,
// 4 must again equal 1.  Prints the max relative difference of 2 and 4 from 1
// and whether 3 threw the reference's domain_error.
static void cmd_chol_mvn_predicted() {
  int N;
  std::cin >> N;
  std::vector<double> a(size_t(N) * N), bad, y(N);
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < N; ++i) a[size_t(j) * N + i] = (i == j ? 2.0 : 0.0) + std::cos(0.37 * (i - j)) * 0.5;
  for (int i = 0; i < N; ++i) y[i] = std::sin(0.1 * i);
  bad = a;
  bad[size_t(N / 2) * N + N / 2] = -1.0;  // a negative pivot in the second half
  auto run = [&](const std::vector<double>& m) {
    start_nested();
    std::vector<double> g;
    try {
      dev_var_matrix A = to_dev_var_matrix(m.data(), N, N);
      var f = multi_normal_cholesky_lpdf(to_dev_data(y), cholesky_decompose(A));
      f.grad();
      g = A.adj();
      g.push_back(f.val());
    } catch (const std::domain_error&) {
      g.clear();
    }
    recover_memory_nested();
    return g;
  };
  std::vector<double> g1 = run(a), g2 = run(a), g3 = run(bad), g4 = run(a);
  auto rel = [&](const std::vector<double>& u) {
    double m = 0.0, s = 0.0;
    for (double v : g1) s = std::max(s, std::fabs(v));
    for (size_t i = 0; i < u.size(); ++i) m = std::max(m, std::fabs(u[i] - g1[i]) / s);
    return m;
  };
  std::printf("rel2 %.3e\n", rel(g2));
  std::printf("threw3 %d\n", g3.empty() ? 1 : 0);
  std::printf("rel4 %.3e\n", rel(g4));
  std::printf("finite %d\n", std::all_of(g4.begin(), g4.end(), [](double v) { return std::isfinite(v); }) ? 1 : 0);
}

// The factor's own adjoint after a sweep whose Cholesky reverse took the
// closed form (never forming it): read through dev_var_matrix::adj() it must
// still hold the MVN's partials, as the reference's varis would.  Prints
// [sum, sum of squares] of L's and A's adjoints.
static void cmd_chol_mvn_ladj() {
  int N;
  std::cin >> N;
  std::vector<double> a(size_t(N) * N), y(N);
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < N; ++i) a[size_t(j) * N + i] = (i == j ? 2.0 : 0.0) + std::cos(0.37 * (i - j)) * 0.5;
  for (int i = 0; i < N; ++i) y[i] = std::sin(0.1 * i);
  start_nested();
  dev_var_matrix A = to_dev_var_matrix(a.data(), N, N);
  dev_var_matrix L = cholesky_decompose(A);
  var f = multi_normal_cholesky_lpdf(to_dev_data(y), L);
  f.grad();
  for (const auto& v : {L.adj(), A.adj()}) {
    double s = 0.0, q = 0.0;
    for (double x : v) {
      s += x;
      q += x * x;
    }
    std::printf("adj %.17g %.17g\n", s, q);
  }
  recover_memory_nested();
}

// One gp_exp_quad_cov output K with two consumers that each take an
// inverse-form adjoint (device API, x_i = 1.1 i: a well-conditioned K):
//   mode 0: two noise terms, K -> add_diag(K, s1) -> chol -> MVN(y1) and
//           K -> add_diag(K, s2) -> chol -> MVN(y2)
//   mode 1: K factored directly and through add_diag(K, s1)
//   mode 2: a nested sweep whose window holds only the Cholesky and MVN
//           nodes: K and Kd = add_diag(K, s1) built outside it (their nodes
//           are not chained), the factor's deposit must still reach Kd.adj()
// `reps` evaluations (the later ones take the predicted closed form with the
// progressive K^{-1}); for the last: "share<mode> lp th' (sigma, l, s1, s2)
// sum / sum of squares of K.adj() and Kd.adj()".  Compared closed form against
// SMG_CHOL_MVN_CLOSED_FORM=0 (tests/test_boundary.py).
static void cmd_gp_share() {
  int N, mode, reps;
  std::cin >> N >> mode >> reps;
  std::vector<double> x(N), y1(N), y2(N);
  for (int i = 0; i < N; ++i) {
    x[i] = 1.1 * i;
    y1[i] = std::sin(0.3 * i);
    y2[i] = std::cos(0.7 * i) * 0.5;
  }
  for (int r = 0; r < reps; ++r) {
    start_nested();
    var sigma = 1.2, l = 0.9, s1 = 0.35, s2 = 0.6;
    dev_var_matrix K = gp_exp_quad_cov(x, sigma, l);
    dev_var_matrix Kd = add_diag(K, s1);
    var lp;
    if (mode == 2) {
      start_nested();
      dev_var_matrix L = cholesky_decompose(Kd);
      lp = multi_normal_cholesky_lpdf(to_dev_data(y1), L);
      grad(lp.vi_);
    } else {
      dev_var_matrix L1 = cholesky_decompose(Kd);
      dev_var_matrix L2 = cholesky_decompose(mode == 0 ? add_diag(K, s2) : K);
      lp = multi_normal_cholesky_lpdf(to_dev_data(y1), L1) + multi_normal_cholesky_lpdf(to_dev_data(y2), L2);
      lp.grad();
    }
    std::vector<double> out = {sigma.adj(), l.adj(), s1.adj(), s2.adj()};
    for (const auto& v : {K.adj(), Kd.adj()}) {
      double a = 0.0, q = 0.0;
      for (double e : v) {
        a += e;
        q += e * e;
      }
      out.push_back(a);
      out.push_back(q);
    }
    if (r + 1 == reps) print("share" + std::to_string(mode), lp.val(), out);
    if (mode == 2) recover_memory_nested();
    recover_memory_nested();
  }
  std::printf("stack %zu %zu\n", ChainableStack::instance_->var_stack_.size(),
              ChainableStack::instance_->host_blocks_.size());
}

// bnd::run_gp_intermediate `reps` times on the same inputs (from the second
// evaluation on the factorisation predicts the closed form and forms K^{-1}
// progressively with its panels); the last one's "gpi lp out..."
static void cmd_gp_inter_rep() {
  int N, variant, reps;
  std::cin >> N >> variant >> reps;
  std::vector<double> x = read_vec(size_t(N)), yv = read_vec(size_t(N)), th = read_vec(3);
  Eigen::VectorXd y = Eigen::Map<Eigen::VectorXd>(yv.data(), N);
  for (int r = 0; r < reps; ++r)
    bnd::run_gp_intermediate(x, y, th.data(), variant, [&](const std::string& name, double f, const std::vector<double>& g) {
      if (r + 1 == reps) print(name, f, g);
    });
  std::printf("stack %zu %zu\n", ChainableStack::instance_->var_stack_.size(),
              ChainableStack::instance_->host_blocks_.size());
}

// bnd::run_gp_intermediate on the fixture's inputs: "gpi lp out..."
static void cmd_gp_inter() {
  int N, variant;
  std::cin >> N >> variant;
  std::vector<double> x = read_vec(size_t(N)), yv = read_vec(size_t(N)), th = read_vec(3);
  Eigen::VectorXd y = Eigen::Map<Eigen::VectorXd>(yv.data(), N);
  bnd::run_gp_intermediate(x, y, th.data(), variant,
                           [](const std::string& name, double f, const std::vector<double>& g) { print(name, f, g); });
  std::printf("stack %zu %zu\n", ChainableStack::instance_->var_stack_.size(),
              ChainableStack::instance_->host_blocks_.size());
}

// The Stan-codegen GP with 1-D x (bnd::gp_marginal<double>, form 0) through
// gradient(), `reps` times (the second and later evaluations take the
// predicted closed form): "gp1d_<r> fx g..." per evaluation
static void cmd_gp_1d() {
  int N, reps;
  std::cin >> N >> reps;
  std::vector<double> x = read_vec(size_t(N)), yv = read_vec(size_t(N)), th = read_vec(3);
  std::vector<Eigen::VectorXd> ys(1, Eigen::Map<Eigen::VectorXd>(yv.data(), N));
  Eigen::VectorXd t = Eigen::Map<Eigen::VectorXd>(th.data(), 3), g;
  for (int r = 0; r < reps; ++r) {
    double fx = 0;
    gradient(bnd::gp_marginal<double>{x, ys, 0}, t, fx, g);
    print("gp1d_" + std::to_string(r), fx, std::vector<double>(g.data(), g.data() + g.size()));
  }
  std::printf("stack %zu %zu\n", ChainableStack::instance_->var_stack_.size(),
              ChainableStack::instance_->host_blocks_.size());
}

int main() {
  std::string cmd;
  while (std::cin >> cmd) {
    if (cmd == "forms") cmd_forms();
    else if (cmd == "errors") cmd_errors();
    else if (cmd == "gp_nd") cmd_gp_nd();
    else if (cmd == "bridge") cmd_bridge();
    else if (cmd == "chol_nan_arena") cmd_chol_nan_arena();
    else if (cmd == "chol_mvn_predicted") cmd_chol_mvn_predicted();
    else if (cmd == "chol_mvn_ladj") cmd_chol_mvn_ladj();
    else if (cmd == "gp_inter") cmd_gp_inter();
    else if (cmd == "gp_1d") cmd_gp_1d();
    else if (cmd == "gp_share") cmd_gp_share();
    else if (cmd == "gp_inter_rep") cmd_gp_inter_rep();
    else {
      std::fprintf(stderr, "unknown command %s\n", cmd.c_str());
      return 2;
    }
    std::fflush(stdout);
  }
  return 0;
}
