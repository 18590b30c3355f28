// Drives every §8 functor of the header-only stan::math layer on the device.
// Reads one command and its inputs from stdin (written by
// tests/test_cpp_functors.py from the golden fixtures), prints the values and
// gradients as %.17g for comparison with the reference's.
//
//   mulchol N nsamp idx...        config 2 via the device-leaf gradient
//   mulchol_eigen N               config 2 via Eigen Matrix<var> (host varis)
//   multiply kind m k n A B W     f = sum(W .* multiply(A, B))
//   mdivide lower kind m n A B W  f = sum(W .* mdivide_left_tri<TriView>(A, B))
//   lse N x                       log_sum_exp(std::vector<var>) and (Matrix<var>)
//   lse_pair n a b                log_sum_exp(var, var)
//   special n x                   lgamma(var), digamma(var) values + derivatives
//   special_vec X(200) W(200)     f = sum(W .* (lgamma(X) + 0.5 digamma(X))), Matrix<var> 10x20
//   normal N theta                gradient of normal_lpdf(theta | 0, 1)
//   normal_vec y mu sigma (9)     all var vectors; f, f(propto), gradients
//   normal_big N y mu sigma       n > 4096: the fused kernel's multi-block path (host vars,
//                                 scalar var mu, device operands)
//   normal_known y mu sigma (4)   double arguments -> values
//   glm R M nb beta               device-filled (x, y); single call and 32 row shards
//   glm_data R M x y theta        explicit data (cutoff branches)
//   mvn N y mu L                  multi_normal_cholesky_lpdf, every argument var (Eigen)
//   errors                        the reference's exceptions
//   hvp N theta v x y             hessian_times_vector of the GP marginal (config 5)
//   hessian N theta x y           hessian() of the GP marginal (3 fwd-over-rev sweeps)
//   hvp_fd N theta v x y h        H v at full size vs the extrapolated central difference of the gradient
//   map_rect_glm R M shards beta  map_rect over GLM row blocks (vs the reference's map_rect32)
//   spd kind n k args... W        mdivide_left_spd / log_determinant_spd /
//                                 multiply_lower_tri_self_transpose / quad_form_sym through the
//                                 Eigen signatures; f = sum(W .* F(args)), gradient over all entries
//   glm2 kind R M y theta         normal_id_glm_lpdf (kind 0) / poisson_log_glm_lpmf (kind 1):
//                                 device x, single call, 7 row shards, propto
//   glm_cat R M C ys y theta      categorical_logit_glm_lpmf: device path (dev_var_matrix alpha /
//                                 beta, 5 row shards), Eigen path (Matrix<var>), mixed and
//                                 all-double operands; x filled on the device (gen.glm_cat_inputs)
//   glm_cat_errors                the reference's exceptions / early returns on small inputs
//   ops_partials y mu sigma (9)   a user lpdf on operands_and_partials (vector / Eigen / device /
//                                 data / broadcast edges)
//   status                        a latched SMG_ERR_SYNC throws from the gradient() / readback that
//                                 ran it, and is cleared
#include <stan/math.hpp>

#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <iostream>
#include <string>
#include <vector>

using namespace stan::math;

// tokens through strtod so inf / -inf / nan parse like any other value
static std::vector<double> read_vec(size_t n) {
  std::vector<double> v(n);
  std::string t;
  for (auto& x : v) {
    std::cin >> t;
    x = std::strtod(t.c_str(), nullptr);
  }
  return v;
}
static void print(const char* tag, const std::vector<double>& v) {
  std::printf("%s", tag);
  for (double x : v) std::printf(" %.17g", x);
  std::printf("\n");
}
static void print1(const char* tag, double v) { std::printf("%s %.17g\n", tag, v); }

static std::vector<var> vars(const std::vector<double>& v) {
  return std::vector<var>(v.begin(), v.end());
}
static std::vector<double> adjs(const std::vector<var>& v) {
  std::vector<double> g(v.size());
  for (size_t i = 0; i < v.size(); ++i) g[i] = v[i].adj();
  return g;
}
// sum_i w_i * c_i over host vars (scalar tape ops)
static var wdot(const std::vector<double>& w, const std::vector<var>& c) {
  var s = 0.0;
  for (size_t i = 0; i < w.size(); ++i) s += w[i] * c[i];
  return s;
}

static void cmd_mulchol() {
  int N, ns;
  std::cin >> N >> ns;
  std::vector<long long> idx(ns);
  for (auto& i : idx) std::cin >> i;
  smg_ctx* c = amd::ctx();
  const size_t nn = size_t(N) * N;
  double* A = amd::alloc_doubles(nn);
  double* G = amd::alloc_doubles(nn);
  amd::check(smg_fill_unif(c, A, (long long)nn, 20260101ull + 2, -1.0, 1.0, std::sqrt(3.0 / N)), "fill");
  auto f = [N](const dev_var_matrix& a) {
    return sum(cholesky_decompose(add_diag(multiply(a, transpose(a)), double(N))));
  };
  for (int rep = 0; rep < 2; ++rep) {
    double fx;
    gradient(f, dev_data<double>(A, nn, N, N), fx, G);
    std::vector<double> g(nn);
    amd::to_host(g.data(), G, nn);
    double s = 0, l2 = 0;
    for (double v : g) {
      s += v;
      l2 += v * v;
    }
    print1("fx", fx);
    print1("grad_sum", s);
    print1("grad_l2", std::sqrt(l2));
    std::vector<double> samp;
    if (ns == 0)
      samp = g;
    else
      for (long long i : idx) samp.push_back(g[i]);
    print("grad", samp);
  }
}

// the Gram product multiply(A, transpose(A)) with the transpose ALSO used
// elsewhere (its adjoint nonzero): f = sum(A A^T) + w sum(transpose(A)) +
// sum(multiply(transpose(A), A)) over an N x M matrix A (host values)
static void cmd_gram_shared() {
  int N, M;
  double w;
  std::cin >> N >> M >> w;
  std::vector<double> a = read_vec(size_t(N) * M);
  smg_ctx* c = amd::ctx();
  const size_t nm = size_t(N) * M;
  double* G = amd::alloc_doubles(nm);
  dev_data<double> A = to_dev_data(a.data(), nm, N, M);
  auto f = [w](const dev_var_matrix& x) {
    dev_var_matrix t = transpose(x);
    return sum(multiply(x, t)) + w * sum(t) + sum(multiply(t, x));
  };
  double fx;
  gradient(f, A, fx, G);
  std::vector<double> g(nm);
  amd::to_host(g.data(), G, nm);
  (void)c;
  print1("fx", fx);
  print("grad", g);
}

static void cmd_mulchol_eigen() {
  int N;
  std::cin >> N;
  std::vector<double> a = read_vec(size_t(N) * N);
  Eigen::VectorXd x = Eigen::Map<Eigen::VectorXd>(a.data(), a.size()), g;
  double fx;
  auto f = [N](const vector_v& v) {
    matrix_v A(N, N);
    for (int i = 0; i < N * N; ++i) A(i) = v(i);
    matrix_v C = multiply(A, transpose(A));
    matrix_v Cd = add_diag(C, double(N));
    return sum(cholesky_decompose(Cd));
  };
  gradient(f, x, fx, g);
  print1("fx", fx);
  print("grad", std::vector<double>(g.data(), g.data() + g.size()));
}

static void cmd_multiply() {
  int kind, m, k, n;
  std::cin >> kind >> m >> k >> n;
  auto A = read_vec(size_t(m) * k), B = read_vec(size_t(k) * n), W = read_vec(size_t(m) * n);
  start_nested();
  std::vector<var> av = vars(A), bv = vars(B);
  dev_var_matrix C;
  if (kind == 0) C = multiply(to_dev(av, m, k), to_dev(bv, k, n));
  if (kind == 1) C = multiply(to_dev(av, m, k), to_dev_data(B.data(), B.size(), k, n));
  if (kind == 2) C = multiply(to_dev_data(A.data(), A.size(), m, k), to_dev(bv, k, n));
  var f = wdot(W, to_var_vector(C));
  f.grad();
  print1("fx", f.val());
  print1("fx_C0", C.val()[0]);
  print("C", C.val());
  print("grad_A", kind == 2 ? std::vector<double>(A.size(), 0.0) : adjs(av));
  print("grad_B", kind == 1 ? std::vector<double>(B.size(), 0.0) : adjs(bv));
  recover_memory_nested();
  // Eigen signature, var * var
  if (kind == 0) {
    start_nested();
    matrix_v Ae(m, k), Be(k, n);
    for (int i = 0; i < m * k; ++i) Ae(i) = A[i];
    for (int i = 0; i < k * n; ++i) Be(i) = B[i];
    matrix_v Ce = multiply(Ae, Be);
    var fe = 0.0;
    for (int i = 0; i < m * n; ++i) fe += W[i] * Ce(i);
    fe.grad();
    std::vector<double> ga(m * k);
    for (int i = 0; i < m * k; ++i) ga[i] = Ae(i).adj();
    print1("fx_eigen", fe.val());
    print("grad_A_eigen", ga);
    recover_memory_nested();
  }
}

static void cmd_mdivide() {
  int lower, kind, m, n;
  std::cin >> lower >> kind >> m >> n;
  auto A = read_vec(size_t(m) * m), B = read_vec(size_t(m) * n), W = read_vec(size_t(m) * n);
  start_nested();
  std::vector<var> av = vars(A), bv = vars(B);
  dev_var_matrix C;
  auto Ad = [&]() { return to_dev(av, m, m); };
  auto Bd = [&]() { return to_dev(bv, m, n); };
  auto Ac = to_dev_data(A.data(), A.size(), m, m);
  auto Bc = to_dev_data(B.data(), B.size(), m, n);
  if (lower) {
    if (kind == 0) C = mdivide_left_tri<1>(Ad(), Bd());
    if (kind == 1) C = mdivide_left_tri<1>(Ac, Bd());
    if (kind == 2) C = mdivide_left_tri<1>(Ad(), Bc);
  } else {
    if (kind == 0) C = mdivide_left_tri<2>(Ad(), Bd());
    if (kind == 1) C = mdivide_left_tri<2>(Ac, Bd());
    if (kind == 2) C = mdivide_left_tri<2>(Ad(), Bc);
  }
  var f = wdot(W, to_var_vector(C));
  f.grad();
  print1("fx", f.val());
  print("C", C.val());
  print("grad_A", kind == 1 ? std::vector<double>(A.size(), 0.0) : adjs(av));
  print("grad_B", kind == 2 ? std::vector<double>(B.size(), 0.0) : adjs(bv));
  recover_memory_nested();
}

static void cmd_lse() {
  int N;
  std::cin >> N;
  auto x = read_vec(N);
  start_nested();
  std::vector<var> xv = vars(x);
  var f = log_sum_exp(xv);
  f.grad();
  print1("fx", f.val());
  print("grad", adjs(xv));
  recover_memory_nested();
  start_nested();
  vector_v xe(N);
  for (int i = 0; i < N; ++i) xe(i) = x[i];
  var fe = log_sum_exp(xe);
  fe.grad();
  std::vector<double> g(N);
  for (int i = 0; i < N; ++i) g[i] = xe(i).adj();
  print1("fx_eigen", fe.val());
  print("grad_eigen", g);
  recover_memory_nested();
}

static void cmd_lse_pair() {
  int n;
  std::cin >> n;
  auto a = read_vec(n), b = read_vec(n);
  std::vector<double> f(n), ga(n), gb(n);
  for (int i = 0; i < n; ++i) {
    start_nested();
    var av = a[i], bv = b[i];
    var r = log_sum_exp(av, bv);
    r.grad();
    f[i] = r.val();
    ga[i] = av.adj();
    gb[i] = bv.adj();
    recover_memory_nested();
  }
  print("f", f);
  print("grad_a", ga);
  print("grad_b", gb);
}

static void cmd_special() {
  int n;
  std::cin >> n;
  auto x = read_vec(n);
  std::vector<double> lg(n), dg(n), glg(n), gdg(n);
  for (int i = 0; i < n; ++i) {
    start_nested();
    var a = x[i];
    var y = lgamma(a);
    y.grad();
    lg[i] = y.val();
    glg[i] = a.adj();
    recover_memory_nested();
    start_nested();
    var b = x[i];
    var z = digamma(b);
    z.grad();
    dg[i] = z.val();
    gdg[i] = b.adj();
    recover_memory_nested();
  }
  print("lgamma", lg);
  print("digamma", dg);
  print("grad_lgamma", glg);
  print("grad_digamma", gdg);
  // vectorised device path over the same inputs (values only)
  start_nested();
  std::vector<var> xv = vars(x);
  std::vector<var> l = lgamma(xv), d = digamma(xv);
  std::vector<double> lv(n), dv(n);
  for (int i = 0; i < n; ++i) {
    lv[i] = l[i].val();
    dv[i] = d[i].val();
  }
  print("lgamma_dev", lv);
  print("digamma_dev", dv);
  recover_memory_nested();
}

static void cmd_special_vec() {
  auto X = read_vec(200), W = read_vec(200);
  start_nested();
  matrix_v Xe(10, 20);
  for (int i = 0; i < 200; ++i) Xe(i) = X[i];
  matrix_v L = lgamma(Xe), D = digamma(Xe);
  var f = 0.0;
  for (int i = 0; i < 200; ++i) f += W[i] * (L(i) + 0.5 * D(i));
  f.grad();
  std::vector<double> g(200);
  for (int i = 0; i < 200; ++i) g[i] = Xe(i).adj();
  print1("fx", f.val());
  print("grad", g);
  recover_memory_nested();
}

static void cmd_normal() {
  int N;
  std::cin >> N;
  auto th = read_vec(N);
  double fx;
  std::vector<double> g;
  for (int rep = 0; rep < 2; ++rep) {
    gradient([](const std::vector<var>& t) { return normal_lpdf(t, 0.0, 1.0); }, th, fx, g);
    print1("fx", fx);
    print("grad", g);
  }
  // device-resident parameters (dev_var_matrix) through the same functor
  start_nested();
  auto d = to_dev_var_matrix(th.data(), N, 1);
  var f = normal_lpdf(d, 0.0, 1.0);
  f.grad();
  print1("fx_dev", f.val());
  print("grad_dev", d.adj());
  recover_memory_nested();
}

// The fused kernel's multi-block path (n > 4096): host vars (zero-copy pinned
// operands above the host gate), mixed scalar var / vector data, and
// dev_var_matrix operands.  Prints f and every gradient for the closed form.
static void cmd_normal_big() {
  int N;
  std::cin >> N;
  auto y = read_vec(N), mu = read_vec(N), s = read_vec(N);
  {  // all vectors host vars
    start_nested();
    std::vector<var> yv = vars(y), mv = vars(mu), sv = vars(s);
    var f = normal_lpdf(yv, mv, sv);
    f.grad();
    print1("fx_vvv", f.val());
    print("gy_vvv", adjs(yv));
    print("gmu_vvv", adjs(mv));
    print("gs_vvv", adjs(sv));
    recover_memory_nested();
  }
  {  // y host vars, mu scalar var, sigma vector data
    start_nested();
    std::vector<var> yv = vars(y);
    var m0 = 0.25;
    var f = normal_lpdf(yv, m0, s);
    f.grad();
    print1("fx_vsd", f.val());
    print("gy_vsd", adjs(yv));
    print1("gmu_vsd", m0.adj());
    recover_memory_nested();
  }
  {  // device-resident y and sigma, mu data vector
    start_nested();
    auto yd = to_dev_var_matrix(y.data(), N, 1);
    auto sd = to_dev_var_matrix(s.data(), N, 1);
    var f = normal_lpdf(yd, mu, sd);
    f.grad();
    print1("fx_dev", f.val());
    print("gy_dev", yd.adj());
    print("gs_dev", sd.adj());
    recover_memory_nested();
  }
}

static void cmd_normal_vec() {
  auto y = read_vec(9), mu = read_vec(9), s = read_vec(9);
  start_nested();
  std::vector<var> yv = vars(y), mv = vars(mu), sv = vars(s);
  var f = normal_lpdf(yv, mv, sv);
  f.grad();
  print1("fx", f.val());
  print("grad_y", adjs(yv));
  print("grad_mu", adjs(mv));
  print("grad_sigma", adjs(sv));
  var fp = normal_lpdf<true>(yv, mv, sv);
  print1("fx_propto", fp.val());
  recover_memory_nested();
}

// A user-written lpdf on the reference's operands_and_partials API
// (rev/scal/meta/operands_and_partials.hpp:72-127): host arithmetic, one
// node over three edges of different kinds.
template <typename T_y, typename T_mu, typename T_s>
static var user_normal_lpdf(const T_y& y, const T_mu& mu, const T_s& sigma, const std::vector<double>& yv,
                            const std::vector<double>& mv, const std::vector<double>& sv) {
  operands_and_partials<T_y, T_mu, T_s> ops_partials(y, mu, sigma);
  double logp = 0.0;
  for (size_t i = 0; i < yv.size(); ++i) {
    const double inv_s = 1.0 / sv[i], z = (yv[i] - mv[i]) * inv_s;
    logp += -0.5 * z * z - std::log(sv[i]) - 0.5 * std::log(2.0 * M_PI);
    ops_partials.edge1_.partials_[int(i)] -= inv_s * z;
    ops_partials.edge2_.partials_[int(i)] += inv_s * z;
    ops_partials.edge3_.partials_[int(i)] += -inv_s + inv_s * z * z;
  }
  return ops_partials.build(logp);
}

static void cmd_ops_partials() {
  auto y = read_vec(9), mu = read_vec(9), s = read_vec(9);
  start_nested();
  {  // std::vector<var>, Eigen::Matrix<var>, std::vector<var> edges
    std::vector<var> yv = vars(y), sv = vars(s);
    Eigen::Matrix<var, Eigen::Dynamic, 1> mv(9);
    for (int i = 0; i < 9; ++i) mv(i) = mu[size_t(i)];
    var f = user_normal_lpdf(yv, mv, sv, y, mu, s);
    f.grad();
    print1("fx", f.val());
    print("grad_y", adjs(yv));
    std::vector<double> gm(9);
    for (int i = 0; i < 9; ++i) gm[size_t(i)] = mv(i).adj();
    print("grad_mu", gm);
    print("grad_sigma", adjs(sv));
  }
  set_zero_all_adjoints_nested();
  {  // a data edge (y), a device edge (mu: dev_var_matrix, partials set from the host), a scalar-broadcast var
    auto md = to_dev_var_matrix(mu.data(), 9, 1);
    var s0 = s[0];
    std::vector<double> s9(9, s[0]);
    operands_and_partials<std::vector<double>, dev_var_matrix, var> op(y, md, s0);
    double logp = 0.0;
    std::vector<double> gmu(9);
    for (int i = 0; i < 9; ++i) {
      const double z = (y[size_t(i)] - mu[size_t(i)]) / s[0];
      logp += -0.5 * z * z - std::log(s[0]) - 0.5 * std::log(2.0 * M_PI);
      op.edge1_.partials_[i] -= z / s[0];  // swallowed: data
      gmu[size_t(i)] = z / s[0];
      op.edge3_.partials_[i] += -1.0 / s[0] + z * z / s[0];  // broadcast: all alias one partial
    }
    op.edge2_.set_partials(gmu.data());
    var f = op.build(logp);
    f.grad();
    print1("fx_mixed", f.val());
    print("grad_mu_dev", md.adj());
    print1("grad_sigma_scalar", s0.adj());
    // all-double operands: build() returns the value
    operands_and_partials<std::vector<double>, double> od(y, 1.0);
    print1("double_build", od.build(3.5));
  }
  recover_memory_nested();
  std::printf("stack %zu %zu\n", ChainableStack::instance_->var_stack_.size(),
              ChainableStack::instance_->dev_adj_stack_.size());
}

static void cmd_normal_known() {
  auto y = read_vec(4), mu = read_vec(4), s = read_vec(4);
  std::vector<double> out(4);
  for (int i = 0; i < 4; ++i) out[i] = normal_lpdf(y[i], mu[i], s[i]);
  print("values", out);
  // propto with all-double arguments drops every term (include_summand)
  print1("propto_double", normal_lpdf<true>(y[0], mu[0], s[0]));
}

static void cmd_glm() {
  long long R;
  int M;
  std::cin >> R >> M;
  auto beta = read_vec(M);
  smg_ctx* c = amd::ctx();
  // resident data outside any nested tape (like the MPI data cache)
  int* y = amd::alloc_ints(size_t(R));
  double* x = amd::alloc_doubles(size_t(R) * M);
  amd::check(smg_fill_unif(c, x, R * M, 20260101ull + 41, -1.0, 1.0, std::sqrt(3.0)), "fill");
  amd::check(smg_fill_bernoulli(c, y, R, 20260101ull + 42, 0.5), "fill");
  std::vector<double> th(M + 1);
  th[0] = 0.1;
  for (int j = 0; j < M; ++j) th[1 + j] = beta[j];
  dev_data<int> yd(y, size_t(R), int(R), 1);
  dev_data<double> xd(x, size_t(R) * M, int(R), M);
  double fx;
  std::vector<double> g;
  for (int rep = 0; rep < 2; ++rep) {
    gradient(
        [&](const std::vector<var>& t) {
          std::vector<var> b(t.begin() + 1, t.end());
          return bernoulli_logit_glm_lpmf(yd, xd, t[0], b);
        },
        th, fx, g);
    print1("fx", fx);
    print("grad", g);
  }
  // 32 contiguous row shards summed on the tape (the map_rect32 decomposition)
  gradient(
      [&](const std::vector<var>& t) {
        std::vector<var> b(t.begin() + 1, t.end());
        var s = 0.0;
        for (int k = 0; k < 32; ++k) {
          long long b0, b1;
          row_partition(R, 32, k, &b0, &b1);
          glm_shard sh;
          sh.y = y + b0;
          sh.x = x + b0;
          sh.rows = b1 - b0;
          sh.M = M;
          sh.ldx = R;
          sh.row0 = b0;
          sh.total_rows = R;
          s += bernoulli_logit_glm_lpmf<false>(sh, t[0], b);
        }
        return s;
      },
      th, fx, g);
  print1("fx_shards32", fx);
  print("grad_shards32", g);
}

static void cmd_spd() {
  int kind, n, k;
  std::cin >> kind >> n >> k;
  size_t na = kind == 2 ? size_t(n) * k : size_t(n) * n;
  size_t nb = (kind == 0 || kind == 3) ? size_t(n) * k : 0;
  auto th = read_vec(na + nb);
  const int wr = kind == 0 ? n : (kind == 3 ? k : n), wc = kind == 0 ? k : (kind == 3 ? k : n);
  std::vector<double> W = kind == 1 ? std::vector<double>() : read_vec(size_t(wr) * wc);
  auto take = [](const std::vector<var>& t, size_t off, int r, int c) {
    matrix_v m(r, c);
    for (int i = 0; i < r * c; ++i) m(i) = t[off + size_t(i)];
    return m;
  };
  auto wsum = [&](const matrix_v& C) {
    var s = 0.0;
    for (int i = 0; i < C.size(); ++i) s += W[size_t(i)] * C(i);
    return s;
  };
  double fx;
  std::vector<double> g;
  gradient(
      [&](const std::vector<var>& t) -> var {
        if (kind == 0) return wsum(mdivide_left_spd(take(t, 0, n, n), take(t, na, n, k)));
        if (kind == 1) return log_determinant_spd(take(t, 0, n, n));
        if (kind == 2) return wsum(multiply_lower_tri_self_transpose(take(t, 0, n, k)));
        return wsum(quad_form_sym(take(t, 0, n, n), take(t, na, n, k)));
      },
      th, fx, g);
  print1("fx", fx);
  print("grad", g);
}

// log_determinant (rev/mat/fun/log_determinant.hpp:14-37): gradient through
// the Eigen signature (host vars bridged to one device node), the device
// signature (dev_var_matrix leaf), the prim double value, and check_square
static void cmd_logdet() {
  int n;
  std::cin >> n;
  auto a = read_vec(size_t(n) * n);
  double fx;
  std::vector<double> g;
  gradient(
      [&](const std::vector<var>& t) -> var {
        matrix_v m(n, n);
        for (int i = 0; i < n * n; ++i) m(i) = t[size_t(i)];
        return log_determinant(m);
      },
      a, fx, g);
  print1("fx", fx);
  print("grad", g);
  smg_ctx* c = amd::ctx();
  double* ad = amd::alloc_doubles(size_t(n) * n);
  amd::to_device(ad, a.data(), size_t(n) * n);
  double* gd = amd::alloc_doubles(size_t(n) * n);
  double fxd;
  gradient([&](const dev_var_matrix& m) { return log_determinant(m); }, dev_data<double>(ad, size_t(n) * n, n, n),
           fxd, gd);
  std::vector<double> gh(size_t(n) * n);
  amd::to_host(gh.data(), gd, gh.size());
  print1("fx_dev", fxd);
  print("grad_dev", gh);
  const Eigen::MatrixXd md = Eigen::Map<const Eigen::MatrixXd>(a.data(), n, n);
  print1("fx_prim", log_determinant(md));
  try {
    matrix_v r(2, 3);
    for (int i = 0; i < 6; ++i) r(i) = var(double(i + 1));
    log_determinant(r);
    std::printf("square none\n");
  } catch (const std::invalid_argument& e) {
    std::printf("square %s\n", e.what());
  }
  matrix_v e0(0, 0);
  print1("empty", log_determinant(e0).val());
  recover_memory();  // the check_square / empty-input vars above live on the outer tape
  std::printf("stack %zu %zu\n", ChainableStack::instance_->var_stack_.size(),
              ChainableStack::instance_->nested_var_stack_sizes_.size());
}

static void cmd_glm2() {
  int kind, M;
  long long R;
  std::cin >> kind >> R >> M;
  auto yv = read_vec(size_t(R));
  auto th = read_vec(size_t(kind == 0 ? M + 2 : M + 1));
  smg_ctx* c = amd::ctx();
  double* x = amd::alloc_doubles(size_t(R) * M);
  amd::check(smg_fill_unif(c, x, R * M, 20260101ull + 41, -1.0, 1.0, std::sqrt(3.0)), "fill");
  std::vector<int> yi(yv.begin(), yv.end());
  dev_data<double> yd = to_dev_data(yv);
  dev_data<int> ydi = to_dev_data(yi);
  dev_data<double> xd(x, size_t(R) * M, int(R), M);
  auto f = [&](const std::vector<var>& t, auto propto_tag) {
    constexpr bool P = decltype(propto_tag)::value;
    std::vector<var> b(t.begin() + 1, t.begin() + 1 + M);
    if (kind == 0) return normal_id_glm_lpdf<P>(yd, xd, t[0], b, t[M + 1]);
    return poisson_log_glm_lpmf<P>(ydi, xd, t[0], b);
  };
  double fx;
  std::vector<double> g;
  gradient([&](const std::vector<var>& t) { return f(t, std::false_type{}); }, th, fx, g);
  print1("fx", fx);
  print("grad", g);
  gradient([&](const std::vector<var>& t) { return f(t, std::true_type{}); }, th, fx, g);
  print1("fx_propto", fx);
  print("grad_propto", g);
  // 7 contiguous row shards summed on the tape (each shard: its own N)
  gradient(
      [&](const std::vector<var>& t) {
        std::vector<var> b(t.begin() + 1, t.begin() + 1 + M);
        var s = 0.0;
        for (int k = 0; k < 7; ++k) {
          long long b0, b1;
          row_partition(R, 7, k, &b0, &b1);
          glm_shard sh;
          sh.y = ydi.data() + b0;
          sh.yd = yd.data() + b0;
          sh.x = x + b0;
          sh.rows = b1 - b0;
          sh.M = M;
          sh.ldx = R;
          sh.row0 = b0;
          sh.total_rows = b1 - b0;
          if (kind == 0) s += normal_id_glm_lpdf<false>(sh, t[0], b, t[M + 1]);
          else s += poisson_log_glm_lpmf<false>(sh, t[0], b);
        }
        return s;
      },
      th, fx, g);
  print1("fx_shards7", fx);
  print("grad_shards7", g);
  // all-double arguments: a plain double, no tape
  std::vector<double> bd(th.begin() + 1, th.begin() + 1 + M);
  start_nested();
  const double v = kind == 0 ? normal_id_glm_lpdf<false>(yd, xd, th[0], bd, th[M + 1])
                             : poisson_log_glm_lpmf<false>(ydi, xd, th[0], bd);
  recover_memory_nested();
  print1("fx_double", v);
}

static void cmd_glm_data() {
  int R, M;
  std::cin >> R >> M;
  auto xv = read_vec(size_t(R) * M), yv = read_vec(R), th = read_vec(M + 1);
  std::vector<int> y(R);
  for (int i = 0; i < R; ++i) y[i] = int(yv[i]);
  double fx;
  std::vector<double> g;
  gradient(
      [&](const std::vector<var>& t) {
        std::vector<var> b(t.begin() + 1, t.end());
        return bernoulli_logit_glm_lpmf(y, xv, M, t[0], b);
      },
      th, fx, g);
  print1("fx", fx);
  print("grad", g);
  // Eigen signature (x MatrixXd, beta Matrix<var,-1,1>)
  start_nested();
  matrix_d xe = Eigen::Map<matrix_d>(xv.data(), R, M);
  vector_v be(M);
  for (int j = 0; j < M; ++j) be(j) = th[1 + j];
  var a = th[0];
  var f = bernoulli_logit_glm_lpmf(y, xe, a, be);
  f.grad();
  std::vector<double> ge(M + 1);
  ge[0] = a.adj();
  for (int j = 0; j < M; ++j) ge[1 + j] = be(j).adj();
  print1("fx_eigen", f.val());
  print("grad_eigen", ge);
  recover_memory_nested();
}

static void cmd_mvn() {
  int N;
  std::cin >> N;
  auto y = read_vec(N), mu = read_vec(N), L = read_vec(size_t(N) * N);
  start_nested();
  std::vector<var> yv = vars(y), mv = vars(mu), Lv = vars(L);
  matrix_v Le(N, N);
  for (int i = 0; i < N * N; ++i) Le(i) = Lv[i];
  vector_v ye(N), me(N);
  for (int i = 0; i < N; ++i) {
    ye(i) = yv[i];
    me(i) = mv[i];
  }
  var f = multi_normal_cholesky_lpdf(ye, me, Le);
  f.grad();
  print1("fx", f.val());
  print("grad_y", adjs(yv));
  print("grad_mu", adjs(mv));
  print("grad_L", adjs(Lv));
  recover_memory_nested();
}

// map_rect job: one block of GLM rows; x_r = the block of x (column-major), x_i = y
// (the reference harness's glm_shard_functor, oracle/ref_harness.cpp)
struct glm_job {
  template <typename T1, typename T2>
  Eigen::Matrix<T1, Eigen::Dynamic, 1> operator()(const Eigen::Matrix<T1, Eigen::Dynamic, 1>& eta,
                                                  const Eigen::Matrix<T2, Eigen::Dynamic, 1>&,
                                                  const std::vector<double>& x_r,
                                                  const std::vector<int>& x_i, std::ostream*) const {
    const int M = int(eta.size()) - 1, r = int(x_i.size());
    matrix_d xs = Eigen::Map<const matrix_d>(x_r.data(), r, M);
    Eigen::Matrix<T1, Eigen::Dynamic, 1> beta = eta.tail(M);
    Eigen::Matrix<T1, Eigen::Dynamic, 1> out(1);
    out(0) = bernoulli_logit_glm_lpmf(x_i, xs, eta(0), beta);
    return out;
  }
};

// map_rect over `shards` row blocks of the config-4 data (generated on the device)
static void cmd_map_rect_glm() {
  long long R;
  int M, shards;
  std::cin >> R >> M >> shards;
  auto beta = read_vec(M);
  smg_ctx* c = amd::ctx();
  std::vector<double> x(size_t(R) * M);
  std::vector<int> y(R);
  {
    double* xd = amd::alloc_doubles(x.size());
    int* yd = amd::alloc_ints(y.size());
    amd::check(smg_fill_unif(c, xd, R * M, 20260101ull + 41, -1.0, 1.0, std::sqrt(3.0)), "fill");
    amd::check(smg_fill_bernoulli(c, yd, R, 20260101ull + 42, 0.5), "fill");
    amd::to_host(x.data(), xd, x.size());
    amd::check(smg_memcpy_d2h(c, y.data(), yd, y.size() * sizeof(int)), "copy");
    amd::check(smg_sync(c), "copy");
  }
  std::vector<std::vector<double>> xr(shards);
  std::vector<std::vector<int>> xi(shards);
  for (int s = 0; s < shards; ++s) {
    long long r0, r1;
    row_partition(R, shards, s, &r0, &r1);
    const long long r = r1 - r0;
    xr[s].resize(size_t(r) * M);
    for (int j = 0; j < M; ++j)
      for (long long i = 0; i < r; ++i) xr[s][size_t(j) * r + i] = x[size_t(j) * R + r0 + i];
    xi[s].assign(y.begin() + r0, y.begin() + r1);
  }
  Eigen::VectorXd th(M + 1), g;
  th(0) = 0.1;
  for (int j = 0; j < M; ++j) th(1 + j) = beta[j];
  double fx;
  gradient(
      [&](const vector_v& t) {
        std::vector<vector_v> job(shards);
        return sum(map_rect<1, glm_job>(t, job, xr, xi));
      },
      th, fx, g);
  print1("fx", fx);
  print("grad", std::vector<double>(g.data(), g.data() + g.size()));
  // double-only instantiation: values
  std::vector<Eigen::VectorXd> jobd(shards);
  Eigen::VectorXd vals = map_rect<2, glm_job>(th, jobd, xr, xi);
  print1("fx_double", vals.sum());
  std::printf("stack %zu %zu\n", ChainableStack::instance_->var_stack_.size(),
              ChainableStack::instance_->dev_adj_stack_.size());
}

struct gp_functor {
  const std::vector<double>& x;
  const std::vector<double>& y;
  template <typename T>
  T operator()(const Eigen::Matrix<T, Eigen::Dynamic, 1>& th) const {
    std::vector<double> mu(x.size(), 0.0);
    auto K = gp_exp_quad_cov(x, th(0), th(1));
    auto Kd = add_diag(K, square(th(2)));
    auto L = cholesky_decompose(Kd);
    return multi_normal_cholesky_lpdf(y, mu, L);
  }
  template <typename T>
  T operator()(const std::vector<T>& th) const {
    Eigen::Matrix<T, Eigen::Dynamic, 1> t(3);
    t << th[0], th[1], th[2];
    return (*this)(t);
  }
};

// hessian_times_vector on the GP marginal (config 5): Eigen and std::vector signatures
static void cmd_hvp() {
  int N;
  std::cin >> N;
  auto th = read_vec(3), v = read_vec(3), x = read_vec(N), y = read_vec(N);
  Eigen::VectorXd te = Eigen::Map<Eigen::VectorXd>(th.data(), 3), ve = Eigen::Map<Eigen::VectorXd>(v.data(), 3), Hv;
  double fx;
  for (int rep = 0; rep < 2; ++rep) {
    hessian_times_vector(gp_functor{x, y}, te, ve, fx, Hv);
    print1("fx", fx);
    print("Hv", std::vector<double>(Hv.data(), Hv.data() + 3));
  }
  std::vector<double> hv;
  hessian_times_vector(gp_functor{x, y}, th, v, fx, hv);
  print1("fx_std", fx);
  print("Hv_std", hv);
  std::printf("stack %zu %zu\n", ChainableStack::instance_->var_stack_.size(),
              ChainableStack::instance_->dev_adj_stack_.size());
}

// config 5 at full size: H v against the Richardson-extrapolated central
// difference of the (pinned) gradient along v:
//   D(h) = (g(th + h v) - g(th - h v)) / 2h,  Hv ~ (4 D(h/2) - D(h)) / 3
static void cmd_hvp_fd() {
  int N;
  double h;
  std::cin >> N;
  auto th = read_vec(3), v = read_vec(3), x = read_vec(N), y = read_vec(N);
  std::cin >> h;
  std::vector<double> hv;
  double fx;
  hessian_times_vector(gp_functor{x, y}, th, v, fx, hv);
  print1("fx", fx);
  print("Hv", hv);
  auto grad_at = [&](double t) {
    std::vector<double> p(3), g;
    for (int i = 0; i < 3; ++i) p[i] = th[i] + t * v[i];
    double f;
    gradient(gp_functor{x, y}, p, f, g);
    return g;
  };
  auto D = [&](double s) {
    std::vector<double> a = grad_at(s), b = grad_at(-s), d(3);
    for (int i = 0; i < 3; ++i) d[i] = (a[i] - b[i]) / (2 * s);
    return d;
  };
  std::vector<double> d1 = D(h), d2 = D(h / 2), r(3);
  for (int i = 0; i < 3; ++i) r[i] = (4 * d2[i] - d1[i]) / 3;
  print("Hv_fd", r);
  print("Hv_fd_plain", d2);
}

static void cmd_hessian() {
  int N;
  std::cin >> N;
  auto th = read_vec(3), x = read_vec(N), y = read_vec(N);
  Eigen::VectorXd te = Eigen::Map<Eigen::VectorXd>(th.data(), 3), g;
  Eigen::MatrixXd H;
  double fx;
  hessian(gp_functor{x, y}, te, fx, g, H);
  print1("fx", fx);
  print("grad", std::vector<double>(g.data(), g.data() + 3));
  print("H", std::vector<double>(H.data(), H.data() + 9));
  std::printf("stack %zu %zu\n", ChainableStack::instance_->var_stack_.size(),
              ChainableStack::instance_->dev_adj_stack_.size());
}

// hessian() (mix/mat/functor/hessian.hpp:39-72) of models built from the
// fvar<var> device functors beyond the GP set:
//   hessian2 mulchol N a(N^2)        sum(cholesky_decompose(add_diag(A A^T, N)))
//   hessian2 lse n x(n)              log_sum_exp(x)
//   hessian2 tri n k theta w(k)      sum(mdivide_left_tri<Lower>(L, B) w)
//   hessian2 glm R M beta(M)         bernoulli_logit_glm_lpmf(y | x, alpha, beta), config-4 streams
// prints fx, grad, H (column-major) and the tape sizes after the call
static void cmd_hessian2() {
  std::string kind;
  std::cin >> kind;
  Eigen::VectorXd x0, g;
  Eigen::MatrixXd H;
  double fx = 0;
  using VF = Eigen::Matrix<fvar<var>, Eigen::Dynamic, 1>;
  if (kind == "mulchol") {
    int N;
    std::cin >> N;
    auto a = read_vec(size_t(N) * N);
    x0 = Eigen::Map<Eigen::VectorXd>(a.data(), N * N);
    hessian(
        [N](const VF& th) {
          dev_fvar_matrix Am = to_dev(th, N, N);
          return sum(cholesky_decompose(add_diag(multiply(Am, transpose(Am)), double(N))));
        },
        x0, fx, g, H);
  } else if (kind == "lse") {
    int n;
    std::cin >> n;
    auto x = read_vec(size_t(n));
    x0 = Eigen::Map<Eigen::VectorXd>(x.data(), n);
    hessian([](const VF& th) { return log_sum_exp(to_dev(th)); }, x0, fx, g, H);
  } else if (kind == "tri") {
    int n, k;
    std::cin >> n >> k;
    auto th = read_vec(size_t(n) * n + size_t(n) * k);
    auto w = read_vec(size_t(k));
    x0 = Eigen::Map<Eigen::VectorXd>(th.data(), Eigen::Index(th.size()));
    hessian(
        [n, k, &w](const VF& t) {
          dev_fvar_matrix L = to_dev(t.head(n * n).eval(), n, n);
          dev_fvar_matrix B = to_dev(t.tail(n * k).eval(), n, k);
          dev_fvar_matrix C = mdivide_left_tri<Eigen::Lower>(L, B);
          return sum(multiply(C, to_dev_data(w.data(), w.size(), k, 1)));
        },
        x0, fx, g, H);
  } else if (kind == "glm") {
    long long R;
    int M;
    std::cin >> R >> M;
    auto beta = read_vec(M);
    smg_ctx* c = amd::ctx();
    int* y = amd::alloc_ints(size_t(R));
    double* x = amd::alloc_doubles(size_t(R) * M);
    amd::check(smg_fill_unif(c, x, R * M, 20260101ull + 41, -1.0, 1.0, std::sqrt(3.0)), "fill");
    amd::check(smg_fill_bernoulli(c, y, R, 20260101ull + 42, 0.5), "fill");
    dev_data<int> yd(y, size_t(R), int(R), 1);
    dev_data<double> xd(x, size_t(R) * M, int(R), M);
    x0.resize(M + 1);
    x0(0) = 0.1;
    for (int j = 0; j < M; ++j) x0(1 + j) = beta[size_t(j)];
    hessian(
        [&](const VF& t) {
          std::vector<fvar<var>> b(t.data() + 1, t.data() + t.size());
          return bernoulli_logit_glm_lpmf(yd, xd, t(0), b);
        },
        x0, fx, g, H);
  }
  print1("fx", fx);
  print("grad", std::vector<double>(g.data(), g.data() + g.size()));
  print("H", std::vector<double>(H.data(), H.data() + H.size()));
  std::printf("stack %zu %zu\n", ChainableStack::instance_->var_stack_.size(),
              ChainableStack::instance_->dev_adj_stack_.size());
}

template <typename F>
static void expect_throw(const char* name, F&& f) {
  start_nested();
  try {
    f();
    std::printf("%s nothrow\n", name);
  } catch (const std::domain_error& e) {
    std::printf("%s domain_error %s\n", name, e.what());
  } catch (const std::invalid_argument& e) {
    std::printf("%s invalid_argument %s\n", name, e.what());
  } catch (const std::exception& e) {
    std::printf("%s other %s\n", name, e.what());
  }
  recover_memory_nested();
}

// the reference's own error cases for the hot-path functors
// (tests/golden/errors_hot_path.json, oracle/ref_harness.cpp fix_errors),
// through the drop-in Eigen / std::vector signatures
static void cmd_errors_hot() {
  const double nan = std::nan("");
  auto M = [](std::initializer_list<double> v, int r, int c) {
    matrix_v m(r, c);
    int i = 0;
    for (double t : v) m(i++) = t;
    return m;
  };
  expect_throw("normal_nan_y", [&] { normal_lpdf(std::vector<var>{1.0, nan}, 0.0, 1.0); });
  expect_throw("normal_inf_mu", [&] { normal_lpdf(var(1.0), INFINITY, 1.0); });
  expect_throw("normal_neg_sigma", [&] { normal_lpdf(var(1.0), 0.0, -1.0); });
  expect_throw("normal_sizes",
               [&] { normal_lpdf(std::vector<var>{1.0, 2.0}, std::vector<double>{0, 0, 0}, 1.0); });
  expect_throw("multiply_sizes", [&] {
    matrix_v A = M({1, 1, 1, 1, 1, 1}, 2, 3);
    multiply(A, A);
  });
  expect_throw("mdivide_square", [&] {
    matrix_v A = M({1, 1, 1, 1, 1, 1}, 2, 3);
    mdivide_left_tri<Eigen::Lower>(A, A);
  });
  expect_throw("chol_not_symmetric", [&] { cholesky_decompose(M({2, 1, 0, 2}, 2, 2)); });
  expect_throw("chol_not_pd", [&] { cholesky_decompose(M({1, 2, 2, 1}, 2, 2)); });
  expect_throw("chol_not_square", [&] { cholesky_decompose(M({1, 2, 2, 1, 3, 3}, 2, 3)); });
  expect_throw("chol_nan", [&] { cholesky_decompose(M({1, nan, nan, 1}, 2, 2)); });
  expect_throw("glm_y_bounds", [&] {
    bernoulli_logit_glm_lpmf(std::vector<int>{0, 2}, std::vector<double>{1, 2}, 1, var(0.0), std::vector<var>{1.0});
  });
  expect_throw("glm_beta_size", [&] {
    bernoulli_logit_glm_lpmf(std::vector<int>{0, 1}, std::vector<double>{1, 2}, 1, var(0.0),
                             std::vector<var>{1.0, 2.0});
  });
  expect_throw("glm_nonfinite_beta", [&] {
    bernoulli_logit_glm_lpmf(std::vector<int>{0, 1}, std::vector<double>{1, 2}, 1, var(0.0),
                             std::vector<var>{INFINITY});
  });
  expect_throw("mvn_not_square", [&] {
    vector_v y(2), mu(2);
    y << 1, 2;
    mu << 0, 0;
    multi_normal_cholesky_lpdf(y, mu, M({1, 0, 0, 1, 0, 0}, 2, 3));
  });
  expect_throw("mvn_size_mu", [&] {
    vector_v y(2), mu(3);
    y << 1, 2;
    mu << 0, 0, 0;
    multi_normal_cholesky_lpdf(y, mu, M({1, 0, 0, 1}, 2, 2));
  });
  expect_throw("mvn_nan_y", [&] {
    vector_v y(2), mu(2);
    y << 1, nan;
    mu << 0, 0;
    multi_normal_cholesky_lpdf(y, mu, M({1, 0, 0, 1}, 2, 2));
  });
  expect_throw("gp_nonpositive_l", [&] { gp_exp_quad_cov(std::vector<double>{1, 2}, var(1.0), var(-1.0)); });
  expect_throw("gp_nan_x", [&] { gp_exp_quad_cov(std::vector<double>{1, nan}, var(1.0), var(1.0)); });
  recover_memory();
  std::printf("stack %zu %zu\n", ChainableStack::instance_->var_stack_.size(),
              ChainableStack::instance_->nested_var_stack_sizes_.size());
}

static void cmd_errors() {
  const double nan = std::nan("");
  expect_throw("normal_nan_y", [&] { normal_lpdf(std::vector<var>{1.0, nan}, 0.0, 1.0); });
  expect_throw("normal_inf_mu", [&] { normal_lpdf(var(1.0), INFINITY, 1.0); });
  expect_throw("normal_neg_sigma", [&] { normal_lpdf(var(1.0), 0.0, -1.0); });
  expect_throw("normal_sizes",
               [&] { normal_lpdf(std::vector<var>{1.0, 2.0}, std::vector<double>{0, 0, 0}, 1.0); });
  expect_throw("multiply_sizes", [&] {
    auto A = to_dev_var_matrix(std::vector<double>(6, 1.0).data(), 2, 3);
    multiply(A, A);
  });
  expect_throw("mdivide_square", [&] {
    auto A = to_dev_var_matrix(std::vector<double>(6, 1.0).data(), 2, 3);
    mdivide_left_tri<1>(A, A);
  });
  expect_throw("chol_not_symmetric", [&] {
    std::vector<double> a = {2, 1, 0, 2};
    cholesky_decompose(to_dev_var_matrix(a.data(), 2, 2));
  });
  expect_throw("chol_not_pd", [&] {
    std::vector<double> a = {1, 2, 2, 1};
    cholesky_decompose(to_dev_var_matrix(a.data(), 2, 2));
  });
  expect_throw("normal_glm_sigma", [&] {
    normal_id_glm_lpdf(std::vector<double>{0.5, 1.0}, std::vector<double>{1, 2}, 1, var(0.0),
                       std::vector<var>{var(1.0)}, var(-1.0));
  });
  expect_throw("normal_glm_beta_size", [&] {
    normal_id_glm_lpdf(std::vector<double>{0.5, 1.0}, std::vector<double>{1, 2}, 1, var(0.0),
                       std::vector<var>{var(1.0), var(2.0)}, var(1.0));
  });
  expect_throw("normal_glm_nonfinite_y", [&] {
    normal_id_glm_lpdf(std::vector<double>{0.5, INFINITY}, std::vector<double>{1, 2}, 1, var(0.0),
                       std::vector<var>{var(1.0)}, var(1.0));
  });
  expect_throw("poisson_glm_negative_y", [&] {
    poisson_log_glm_lpmf(std::vector<int>{0, 3, -2}, std::vector<double>{1, 2, 3}, 1, var(0.0),
                         std::vector<var>{var(1.0)});
  });
  expect_throw("poisson_glm_nonfinite_beta", [&] {
    poisson_log_glm_lpmf(std::vector<int>{0, 3}, std::vector<double>{1, 2}, 1, var(0.0),
                         std::vector<var>{var(INFINITY)});
  });
  expect_throw("spd_mdivide_sizes", [&] {
    mdivide_left_spd(matrix_v(matrix_d::Identity(3, 3).cast<var>()), matrix_v(matrix_d::Ones(2, 1).cast<var>()));
  });
  expect_throw("spd_mdivide_not_pd", [&] {
    matrix_d A = matrix_d::Identity(3, 3);
    A(1, 1) = -1.0;
    mdivide_left_spd(matrix_v(A.cast<var>()), matrix_v(matrix_d::Ones(3, 1).cast<var>()));
  });
  expect_throw("spd_logdet_not_symmetric", [&] {
    matrix_d A = matrix_d::Identity(3, 3);
    A(2, 0) = 0.5;
    log_determinant_spd(matrix_v(A.cast<var>()));
  });
  expect_throw("spd_logdet_negative", [&] {
    matrix_d A = matrix_d::Identity(3, 3);
    A(1, 1) = -1.0;
    log_determinant_spd(matrix_v(A.cast<var>()));
  });
  expect_throw("spd_quad_form_sizes", [&] {
    quad_form_sym(matrix_v(matrix_d::Identity(3, 3).cast<var>()), matrix_v(matrix_d::Ones(2, 2).cast<var>()));
  });
  expect_throw("spd_quad_form_not_symmetric", [&] {
    matrix_d A = matrix_d::Identity(3, 3);
    A(2, 0) = 0.5;
    quad_form_sym(matrix_v(A.cast<var>()), matrix_v(matrix_d::Ones(3, 2).cast<var>()));
  });
  expect_throw("glm_y_bounds", [&] {
    bernoulli_logit_glm_lpmf(std::vector<int>{0, 2}, std::vector<double>{1, 2}, 1, var(0.0),
                             std::vector<var>{1.0});
  });
  expect_throw("glm_beta_size", [&] {
    bernoulli_logit_glm_lpmf(std::vector<int>{0, 1}, std::vector<double>{1, 2}, 1, var(0.0),
                             std::vector<var>{1.0, 2.0});
  });
  expect_throw("glm_nonfinite_beta", [&] {
    bernoulli_logit_glm_lpmf(std::vector<int>{0, 1}, std::vector<double>{1, 2}, 1, var(0.0),
                             std::vector<var>{INFINITY});
  });
  // empty containers
  start_nested();
  var e1 = log_sum_exp(std::vector<var>{});
  std::printf("lse_empty %.17g\n", e1.val());
  var e2 = normal_lpdf(std::vector<var>{}, 0.0, 1.0);
  std::printf("normal_empty %.17g\n", e2.val());
  recover_memory_nested();
  std::printf("stack %zu %zu\n", ChainableStack::instance_->var_stack_.size(),
              ChainableStack::instance_->dev_adj_stack_.size());
}

static void cmd_glm_cat() {
  int M, C, ys;
  long long R;
  std::cin >> R >> M >> C >> ys;
  auto yv = read_vec(size_t(R));
  auto th = read_vec(size_t(C + M * C));
  smg_ctx* c = amd::ctx();
  double* x = amd::alloc_doubles(size_t(R) * M);
  amd::check(smg_fill_unif(c, x, R * M, 20260101ull + 81, -1.0, 1.0, std::sqrt(3.0)), "fill");
  std::vector<int> yi(yv.begin(), yv.end());
  dev_data<int> ydi = to_dev_data(yi);
  dev_data<double> xd(x, size_t(R) * M, int(R), M);
  std::vector<double> xh(size_t(R) * M);
  amd::to_host(xh.data(), x, xh.size());
  const matrix_d xm = Eigen::Map<matrix_d>(xh.data(), R, M);
  auto split = [&](const std::vector<var>& t, dev_var_matrix& a, dev_var_matrix& b) {
    a = to_dev(std::vector<var>(t.begin(), t.begin() + C), C, 1);
    b = to_dev(std::vector<var>(t.begin() + C, t.end()), M, C);
  };
  double fx;
  std::vector<double> g;
  // device operands, one call
  gradient(
      [&](const std::vector<var>& t) {
        dev_var_matrix a, b;
        split(t, a, b);
        return categorical_logit_glm_lpmf<false>(ydi, xd, a, b);
      },
      th, fx, g);
  print1("fx", fx);
  print("grad", g);
  gradient(
      [&](const std::vector<var>& t) {
        dev_var_matrix a, b;
        split(t, a, b);
        return categorical_logit_glm_lpmf<true>(ydi, xd, a, b);
      },
      th, fx, g);
  print1("fx_propto", fx);
  print("grad_propto", g);
  // 5 contiguous row shards summed on the tape
  gradient(
      [&](const std::vector<var>& t) {
        dev_var_matrix a, b;
        split(t, a, b);
        var s = 0.0;
        for (int k = 0; k < 5; ++k) {
          long long b0, b1;
          row_partition(R, 5, k, &b0, &b1);
          glm_shard sh;
          sh.y = ydi.data() + b0;
          sh.x = x + b0;
          sh.rows = b1 - b0;
          sh.M = M;
          sh.ldx = R;
          sh.row0 = b0;
          sh.total_rows = b1 - b0;
          s += categorical_logit_glm_lpmf<false>(sh, a, b);
        }
        return s;
      },
      th, fx, g);
  print1("fx_shards5", fx);
  print("grad_shards5", g);
  // Eigen signature, Matrix<var> alpha and beta (scalar y when ys > 0)
  gradient(
      [&](const std::vector<var>& t) {
        Eigen::Matrix<var, Eigen::Dynamic, 1> a(C);
        Eigen::Matrix<var, Eigen::Dynamic, Eigen::Dynamic> b(M, C);
        for (int k = 0; k < C; ++k) a(k) = t[k];
        for (int k = 0; k < M * C; ++k) b(k) = t[C + k];
        if (ys > 0) return categorical_logit_glm_lpmf(ys, xm, a, b);
        return categorical_logit_glm_lpmf(yi, xm, a, b);
      },
      th, fx, g);
  print1("fx_eigen", fx);
  print("grad_eigen", g);
  // double alpha, var beta: the beta block of the gradient
  std::vector<double> tb(th.begin() + C, th.end());
  gradient(
      [&](const std::vector<var>& t) {
        Eigen::VectorXd a = Eigen::Map<const Eigen::VectorXd>(th.data(), C);
        Eigen::Matrix<var, Eigen::Dynamic, Eigen::Dynamic> b(M, C);
        for (int k = 0; k < M * C; ++k) b(k) = t[k];
        return categorical_logit_glm_lpmf(yi, xm, a, b);
      },
      tb, fx, g);
  print1("fx_mixed", fx);
  print("grad_mixed", g);
  // all double: a plain double; with propto: 0
  const Eigen::VectorXd a = Eigen::Map<const Eigen::VectorXd>(th.data(), C);
  const matrix_d b = Eigen::Map<const matrix_d>(th.data() + C, M, C);
  print1("fx_double", categorical_logit_glm_lpmf(yi, xm, a, b));
  print1("fx_double_propto", categorical_logit_glm_lpmf<true>(yi, xm, a, b));
  std::printf("stack %zu %zu\n", ChainableStack::instance_->var_stack_.size(),
              ChainableStack::instance_->dev_adj_stack_.size());
}

static void cmd_glm_cat_errors() {
  using VV = Eigen::Matrix<var, Eigen::Dynamic, 1>;
  using MV = Eigen::Matrix<var, Eigen::Dynamic, Eigen::Dynamic>;
  auto X = [](std::initializer_list<double> v, int r, int c) {
    matrix_d m(r, c);
    int i = 0;
    for (double t : v) m(i++) = t;
    return m;
  };
  auto A = [](std::initializer_list<double> v) {
    VV a((Eigen::Index)v.size());
    int i = 0;
    for (double t : v) a(i++) = t;
    return a;
  };
  auto B = [](std::initializer_list<double> v, int r, int c) {
    MV m(r, c);
    int i = 0;
    for (double t : v) m(i++) = t;
    return m;
  };
  auto run = [&](const char* name, auto&& f) {
    start_nested();
    try {
      const var v = f();
      std::printf("%s value %.17g\n", name, v.val());
    } catch (const std::domain_error& e) {
      std::printf("%s domain_error %s\n", name, e.what());
    } catch (const std::invalid_argument& e) {
      std::printf("%s invalid_argument %s\n", name, e.what());
    } catch (const std::exception& e) {
      std::printf("%s other %s\n", name, e.what());
    }
    recover_memory_nested();
  };
  const matrix_d x = X({1, 2}, 2, 1);
  run("cat_y_support", [&] { return categorical_logit_glm_lpmf(std::vector<int>{1, 4}, x, A({0, 1, 2}), B({1, 2, 3}, 1, 3)); });
  run("cat_y_zero", [&] { return categorical_logit_glm_lpmf(std::vector<int>{0, 1}, x, A({0, 1, 2}), B({1, 2, 3}, 1, 3)); });
  run("cat_y_size", [&] { return categorical_logit_glm_lpmf(std::vector<int>{1, 2, 3}, x, A({0, 1, 2}), B({1, 2, 3}, 1, 3)); });
  run("cat_alpha_size", [&] { return categorical_logit_glm_lpmf(std::vector<int>{1, 2}, x, A({0, 1}), B({1, 2, 3}, 1, 3)); });
  run("cat_x_beta", [&] { return categorical_logit_glm_lpmf(std::vector<int>{1, 2}, x, A({0, 1, 2}), B({1, 2, 3, 4, 5, 6}, 2, 3)); });
  run("cat_nonfinite_beta", [&] { return categorical_logit_glm_lpmf(std::vector<int>{1, 2}, x, A({0, 1, 2}), B({1, INFINITY, 3}, 1, 3)); });
  run("cat_nonfinite_alpha", [&] { return categorical_logit_glm_lpmf(std::vector<int>{1, 2}, x, A({0, 1, NAN}), B({1, 2, 3}, 1, 3)); });
  run("cat_nonfinite_x", [&] { return categorical_logit_glm_lpmf(std::vector<int>{1, 2}, X({1, INFINITY}, 2, 1), A({0, 1, 2}), B({1, 2, 3}, 1, 3)); });
  run("cat_y_scalar_support", [&] { return categorical_logit_glm_lpmf(5, x, A({0, 1, 2}), B({1, 2, 3}, 1, 3)); });
  run("cat_one_class", [&] { return categorical_logit_glm_lpmf(std::vector<int>{1, 1}, x, A({0.5}), B({2}, 1, 1)); });
  run("cat_one_class_y2", [&] { return categorical_logit_glm_lpmf(std::vector<int>{1, 2}, x, A({0.5}), B({2}, 1, 1)); });
  run("cat_empty", [&] { return categorical_logit_glm_lpmf(std::vector<int>{}, matrix_d(0, 1), A({0, 1, 2}), B({1, 2, 3}, 1, 3)); });
  run("cat_small", [&] { return categorical_logit_glm_lpmf(std::vector<int>{3, 1}, x, A({0, 1, 2}), B({1, -2, 0.5}, 1, 3)); });
  std::printf("stack %zu %zu\n", ChainableStack::instance_->var_stack_.size(),
              ChainableStack::instance_->dev_adj_stack_.size());
}

// a node whose reverse step latches SMG_ERR_SYNC, as a persistent solve whose
// hand-off timed out would
struct inject_sync_vari : public vari {
  inject_sync_vari() : vari(0.0) {}
  void chain() override { amd::check(smg_status_inject(amd::ctx(), SMG_ERR_SYNC), "inject"); }
};

static void cmd_status() {
  std::vector<double> x = {0.5, -1.0, 2.0}, g;
  double fx = 0;
  expect_throw("sync_in_reverse", [&] {
    gradient(
        [](const std::vector<var>& t) {
          var a(new inject_sync_vari());  // first on the tape: its chain() runs last
          var b = normal_lpdf(t, 0.0, 1.0);
          return a + b;
        },
        x, fx, g);
  });
  expect_throw("sync_in_forward_readback", [&] {
    auto A = to_dev_var_matrix(x.data(), 3, 1);
    amd::check(smg_status_inject(amd::ctx(), SMG_ERR_SYNC), "inject");
    A.val();
  });
  // the latch is cleared by the throw: the next gradient is clean
  gradient([](const std::vector<var>& t) { return normal_lpdf(t, 0.0, 1.0); }, x, fx, g);
  print1("fx", fx);
  print("grad", g);
  std::printf("stack %zu %zu\n", ChainableStack::instance_->var_stack_.size(),
              ChainableStack::instance_->dev_adj_stack_.size());
}

int main() {
  std::string cmd;
  std::cin >> cmd;
  try {
    if (cmd == "mulchol") cmd_mulchol();
    else if (cmd == "mulchol_eigen") cmd_mulchol_eigen();
    else if (cmd == "gram_shared") cmd_gram_shared();
    else if (cmd == "multiply") cmd_multiply();
    else if (cmd == "mdivide") cmd_mdivide();
    else if (cmd == "lse") cmd_lse();
    else if (cmd == "lse_pair") cmd_lse_pair();
    else if (cmd == "special") cmd_special();
    else if (cmd == "special_vec") cmd_special_vec();
    else if (cmd == "normal") cmd_normal();
    else if (cmd == "normal_vec") cmd_normal_vec();
    else if (cmd == "normal_big") cmd_normal_big();
    else if (cmd == "normal_known") cmd_normal_known();
    else if (cmd == "glm") cmd_glm();
    else if (cmd == "glm_data") cmd_glm_data();
    else if (cmd == "glm2") cmd_glm2();
    else if (cmd == "glm_cat") cmd_glm_cat();
    else if (cmd == "glm_cat_errors") cmd_glm_cat_errors();
    else if (cmd == "spd") cmd_spd();
    else if (cmd == "logdet") cmd_logdet();
    else if (cmd == "mvn") cmd_mvn();
    else if (cmd == "errors") cmd_errors();
    else if (cmd == "errors_hot") cmd_errors_hot();
    else if (cmd == "hvp") cmd_hvp();
    else if (cmd == "hessian") cmd_hessian();
    else if (cmd == "hvp_fd") cmd_hvp_fd();
    else if (cmd == "hessian2") cmd_hessian2();
    else if (cmd == "map_rect_glm") cmd_map_rect_glm();
    else if (cmd == "status") cmd_status();
    else if (cmd == "ops_partials") cmd_ops_partials();
    else {
      std::fprintf(stderr, "unknown command %s\n", cmd.c_str());
      return 2;
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "exception: %s\n", e.what());
    return 1;
  }
  return 0;
}
