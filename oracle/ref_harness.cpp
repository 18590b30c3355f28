/*
 * oracle/ref_harness.cpp — drives the REAL reference (Stan Math 3.0.0 headers
 * under /root/reference, compiled by oracle/Makefile into oracle/_ref/) to
 *   (1) generate the golden fixtures committed under tests/golden/  ("gen")
 *   (2) time the reference CPU path for bench.py's cpu_baseline     ("bench")
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in math_amd/ links or calls this; it is
 * the checker / baseline, never the product.
 *
 * Build note: the reference always includes rev/core/init_chainablestack.hpp,
 * whose TBB task-scheduler observer needs libtbb at link time.  It is only
 * there to give STAN_THREADS worker threads their tapes; this harness is
 * single-threaded, so it defines that header's include guard and owns the
 * main-thread tape through the documented AutodiffStackSingleton instance
 * (rev/core/autodiffstackstorage.hpp:55-60).  No reference source is copied
 * or replaced: everything below calls the reference's own functions.
 *
 * Functions exercised (reference file:line):
 *   gradient                 stan/math/rev/mat/functor/gradient.hpp:41-57
 *   gp_exp_quad_cov (var)    stan/math/rev/mat/fun/gp_exp_quad_cov.hpp:213-242
 *   add_diag                 stan/math/prim/mat/fun/add_diag.hpp:20-55
 *   cholesky_decompose       stan/math/rev/mat/fun/cholesky_decompose.hpp:378-427
 *   multi_normal_cholesky    stan/math/prim/mat/prob/multi_normal_cholesky_lpdf.hpp:40-160
 *   multiply                 stan/math/rev/mat/fun/multiply.hpp:562-661
 *   mdivide_left_tri         stan/math/rev/mat/fun/mdivide_left_tri.hpp:311-373
 *   log_sum_exp              stan/math/rev/mat/fun/log_sum_exp.hpp:20-53,
 *                            stan/math/rev/scal/fun/log_sum_exp.hpp:15-68
 *   lgamma / digamma (var)   stan/math/rev/scal/fun/lgamma.hpp:13-32, digamma.hpp:13-22
 *   trigamma (double)        stan/math/prim/scal/fun/trigamma.hpp:33-125
 *   normal_lpdf              stan/math/prim/scal/prob/normal_lpdf.hpp:36-119
 *   bernoulli_logit_glm_lpmf stan/math/prim/mat/prob/bernoulli_logit_glm_lpmf.hpp:46-138
 *   normal_id_glm_lpdf       stan/math/prim/mat/prob/normal_id_glm_lpdf.hpp:40-150
 *   poisson_log_glm_lpmf     stan/math/prim/mat/prob/poisson_log_glm_lpmf.hpp:37-123
 *   categorical_logit_glm_lpmf stan/math/prim/mat/prob/categorical_logit_glm_lpmf.hpp:38-183
 *   mdivide_left_spd         stan/math/rev/mat/fun/mdivide_left_spd.hpp:232-260
 *   log_determinant_spd      stan/math/rev/mat/fun/log_determinant_spd.hpp:16-57
 *   log_determinant          stan/math/rev/mat/fun/log_determinant.hpp:14-37
 *   multiply_lower_tri_self_transpose  stan/math/rev/mat/fun/multiply_lower_tri_self_transpose.hpp:14-44
 *   quad_form_sym            stan/math/rev/mat/fun/quad_form_sym.hpp:15-27
 *   map_rect                 stan/math/prim/mat/functor/map_rect.hpp:120-177
 *   hessian_times_vector     stan/math/mix/mat/functor/hessian_times_vector.hpp:13-40
 *   hessian                  stan/math/mix/mat/functor/hessian.hpp:39-72
 *   the boundary call forms  tests/cpp/boundary_cases.hpp (multiply / add_diag / sum /
 *                            multi_normal_cholesky_lpdf / D-dimensional gp_exp_quad_cov)
 */
#define STAN_MATH_REV_CORE_INIT_CHAINABLESTACK_HPP
#include <stan/math/mix/mat.hpp>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "gen.h"
#include "../tests/cpp/boundary_cases.hpp"  // the call forms, shared with tests/cpp/test_boundary.cpp

stan::math::ChainableStack main_thread_tape;  // owns the main-thread tape

using Eigen::Dynamic;
using Eigen::Matrix;
using Eigen::MatrixXd;
using Eigen::VectorXd;
using stan::math::var;

// ----------------------------------------------------------------- JSON out
struct Json {
  std::ostringstream os;
  bool first = true;
  Json() { os << "{"; }
  void key(const std::string& k) {
    os << (first ? "\n" : ",\n") << "  \"" << k << "\": ";
    first = false;
  }
  static std::string num(double v) {
    if (std::isnan(v)) return "\"nan\"";
    if (std::isinf(v)) return v > 0 ? "\"inf\"" : "\"-inf\"";
    char b[40];
    std::snprintf(b, sizeof b, "%.17g", v);
    return b;
  }
  void put(const std::string& k, double v) {
    key(k);
    os << num(v);
  }
  void put_int(const std::string& k, long long v) {
    key(k);
    os << v;
  }
  void put_str(const std::string& k, const std::string& v) {
    key(k);
    os << "\"" << v << "\"";
  }
  template <typename V>
  void put_vec(const std::string& k, const V& v, size_t n) {
    key(k);
    os << "[";
    for (size_t i = 0; i < n; ++i) os << (i ? ", " : "") << num(v[i]);
    os << "]";
  }
  void put_vec(const std::string& k, const std::vector<double>& v) {
    put_vec(k, v, v.size());
  }
  void put_vec(const std::string& k, const VectorXd& v) {
    put_vec(k, v.data(), (size_t)v.size());
  }
  void put_mat(const std::string& k, const MatrixXd& m) {  // column-major
    put_vec(k, m.data(), (size_t)m.size());
  }
  void put_ivec(const std::string& k, const std::vector<int>& v) {
    key(k);
    os << "[";
    for (size_t i = 0; i < v.size(); ++i) os << (i ? ", " : "") << v[i];
    os << "]";
  }
  std::string str() { return os.str() + "\n}\n"; }
};

static std::string g_outdir = "tests/golden";
static void write_fixture(const std::string& name, Json& j) {
  std::string path = g_outdir + "/" + name + ".json";
  std::ofstream f(path);
  f << j.str();
  std::fprintf(stderr, "wrote %s\n", path.c_str());
}

// -------------------------------------------------------------- generators
static std::vector<double> unif(uint64_t seed, size_t n, double a, double b) {
  std::vector<double> v(n);
  smg_fill_unif(seed, n, a, b, v.data());
  return v;
}
// Box-Muller normals (stored in fixtures, never regenerated elsewhere)
static std::vector<double> normals(uint64_t seed, size_t n) {
  smg_rng r = smg_rng_make(seed);
  std::vector<double> v(n);
  for (size_t i = 0; i < n; i += 2) {
    double u1 = 1.0 - smg_rng_u01(&r), u2 = smg_rng_u01(&r);
    double rad = std::sqrt(-2.0 * std::log(u1));
    v[i] = rad * std::cos(2 * M_PI * u2);
    if (i + 1 < n) v[i + 1] = rad * std::sin(2 * M_PI * u2);
  }
  return v;
}

static const uint64_t SEED = 20260101ULL;

// GP inputs (config 3): x ~ U(-10,10), y = sin(x) + 0.3 eps
static void gp_inputs(int N, std::vector<double>& x, VectorXd& y) {
  x = unif(SEED + 3, N, -10.0, 10.0);
  std::vector<double> e = normals(SEED + 33, N);
  y.resize(N);
  for (int i = 0; i < N; ++i) y(i) = std::sin(x[i]) + 0.3 * e[i];
}

struct gp_functor {
  const std::vector<double>& x;
  const VectorXd& y;
  template <typename T>
  T operator()(const Matrix<T, Dynamic, 1>& th) const {
    using namespace stan::math;
    const int N = (int)x.size();
    Matrix<T, Dynamic, Dynamic> K = gp_exp_quad_cov(x, th(0), th(1));
    Matrix<T, Dynamic, Dynamic> Kd = add_diag(K, square(th(2)));
    Matrix<T, Dynamic, Dynamic> L = cholesky_decompose(Kd);
    VectorXd mu = VectorXd::Zero(N);
    return multi_normal_cholesky_lpdf(y, mu, L);
  }
};

// config 2: f(A) = sum(cholesky_decompose(add_diag(multiply(A, A'), N)))
struct mulchol_functor {
  int N;
  template <typename T>
  T operator()(const Matrix<T, Dynamic, 1>& a) const {
    using namespace stan::math;
    Matrix<T, Dynamic, Dynamic> A(N, N);
    for (int i = 0; i < N * N; ++i) A(i) = a(i);
    Matrix<T, Dynamic, Dynamic> C = multiply(A, transpose(A));
    Matrix<T, Dynamic, Dynamic> Cd = add_diag(C, (double)N);
    return sum(cholesky_decompose(Cd));
  }
};
static VectorXd mulchol_input(int N) {
  std::vector<double> a = unif(SEED + 2, (size_t)N * N, -1.0, 1.0);
  const double s = std::sqrt(3.0 / N);
  VectorXd v(N * N);
  for (int i = 0; i < N * N; ++i) v(i) = a[i] * s;
  return v;
}

// config 4 inputs (column-major x, R x M)
struct glm_data {
  int R, M;
  MatrixXd x;
  std::vector<int> y;
  VectorXd theta;  // (alpha, beta_1..M)
};
static glm_data glm_inputs(int R, int M) {
  glm_data d;
  d.R = R;
  d.M = M;
  std::vector<double> xv = unif(SEED + 41, (size_t)R * M, -1.0, 1.0);
  const double s3 = std::sqrt(3.0);
  d.x.resize(R, M);
  for (size_t i = 0; i < (size_t)R * M; ++i) d.x.data()[i] = xv[i] * s3;
  d.y.resize(R);
  smg_fill_bernoulli(SEED + 42, R, 0.5, d.y.data());
  std::vector<double> b = unif(SEED + 43, M, -1.0, 1.0);
  const double sb = std::sqrt(3.0 / M);
  d.theta.resize(M + 1);
  d.theta(0) = 0.1;
  for (int j = 0; j < M; ++j) d.theta(j + 1) = b[j] * sb;
  return d;
}
struct glm_functor {
  const glm_data& d;
  template <typename T>
  T operator()(const Matrix<T, Dynamic, 1>& th) const {
    Matrix<T, Dynamic, 1> beta = th.tail(d.M);
    return stan::math::bernoulli_logit_glm_lpmf(d.y, d.x, th(0), beta);
  }
};

// map_rect job functor: one shard of rows; x_r = shard of x (col-major), x_i = y
struct glm_shard_functor {
  template <typename T1, typename T2>
  Matrix<stan::return_type_t<T1, T2>, Dynamic, 1> operator()(
      const Matrix<T1, Dynamic, 1>& eta, const Matrix<T2, Dynamic, 1>& /*phi*/,
      const std::vector<double>& x_r, const std::vector<int>& x_i,
      std::ostream* /*msgs*/) const {
    const int M = eta.size() - 1;
    const int r = (int)x_i.size();
    MatrixXd xs = Eigen::Map<const MatrixXd>(x_r.data(), r, M);
    Matrix<T1, Dynamic, 1> beta = eta.tail(M);
    Matrix<stan::return_type_t<T1, T2>, Dynamic, 1> out(1);
    out(0) = stan::math::bernoulli_logit_glm_lpmf(x_i, xs, eta(0), beta);
    return out;
  }
};
struct glm_maprect_functor {
  const std::vector<std::vector<double>>& xr;
  const std::vector<std::vector<int>>& xi;
  template <typename T>
  T operator()(const Matrix<T, Dynamic, 1>& th) const {
    std::vector<Matrix<double, Dynamic, 1>> job(xr.size());
    return stan::math::sum(
        stan::math::map_rect<1, glm_shard_functor>(th, job, xr, xi));
  }
};

static void shard_glm(const glm_data& d, int shards,
                      std::vector<std::vector<double>>& xr,
                      std::vector<std::vector<int>>& xi) {
  xr.assign(shards, {});
  xi.assign(shards, {});
  for (int s = 0; s < shards; ++s) {
    int r0 = (int)((long long)d.R * s / shards);
    int r1 = (int)((long long)d.R * (s + 1) / shards);
    int r = r1 - r0;
    xr[s].resize((size_t)r * d.M);
    for (int j = 0; j < d.M; ++j)
      for (int i = 0; i < r; ++i) xr[s][(size_t)j * r + i] = d.x(r0 + i, j);
    xi[s].assign(d.y.begin() + r0, d.y.begin() + r1);
  }
}

// normal_lpdf (config 1)
struct normal_functor {
  template <typename T>
  T operator()(const Matrix<T, Dynamic, 1>& th) const {
    return stan::math::normal_lpdf(th, 0.0, 1.0);
  }
};

// --------------------------------------------------------------- fixtures
static void fix_gp() {
  for (int N : {16, 64, 256, 1024, 4096}) {
    std::vector<double> x;
    VectorXd y;
    gp_inputs(N, x, y);
    VectorXd th(3);
    th << 1.0, 1.5, 0.3;
    double fx;
    VectorXd g;
    auto t0 = std::chrono::steady_clock::now();
    stan::math::gradient(gp_functor{x, y}, th, fx, g);
    double sec = std::chrono::duration<double>(
                     std::chrono::steady_clock::now() - t0).count();
    Json j;
    j.put_str("what", "gradient of multi_normal_cholesky_lpdf(y|0,cholesky_decompose(add_diag(gp_exp_quad_cov(x,alpha,rho),sigma^2))) wrt (alpha,rho,sigma)");
    j.put_int("N", N);
    j.put_vec("theta", th);
    j.put_vec("x", x);
    j.put_vec("y", y);
    j.put("fx", fx);
    j.put_vec("grad", g);
    j.put("ref_seconds", sec);
    write_fixture("gp_N" + std::to_string(N), j);
  }
}

static void fix_mulchol() {
  for (int N : {8, 40, 128, 2048}) {
    VectorXd a = mulchol_input(N);
    double fx;
    VectorXd g;
    auto t0 = std::chrono::steady_clock::now();
    stan::math::gradient(mulchol_functor{N}, a, fx, g);
    double sec = std::chrono::duration<double>(
                     std::chrono::steady_clock::now() - t0).count();
    Json j;
    j.put_str("what", "gradient of sum(cholesky_decompose(add_diag(multiply(A,A^T),N))) wrt A (col-major); A = unif(seed 20260102)*sqrt(3/N)");
    j.put_int("N", N);
    j.put("fx", fx);
    j.put("grad_sum", g.sum());
    j.put("grad_l2", g.norm());
    if (N <= 128) {
      j.put_vec("grad", g);
    } else {
      smg_rng r = smg_rng_make(SEED + 222);
      std::vector<double> idx, val;
      for (int s = 0; s < 1024; ++s) {
        size_t k = smg_rng_next(&r) % ((size_t)N * N);
        idx.push_back((double)k);
        val.push_back(g((Eigen::Index)k));
      }
      j.put_vec("sample_index", idx);
      j.put_vec("sample_grad", val);
    }
    j.put("ref_seconds", sec);
    write_fixture("mulchol_N" + std::to_string(N), j);
  }
}

// weighted-sum seeds: f = sum_ij W_ij out_ij, W = unif(-1,1)
static std::vector<double> weights(uint64_t seed, size_t n) {
  return unif(seed, n, -1.0, 1.0);
}

static MatrixXd spd(int N, uint64_t seed) {
  std::vector<double> b = unif(seed, (size_t)N * N, -1.0, 1.0);
  MatrixXd B = Eigen::Map<MatrixXd>(b.data(), N, N);
  MatrixXd A = B * B.transpose() / N;
  A.diagonal().array() += 1.0;
  A = 0.5 * (A + A.transpose()).eval();
  return A;
}

static void fix_cholesky() {
  for (int N : {1, 5, 35, 36, 100, 200}) {
    MatrixXd A = spd(N, SEED + 100 + N);
    std::vector<double> W = weights(SEED + 500 + N, (size_t)N * N);
    Matrix<var, Dynamic, Dynamic> Av(N, N);
    for (int i = 0; i < N * N; ++i) Av(i) = A(i);
    Matrix<var, Dynamic, Dynamic> L = stan::math::cholesky_decompose(Av);
    var f = 0;
    for (int jj = 0; jj < N; ++jj)
      for (int ii = jj; ii < N; ++ii) f += W[(size_t)jj * N + ii] * L(ii, jj);
    f.grad();
    MatrixXd Lv(N, N), Ag(N, N);
    for (int i = 0; i < N * N; ++i) {
      Lv(i) = L(i).val();
      Ag(i) = Av(i).adj();
    }
    Json j;
    j.put_str("what", "cholesky_decompose(A) value and gradient of f=sum_{i>=j} W_ij L_ij wrt every A_ij (independent varis; upper triangle gets 0)");
    j.put_int("N", N);
    j.put_mat("A", A);
    j.put_vec("W", W);
    j.put("fx", f.val());
    j.put_mat("L", Lv);
    j.put_mat("grad_A", Ag);
    write_fixture("cholesky_N" + std::to_string(N), j);
    stan::math::recover_memory();
  }
}

static void fix_multiply() {
  struct Case {
    int m, k, n;
    int kind;  // 0 vv, 1 vd, 2 dv
  };
  for (Case c : {Case{5, 7, 4, 0}, Case{5, 7, 4, 1}, Case{5, 7, 4, 2},
                 Case{64, 48, 33, 0}, Case{1, 9, 1, 0}}) {
    std::vector<double> a = unif(SEED + 600 + c.m, (size_t)c.m * c.k, -1, 1);
    std::vector<double> b = unif(SEED + 700 + c.n, (size_t)c.k * c.n, -1, 1);
    std::vector<double> W = weights(SEED + 800, (size_t)c.m * c.n);
    MatrixXd Ad = Eigen::Map<MatrixXd>(a.data(), c.m, c.k);
    MatrixXd Bd = Eigen::Map<MatrixXd>(b.data(), c.k, c.n);
    Matrix<var, Dynamic, Dynamic> Av = Ad.cast<var>(), Bv = Bd.cast<var>();
    Matrix<var, Dynamic, Dynamic> C;
    if (c.kind == 0) C = stan::math::multiply(Av, Bv);
    if (c.kind == 1) C = stan::math::multiply(Av, Bd);
    if (c.kind == 2) C = stan::math::multiply(Ad, Bv);
    var f = 0;
    for (int i = 0; i < c.m * c.n; ++i) f += W[i] * C(i);
    f.grad();
    MatrixXd Cv(c.m, c.n), Ag(c.m, c.k), Bg(c.k, c.n);
    for (int i = 0; i < c.m * c.n; ++i) Cv(i) = C(i).val();
    for (int i = 0; i < c.m * c.k; ++i) Ag(i) = Av(i).adj();
    for (int i = 0; i < c.k * c.n; ++i) Bg(i) = Bv(i).adj();
    Json j;
    j.put_str("what", "multiply(A,B) (kind 0 var*var, 1 var*double, 2 double*var) and gradient of sum W.*C");
    j.put_int("m", c.m);
    j.put_int("k", c.k);
    j.put_int("n", c.n);
    j.put_int("kind", c.kind);
    j.put_mat("A", Ad);
    j.put_mat("B", Bd);
    j.put_vec("W", W);
    j.put_mat("C", Cv);
    j.put("fx", f.val());
    j.put_mat("grad_A", Ag);
    j.put_mat("grad_B", Bg);
    write_fixture("multiply_" + std::to_string(c.m) + "x" + std::to_string(c.k) +
                      "x" + std::to_string(c.n) + "_k" + std::to_string(c.kind),
                  j);
    stan::math::recover_memory();
  }
}

static void fix_mdivide() {
  struct Case {
    int m, n;
    int lower;  // 1 Lower, 0 Upper
    int kind;   // 0 vv, 1 dv, 2 vd
  };
  for (Case c : {Case{6, 3, 1, 0}, Case{6, 3, 0, 0}, Case{6, 3, 1, 1},
                 Case{6, 3, 1, 2}, Case{50, 20, 1, 0}, Case{50, 1, 0, 0}}) {
    MatrixXd S = spd(c.m, SEED + 900 + c.m);
    MatrixXd T = S.llt().matrixL();
    if (!c.lower) T = T.transpose().eval();
    // put junk in the unused triangle: the reference must ignore it
    std::vector<double> junk = unif(SEED + 901, (size_t)c.m * c.m, -3, 3);
    for (int jj = 0; jj < c.m; ++jj)
      for (int ii = 0; ii < c.m; ++ii)
        if ((c.lower && ii < jj) || (!c.lower && ii > jj))
          T(ii, jj) = junk[(size_t)jj * c.m + ii];
    std::vector<double> b = unif(SEED + 902, (size_t)c.m * c.n, -1, 1);
    MatrixXd Bd = Eigen::Map<MatrixXd>(b.data(), c.m, c.n);
    std::vector<double> W = weights(SEED + 903, (size_t)c.m * c.n);
    Matrix<var, Dynamic, Dynamic> Av = T.cast<var>(), Bv = Bd.cast<var>();
    Matrix<var, Dynamic, Dynamic> C;
    using stan::math::mdivide_left_tri;
    if (c.lower) {
      if (c.kind == 0) C = mdivide_left_tri<Eigen::Lower>(Av, Bv);
      if (c.kind == 1) C = mdivide_left_tri<Eigen::Lower>(T, Bv);
      if (c.kind == 2) C = mdivide_left_tri<Eigen::Lower>(Av, Bd);
    } else {
      if (c.kind == 0) C = mdivide_left_tri<Eigen::Upper>(Av, Bv);
      if (c.kind == 1) C = mdivide_left_tri<Eigen::Upper>(T, Bv);
      if (c.kind == 2) C = mdivide_left_tri<Eigen::Upper>(Av, Bd);
    }
    var f = 0;
    for (int i = 0; i < c.m * c.n; ++i) f += W[i] * C(i);
    f.grad();
    MatrixXd Cv(c.m, c.n), Ag(c.m, c.m), Bg(c.m, c.n);
    for (int i = 0; i < c.m * c.n; ++i) Cv(i) = C(i).val();
    for (int i = 0; i < c.m * c.m; ++i) Ag(i) = Av(i).adj();
    for (int i = 0; i < c.m * c.n; ++i) Bg(i) = Bv(i).adj();
    Json j;
    j.put_str("what", "mdivide_left_tri<TriView>(A,B) (kind 0 vv, 1 dv, 2 vd) and gradient of sum W.*C; unused triangle of A holds junk");
    j.put_int("m", c.m);
    j.put_int("n", c.n);
    j.put_int("lower", c.lower);
    j.put_int("kind", c.kind);
    j.put_mat("A", T);
    j.put_mat("B", Bd);
    j.put_vec("W", W);
    j.put_mat("C", Cv);
    j.put("fx", f.val());
    j.put_mat("grad_A", Ag);
    j.put_mat("grad_B", Bg);
    write_fixture("mdivide_left_tri_" + std::string(c.lower ? "L" : "U") +
                      std::to_string(c.m) + "x" + std::to_string(c.n) + "_k" +
                      std::to_string(c.kind),
                  j);
    stan::math::recover_memory();
  }
}

static void fix_mvn() {
  for (int N : {3, 20, 100}) {
    MatrixXd S = spd(N, SEED + 1000 + N);
    MatrixXd L = S.llt().matrixL();
    std::vector<double> yv = unif(SEED + 1001, N, -2, 2);
    std::vector<double> mv = unif(SEED + 1002, N, -1, 1);
    VectorXd y = Eigen::Map<VectorXd>(yv.data(), N);
    VectorXd mu = Eigen::Map<VectorXd>(mv.data(), N);
    // all of y, mu, L var: full reference partials, upper triangle included
    Matrix<var, Dynamic, 1> yvv = y.cast<var>(), muv = mu.cast<var>();
    Matrix<var, Dynamic, Dynamic> Lv = L.cast<var>();
    var lp = stan::math::multi_normal_cholesky_lpdf(yvv, muv, Lv);
    lp.grad();
    MatrixXd gL(N, N);
    VectorXd gy(N), gm(N);
    for (int i = 0; i < N * N; ++i) gL(i) = Lv(i).adj();
    for (int i = 0; i < N; ++i) {
      gy(i) = yvv(i).adj();
      gm(i) = muv(i).adj();
    }
    Json j;
    j.put_str("what", "multi_normal_cholesky_lpdf(y|mu,L) with y,mu,L all var; gradient wrt every entry (upper triangle of L included)");
    j.put_int("N", N);
    j.put_vec("y", y);
    j.put_vec("mu", mu);
    j.put_mat("L", L);
    j.put("fx", lp.val());
    j.put_vec("grad_y", gy);
    j.put_vec("grad_mu", gm);
    j.put_mat("grad_L", gL);
    write_fixture("mvn_cholesky_N" + std::to_string(N), j);
    stan::math::recover_memory();
  }
  {  // reference known answer: test/unit/math/rev/mat/prob/multi_normal_cholesky_test.cpp:9-20
    Json j;
    j.put_str("what", "known answer from the reference's own test (multi_normal_cholesky_test.cpp:9-20), EXPECT_FLOAT_EQ");
    j.put_vec("y", std::vector<double>{2.0, -2.0, 11.0});
    j.put_vec("mu", std::vector<double>{1.0, -1.0, 3.0});
    j.put_vec("Sigma", std::vector<double>{9.0, -3.0, 0.0, -3.0, 4.0, 0.0, 0.0, 0.0, 5.0});
    j.put("expected", -11.73908);
    write_fixture("mvn_cholesky_known", j);
  }
}

static void fix_lse() {
  for (int kind = 0; kind < 3; ++kind) {
    int N = kind == 2 ? 1000 : 50;
    std::vector<double> v = unif(SEED + 1100 + kind, N, -5, 5);
    if (kind == 1)
      for (auto& e : v) e += 700.0;  // would overflow exp without the shift
    Matrix<var, Dynamic, 1> xv(N);
    for (int i = 0; i < N; ++i) xv(i) = v[i];
    var f = stan::math::log_sum_exp(xv);
    f.grad();
    VectorXd g(N);
    for (int i = 0; i < N; ++i) g(i) = xv(i).adj();
    Json j;
    j.put_str("what", "log_sum_exp(Matrix<var,-1,1>) value and gradient");
    j.put_int("N", N);
    j.put_vec("x", v);
    j.put("fx", f.val());
    j.put_vec("grad", g);
    write_fixture("log_sum_exp_" + std::to_string(kind), j);
    stan::math::recover_memory();
  }
  {  // scalar pairs
    std::vector<double> a = {1.0, -3.0, 1000.0, 0.0, -INFINITY};
    std::vector<double> b = {2.0, -3.0, 999.0, -50.0, 1.0};
    std::vector<double> f, ga, gb;
    for (size_t i = 0; i < a.size(); ++i) {
      var av = a[i], bv = b[i];
      var r = stan::math::log_sum_exp(av, bv);
      r.grad();
      f.push_back(r.val());
      ga.push_back(av.adj());
      gb.push_back(bv.adj());
      stan::math::recover_memory();
    }
    Json j;
    j.put_str("what", "log_sum_exp(var a, var b) values and gradients");
    j.put_vec("a", a);
    j.put_vec("b", b);
    j.put_vec("f", f);
    j.put_vec("grad_a", ga);
    j.put_vec("grad_b", gb);
    write_fixture("log_sum_exp_pair", j);
  }
}

static void fix_special() {
  std::vector<double> xs = {-4.5, -3.7, -2.5, -1.5, -1.25, -0.5, -1e-5, 1e-8,
                            1e-4, 1e-3, 0.1, 0.25, 0.5, 0.9, 1.0, 1.4616321449683623,
                            1.5, 2.0, 2.5, 3.0, 4.99, 5.0, 7.5, 9.99, 10.0, 10.01,
                            20.0, 55.5, 100.0, 1e3, 1e5, 1e10, 1e15};
  std::vector<double> more = unif(SEED + 1200, 64, 0.01, 30.0);
  std::vector<double> neg = unif(SEED + 1201, 16, -20.0, -0.01);
  xs.insert(xs.end(), more.begin(), more.end());
  xs.insert(xs.end(), neg.begin(), neg.end());
  std::vector<double> lg, dg, tg, dlg, ddg;
  for (double x : xs) {
    lg.push_back(stan::math::lgamma(x));
    dg.push_back(stan::math::digamma(x));
    tg.push_back(stan::math::trigamma(x));
    var xv = x;
    var y = stan::math::lgamma(xv);
    y.grad();
    dlg.push_back(xv.adj());
    stan::math::recover_memory();
    var xv2 = x;
    var y2 = stan::math::digamma(xv2);
    y2.grad();
    ddg.push_back(xv2.adj());
    stan::math::recover_memory();
  }
  Json j;
  j.put_str("what", "lgamma (glibc lgamma_r), digamma (boost, boost_policy_t), trigamma (stan AS121-style) values; d/dx lgamma(var) and d/dx digamma(var)");
  j.put_vec("x", xs);
  j.put_vec("lgamma", lg);
  j.put_vec("digamma", dg);
  j.put_vec("trigamma", tg);
  j.put_vec("grad_lgamma", dlg);
  j.put_vec("grad_digamma", ddg);
  write_fixture("special", j);
  // vectorised form on a matrix of vars
  {
    int N = 200;
    std::vector<double> v = unif(SEED + 1202, N, 0.05, 50.0);
    std::vector<double> W = weights(SEED + 1203, N);
    Matrix<var, Dynamic, Dynamic> X(10, 20);
    for (int i = 0; i < N; ++i) X(i) = v[i];
    Matrix<var, Dynamic, Dynamic> Y = stan::math::lgamma(X);
    Matrix<var, Dynamic, Dynamic> Z = stan::math::digamma(X);
    var f = 0;
    for (int i = 0; i < N; ++i) f += W[i] * (Y(i) + 0.5 * Z(i));
    f.grad();
    std::vector<double> g(N);
    for (int i = 0; i < N; ++i) g[i] = X(i).adj();
    Json k;
    k.put_str("what", "vectorised lgamma/digamma on Matrix<var> 10x20; f = sum W.*(lgamma(X) + 0.5 digamma(X))");
    k.put_vec("x", v);
    k.put_vec("W", W);
    k.put("fx", f.val());
    k.put_vec("grad", g);
    write_fixture("special_vectorised", k);
    stan::math::recover_memory();
  }
}

static void fix_normal() {
  {
    int N = 1024;
    std::vector<double> th = normals(SEED + 1, N);
    VectorXd x = Eigen::Map<VectorXd>(th.data(), N);
    double fx;
    VectorXd g;
    stan::math::gradient(normal_functor{}, x, fx, g);
    Json j;
    j.put_str("what", "gradient of normal_lpdf(theta|0,1), N=1024 (config 1)");
    j.put_int("N", N);
    j.put_vec("theta", x);
    j.put("fx", fx);
    j.put_vec("grad", g);
    write_fixture("normal_N1024", j);
  }
  {  // vector y, mu, sigma all var
    int N = 9;
    std::vector<double> y = unif(SEED + 1301, N, -3, 3),
                        mu = unif(SEED + 1302, N, -1, 1),
                        sg = unif(SEED + 1303, N, 0.2, 3);
    Matrix<var, Dynamic, 1> yv(N), mv(N), sv(N);
    for (int i = 0; i < N; ++i) {
      yv(i) = y[i];
      mv(i) = mu[i];
      sv(i) = sg[i];
    }
    var f = stan::math::normal_lpdf(yv, mv, sv);
    var fp = stan::math::normal_lpdf<true>(yv, mv, sv);
    f.grad();
    std::vector<double> gy(N), gm(N), gs(N);
    for (int i = 0; i < N; ++i) {
      gy[i] = yv(i).adj();
      gm[i] = mv(i).adj();
      gs[i] = sv(i).adj();
    }
    Json j;
    j.put_str("what", "normal_lpdf(y|mu,sigma) all vector var; propto=false value+grad, propto=true value");
    j.put_vec("y", y);
    j.put_vec("mu", mu);
    j.put_vec("sigma", sg);
    j.put("fx", f.val());
    j.put("fx_propto", fp.val());
    j.put_vec("grad_y", gy);
    j.put_vec("grad_mu", gm);
    j.put_vec("grad_sigma", gs);
    write_fixture("normal_vec9", j);
    stan::math::recover_memory();
  }
  {  // the reference's own golden values (test/prob/normal/normal_test.hpp:9-32)
    Json j;
    j.put_str("what", "known answers from test/prob/normal/normal_test.hpp:9-32 (checked to 1e-8 by test_fixture_distr.hpp:120)");
    j.put_vec("y", std::vector<double>{0, 1, -2, -3.5});
    j.put_vec("mu", std::vector<double>{0, 0, 0, 1.9});
    j.put_vec("sigma", std::vector<double>{1, 1, 1, 7.2});
    j.put_vec("expected", std::vector<double>{-0.918938533204672669541, -1.418938533204672669541,
                                              -2.918938533204672669541, -3.174269559226682080322});
    write_fixture("normal_known", j);
  }
}

static void fix_glm() {
  struct Case {
    int R, M;
  };
  for (Case c : {Case{1000, 8}, Case{10000, 256}, Case{100000, 256}}) {
    glm_data d = glm_inputs(c.R, c.M);
    double fx;
    VectorXd g;
    stan::math::gradient(glm_functor{d}, d.theta, fx, g);
    Json j;
    j.put_str("what", "gradient of bernoulli_logit_glm_lpmf(y|x,alpha,beta) wrt (alpha,beta); inputs regenerated from oracle/gen.h seeds 20260142/43/44");
    j.put_int("R", c.R);
    j.put_int("M", c.M);
    j.put("fx", fx);
    j.put_vec("grad", g);
#ifndef STAN_THREADS  // (the threaded map_rect needs libtbb: the STAN_THREADS build only benches)
    if (c.R == 100000) {
      std::vector<std::vector<double>> xr;
      std::vector<std::vector<int>> xi;
      shard_glm(d, 32, xr, xi);
      double fx2;
      VectorXd g2;
      stan::math::gradient(glm_maprect_functor{xr, xi}, d.theta, fx2, g2);
      j.put("fx_map_rect32", fx2);
      j.put_vec("grad_map_rect32", g2);
    }
#endif
    write_fixture("glm_R" + std::to_string(c.R) + "_M" + std::to_string(c.M), j);
  }
  {  // extreme linear predictors exercise the +-20 cutoff branches
    int R = 64, M = 2;
    MatrixXd x(R, M);
    std::vector<int> y(R);
    std::vector<double> xv = unif(SEED + 1401, (size_t)R * M, -30, 30);
    for (int i = 0; i < R * M; ++i) x.data()[i] = xv[i];
    smg_fill_bernoulli(SEED + 1402, R, 0.5, y.data());
    glm_data d;
    d.R = R;
    d.M = M;
    d.x = x;
    d.y = y;
    d.theta.resize(M + 1);
    d.theta << 0.5, 1.3, -0.9;
    double fx;
    VectorXd g;
    stan::math::gradient(glm_functor{d}, d.theta, fx, g);
    Json j;
    j.put_str("what", "bernoulli_logit_glm_lpmf with |eta| > 20 rows (cutoff branches)");
    j.put_int("R", R);
    j.put_int("M", M);
    j.put_mat("x", x);
    j.put_ivec("y", y);
    j.put_vec("theta", d.theta);
    j.put("fx", fx);
    j.put_vec("grad", g);
    write_fixture("glm_extreme", j);
  }
}

// normal_id / poisson_log GLM inputs (tests/gen.py glm2_inputs)
static void glm2_inputs(int R, int M, bool normal, glm_data& d, VectorXd& yd) {
  d = glm_inputs(R, M);
  if (normal) {
    std::vector<double> y = unif(SEED + 51, R, -2.0, 2.0);
    yd = Eigen::Map<VectorXd>(y.data(), R);
    d.theta.conservativeResize(M + 2);
    d.theta(M + 1) = 1.3;
  } else {
    std::vector<double> u = unif(SEED + 52, R, 0.0, 6.0);
    for (int i = 0; i < R; ++i) d.y[i] = (int)u[i];
    for (int j = 0; j < M; ++j) d.theta(j + 1) *= 0.5;
  }
}
template <bool propto>
struct normal_glm_functor {
  const glm_data& d;
  const VectorXd& y;
  template <typename T>
  T operator()(const Matrix<T, Dynamic, 1>& th) const {
    Matrix<T, Dynamic, 1> beta = th.segment(1, d.M);
    return stan::math::normal_id_glm_lpdf<propto>(y, d.x, th(0), beta, th(d.M + 1));
  }
};
template <bool propto>
struct poisson_glm_functor {
  const glm_data& d;
  template <typename T>
  T operator()(const Matrix<T, Dynamic, 1>& th) const {
    Matrix<T, Dynamic, 1> beta = th.tail(d.M);
    return stan::math::poisson_log_glm_lpmf<propto>(d.y, d.x, th(0), beta);
  }
};

static void fix_glm2() {
  struct Case {
    int R, M;
  };
  for (Case c : {Case{1000, 8}, Case{20000, 64}}) {
    for (int normal = 1; normal >= 0; --normal) {
      glm_data d;
      VectorXd yd;
      glm2_inputs(c.R, c.M, normal, d, yd);
      double fx, fxp;
      VectorXd g, gp;
      Json j;
      if (normal) {
        stan::math::gradient(normal_glm_functor<false>{d, yd}, d.theta, fx, g);
        stan::math::gradient(normal_glm_functor<true>{d, yd}, d.theta, fxp, gp);
        j.put_str("what", "gradient of normal_id_glm_lpdf(y|x,alpha,beta,sigma) wrt (alpha,beta,sigma); inputs: tests/gen.py glm2_inputs");
      } else {
        stan::math::gradient(poisson_glm_functor<false>{d}, d.theta, fx, g);
        stan::math::gradient(poisson_glm_functor<true>{d}, d.theta, fxp, gp);
        j.put_str("what", "gradient of poisson_log_glm_lpmf(y|x,alpha,beta) wrt (alpha,beta); inputs: tests/gen.py glm2_inputs");
      }
      j.put_int("R", c.R);
      j.put_int("M", c.M);
      j.put("fx", fx);
      j.put_vec("grad", g);
      j.put("fx_propto", fxp);
      j.put_vec("grad_propto", gp);
      write_fixture(std::string(normal ? "normal_id_glm" : "poisson_log_glm") + "_R" +
                        std::to_string(c.R) + "_M" + std::to_string(c.M),
                    j);
    }
  }
}

// categorical_logit_glm inputs (tests/gen.py glm_cat_inputs): x R x M
// col-major U[-1,1) sqrt 3, alpha U[-1,1) (C), beta U[-1,1) sqrt(3/M) (M x C
// col-major), y = floor(U[0, C)) + 1; theta = (alpha, beta).
struct glm_cat_data {
  int R, M, C;
  MatrixXd x;
  std::vector<int> y;
  VectorXd theta;
};
static glm_cat_data glm_cat_inputs(int R, int M, int C) {
  glm_cat_data d;
  d.R = R, d.M = M, d.C = C;
  std::vector<double> x = unif(SEED + 81, (size_t)R * M, -1.0, 1.0);
  for (double& v : x) v *= std::sqrt(3.0);
  d.x = Eigen::Map<MatrixXd>(x.data(), R, M);
  std::vector<double> a = unif(SEED + 82, C, -1.0, 1.0);
  std::vector<double> b = unif(SEED + 83, (size_t)M * C, -1.0, 1.0);
  d.theta.resize(C + (Eigen::Index)M * C);
  for (int c = 0; c < C; ++c) d.theta(c) = a[c];
  for (int e = 0; e < M * C; ++e) d.theta(C + e) = b[e] * std::sqrt(3.0 / M);
  std::vector<double> u = unif(SEED + 84, R, 0.0, (double)C);
  d.y.resize(R);
  for (int i = 0; i < R; ++i) d.y[i] = (int)u[i] + 1;
  return d;
}
template <bool propto>
struct glm_cat_functor {
  const glm_cat_data& d;
  int y_scalar;  // > 0: the broadcast-scalar overload
  template <typename T>
  T operator()(const Matrix<T, Dynamic, 1>& th) const {
    Matrix<T, Dynamic, 1> alpha = th.head(d.C);
    Matrix<T, Dynamic, Dynamic> beta(d.M, d.C);
    for (int e = 0; e < d.M * d.C; ++e) beta(e) = th(d.C + e);
    if (y_scalar > 0) return stan::math::categorical_logit_glm_lpmf<propto>(y_scalar, d.x, alpha, beta);
    return stan::math::categorical_logit_glm_lpmf<propto>(d.y, d.x, alpha, beta);
  }
};
static void fix_glm_cat() {
  struct Case {
    int R, M, C, ys;
  };
  for (Case c : {Case{1000, 8, 5, 0}, Case{20000, 64, 16, 0}, Case{3000, 200, 3, 0}, Case{50, 6, 4, 3}}) {
    glm_cat_data d = glm_cat_inputs(c.R, c.M, c.C);
    double fx, fxp;
    VectorXd g, gp;
    stan::math::gradient(glm_cat_functor<false>{d, c.ys}, d.theta, fx, g);
    stan::math::gradient(glm_cat_functor<true>{d, c.ys}, d.theta, fxp, gp);
    Json j;
    j.put_str("what", "gradient of categorical_logit_glm_lpmf(y|x,alpha,beta) wrt (alpha, beta col-major); inputs: tests/gen.py glm_cat_inputs");
    j.put_int("R", c.R);
    j.put_int("M", c.M);
    j.put_int("C", c.C);
    j.put_int("y_scalar", c.ys);
    j.put("fx", fx);
    j.put_vec("grad", g);
    j.put("fx_propto", fxp);
    j.put_vec("grad_propto", gp);
    write_fixture("categorical_logit_glm_R" + std::to_string(c.R) + "_M" + std::to_string(c.M) + "_C" +
                      std::to_string(c.C) + (c.ys ? "_yscalar" : ""),
                  j);
  }
}

// The reference's exceptions (and early returns) for categorical_logit_glm on
// small hand-made inputs; tests/cpp/test_functors.cpp "glm_cat_errors" runs
// the same cases through the layer and the test compares the strings.
static void fix_glm_cat_errors() {
  using stan::math::var;
  using VV = Matrix<var, Dynamic, 1>;
  using MV = Matrix<var, Dynamic, Dynamic>;
  Json j;
  auto run = [&](const char* name, auto&& f) {
    std::string out;
    try {
      const double v = stan::math::value_of(f());
      std::ostringstream o;
      o.precision(17);
      o << "value " << v;
      out = o.str();
    } catch (const std::domain_error& e) {
      out = std::string("domain_error ") + e.what();
    } catch (const std::invalid_argument& e) {
      out = std::string("invalid_argument ") + e.what();
    }
    stan::math::recover_memory();
    j.put_str(name, out.c_str());
  };
  auto X = [](std::initializer_list<double> v, int r, int c) {
    MatrixXd m(r, c);
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
  const MatrixXd x = X({1, 2}, 2, 1);
  using stan::math::categorical_logit_glm_lpmf;
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
  run("cat_empty", [&] { return categorical_logit_glm_lpmf(std::vector<int>{}, MatrixXd(0, 1), A({0, 1, 2}), B({1, 2, 3}, 1, 3)); });
  run("cat_small", [&] { return categorical_logit_glm_lpmf(std::vector<int>{3, 1}, x, A({0, 1, 2}), B({1, -2, 0.5}, 1, 3)); });
  write_fixture("categorical_logit_glm_errors", j);
}

// ---- map_rect with a generic user functor whose jobs
// return different numbers of outputs (x_i[0] = outputs of the job).  Host
// scalar arithmetic only; the same functor is written out in
// tests/cpp/maprect_dist.cpp.  f = sum_i (1 + 0.1 i) out_i over the
// concatenated outputs; gradient over (phi(2), theta(J)).
struct hier_job {
  template <typename T1, typename T2>
  Matrix<stan::return_type_t<T1, T2>, Dynamic, 1> operator()(
      const Matrix<T1, Dynamic, 1>& phi, const Matrix<T2, Dynamic, 1>& theta,
      const std::vector<double>& x_r, const std::vector<int>& x_i, std::ostream*) const {
    using stan::math::exp;
    using stan::math::log;
    using stan::math::square;
    const int nout = x_i[0];
    Matrix<stan::return_type_t<T1, T2>, Dynamic, 1> out(nout);
    const auto sigma = exp(phi(1));
    for (int k = 0; k < nout; ++k) {
      stan::return_type_t<T1, T2> acc = 0.0;
      for (size_t i = k; i < x_r.size(); i += nout)
        acc += -0.5 * square((x_r[i] - (phi(0) + theta(0))) / sigma) - log(sigma);
      out(k) = acc;
    }
    return out;
  }
};
static void maprect_inputs(int J, std::vector<std::vector<double>>& xr, std::vector<std::vector<int>>& xi,
                           VectorXd& th) {
  std::vector<double> u = unif(SEED + 91, (size_t)J * 6, -2.0, 2.0);
  xr.assign(J, std::vector<double>(6));
  xi.assign(J, std::vector<int>(2, 0));
  for (int j = 0; j < J; ++j) {
    for (int i = 0; i < 6; ++i) xr[j][i] = u[(size_t)j * 6 + i];
    xi[j][0] = 1 + j % 3;
  }
  th.resize(2 + J);
  th(0) = 0.3;
  th(1) = -0.2;
  for (int j = 0; j < J; ++j) th(2 + j) = 0.1 * j - 0.25;
}
struct hier_maprect_functor {
  int J;
  const std::vector<std::vector<double>>& xr;
  const std::vector<std::vector<int>>& xi;
  template <typename T>
  T operator()(const Matrix<T, Dynamic, 1>& th) const {
    Matrix<T, Dynamic, 1> phi = th.head(2);
    std::vector<Matrix<T, Dynamic, 1>> job(J, Matrix<T, Dynamic, 1>(1));
    for (int j = 0; j < J; ++j) job[j](0) = th(2 + j);
    Matrix<T, Dynamic, 1> out = stan::math::map_rect<3, hier_job>(phi, job, xr, xi);
    T f = 0.0;
    for (int i = 0; i < out.size(); ++i) f += (1.0 + 0.1 * i) * out(i);
    return f;
  }
};
static void fix_maprect() {
#ifndef STAN_THREADS
  for (int J : {7, 1, 16}) {
    std::vector<std::vector<double>> xr;
    std::vector<std::vector<int>> xi;
    VectorXd th, g;
    maprect_inputs(J, xr, xi, th);
    double fx;
    stan::math::gradient(hier_maprect_functor{J, xr, xi}, th, fx, g);
    std::vector<Matrix<double, Dynamic, 1>> jobd(J, Matrix<double, Dynamic, 1>(1));
    for (int j = 0; j < J; ++j) jobd[j](0) = th(2 + j);
    VectorXd vals = stan::math::map_rect<4, hier_job>(VectorXd(th.head(2)), jobd, xr, xi);
    Json j;
    j.put_str("what", "map_rect<hier_job>: f = sum_i (1 + 0.1 i) out_i, gradient over (phi(2), theta(J)); inputs: tests/gen.py maprect_inputs");
    j.put_int("J", J);
    j.put("fx", fx);
    j.put_vec("grad", g);
    j.put_vec("values", vals);
    write_fixture("map_rect_hier_J" + std::to_string(J), j);
  }
#endif
}

// ---- mdivide_left_spd, log_determinant_spd,
// multiply_lower_tri_self_transpose, quad_form_sym.  Inputs are exact
// element-wise constructions (tests/gen.py spd_inputs mirrors them bit for
// bit): S_ij = S_ji = u_ij (i > j), S_ii = n + u_ii (diagonally dominant,
// so SPD); B, L, W uniform on [-1, 1).  f = sum(W .* F(args)); the gradient
// runs over every entry of every argument (col-major, args concatenated).
static MatrixXd spd_exact(int n, uint64_t seed) {
  std::vector<double> u = unif(seed, (size_t)n * n, -1.0, 1.0);
  MatrixXd S(n, n);
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) {
      const int a = i > j ? i : j, b = i > j ? j : i;  // lower-triangle source
      S(i, j) = u[(size_t)b * n + a];
    }
  for (int i = 0; i < n; ++i) S(i, i) = n + u[(size_t)i * n + i];
  return S;
}
static MatrixXd unif_mat(int r, int c, uint64_t seed) {
  std::vector<double> u = unif(seed, (size_t)r * c, -1.0, 1.0);
  return Eigen::Map<MatrixXd>(u.data(), r, c);
}
static Matrix<var, Dynamic, Dynamic> take(const Matrix<var, Dynamic, 1>& th, size_t off, int r, int c) {
  Matrix<var, Dynamic, Dynamic> m(r, c);
  for (int i = 0; i < r * c; ++i) m(i) = th((Eigen::Index)(off + i));
  return m;
}
struct spd_functor {
  int kind, n, k;  // kind 0 mdivide_left_spd(A n x n, B n x k); 1 log_determinant_spd(A);
                   // 2 multiply_lower_tri_self_transpose(L n x k); 3 quad_form_sym(A, B n x k)
  MatrixXd W;
  var operator()(const Matrix<var, Dynamic, 1>& th) const {
    using stan::math::sum;
    if (kind == 0) {
      auto A = take(th, 0, n, n), B = take(th, (size_t)n * n, n, k);
      Matrix<var, Dynamic, Dynamic> C = stan::math::mdivide_left_spd(A, B);
      return sum(stan::math::elt_multiply(C, W));
    }
    if (kind == 1) return stan::math::log_determinant_spd(take(th, 0, n, n));
    if (kind == 2) {
      Matrix<var, Dynamic, Dynamic> C = stan::math::multiply_lower_tri_self_transpose(take(th, 0, n, k));
      return sum(stan::math::elt_multiply(C, W));
    }
    auto A = take(th, 0, n, n), B = take(th, (size_t)n * n, n, k);
    Matrix<var, Dynamic, Dynamic> C = stan::math::quad_form_sym(A, B);
    return sum(stan::math::elt_multiply(C, W));
  }
};
static void fix_spd() {
  struct Case {
    int kind, n, k;
  };
  const char* names[] = {"mdivide_left_spd", "log_determinant_spd", "multiply_lower_tri_self_transpose",
                         "quad_form_sym"};
  for (Case c : {Case{0, 5, 3}, Case{0, 40, 7}, Case{0, 130, 17}, Case{1, 5, 0}, Case{1, 40, 0},
                 Case{1, 130, 0}, Case{2, 5, 5}, Case{2, 40, 25}, Case{2, 25, 40}, Case{2, 130, 130},
                 Case{3, 5, 3}, Case{3, 40, 12}, Case{3, 130, 60}}) {
    const uint64_t s0 = SEED + 60 + 10 * c.kind;
    VectorXd th;
    int wr = 0, wc = 0;
    if (c.kind == 0 || c.kind == 3) {
      MatrixXd A = spd_exact(c.n, s0), B = unif_mat(c.n, c.k, s0 + 1);
      th.resize((Eigen::Index)c.n * c.n + (Eigen::Index)c.n * c.k);
      th << Eigen::Map<VectorXd>(A.data(), A.size()), Eigen::Map<VectorXd>(B.data(), B.size());
      wr = c.kind == 0 ? c.n : c.k;
      wc = c.k;
    } else if (c.kind == 1) {
      MatrixXd A = spd_exact(c.n, s0);
      th = Eigen::Map<VectorXd>(A.data(), A.size());
    } else {
      MatrixXd L = unif_mat(c.n, c.k, s0 + 1);
      th = Eigen::Map<VectorXd>(L.data(), L.size());
      wr = wc = c.n;
    }
    spd_functor f{c.kind, c.n, c.k, unif_mat(wr, wc, s0 + 2)};
    double fx;
    VectorXd g;
    stan::math::gradient(f, th, fx, g);
    Json j;
    j.put_str("what", std::string("gradient of sum(W .* ") + names[c.kind] +
                          "(...)) (log_determinant_spd: the value itself) wrt every argument entry; "
                          "inputs: tests/gen.py spd_inputs");
    j.put_int("kind", c.kind);
    j.put_int("n", c.n);
    j.put_int("k", c.k);
    j.put("fx", fx);
    j.put("grad_sum", g.sum());
    j.put("grad_l2", g.norm());
    if (g.size() <= 4000) {
      j.put_vec("grad", g);
    } else {
      smg_rng r = smg_rng_make(SEED + 223);
      std::vector<double> idx, val;
      for (int q = 0; q < 512; ++q) {
        size_t kk = smg_rng_next(&r) % (size_t)g.size();
        idx.push_back((double)kk);
        val.push_back(g((Eigen::Index)kk));
      }
      j.put_vec("sample_index", idx);
      j.put_vec("sample_grad", val);
    }
    write_fixture(std::string(names[c.kind]) + "_n" + std::to_string(c.n) + "_k" + std::to_string(c.k), j);
  }
}

// ---- log_determinant (rev/mat/fun/log_determinant.hpp:14-37)
// of general square matrices: A = U[-1, 1) (n x n, col-major, tests/gen.py
// logdet_input) + shift sqrt(n) I, row 0 negated when flip (det < 0);
// gradient wrt every entry.  Plus the prim value of a singular matrix.
struct logdet_functor {
  int n;
  var operator()(const Matrix<var, Dynamic, 1>& th) const { return stan::math::log_determinant(take(th, 0, n, n)); }
};
static void fix_logdet() {
  struct Case {
    int n, shift, flip;
  };
  for (Case c : {Case{1, 1, 1}, Case{5, 1, 1}, Case{40, 0, 0}, Case{40, 1, 1}, Case{130, 1, 0}}) {
    MatrixXd A = unif_mat(c.n, c.n, SEED + 130 + c.n);
    for (int i = 0; i < c.n; ++i) A(i, i) += c.shift * std::sqrt((double)c.n);
    if (c.flip) A.row(0) *= -1.0;
    VectorXd th = Eigen::Map<VectorXd>(A.data(), A.size()), g;
    double fx;
    stan::math::gradient(logdet_functor{c.n}, th, fx, g);
    Json j;
    j.put_str("what", "gradient of log_determinant(A) (log|det A|) wrt every entry of A; input: tests/gen.py "
                      "logdet_input");
    j.put_int("n", c.n);
    j.put_int("shift", c.shift);
    j.put_int("flip", c.flip);
    j.put("fx", fx);
    j.put("fx_prim", stan::math::log_determinant(A));
    j.put_vec("grad", g);
    write_fixture("log_determinant_n" + std::to_string(c.n) + "_s" + std::to_string(c.shift), j);
  }
  MatrixXd S(3, 3);
  S << 1, 2, 3, 2, 4, 6, 1, 0, 1;  // rank 2
  Json j;
  j.put_str("what", "prim log_determinant of the rank-2 matrix [[1,2,3],[2,4,6],[1,0,1]] (row-major)");
  j.put("fx", stan::math::log_determinant(S));
  write_fixture("log_determinant_singular3", j);
}

// ---- hessian() (mix/mat/functor/hessian.hpp:39-72) of
// models built from multiply, mdivide_left_tri_low, log_sum_exp and the
// bernoulli logit GLM (fvar<var> instantiations of the reference).
struct lse_h_functor {
  template <typename T>
  T operator()(const Matrix<T, Dynamic, 1>& th) const {
    return stan::math::log_sum_exp(th);
  }
};
struct tri_h_functor {  // sum(mdivide_left_tri_low(L, B) w), L n x n (lower used), B n x k
  int n, k;
  VectorXd w;
  template <typename T>
  T operator()(const Matrix<T, Dynamic, 1>& th) const {
    Matrix<T, Dynamic, Dynamic> L(n, n), B(n, k);
    for (int i = 0; i < n * n; ++i) L(i) = th(i);
    for (int i = 0; i < n * k; ++i) B(i) = th(n * n + i);
    Matrix<T, Dynamic, Dynamic> C = stan::math::mdivide_left_tri_low(L, B);
    return stan::math::sum(stan::math::multiply(C, w));
  }
};
static void put_hessian(Json& j, const MatrixXd& H, bool full) {
  j.put("H_sum", H.sum());
  j.put("H_l2", H.norm());
  if (full) {
    j.put_mat("H", H);
    return;
  }
  smg_rng r = smg_rng_make(SEED + 224);
  std::vector<double> idx, val;
  for (int s = 0; s < 2048; ++s) {
    size_t kk = smg_rng_next(&r) % (size_t)H.size();
    idx.push_back((double)kk);
    val.push_back(H((Eigen::Index)kk));
  }
  j.put_vec("H_sample_index", idx);
  j.put_vec("H_sample", val);
}
static void fix_hessian2() {
  for (int N : {8, 40}) {  // config 2: sum(cholesky_decompose(add_diag(A A^T, N)))
    VectorXd a = mulchol_input(N), g;
    double fx;
    MatrixXd H;
    stan::math::hessian(mulchol_functor{N}, a, fx, g, H);
    Json j;
    j.put_str("what", "hessian of sum(cholesky_decompose(add_diag(multiply(A,A^T),N))) wrt A (col-major), "
                      "A = tests/gen.py mulchol_input");
    j.put_int("N", N);
    j.put("fx", fx);
    j.put_vec("grad", g);
    put_hessian(j, H, N <= 8);
    write_fixture("hessian_mulchol_N" + std::to_string(N), j);
  }
  // (the bernoulli logit GLM does not instantiate at fvar<var> in the
  // reference: prim/mat/prob/bernoulli_logit_glm_lpmf.hpp:106 calls
  // std::isfinite on a var; its Hessian is pinned in tests/ by the closed form)
  {  // log_sum_exp of 7 values with a wide spread
    VectorXd th(7), g;
    th << -3.0, 0.5, 2.0, -0.25, 10.0, 9.5, -40.0;
    double fx;
    MatrixXd H;
    stan::math::hessian(lse_h_functor{}, th, fx, g, H);
    Json j;
    j.put_str("what", "hessian of log_sum_exp(x)");
    j.put_vec("x", th);
    j.put("fx", fx);
    j.put_vec("grad", g);
    put_hessian(j, H, true);
    write_fixture("hessian_lse7", j);
  }
  {  // mdivide_left_tri_low: L 6 x 6 (lower: U[-1,1) + 4 on the diagonal; upper entries unused), B 6 x 2
    const int n = 6, k = 2;
    MatrixXd L = unif_mat(n, n, SEED + 140);
    for (int i = 0; i < n; ++i) L(i, i) += 4.0;
    MatrixXd B = unif_mat(n, k, SEED + 141);
    VectorXd w = Eigen::Map<VectorXd>(unif_mat(k, 1, SEED + 142).data(), k);
    VectorXd th(n * n + n * k), g;
    th << Eigen::Map<VectorXd>(L.data(), L.size()), Eigen::Map<VectorXd>(B.data(), B.size());
    double fx;
    MatrixXd H;
    stan::math::hessian(tri_h_functor{n, k, w}, th, fx, g, H);
    Json j;
    j.put_str("what", "hessian of sum(mdivide_left_tri_low(L, B) w) wrt (L (all n^2 entries, lower used), B); "
                      "inputs tests/gen.py tri_h_inputs");
    j.put_vec("theta", th);
    j.put_vec("w", w);
    j.put("fx", fx);
    j.put_vec("grad", g);
    put_hessian(j, H, true);
    write_fixture("hessian_tri_n6_k2", j);
  }
}

// The error messages of the hot-path functors (the cases of
// tests/cpp/test_functors.cpp cmd_errors, with the reference's own argument
// types): "<kind> <what()>" per case.
static void fix_errors() {
  using stan::math::var;
  using VV = Matrix<var, Dynamic, 1>;
  using MV = Matrix<var, Dynamic, Dynamic>;
  Json j;
  auto run = [&](const char* name, auto&& f) {
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
    stan::math::recover_memory();
    j.put_str(name, out.c_str());
  };
  auto M = [](std::initializer_list<double> v, int r, int c) {
    MV m(r, c);
    int i = 0;
    for (double t : v) m(i++) = t;
    return m;
  };
  const double nan = std::nan("");
  run("normal_nan_y", [&] { return stan::math::normal_lpdf(std::vector<var>{1.0, nan}, 0.0, 1.0); });
  run("normal_inf_mu", [&] { return stan::math::normal_lpdf(var(1.0), INFINITY, 1.0); });
  run("normal_neg_sigma", [&] { return stan::math::normal_lpdf(var(1.0), 0.0, -1.0); });
  run("normal_sizes", [&] {
    return stan::math::normal_lpdf(std::vector<var>{1.0, 2.0}, std::vector<double>{0, 0, 0}, 1.0);
  });
  run("multiply_sizes", [&] {
    MV A = M({1, 1, 1, 1, 1, 1}, 2, 3);
    return stan::math::multiply(A, A);
  });
  run("mdivide_square", [&] {
    MV A = M({1, 1, 1, 1, 1, 1}, 2, 3);
    return stan::math::mdivide_left_tri<Eigen::Lower>(A, A);
  });
  run("chol_not_symmetric", [&] { return stan::math::cholesky_decompose(M({2, 1, 0, 2}, 2, 2)); });
  run("chol_not_pd", [&] { return stan::math::cholesky_decompose(M({1, 2, 2, 1}, 2, 2)); });
  run("chol_not_square", [&] { return stan::math::cholesky_decompose(M({1, 2, 2, 1, 3, 3}, 2, 3)); });
  run("chol_nan", [&] { return stan::math::cholesky_decompose(M({1, nan, nan, 1}, 2, 2)); });
  const MatrixXd x = Eigen::Map<const MatrixXd>(std::vector<double>{1, 2}.data(), 2, 1);
  run("glm_y_bounds", [&] {
    VV b(1);
    b << 1.0;
    return stan::math::bernoulli_logit_glm_lpmf(std::vector<int>{0, 2}, x, var(0.0), b);
  });
  run("glm_beta_size", [&] {
    VV b(2);
    b << 1.0, 2.0;
    return stan::math::bernoulli_logit_glm_lpmf(std::vector<int>{0, 1}, x, var(0.0), b);
  });
  run("glm_nonfinite_beta", [&] {
    VV b(1);
    b << INFINITY;
    return stan::math::bernoulli_logit_glm_lpmf(std::vector<int>{0, 1}, x, var(0.0), b);
  });
  run("mvn_not_square", [&] {
    VV y(2), mu(2);
    y << 1, 2;
    mu << 0, 0;
    return stan::math::multi_normal_cholesky_lpdf(y, mu, M({1, 0, 0, 1, 0, 0}, 2, 3));
  });
  run("mvn_size_mu", [&] {
    VV y(2), mu(3);
    y << 1, 2;
    mu << 0, 0, 0;
    return stan::math::multi_normal_cholesky_lpdf(y, mu, M({1, 0, 0, 1}, 2, 2));
  });
  run("mvn_nan_y", [&] {
    VV y(2), mu(2);
    y << 1, nan;
    mu << 0, 0;
    return stan::math::multi_normal_cholesky_lpdf(y, mu, M({1, 0, 0, 1}, 2, 2));
  });
  run("gp_nonpositive_l", [&] {
    return stan::math::gp_exp_quad_cov(std::vector<double>{1, 2}, var(1.0), var(-1.0));
  });
  run("gp_nan_x", [&] {
    return stan::math::gp_exp_quad_cov(std::vector<double>{1, nan}, var(1.0), var(1.0));
  });
  write_fixture("errors_hot_path", j);
}

static void fix_hessian() {  // mix/mat/functor/hessian.hpp on the GP marginal
  for (int N : {8, 32, 100}) {
    std::vector<double> x;
    VectorXd y;
    gp_inputs(N, x, y);
    VectorXd th(3), g;
    th << 1.0, 1.5, 0.3;
    double fx;
    MatrixXd H;
    stan::math::hessian(gp_functor{x, y}, th, fx, g, H);
    Json j;
    j.put_str("what", "hessian (fwd-over-rev, mix/mat/functor/hessian.hpp) of the GP marginal log density");
    j.put_int("N", N);
    j.put_vec("theta", th);
    j.put_vec("x", x);
    j.put_vec("y", y);
    j.put("fx", fx);
    j.put_vec("grad", g);
    j.put_mat("H", H);
    write_fixture("hessian_gp_N" + std::to_string(N), j);
  }
}

static void fix_hvp() {
  for (int N : {8, 32, 100, 256}) {
    std::vector<double> x;
    VectorXd y;
    gp_inputs(N, x, y);
    VectorXd th(3), v(3);
    th << 1.0, 1.5, 0.3;
    v << 1.0, -0.5, 0.25;
    double fx;
    VectorXd Hv;
    stan::math::hessian_times_vector(gp_functor{x, y}, th, v, fx, Hv);
    Json j;
    j.put_str("what", "hessian_times_vector (fwd-over-rev) of the GP marginal log density");
    j.put_int("N", N);
    j.put_vec("theta", th);
    j.put_vec("v", v);
    j.put_vec("x", x);
    j.put_vec("y", y);
    j.put("fx", fx);
    j.put_vec("Hv", Hv);
    write_fixture("hvp_gp_N" + std::to_string(N), j);
  }
}


// The reference's call forms at the drop-in boundary (tests/cpp/boundary_cases.hpp,
// compiled here against the reference and in tests/cpp/test_boundary.cpp
// against math_amd): multiply row x col / matrix x vector / scalar forms,
// add_diag with a vector, sum(std::vector<var>), every var / double mix and
// the array forms of multi_normal_cholesky_lpdf, the D-dimensional GP.
static bnd::form_inputs boundary_inputs() {
  bnd::form_inputs in;
  in.A = unif(SEED + 2000, (size_t)in.m * in.k, -1, 1);
  in.B = unif(SEED + 2001, (size_t)in.k * in.n, -1, 1);
  in.v = unif(SEED + 2002, in.k, -1, 1);
  in.r = unif(SEED + 2003, in.k, -1, 1);
  in.r5 = unif(SEED + 2004, in.m, -1, 1);
  MatrixXd S = spd(in.s, SEED + 2005);
  in.S.assign(S.data(), S.data() + S.size());
  in.d = unif(SEED + 2006, in.s, 0.5, 1.5);
  MatrixXd L = spd(in.s, SEED + 2007).llt().matrixL();
  in.L.assign(L.data(), L.data() + L.size());
  in.ys = unif(SEED + 2008, (size_t)in.s * in.nobs, -2, 2);
  in.mu = unif(SEED + 2009, in.s, -1, 1);
  in.W = unif(SEED + 2010, 64, -1, 1);
  in.c = 0.7;
  return in;
}

static void gp_nd_inputs(int N, int D, int nobs, std::vector<VectorXd>& x, std::vector<VectorXd>& ys) {
  std::vector<double> xv = unif(SEED + 2100, (size_t)N * D, -5.0, 5.0);
  x.assign(N, VectorXd(D));
  for (int i = 0; i < N; ++i)
    for (int d = 0; d < D; ++d) x[i](d) = xv[(size_t)i * D + d];
  ys.assign(nobs, VectorXd(N));
  for (int j = 0; j < nobs; ++j) {
    std::vector<double> e = normals(SEED + 2101 + j, N);
    for (int i = 0; i < N; ++i) {
      double t = 0;
      for (int d = 0; d < D; ++d) t += (d % 2 ? -0.5 : 1.0) * x[i](d);
      ys[j](i) = std::sin(t) + 0.3 * e[i];
    }
  }
}

static void fix_boundary() {
  {
    bnd::form_inputs in = boundary_inputs();
    Json j;
    j.put_str("what", "the reference's boundary call forms (tests/cpp/boundary_cases.hpp): per case f and the gradient of every var input in argument order");
    j.put_int("m", in.m);
    j.put_int("k", in.k);
    j.put_int("n", in.n);
    j.put_int("s", in.s);
    j.put_int("nobs", in.nobs);
    j.put_vec("A", in.A);
    j.put_vec("B", in.B);
    j.put_vec("v", in.v);
    j.put_vec("r", in.r);
    j.put_vec("r5", in.r5);
    j.put_vec("S", in.S);
    j.put_vec("d", in.d);
    j.put_vec("L", in.L);
    j.put_vec("ys", in.ys);
    j.put_vec("mu", in.mu);
    j.put_vec("W", in.W);
    j.put("c", in.c);
    bnd::run_form_cases(in, [&](const std::string& name, double f, const std::vector<double>& g) {
      j.put(name + "_fx", f);
      j.put_vec(name + "_grad", g);
    });
    write_fixture("boundary_forms", j);
  }
  {
    Json j;
    bnd::run_error_cases([&](const std::string& name, const std::function<void()>& f) {
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
      stan::math::recover_memory();
      j.put_str(name, out);
    });
    write_fixture("boundary_errors", j);
  }
  for (int N : {64, 256}) {
    const int D = 3, nobs = 5;
    std::vector<VectorXd> x, ys;
    gp_nd_inputs(N, D, nobs, x, ys);
    Json j;
    j.put_str("what", "Stan-codegen-shaped GP marginal with D-dimensional x (std::vector<VectorXd>): form 0 gp_exp_quad_cov(x, alpha, rho); form 1 gp_exp_quad_cov(x, 1.3, rho); form 2 form 0 with nobs observations and a var mean theta(3)");
    j.put_int("N", N);
    j.put_int("D", D);
    j.put_int("nobs", nobs);
    std::vector<double> xf, yf;
    for (auto& p : x) xf.insert(xf.end(), p.data(), p.data() + D);
    for (auto& y : ys) yf.insert(yf.end(), y.data(), y.data() + N);
    j.put_vec("x", xf);
    j.put_vec("ys", yf);
    const double th0[] = {1.0, 1.5, 0.3, 0.2};
    for (int form = 0; form < 3; ++form) {
      const int P = form == 1 ? 2 : form == 2 ? 4 : 3;
      VectorXd th(P);
      if (form == 1)
        th << 1.5, 0.3;
      else
        for (int i = 0; i < P; ++i) th(i) = th0[i];
      double fx;
      VectorXd g;
      stan::math::gradient(bnd::gp_marginal<VectorXd>{x, ys, form}, th, fx, g);
      const std::string f = "_f" + std::to_string(form);
      j.put_vec("theta" + f, th);
      j.put("fx" + f, fx);
      j.put_vec("grad" + f, g);
    }
    write_fixture("gp_nd_D3_N" + std::to_string(N), j);
  }
  // intermediate adjoints and vari identity after a top-level lp.grad()
  // (bnd::run_gp_intermediate): the config-3 inputs at N = 64 (variants 0-2)
  // and N = 256 (variants 0, 1)
  for (int N : {64, 256}) {
    std::vector<double> x;
    VectorXd y;
    gp_inputs(N, x, y);
    const double th[3] = {1.0, 1.5, 0.3};
    Json j;
    j.put_str("what", "after lp.grad() of the Stan-codegen GP marginal (K = gp_exp_quad_cov(x, th0, th1), Kd = add_diag(K, th2^2), L = cholesky_decompose(Kd), lp = multi_normal_cholesky_lpdf(y | 0, L); variant 1 + host uses of L, variant 2 + host uses of K and Kd's diagonal): v<k> = [grad th | K adj lower packed | Kd diag adj | L adj lower packed | L val lower packed | K sym-shared, Kd shares K, Kd diag new, L upper dummy, #varis K, #varis K+Kd, #varis L]");
    j.put_int("N", N);
    j.put_vec("x", x);
    j.put_vec("y", y);
    j.put_vec("theta", std::vector<double>(th, th + 3));
    for (int v = 0; v < (N == 64 ? 3 : 2); ++v)
      bnd::run_gp_intermediate(x, y, th, v, [&](const std::string&, double f, const std::vector<double>& out) {
        j.put("fx_v" + std::to_string(v), f);
        j.put_vec("v" + std::to_string(v), out);
      });
    write_fixture("gp_intermediate_N" + std::to_string(N), j);
  }
}

// ------------------------------------------------------------------ bench
static double now() {
  return std::chrono::duration<double>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

#ifdef STAN_THREADS
// config 4 on every host core the way the reference's threaded map_rect
// runs it (rev/mat/functor/map_rect_concurrent.hpp:39-57: the jobs' nested
// gradients -- map_rect_reduce -- in parallel, here on std::threads instead
// of TBB, each with its own thread-local tape; STAN_THREADS build
// oracle/_ref/ref_harness_mt): 32 row-shard jobs of bernoulli_logit_glm_lpmf,
// their values and gradients summed in job order.
struct glm_rows_functor {
  const MatrixXd& x;
  const std::vector<int>& y;
  template <typename T>
  T operator()(const Matrix<T, Dynamic, 1>& th) const {
    Matrix<T, Dynamic, 1> beta = th.tail(x.cols());
    return stan::math::bernoulli_logit_glm_lpmf(y, x, th(0), beta);
  }
};
static int bench_glm_mt(int R, int reps, int threads) {
  const int shards = 32, M = 256;
  glm_data d = glm_inputs(R, M);
  std::vector<MatrixXd> xs(shards);
  std::vector<std::vector<int>> ys(shards);
  for (int s = 0; s < shards; ++s) {
    const int r0 = (int)((long long)R * s / shards), r1 = (int)((long long)R * (s + 1) / shards);
    xs[s] = d.x.middleRows(r0, r1 - r0);
    ys[s].assign(d.y.begin() + r0, d.y.begin() + r1);
  }
  std::vector<double> fxs(shards);
  std::vector<VectorXd> gs(shards);
  double fx = 0.0;
  VectorXd g = VectorXd::Zero(M + 1);
  const double t0 = now();
  for (int rep = 0; rep < reps; ++rep) {
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t)
      pool.emplace_back([&, t] {
        stan::math::ChainableStack tape;  // this thread's tape (the reference's STAN_THREADS contract)
        for (int s = t; s < shards; s += threads)
          stan::math::gradient(glm_rows_functor{xs[s], ys[s]}, d.theta, fxs[s], gs[s]);
      });
    for (auto& th : pool) th.join();
    fx = 0.0;
    g.setZero();
    for (int s = 0; s < shards; ++s) {
      fx += fxs[s];
      g += gs[s];
    }
  }
  const double per = (now() - t0) / reps;
  std::printf("{\"config\": \"glm_mt\", \"N\": %d, \"reps\": %d, \"seconds_per_eval\": %.9g, "
              "\"evals_per_sec\": %.9g, \"fx\": %.17g, \"threads\": %d, \"shards\": %d, \"grad0\": %.17g}\n",
              R, reps, per, 1.0 / per, fx, threads, shards, g(0));
  return 0;
}
#endif

static int bench(const std::string& cfg, int N, int reps) {
  double t0 = 0, t1 = 0, fx = 0;
  VectorXd g;
  if (cfg == "gp") {
    std::vector<double> x;
    VectorXd y;
    gp_inputs(N, x, y);
    VectorXd th(3);
    th << 1.0, 1.5, 0.3;
    t0 = now();
    for (int r = 0; r < reps; ++r)
      stan::math::gradient(gp_functor{x, y}, th, fx, g);
    t1 = now();
  } else if (cfg == "mulchol") {
    VectorXd a = mulchol_input(N);
    t0 = now();
    for (int r = 0; r < reps; ++r)
      stan::math::gradient(mulchol_functor{N}, a, fx, g);
    t1 = now();
  } else if (cfg == "glm") {
    glm_data d = glm_inputs(N, 256);
    t0 = now();
    for (int r = 0; r < reps; ++r)
      stan::math::gradient(glm_functor{d}, d.theta, fx, g);
    t1 = now();
  } else if (cfg == "hvp") {
    std::vector<double> x;
    VectorXd y;
    gp_inputs(N, x, y);
    VectorXd th(3), v(3), hv;
    th << 1.0, 1.5, 0.3;
    v << 1.0, -0.5, 0.25;
    t0 = now();
    for (int r = 0; r < reps; ++r)
      stan::math::hessian_times_vector(gp_functor{x, y}, th, v, fx, hv);
    t1 = now();
  } else if (cfg == "normal") {
    std::vector<double> th = normals(SEED + 1, N);
    VectorXd x = Eigen::Map<VectorXd>(th.data(), N);
    t0 = now();
    for (int r = 0; r < reps; ++r)
      stan::math::gradient(normal_functor{}, x, fx, g);
    t1 = now();
  } else {
    std::fprintf(stderr, "unknown bench config %s\n", cfg.c_str());
    return 2;
  }
  double per = (t1 - t0) / reps;
  std::printf("{\"config\": \"%s\", \"N\": %d, \"reps\": %d, \"seconds_per_eval\": %.9g, "
              "\"evals_per_sec\": %.9g, \"fx\": %.17g, \"threads\": 1}\n",
              cfg.c_str(), N, reps, per, 1.0 / per, fx);
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 2 && std::string(argv[1]) == "gen") {
    if (argc >= 3) g_outdir = argv[2];
    std::string only = argc >= 4 ? argv[3] : "";
    auto want = [&](const char* s) { return only.empty() || only == s; };
    if (want("normal")) fix_normal();
    if (want("special")) fix_special();
    if (want("lse")) fix_lse();
    if (want("multiply")) fix_multiply();
    if (want("mdivide")) fix_mdivide();
    if (want("cholesky")) fix_cholesky();
    if (want("mvn")) fix_mvn();
    if (want("glm")) fix_glm();
    if (want("glm2")) fix_glm2();
    if (want("glm_cat")) {
      fix_glm_cat();
      fix_glm_cat_errors();
    }
    if (want("spd")) fix_spd();
    if (want("logdet")) fix_logdet();
    if (want("maprect")) fix_maprect();
    if (want("hessian")) fix_hessian();
    if (want("hessian2")) fix_hessian2();
    if (want("errors")) fix_errors();
    if (want("hvp")) fix_hvp();
    if (want("mulchol")) fix_mulchol();
    if (want("gp")) fix_gp();
    if (want("boundary")) fix_boundary();
    return 0;
  }
#ifdef STAN_THREADS
  if (argc >= 5 && std::string(argv[1]) == "bench" && std::string(argv[2]) == "glm_mt") {
    int threads = argc >= 6 ? std::atoi(argv[5]) : 0;
    if (threads <= 0) threads = std::max(1, std::min(16, (int)std::thread::hardware_concurrency()));
    return bench_glm_mt(std::atoi(argv[3]), std::atoi(argv[4]), threads);
  }
#endif
  if (argc >= 5 && std::string(argv[1]) == "bench")
    return bench(argv[2], std::atoi(argv[3]), std::atoi(argv[4]));
  std::fprintf(stderr,
               "usage: %s gen [outdir] [only]\n       %s bench gp|mulchol|glm|normal|hvp N reps\n",
               argv[0], argv[0]);
  return 2;
}
