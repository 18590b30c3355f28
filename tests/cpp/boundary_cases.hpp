// The reference's call forms at the drop-in boundary, written ONCE and
// compiled twice (TEST INFRASTRUCTURE):
//   - by oracle/ref_harness.cpp against the real Stan Math 3.0.0 headers, to
//     write the golden fixtures tests/golden/boundary_*.json, gp_nd_*.json;
//   - by tests/cpp/test_boundary.cpp against math_amd/include (the compile
//     probe: every form below must resolve to a math_amd overload), whose
//     output tests/test_boundary.py compares with those fixtures.
// Every case builds its var inputs from the given doubles, evaluates one
// scalar f (a weighted sum W .* out for matrix outputs), runs f.grad() and
// emits (name, f, gradients of every var input in argument order, each
// column-major), then recovers the tape.
//
// Reference overloads exercised (file:line):
//   multiply         rev/mat/fun/multiply.hpp:562-661 (row x col -> var :647-661,
//                    matrix x matrix / vector / row vector :619-645, scalar x matrix :574-600)
//   add_diag         prim/mat/fun/add_diag.hpp:20-55 (scalar and vector to_add)
//   sum              rev/arr/fun/sum.hpp:54 (std::vector<var>)
//   multi_normal_cholesky_lpdf  prim/mat/prob/multi_normal_cholesky_lpdf.hpp:40-166
//                    (any var/double mix of y / mu / L, vector_seq_view arrays :59-80)
//   gp_exp_quad_cov  rev/mat/fun/gp_exp_quad_cov.hpp:211-286 (std::vector<T_x>, T_x = VectorXd)
#ifndef SMG_TESTS_BOUNDARY_CASES_HPP
#define SMG_TESTS_BOUNDARY_CASES_HPP

#include <functional>
#include <string>
#include <unordered_set>
#include <vector>

namespace bnd {

using stan::math::var;
using MV = Eigen::Matrix<var, Eigen::Dynamic, Eigen::Dynamic>;
using VV = Eigen::Matrix<var, Eigen::Dynamic, 1>;
using RV = Eigen::Matrix<var, 1, Eigen::Dynamic>;
using MD = Eigen::Matrix<double, Eigen::Dynamic, Eigen::Dynamic>;
using VD = Eigen::Matrix<double, Eigen::Dynamic, 1>;
using RD = Eigen::Matrix<double, 1, Eigen::Dynamic>;

using emit_fn = std::function<void(const std::string&, double, const std::vector<double>&)>;

/** Inputs of the form cases (all column-major). */
struct form_inputs {
  int m = 5, k = 7, n = 4, s = 6, nobs = 5;
  std::vector<double> A, B, v, r, r5, S, d, L, ys, mu, W;
  double c = 0.0;
};

template <typename T, int R, int C>
inline Eigen::Matrix<T, R, C> mat(const std::vector<double>& a, int rows, int cols, size_t off = 0) {
  Eigen::Matrix<T, R, C> out(rows, cols);
  for (int i = 0; i < rows * cols; ++i) out(i) = a[off + size_t(i)];
  return out;
}

// collected adjoints of the var inputs, in argument order
struct grads {
  std::vector<double> g;
  template <int R, int C>
  grads& add(const Eigen::Matrix<var, R, C>& x) {
    for (int i = 0; i < x.size(); ++i) g.push_back(x(i).adj());
    return *this;
  }
  grads& add(const var& x) {
    g.push_back(x.adj());
    return *this;
  }
  grads& add(const std::vector<var>& x) {
    for (const var& e : x) g.push_back(e.adj());
    return *this;
  }
  template <int R, int C>
  grads& add(const std::vector<Eigen::Matrix<var, R, C>>& x) {
    for (const auto& e : x) add(e);
    return *this;
  }
};

// f = sum_i W_i out_i over a var matrix / vector output
template <int R, int C>
inline var wsum(const Eigen::Matrix<var, R, C>& out, const std::vector<double>& W) {
  var f = 0.0;
  for (int i = 0; i < out.size(); ++i) f += W[size_t(i)] * out(i);
  return f;
}

inline void finish(const emit_fn& emit, const std::string& name, var f, const grads& g) {
  (void)f;
  emit(name, f.val(), g.g);
  stan::math::recover_memory();
}

inline void run_form_cases(const form_inputs& in, const emit_fn& emit) {
  using stan::math::add_diag;
  using stan::math::multi_normal_cholesky_lpdf;
  using stan::math::multiply;
  using stan::math::sum;
  const int m = in.m, k = in.k, n = in.n, s = in.s, K = in.nobs;

  // ---- multiply: row vector x vector -> var (multiply.hpp:647-661)
  {
    RV r = mat<var, 1, -1>(in.r, 1, k);
    VV v = mat<var, -1, 1>(in.v, k, 1);
    var f = multiply(r, v);
    f.grad();
    finish(emit, "mul_rv_v", f, grads().add(r).add(v));
  }
  {
    RD r = mat<double, 1, -1>(in.r, 1, k);
    VV v = mat<var, -1, 1>(in.v, k, 1);
    var f = multiply(r, v);
    f.grad();
    finish(emit, "mul_rd_v", f, grads().add(v));
  }
  {
    RV r = mat<var, 1, -1>(in.r, 1, k);
    VD v = mat<double, -1, 1>(in.v, k, 1);
    var f = multiply(r, v);
    f.grad();
    finish(emit, "mul_rv_vd", f, grads().add(r));
  }
  // ---- matrix x vector, row vector x matrix (:619-645)
  {
    MV A = mat<var, -1, -1>(in.A, m, k);
    VV v = mat<var, -1, 1>(in.v, k, 1);
    VV out = multiply(A, v);
    var f = wsum(out, in.W);
    f.grad();
    finish(emit, "mul_m_v", f, grads().add(A).add(v));
  }
  {
    MD A = mat<double, -1, -1>(in.A, m, k);
    VV v = mat<var, -1, 1>(in.v, k, 1);
    VV out = multiply(A, v);
    var f = wsum(out, in.W);
    f.grad();
    finish(emit, "mul_md_v", f, grads().add(v));
  }
  {
    MV A = mat<var, -1, -1>(in.A, m, k);
    VD v = mat<double, -1, 1>(in.v, k, 1);
    VV out = multiply(A, v);
    var f = wsum(out, in.W);
    f.grad();
    finish(emit, "mul_m_vd", f, grads().add(A));
  }
  {
    RV r = mat<var, 1, -1>(in.r5, 1, m);
    MV A = mat<var, -1, -1>(in.A, m, k);
    RV out = multiply(r, A);
    var f = wsum(out, in.W);
    f.grad();
    finish(emit, "mul_rv_m", f, grads().add(r).add(A));
  }
  {
    MV A = mat<var, -1, -1>(in.A, m, k);
    MD B = mat<double, -1, -1>(in.B, k, n);
    MV out = multiply(A, B);
    var f = wsum(out, in.W);
    f.grad();
    finish(emit, "mul_m_md", f, grads().add(A));
  }
  // ---- scalar x matrix (:574-600) and scalar x scalar (:561-565)
  {
    var c = in.c;
    MV A = mat<var, -1, -1>(in.A, m, k);
    MV o1 = multiply(c, A);
    MV o2 = multiply(A, c);
    var f = wsum(o1, in.W) + 0.5 * wsum(o2, in.W);
    f.grad();
    finish(emit, "mul_c_m", f, grads().add(c).add(A));
  }
  {
    var c = in.c;
    MD A = mat<double, -1, -1>(in.A, m, k);
    MV o1 = multiply(c, A);
    MV o2 = multiply(A, c);
    var f = wsum(o1, in.W) + 0.5 * wsum(o2, in.W);
    f.grad();
    finish(emit, "mul_c_md", f, grads().add(c));
  }
  {
    MV A = mat<var, -1, -1>(in.A, m, k);
    MV o = multiply(2.5, A);
    var f = wsum(o, in.W);
    f.grad();
    finish(emit, "mul_d_m", f, grads().add(A));
  }
  {
    var c = in.c, e = in.v[0];
    var f = multiply(c, e) + multiply(c, 3.0) + multiply(2.0, e);
    f.grad();
    finish(emit, "mul_scalars", f, grads().add(c).add(e));
  }

  // ---- add_diag (prim/mat/fun/add_diag.hpp:20-55)
  {
    MV S = mat<var, -1, -1>(in.S, s, s);
    VV d = mat<var, -1, 1>(in.d, s, 1);
    MV o = add_diag(S, d);
    var f = wsum(o, in.W);
    f.grad();
    finish(emit, "ad_m_v", f, grads().add(S).add(d));
  }
  {
    MV S = mat<var, -1, -1>(in.S, s, s);
    VD d = mat<double, -1, 1>(in.d, s, 1);
    MV o = add_diag(S, d);
    var f = wsum(o, in.W);
    f.grad();
    finish(emit, "ad_m_vd", f, grads().add(S));
  }
  {
    MD S = mat<double, -1, -1>(in.S, s, s);
    VV d = mat<var, -1, 1>(in.d, s, 1);
    MV o = add_diag(S, d);
    var f = wsum(o, in.W);
    f.grad();
    finish(emit, "ad_md_v", f, grads().add(d));
  }
  {
    MD S = mat<double, -1, -1>(in.S, s, s);
    var c = in.c;
    MV o = add_diag(S, c);
    var f = wsum(o, in.W);
    f.grad();
    finish(emit, "ad_md_c", f, grads().add(c));
  }
  {
    MV R = mat<var, -1, -1>(in.S, 4, s);  // non-square: min(rows, cols) = 4 diagonal entries
    VV d = mat<var, -1, 1>(in.d, 4, 1);
    MV o = add_diag(R, d);
    var f = wsum(o, in.W);
    f.grad();
    finish(emit, "ad_rect_v", f, grads().add(R).add(d));
  }
  {
    MV R = mat<var, -1, -1>(in.S, s, 4);
    var c = in.c;
    MV o = add_diag(R, c);
    var f = wsum(o, in.W);
    f.grad();
    finish(emit, "ad_rect_c", f, grads().add(R).add(c));
  }

  // ---- sum(std::vector<var>) (rev/arr/fun/sum.hpp:54)
  {
    std::vector<var> v(in.v.begin(), in.v.end());
    var f = sum(v);
    f.grad();
    finish(emit, "sum_vec", f, grads().add(v));
  }
  {
    std::vector<var> v;
    var f = sum(v);
    finish(emit, "sum_empty", f, grads());
  }

  // ---- multi_normal_cholesky_lpdf, every var / double mix and the array forms
  auto obs_v = [&](int j) { return mat<var, -1, 1>(in.ys, s, 1, size_t(j) * s); };
  auto obs_d = [&](int j) { return mat<double, -1, 1>(in.ys, s, 1, size_t(j) * s); };
  {
    VV y = obs_v(0);
    VD mu = mat<double, -1, 1>(in.mu, s, 1);
    MV L = mat<var, -1, -1>(in.L, s, s);
    var f = multi_normal_cholesky_lpdf(y, mu, L);
    f.grad();
    finish(emit, "mvn_v_d_m", f, grads().add(y).add(L));
  }
  {
    VD y = obs_d(0);
    VV mu = mat<var, -1, 1>(in.mu, s, 1);
    MV L = mat<var, -1, -1>(in.L, s, s);
    var f = multi_normal_cholesky_lpdf(y, mu, L);
    f.grad();
    finish(emit, "mvn_d_v_m", f, grads().add(mu).add(L));
  }
  {
    VV y = obs_v(0);
    VV mu = mat<var, -1, 1>(in.mu, s, 1);
    MD L = mat<double, -1, -1>(in.L, s, s);
    var f = multi_normal_cholesky_lpdf(y, mu, L);
    f.grad();
    finish(emit, "mvn_v_v_md", f, grads().add(y).add(mu));
  }
  {
    std::vector<VD> y;
    for (int j = 0; j < K; ++j) y.push_back(obs_d(j));
    VV mu = mat<var, -1, 1>(in.mu, s, 1);
    MV L = mat<var, -1, -1>(in.L, s, s);
    var f = multi_normal_cholesky_lpdf(y, mu, L);
    f.grad();
    finish(emit, "mvn_arr_d_v_m", f, grads().add(mu).add(L));
  }
  {
    std::vector<VD> y;
    for (int j = 0; j < K; ++j) y.push_back(obs_d(j));
    VV mu = mat<var, -1, 1>(in.mu, s, 1);
    MV L = mat<var, -1, -1>(in.L, s, s);
    var f = multi_normal_cholesky_lpdf<true>(y, mu, L);
    f.grad();
    finish(emit, "mvn_arr_d_v_m_propto", f, grads().add(mu).add(L));
  }
  {
    std::vector<VV> y;
    std::vector<VD> mu;
    for (int j = 0; j < K; ++j) {
      y.push_back(obs_v(j));
      mu.push_back(mat<double, -1, 1>(in.ys, s, 1, size_t(K - 1 - j) * s) * 0.5);
    }
    MV L = mat<var, -1, -1>(in.L, s, s);
    var f = multi_normal_cholesky_lpdf(y, mu, L);
    f.grad();
    finish(emit, "mvn_arr_v_arr_d_m", f, grads().add(y).add(L));
  }
  {
    std::vector<VV> y;
    for (int j = 0; j < K; ++j) y.push_back(obs_v(j));
    MD L = mat<double, -1, -1>(in.L, s, s);
    VD mu = mat<double, -1, 1>(in.mu, s, 1);
    var f = multi_normal_cholesky_lpdf(y, mu, L);
    f.grad();
    finish(emit, "mvn_arr_v_d_md", f, grads().add(y));
  }
  {
    RV y = mat<var, 1, -1>(in.ys, 1, s);
    RD mu = mat<double, 1, -1>(in.mu, 1, s);
    MV L = mat<var, -1, -1>(in.L, s, s);
    var f = multi_normal_cholesky_lpdf(y, mu, L);
    f.grad();
    finish(emit, "mvn_rv_rd_m", f, grads().add(y).add(L));
  }
  {
    // the GP-shaped form: L from cholesky_decompose of a var matrix (its
    // upper triangle is the reference's dummy vari), K observations
    MV S = mat<var, -1, -1>(in.S, s, s);
    MV L = stan::math::cholesky_decompose(S);
    std::vector<VD> y;
    for (int j = 0; j < K; ++j) y.push_back(obs_d(j));
    VD mu = mat<double, -1, 1>(in.mu, s, 1);
    var f = multi_normal_cholesky_lpdf(y, mu, L);
    f.grad();
    finish(emit, "mvn_arr_chol", f, grads().add(S));
  }
  // ---- mdivide_left_tri_low / mdivide_right_tri_low, the names Stan-generated
  // code emits (prim/mat/fun/mdivide_left_tri_low.hpp:33-47,
  // mdivide_right_tri_low.hpp:25-31): L s x s (its strict upper is ignored),
  // b s x 2 / 2 x s
  {
    using stan::math::mdivide_left_tri_low;
    using stan::math::mdivide_right_tri_low;
    MV L = mat<var, -1, -1>(in.S, s, s);  // a full matrix: only its lower triangle is read
    MV b = mat<var, -1, -1>(in.ys, s, 2);
    MV out = mdivide_left_tri_low(L, b);
    var f = wsum(out, in.W);
    f.grad();
    finish(emit, "mdl_tri_low_vv", f, grads().add(L).add(b));
  }
  {
    using stan::math::mdivide_left_tri_low;
    MD L = mat<double, -1, -1>(in.S, s, s);
    VV b = mat<var, -1, 1>(in.ys, s, 1);
    VV out = mdivide_left_tri_low(L, b);
    var f = wsum(out, in.W);
    f.grad();
    finish(emit, "mdl_tri_low_dv", f, grads().add(b));
  }
  {
    using stan::math::mdivide_left_tri_low;
    MV L = mat<var, -1, -1>(in.S, s, s);
    MD b = mat<double, -1, -1>(in.ys, s, 2);
    MV out = mdivide_left_tri_low(L, b);
    var f = wsum(out, in.W);
    f.grad();
    finish(emit, "mdl_tri_low_vd", f, grads().add(L));
  }
  {
    using stan::math::mdivide_left_tri_low;
    MV L = mat<var, -1, -1>(in.S, s, s);
    MV out = mdivide_left_tri_low(L);
    var f = wsum(out, in.W);
    f.grad();
    finish(emit, "mdl_tri_low_inv", f, grads().add(L));
  }
  {
    using stan::math::mdivide_right_tri_low;
    MV b = mat<var, -1, -1>(in.ys, 2, s);
    MV L = mat<var, -1, -1>(in.S, s, s);
    MV out = mdivide_right_tri_low(b, L);
    var f = wsum(out, in.W);
    f.grad();
    finish(emit, "mdr_tri_low_vv", f, grads().add(b).add(L));
  }
  {
    using stan::math::mdivide_right_tri_low;
    RV b = mat<var, 1, -1>(in.ys, 1, s);
    MD L = mat<double, -1, -1>(in.S, s, s);
    RV out = mdivide_right_tri_low(b, L);
    var f = wsum(out, in.W);
    f.grad();
    finish(emit, "mdr_tri_low_rv_d", f, grads().add(b));
  }
  {
    using stan::math::mdivide_left_tri_low;
    using stan::math::mdivide_right_tri_low;
    MD L = mat<double, -1, -1>(in.S, s, s);
    MD b = mat<double, -1, -1>(in.ys, s, 2);
    MD o1 = mdivide_left_tri_low(L, b);
    MD o2 = mdivide_right_tri_low(MD(b.transpose()), L);
    double f = 0.0;
    for (int i = 0; i < o1.size(); ++i) f += in.W[size_t(i)] * o1(i) + 0.5 * in.W[size_t(i)] * o2(i);
    emit("mdl_mdr_tri_low_dd", f, {});
    stan::math::recover_memory();
  }
}

// The Stan-codegen-shaped GP marginal: `matrix[N,N] K = ...` is an
// Eigen::Matrix<var,-1,-1>, so every stage crosses the Eigen boundary.
//   form 0: gp_exp_quad_cov(x, alpha, rho)          (var, var), theta = (alpha, rho, sigma)
//   form 1: gp_exp_quad_cov(x, 1.3, rho)            (double, var), theta = (rho, sigma)
//   form 2: form 0 with nobs observations y_j and a var mean theta(3)
template <typename T_x>
struct gp_marginal {
  const std::vector<T_x>& x;
  const std::vector<Eigen::VectorXd>& ys;  // ys[0] is the single-observation y
  int form;
  template <typename T>
  T operator()(const Eigen::Matrix<T, Eigen::Dynamic, 1>& th) const {
    using stan::math::add_diag;
    using stan::math::cholesky_decompose;
    using stan::math::gp_exp_quad_cov;
    using stan::math::multi_normal_cholesky_lpdf;
    using stan::math::square;
    const int N = int(x.size());
    if (form == 1) {
      Eigen::Matrix<T, -1, -1> K = gp_exp_quad_cov(x, 1.3, th(0));
      Eigen::Matrix<T, -1, -1> Kd = add_diag(K, square(th(1)));
      Eigen::Matrix<T, -1, -1> L = cholesky_decompose(Kd);
      Eigen::VectorXd mu = Eigen::VectorXd::Zero(N);
      return multi_normal_cholesky_lpdf(ys[0], mu, L);
    }
    Eigen::Matrix<T, -1, -1> K = gp_exp_quad_cov(x, th(0), th(1));
    Eigen::Matrix<T, -1, -1> Kd = add_diag(K, square(th(2)));
    Eigen::Matrix<T, -1, -1> L = cholesky_decompose(Kd);
    if (form == 2) {
      Eigen::Matrix<T, -1, 1> mu(N);
      for (int i = 0; i < N; ++i) mu(i) = th(3);
      return multi_normal_cholesky_lpdf(ys, mu, L);
    }
    Eigen::VectorXd mu = Eigen::VectorXd::Zero(N);
    return multi_normal_cholesky_lpdf(ys[0], mu, L);
  }
};

/**
 * What the varis of a Stan-codegen GP hold after a top-level lp.grad()
 * (intermediate adjoints and vari identity at the Eigen boundary):
 *   K = gp_exp_quad_cov(x, th0, th1)  (1-D x; rev/mat/fun/gp_exp_quad_cov.hpp:211-244:
 *                                      K(i, j) and K(j, i) one vari)
 *   Kd = add_diag(K, square(th2))      (prim/mat/fun/add_diag.hpp:25-27: K's varis
 *                                      off the diagonal, new ones on it)
 *   L = cholesky_decompose(Kd)         (rev/mat/fun/cholesky_decompose.hpp:378-427:
 *                                      new lower varis, one dummy above)
 *   lp = multi_normal_cholesky_lpdf(y | 0, L)
 * variant 1 adds a host consumer of L (0.25 L(n-1, 0) + 0.5 L(n/2, n/4): the
 * factor's adjoint then has a second writer), variant 2 host consumers of K's
 * shared varis and of add_diag's own (0.5 K(1, 0) + 0.25 K(0, 1) + 0.125 Kd(2, 2)).
 * emit("gpi", lp, [grad th (3) | K(i, j).adj() lower packed | Kd(i, i).adj() |
 *                 L(i, j).adj() lower packed | L(i, j).val() lower packed |
 *                 identity: K symmetric-shared, Kd shares K off the diagonal,
 *                 Kd's diagonal new and distinct, L's strict upper one dummy,
 *                 distinct varis in K, in K and Kd, in L]).
 */
inline void run_gp_intermediate(const std::vector<double>& x, const VD& y, const double* th3, int variant,
                                const emit_fn& emit) {
  using stan::math::add_diag;
  using stan::math::cholesky_decompose;
  using stan::math::gp_exp_quad_cov;
  using stan::math::multi_normal_cholesky_lpdf;
  using stan::math::square;
  const int N = int(x.size());
  VV th(3);
  for (int i = 0; i < 3; ++i) th(i) = th3[i];
  MV K = gp_exp_quad_cov(x, th(0), th(1));
  MV Kd = add_diag(K, square(th(2)));
  // variant 3 (math_amd only: no fixture of its own): one element of Kd
  // replaced by a new vari of the same value, 0.5 (x + x) = x exactly
  if (variant == 3) Kd(N - 1, N / 2) = 0.5 * (Kd(N - 1, N / 2) + Kd(N - 1, N / 2));
  MV L = cholesky_decompose(Kd);
  VD mu = VD::Zero(N);
  var lp = multi_normal_cholesky_lpdf(y, mu, L);
  if (variant == 1) lp = lp + 0.25 * L(N - 1, 0) + 0.5 * L(N / 2, N / 4);
  if (variant == 2) lp = lp + 0.5 * K(1, 0) + 0.25 * K(0, 1) + 0.125 * Kd(2, 2);
  lp.grad();
  std::vector<double> out;
  for (int i = 0; i < 3; ++i) out.push_back(th(i).adj());
  for (int j = 0; j < N; ++j)
    for (int i = j; i < N; ++i) out.push_back(K(i, j).adj());
  for (int i = 0; i < N; ++i) out.push_back(Kd(i, i).adj());
  for (int j = 0; j < N; ++j)
    for (int i = j; i < N; ++i) out.push_back(L(i, j).adj());
  for (int j = 0; j < N; ++j)
    for (int i = j; i < N; ++i) out.push_back(L(i, j).val());
  bool k_sym = true, kd_shares = true, kd_new = true, l_dummy = true;
  std::unordered_set<const void*> sk, skd, sl;
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < N; ++i) {
      k_sym &= K(i, j).vi_ == K(j, i).vi_;
      if (i != j) kd_shares &= Kd(i, j).vi_ == K(i, j).vi_;
      if (i < j) l_dummy &= L(i, j).vi_ == L(0, 1).vi_ && L(i, j).val() == 0.0;
      sk.insert(K(i, j).vi_);
      skd.insert(K(i, j).vi_);
      skd.insert(Kd(i, j).vi_);
      sl.insert(L(i, j).vi_);
    }
  for (int i = 0; i < N; ++i) kd_new &= Kd(i, i).vi_ != K(i, i).vi_;
  out.push_back(k_sym);
  out.push_back(kd_shares);
  out.push_back(kd_new && skd.size() == sk.size() + size_t(N));
  out.push_back(l_dummy);
  out.push_back(double(sk.size()));
  out.push_back(double(skd.size()));
  out.push_back(double(sl.size()));
  emit("gpi", lp.val(), out);
  stan::math::recover_memory();
}

/** Error cases of the new forms: name -> "<kind> <what()>". */
inline void run_error_cases(const std::function<void(const std::string&, const std::function<void()>&)>& expect) {
  using stan::math::add_diag;
  using stan::math::gp_exp_quad_cov;
  using stan::math::multi_normal_cholesky_lpdf;
  using stan::math::multiply;
  const double nan = std::nan("");
  expect("mul_rv_v_sizes", [] {
    RV r(3);
    VV v(2);
    for (int i = 0; i < 3; ++i) r(i) = 1.0;
    for (int i = 0; i < 2; ++i) v(i) = 1.0;
    multiply(r, v);
  });
  expect("mul_m_v_nan", [&] {
    MV A(2, 2);
    VV v(2);
    A << 1, 2, nan, 4;
    v << 1, 1;
    multiply(A, v);
  });
  expect("mul_m_v_nan_b", [&] {
    MD A(2, 2);
    VV v(2);
    A << 1, 2, 3, 4;
    v << 1, nan;
    multiply(A, v);
  });
  expect("ad_vec_size", [] {
    MV S(3, 3);
    VV d(2);
    for (int i = 0; i < 9; ++i) S(i) = double(i);
    d << 1, 2;
    add_diag(S, d);
  });
  expect("mvn_ragged_y", [] {
    std::vector<Eigen::VectorXd> y{Eigen::VectorXd::Zero(2), Eigen::VectorXd::Zero(3)};
    VV mu(2);
    mu << 0, 0;
    MV L(2, 2);
    L << 1, 0, 0, 1;
    multi_normal_cholesky_lpdf(y, mu, L);
  });
  expect("mvn_count_mismatch", [] {
    std::vector<Eigen::VectorXd> y(3, Eigen::VectorXd::Zero(2)), mu(2, Eigen::VectorXd::Zero(2));
    MV L(2, 2);
    L << 1, 0, 0, 1;
    multi_normal_cholesky_lpdf(y, mu, L);
  });
  expect("mvn_arr_nan_mu", [&] {
    std::vector<Eigen::VectorXd> y(2, Eigen::VectorXd::Zero(2));
    VV mu(2);
    mu << 0, nan;
    MV L(2, 2);
    L << 1, 0, 0, 1;
    multi_normal_cholesky_lpdf(y, mu, L);
  });
  expect("gp_nd_nan_x", [&] {
    std::vector<Eigen::VectorXd> x(2, Eigen::VectorXd::Zero(3));
    x[1](2) = nan;
    gp_exp_quad_cov(x, var(1.0), var(1.0));
  });
  expect("gp_nd_ragged_x", [] {
    std::vector<Eigen::VectorXd> x{Eigen::VectorXd::Zero(3), Eigen::VectorXd::Zero(2)};
    gp_exp_quad_cov(x, var(1.0), var(1.0));
  });
  expect("gp_nd_sigma_data", [] {
    std::vector<Eigen::VectorXd> x(2, Eigen::VectorXd::Zero(3));
    gp_exp_quad_cov(x, -1.0, var(1.0));
  });
  expect("mdl_tri_low_not_square", [] {
    MV L(3, 2);
    MV b(3, 1);
    for (int i = 0; i < L.size(); ++i) L(i) = 1.0;
    for (int i = 0; i < b.size(); ++i) b(i) = 1.0;
    stan::math::mdivide_left_tri_low(L, b);
  });
  expect("mdl_tri_low_sizes", [] {
    MV L(3, 3);
    MV b(2, 1);
    for (int i = 0; i < L.size(); ++i) L(i) = 1.0;
    for (int i = 0; i < b.size(); ++i) b(i) = 1.0;
    stan::math::mdivide_left_tri_low(L, b);
  });
  expect("mdl_tri_low_empty_b", [] {
    MV L(3, 3);
    MV b(3, 0);
    for (int i = 0; i < L.size(); ++i) L(i) = 1.0;
    stan::math::mdivide_left_tri_low(L, b);
  });
  expect("mdr_tri_low_sizes", [] {
    MV L(3, 3);
    MV b(1, 2);
    for (int i = 0; i < L.size(); ++i) L(i) = 1.0;
    for (int i = 0; i < b.size(); ++i) b(i) = 1.0;
    stan::math::mdivide_right_tri_low(b, L);
  });
  expect("mul_empty", [] {
    MV A(0, 2);
    MV B(2, 3);
    for (int i = 0; i < B.size(); ++i) B(i) = 1.0;
    multiply(A, B);
  });
}

}  // namespace bnd
#endif
