/*
 * oracle/cpu_ref.cpp — CPU restatement of the reference algorithms
 * (TEST INFRASTRUCTURE ONLY: parity checker + "port" CPU baseline).
 * See cpu_ref.h for the reference file:line each function restates.
 * Pinned against the golden fixtures the real reference produced
 * (tests/golden, oracle/ref_harness.cpp) by tests/test_oracle.py.
 * Build: make -C oracle cpu  ->  oracle/_build/libsmg_oracle.so
 */
#include "cpu_ref.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <vector>

namespace {

const double kPi = 3.14159265358979323846;
const double kNegLogSqrtTwoPi = -std::log(std::sqrt(2.0 * kPi));

// column-major helpers
struct Mat {
  int r, c;
  std::vector<double> v;
  Mat(int r_, int c_) : r(r_), c(c_), v((size_t)r_ * c_, 0.0) {}
  double& operator()(int i, int j) { return v[(size_t)j * r + i]; }
  double operator()(int i, int j) const { return v[(size_t)j * r + i]; }
};

// Solve X * D = Y in place (D lower triangular b x b), Y is m x b.
// == Y <- Y D^{-1}   (cholesky_decompose.hpp:136-139)
void right_solve_lower(const Mat& L, int j0, int b, Mat& A, int r0, int m) {
  // columns of X from last to first: X(:,c) = (Y(:,c) - sum_{t>c} X(:,t) D(t,c)) / D(c,c)
  for (int c = b - 1; c >= 0; --c) {
    for (int i = 0; i < m; ++i) {
      double s = A(r0 + i, j0 + c);
      for (int t = c + 1; t < b; ++t) s -= A(r0 + i, j0 + t) * L(j0 + t, j0 + c);
      A(r0 + i, j0 + c) = s / L(j0 + c, j0 + c);
    }
  }
}

}  // namespace

extern "C" {

void oracle_gp_cov(const double* x, int n, double sigma, double l, double* K) {
  const double s2 = sigma * sigma;
  const double inv_half_sq_l = 0.5 / (l * l);
  for (int j = 0; j < n; ++j) {
    K[(size_t)j * n + j] = s2;
    for (int i = j + 1; i < n; ++i) {
      const double d = x[i] - x[j];
      const double v = s2 * std::exp(-(d * d) * inv_half_sq_l);
      K[(size_t)j * n + i] = v;
      K[(size_t)i * n + j] = v;
    }
  }
}

void oracle_gp_cov_rev(const double* x, int n, double sigma, double l,
                       const double* Kadj, double* adj_sigma, double* adj_l) {
  const double s2 = sigma * sigma;
  const double inv_half_sq_l = 0.5 / (l * l);
  double adjl = 0.0, adjs = 0.0;
  for (int j = 0; j + 1 < n; ++j) {
    for (int i = j + 1; i < n; ++i) {
      const double d = x[i] - x[j];
      const double dist = d * d;
      const double val = s2 * std::exp(-dist * inv_half_sq_l);
      const double adj = Kadj[(size_t)j * n + i] + Kadj[(size_t)i * n + j];
      const double prod = adj * val;
      adjl += prod * dist;
      adjs += prod;
    }
  }
  for (int i = 0; i < n; ++i) adjs += Kadj[(size_t)i * n + i] * s2;
  *adj_l += adjl / (l * l * l);
  *adj_sigma += adjs * 2 / sigma;
}

int oracle_cholesky(const double* A, int n, double* L) {
  std::memset(L, 0, sizeof(double) * (size_t)n * n);
  for (int j = 0; j < n; ++j) {
    double d = A[(size_t)j * n + j];
    for (int k = 0; k < j; ++k) d -= L[(size_t)k * n + j] * L[(size_t)k * n + j];
    if (!(d > 0.0) || !std::isfinite(d)) return 1;
    const double ljj = std::sqrt(d);
    L[(size_t)j * n + j] = ljj;
    for (int i = j + 1; i < n; ++i) {
      double s = A[(size_t)j * n + i];
      for (int k = 0; k < j; ++k) s -= L[(size_t)k * n + i] * L[(size_t)k * n + j];
      L[(size_t)j * n + i] = s / ljj;
    }
  }
  return 0;
}

void oracle_cholesky_rev(const double* Lp, const double* Ladjp, int M,
                         double* Aadj) {
  Mat L(M, M), La(M, M);
  for (int j = 0; j < M; ++j)
    for (int i = j; i < M; ++i) {
      L(i, j) = Lp[(size_t)j * M + i];
      La(i, j) = Ladjp[(size_t)j * M + i];
    }
  if (M <= 35) {
    // cholesky_scalar::chain (Giles), cholesky_decompose.hpp:221-254
    Mat adjA(M, M);
    for (int i = M - 1; i >= 0; --i) {
      for (int j = i; j >= 0; --j) {
        if (i == j) {
          adjA(i, j) = 0.5 * La(i, j) / L(i, j);
        } else {
          adjA(i, j) = La(i, j) / L(j, j);
          La(j, j) -= La(i, j) * L(i, j) / L(j, j);
        }
        for (int k = j - 1; k >= 0; --k) {
          La(i, k) -= adjA(i, j) * L(j, k);
          La(j, k) -= adjA(i, j) * L(i, k);
        }
        Aadj[(size_t)j * M + i] += adjA(i, j);
      }
    }
    return;
  }
  // cholesky_block::chain (Murray 2016), cholesky_decompose.hpp:118-165
  int bs = std::min(std::max(M / 8, 8), 128);
  for (int k = M; k > 0; k -= bs) {
    const int j = std::max(0, k - bs);
    const int b = k - j, m = M - k;
    if (m > 0) {
      right_solve_lower(L, j, b, La, k, m);  // C_adj = C_adj D^{-1}
      // B_adj -= C_adj * R   (m x j) -= (m x b)(b x j)
      for (int c = 0; c < j; ++c)
        for (int i = 0; i < m; ++i) {
          double s = 0;
          for (int t = 0; t < b; ++t) s += La(k + i, j + t) * L(j + t, c);
          La(k + i, c) -= s;
        }
      // D_adj -= C_adj^T * C   (b x b) -= (b x m)(m x b)
      for (int c = 0; c < b; ++c)
        for (int r = 0; r < b; ++r) {
          double s = 0;
          for (int t = 0; t < m; ++t) s += La(k + t, j + r) * L(k + t, j + c);
          La(j + r, j + c) -= s;
        }
    }
    // symbolic_rev(D, D_adj), cholesky_decompose.hpp:101-111:
    //   S = D^T tril(D_adj); mirror lower->upper; S = D^-T S D^-1
    Mat S(b, b);
    for (int c = 0; c < b; ++c)
      for (int r = 0; r < b; ++r) {
        double s = 0;  // (D^T)(r,t) = D(t,r), nonzero for t >= r; tril(Dadj)(t,c) nonzero for t >= c
        for (int t = std::max(r, c); t < b; ++t) s += L(j + t, j + r) * La(j + t, j + c);
        S(r, c) = s;
      }
    for (int c = 0; c < b; ++c)
      for (int r = 0; r < c; ++r) S(r, c) = S(c, r);
    // S <- D^{-T} S  (upper-triangular solve, Lt = D^T)
    for (int c = 0; c < b; ++c)
      for (int r = b - 1; r >= 0; --r) {
        double s = S(r, c);
        for (int t = r + 1; t < b; ++t) s -= L(j + t, j + r) * S(t, c);
        S(r, c) = s / L(j + r, j + r);
      }
    // S <- S D^{-1}
    for (int c = b - 1; c >= 0; --c)
      for (int r = 0; r < b; ++r) {
        double s = S(r, c);
        for (int t = c + 1; t < b; ++t) s -= S(r, t) * L(j + t, j + c);
        S(r, c) = s / L(j + c, j + c);
      }
    // R_adj -= C_adj^T B ; R_adj -= sym_lower(D_adj) R
    for (int c = 0; c < j; ++c)
      for (int r = 0; r < b; ++r) {
        double s = 0;
        for (int t = 0; t < m; ++t) s += La(k + t, j + r) * L(k + t, c);
        double s2 = 0;
        for (int t = 0; t < b; ++t) {
          const double dsym = (t <= r) ? S(r, t) : S(t, r);
          s2 += dsym * L(j + t, c);
        }
        La(j + r, c) -= s + s2;
      }
    for (int c = 0; c < b; ++c)
      for (int r = 0; r < b; ++r)
        La(j + r, j + c) = (r > c) ? S(r, c) : (r == c ? 0.5 * S(r, c) : 0.0);
  }
  for (int j = 0; j < M; ++j)
    for (int i = j; i < M; ++i) Aadj[(size_t)j * M + i] += La(i, j);
}

void oracle_mvn_cholesky(const double* y, const double* mu, const double* Lp,
                         int n, double* lp, double* gy, double* gmu,
                         double* gL) {
  // inv_L = mdivide_left_tri<Lower>(L): explicit inverse (:117-118)
  Mat inv(n, n);
  for (int c = 0; c < n; ++c)
    for (int r = c; r < n; ++r) {
      double s = (r == c) ? 1.0 : 0.0;
      for (int t = c; t < r; ++t) s -= Lp[(size_t)t * n + r] * inv(t, c);
      inv(r, c) = s / Lp[(size_t)r * n + r];
    }
  std::vector<double> d(n), half(n, 0.0), sd(n, 0.0);
  for (int i = 0; i < n; ++i) d[i] = y[i] - mu[i];
  for (int r = 0; r < n; ++r) {
    double s = 0;
    for (int t = 0; t <= r; ++t) s += inv(r, t) * d[t];
    half[r] = s;
  }
  for (int c = 0; c < n; ++c) {
    double s = 0;
    for (int t = c; t < n; ++t) s += half[t] * inv(t, c);
    sd[c] = s;
  }
  double logp = kNegLogSqrtTwoPi * n;
  double dot = 0;
  for (int i = 0; i < n; ++i) dot += half[i] * half[i];
  logp -= 0.5 * dot;
  double ld = 0;
  for (int i = 0; i < n; ++i) ld += std::log(inv(i, i));
  logp += ld;
  *lp = logp;
  for (int i = 0; i < n; ++i) {
    if (gy) gy[i] = -sd[i];
    if (gmu) gmu[i] = sd[i];
  }
  if (gL)
    for (int c = 0; c < n; ++c)
      for (int r = 0; r < n; ++r)
        gL[(size_t)c * n + r] = sd[r] * half[c] - inv(c, r);
}

void oracle_multiply(const double* A, const double* B, int m, int k, int n,
                     double* C) {
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < m; ++i) {
      double s = 0;
      for (int t = 0; t < k; ++t) s += A[(size_t)t * m + i] * B[(size_t)j * k + t];
      C[(size_t)j * m + i] = s;
    }
}

void oracle_multiply_rev(const double* A, const double* B, const double* Cadj,
                         int m, int k, int n, double* Aadj, double* Badj) {
  if (Aadj)
    for (int t = 0; t < k; ++t)
      for (int i = 0; i < m; ++i) {
        double s = 0;
        for (int j = 0; j < n; ++j) s += Cadj[(size_t)j * m + i] * B[(size_t)j * k + t];
        Aadj[(size_t)t * m + i] += s;
      }
  if (Badj)
    for (int j = 0; j < n; ++j)
      for (int t = 0; t < k; ++t) {
        double s = 0;
        for (int i = 0; i < m; ++i) s += A[(size_t)t * m + i] * Cadj[(size_t)j * m + i];
        Badj[(size_t)j * k + t] += s;
      }
}

static inline double tri(int lower, const double* A, int m, int i, int j) {
  const bool in = lower ? (i >= j) : (i <= j);
  return in ? A[(size_t)j * m + i] : 0.0;
}

void oracle_mdivide_left_tri(int lower, const double* A, const double* B,
                             int m, int n, double* C) {
  for (int c = 0; c < n; ++c) {
    if (lower) {
      for (int r = 0; r < m; ++r) {
        double s = B[(size_t)c * m + r];
        for (int t = 0; t < r; ++t) s -= tri(1, A, m, r, t) * C[(size_t)c * m + t];
        C[(size_t)c * m + r] = s / tri(1, A, m, r, r);
      }
    } else {
      for (int r = m - 1; r >= 0; --r) {
        double s = B[(size_t)c * m + r];
        for (int t = r + 1; t < m; ++t) s -= tri(0, A, m, r, t) * C[(size_t)c * m + t];
        C[(size_t)c * m + r] = s / tri(0, A, m, r, r);
      }
    }
  }
}

void oracle_mdivide_left_tri_rev(int lower, const double* A, const double* C,
                                 const double* Cadj, int m, int n,
                                 double* Aadj, double* Badj) {
  // adjB = tri(A)^{-T} Cadj  (transpose flips the triangle)
  std::vector<double> adjB((size_t)m * n);
  for (int c = 0; c < n; ++c) {
    if (lower) {  // A^T upper: back substitution
      for (int r = m - 1; r >= 0; --r) {
        double s = Cadj[(size_t)c * m + r];
        for (int t = r + 1; t < m; ++t) s -= tri(1, A, m, t, r) * adjB[(size_t)c * m + t];
        adjB[(size_t)c * m + r] = s / tri(1, A, m, r, r);
      }
    } else {
      for (int r = 0; r < m; ++r) {
        double s = Cadj[(size_t)c * m + r];
        for (int t = 0; t < r; ++t) s -= tri(0, A, m, t, r) * adjB[(size_t)c * m + t];
        adjB[(size_t)c * m + r] = s / tri(0, A, m, r, r);
      }
    }
  }
  if (Aadj)
    for (int j = 0; j < m; ++j)
      for (int i = 0; i < m; ++i) {
        if (lower ? (i < j) : (i > j)) continue;
        double s = 0;
        for (int c = 0; c < n; ++c) s += adjB[(size_t)c * m + i] * C[(size_t)c * m + j];
        Aadj[(size_t)j * m + i] -= s;
      }
  if (Badj)
    for (size_t i = 0; i < (size_t)m * n; ++i) Badj[i] += adjB[i];
}

double oracle_log_sum_exp(const double* x, int n) {
  if (n == 0) return -std::numeric_limits<double>::infinity();
  double mx = x[0];
  for (int i = 1; i < n; ++i) mx = std::max(mx, x[i]);
  if (!std::isfinite(mx)) return mx;
  double s = 0;
  for (int i = 0; i < n; ++i) s += std::exp(x[i] - mx);
  return mx + std::log(s);
}

void oracle_log_sum_exp_rev(const double* x, int n, double lse, double adj,
                            double* xadj) {
  for (int i = 0; i < n; ++i) xadj[i] += adj * std::exp(x[i] - lse);
}

double oracle_lgamma(double x) {
  int sign;
  return ::lgamma_r(x, &sign);
}

// Boost 1.69 digamma, 53-bit tag (boost/math/special_functions/digamma.hpp)
static double digamma_large(double x) {  // :108-128, x >= 10
  static const double P[] = {0.083333333333333333333333333333333333333333333333333,
                             -0.0083333333333333333333333333333333333333333333333333,
                             0.003968253968253968253968253968253968253968253968254,
                             -0.0041666666666666666666666666666666666666666666666667,
                             0.0075757575757575757575757575757575757575757575757576,
                             -0.021092796092796092796092796092796092796092796092796,
                             0.083333333333333333333333333333333333333333333333333,
                             -0.44325980392156862745098039215686274509803921568627};
  x -= 1;
  double result = std::log(x);
  result += 1 / (2 * x);
  const double z = 1 / (x * x);
  double p = P[7];
  for (int i = 6; i >= 0; --i) p = p * z + P[i];
  result -= z * p;
  return result;
}
static double digamma_1_2(double x) {  // :300-347
  const float Y = 0.99558162689208984F;
  const double root1 = 1569415565.0 / 1073741824.0;
  const double root2 = (381566830.0 / 1073741824.0) / 1073741824.0;
  const double root3 = 0.9016312093258695918615325266959189453125e-19;
  static const double P[] = {0.25479851061131551, -0.32555031186804491,
                             -0.65031853770896507, -0.28919126444774784,
                             -0.045251321448739056, -0.0020713321167745952};
  static const double Q[] = {1.0, 2.0767117023730469, 1.4606242909763515,
                             0.43593529692665969, 0.054151797245674225,
                             0.0021284987017821144, -0.55789841321675513e-6};
  double g = x - root1;
  g -= root2;
  g -= root3;
  const double t = x - 1;
  double p = P[5], q = Q[6];
  for (int i = 4; i >= 0; --i) p = p * t + P[i];
  for (int i = 5; i >= 0; --i) q = q * t + Q[i];
  const double r = p / q;
  return g * Y + g * r;
}
double oracle_digamma(double x) {  // :381-449, pole -> NaN (errno_on_error)
  double result = 0;
  if (x <= -1) {
    x = 1 - x;
    double rem = x - std::floor(x);
    if (rem > 0.5) rem -= 1;
    if (rem == 0) return std::numeric_limits<double>::quiet_NaN();
    result = kPi / std::tan(kPi * rem);
  }
  if (x == 0) return std::numeric_limits<double>::quiet_NaN();
  if (x >= 10) {
    result += digamma_large(x);
  } else {
    while (x > 2) {
      x -= 1;
      result += 1 / x;
    }
    while (x < 1) {
      result -= 1 / x;
      x += 1;
    }
    result += digamma_1_2(x);
  }
  return result;
}

double oracle_trigamma(double x) {  // prim/scal/fun/trigamma.hpp:33-80
  const double small = 0.0001, large = 5.0;
  const double b2 = 1.0 / 6.0, b4 = -1.0 / 30.0, b6 = 1.0 / 42.0, b8 = -1.0 / 30.0;
  if (x <= 0.0 && std::floor(x) == x) return std::numeric_limits<double>::infinity();
  if (x <= 0 && std::floor(x) != x) {
    const double s = kPi / std::sin(-kPi * x);
    return -oracle_trigamma(-x + 1.0) + s * s;
  }
  if (x <= small) return 1.0 / (x * x);
  double z = x, value = 0.0;
  while (z < large) {
    value += 1.0 / (z * z);
    z += 1.0;
  }
  const double y = 1.0 / (z * z);
  value += 0.5 * y + (1.0 + y * (b2 + y * (b4 + y * (b6 + y * b8)))) / z;
  return value;
}

double oracle_normal_lpdf(const double* y, int sy, const double* mu, int smu,
                          const double* sigma, int ssig, int n, double* gy,
                          double* gmu, double* gsigma) {
  double logp = 0;
  for (int i = 0; i < n; ++i) {
    const double s = sigma[i * ssig];
    const double inv_s = 1.0 / s;
    const double z = (y[i * sy] - mu[i * smu]) * inv_s;
    const double z2 = z * z;
    logp += kNegLogSqrtTwoPi;
    logp -= std::log(s);
    logp += -0.5 * z2;
    const double sc = inv_s * z;
    if (gy) gy[i] -= sc;
    if (gmu) gmu[i] += sc;
    if (gsigma) gsigma[i] += -inv_s + inv_s * z2;
  }
  return logp;
}

double oracle_glm(const int* y, const double* x, long long R, int M,
                  double alpha, const double* beta, double* galpha,
                  double* gbeta) {
  std::vector<double> eta((size_t)R, 0.0);
  for (int j = 0; j < M; ++j) {
    const double b = beta[j];
    const double* col = x + (size_t)j * R;
    for (long long i = 0; i < R; ++i) eta[i] += col[i] * b;
  }
  const double cutoff = 20.0;
  double logp = 0, ga = 0;
  std::vector<double> td((size_t)R);
  for (long long i = 0; i < R; ++i) {
    const double sgn = 2.0 * y[i] - 1.0;
    const double yt = sgn * (eta[i] + alpha);
    const double e = std::exp(-yt);
    logp += yt > cutoff ? -e : (yt < -cutoff ? yt : -std::log1p(e));
    td[i] = yt > cutoff ? -e : (yt < -cutoff ? sgn : sgn * e / (e + 1));
    ga += td[i];
  }
  if (galpha) *galpha = ga;
  if (gbeta)
    for (int j = 0; j < M; ++j) {
      const double* col = x + (size_t)j * R;
      double s = 0;
      for (long long i = 0; i < R; ++i) s += col[i] * td[i];
      gbeta[j] = s;
    }
  return logp;
}

// x beta over the rows (column by column, like Eigen's col-major GEMV)
static std::vector<double> glm_eta(const double* x, long long R, int M, const double* beta) {
  std::vector<double> eta((size_t)R, 0.0);
  for (int j = 0; j < M; ++j) {
    const double b = beta[j];
    const double* col = x + (size_t)j * R;
    for (long long i = 0; i < R; ++i) eta[i] += col[i] * b;
  }
  return eta;
}

// g[1 + j] = x_j . d
static void glm_xt(const double* x, long long R, int M, const double* d, double* g) {
  for (int j = 0; j < M; ++j) {
    const double* col = x + (size_t)j * R;
    double s = 0;
    for (long long i = 0; i < R; ++i) s += col[i] * d[i];
    g[1 + j] = s;
  }
}

double oracle_normal_id_glm(const double* y, const double* x, long long R, int M,
                            double alpha, const double* beta, double sigma, double* g) {
  // normal_id_glm_lpdf.hpp:84-86: y_scaled = (y - x beta - alpha) * inv_sigma
  const double inv_sigma = 1.0 / sigma;
  std::vector<double> ys = glm_eta(x, R, M, beta), mu((size_t)R);
  double sq = 0, sa = 0;
  for (long long i = 0; i < R; ++i) {
    ys[i] = (y[i] - ys[i] - alpha) * inv_sigma;
    mu[i] = inv_sigma * ys[i];  // :92 mu_derivative
    sq += ys[i] * ys[i];
    sa += mu[i];
  }
  if (g) {
    g[0] = sa;                                // :104-109 alpha
    glm_xt(x, R, M, mu.data(), g);            // :101-103 beta
    g[M + 1] = (sq - (double)R) * inv_sigma;  // :116-118 sigma
  }
  // :131-142
  const double NEG_LOG_SQRT_TWO_PI = -0.91893853320467274178;
  return NEG_LOG_SQRT_TWO_PI * (double)R - (double)R * std::log(sigma) - 0.5 * sq;
}

double oracle_poisson_log_glm(const int* y, const double* x, long long R, int M,
                              double alpha, const double* beta, double* g) {
  // poisson_log_glm_lpmf.hpp:81-106
  std::vector<double> th = glm_eta(x, R, M, beta), d((size_t)R);
  double sd = 0, lg = 0, s2 = 0;
  for (long long i = 0; i < R; ++i) {
    th[i] += alpha;
    const double e = std::exp(th[i]);
    d[i] = y[i] - e;
    sd += d[i];
    lg += std::lgamma(y[i] + 1.0);
    s2 += y[i] * th[i] - e;
  }
  if (g) {
    g[0] = sd;
    glm_xt(x, R, M, d.data(), g);
  }
  return -lg + s2;
}

double oracle_categorical_logit_glm(const int* y, const double* x, long long R, int M, int C,
                                    const double* alpha, const double* beta, double* g) {
  // categorical_logit_glm_lpmf.hpp:84-183 (x an R x M matrix, beta M x C):
  // lin = x beta + alpha; logp = sum log(1 / sum exp(lin - max)) - sum max
  // + sum lin(i, y_i - 1); alpha' = colsum(-softmax) + counts; beta' = x^T (-softmax)
  // + the one-hot rows of x
  if (R == 0 || C == 1) {
    if (g)
      for (long long e = 0; e < C + (long long)M * C; ++e) g[e] = 0.0;
    return 0.0;
  }
  std::vector<double> lin((size_t)C);
  double lsum = 0, msum = 0, ysum = 0;
  if (g)
    for (long long e = 0; e < C + (long long)M * C; ++e) g[e] = 0.0;
  for (long long i = 0; i < R; ++i) {
    for (int c = 0; c < C; ++c) {
      double s = 0;
      for (int m = 0; m < M; ++m) s += x[i + (size_t)m * R] * beta[m + (size_t)c * M];
      lin[c] = s + alpha[c];
    }
    double mx = lin[0];
    for (int c = 1; c < C; ++c) mx = std::max(mx, lin[c]);
    double se = 0;
    for (int c = 0; c < C; ++c) se += std::exp(lin[c] - mx);
    const double inv = 1.0 / se;
    lsum += std::log(inv);
    msum += mx;
    ysum += lin[y[i] - 1];
    if (g)
      for (int c = 0; c < C; ++c) {
        const double d = (c == y[i] - 1 ? 1.0 : 0.0) - std::exp(lin[c] - mx) * inv;
        g[c] += d;
        for (int m = 0; m < M; ++m) g[C + m + (size_t)c * M] += x[i + (size_t)m * R] * d;
      }
  }
  return lsum - msum + ysum;
}

// X (n x k) <- A^{-1} X through L = chol(A): forward then backward substitution
static void spd_solve(const double* L, int n, double* X, int k) {
  for (int c = 0; c < k; ++c) {
    double* x = X + (size_t)c * n;
    for (int i = 0; i < n; ++i) {
      double s = x[i];
      for (int j = 0; j < i; ++j) s -= L[i + (size_t)j * n] * x[j];
      x[i] = s / L[i + (size_t)i * n];
    }
    for (int i = n - 1; i >= 0; --i) {
      double s = x[i];
      for (int j = i + 1; j < n; ++j) s -= L[j + (size_t)i * n] * x[j];
      x[i] = s / L[i + (size_t)i * n];
    }
  }
}

int oracle_mdivide_left_spd(const double* A, const double* B, int n, int k, const double* W,
                            double* fx, double* gA, double* gB) {
  std::vector<double> L((size_t)n * n);
  if (oracle_cholesky(A, n, L.data()) != 0) return -1;
  std::vector<double> C(B, B + (size_t)n * k), Wa(W, W + (size_t)n * k);
  spd_solve(L.data(), n, C.data(), k);  // C = A^{-1} B (:57-62)
  double f = 0;
  for (size_t e = 0; e < (size_t)n * k; ++e) f += W[e] * C[e];
  *fx = f;
  spd_solve(L.data(), n, Wa.data(), k);  // adjB = A^{-1} Cadj (:95-96)
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) {
      double s = 0;
      for (int c = 0; c < k; ++c) s += Wa[i + (size_t)c * n] * C[j + (size_t)c * n];
      gA[i + (size_t)j * n] = -s;  // Aadj -= adjB C^T (:97-98)
    }
  for (size_t e = 0; e < (size_t)n * k; ++e) gB[e] = Wa[e];
  return 0;
}

int oracle_log_determinant_spd(const double* A, int n, double* fx, double* gA) {
  std::vector<double> L((size_t)n * n);
  if (oracle_cholesky(A, n, L.data()) != 0) return -1;
  double s = 0;
  for (int i = 0; i < n; ++i) s += std::log(L[i + (size_t)i * n]);
  *fx = 2 * s;
  std::fill(gA, gA + (size_t)n * n, 0.0);
  for (int i = 0; i < n; ++i) gA[i + (size_t)i * n] = 1.0;
  spd_solve(L.data(), n, gA, n);  // A^{-1} (:46-53)
  return 0;
}

void oracle_mlt_self_transpose(const double* L, int K, int J, const double* W, double* fx,
                               double* gL) {
  auto T = [&](int i, int j) { return i >= j ? L[i + (size_t)j * K] : 0.0; };
  double f = 0;
  for (int m = 0; m < K; ++m)
    for (int q = 0; q < K; ++q) {
      double c = 0;
      for (int j = 0; j < J; ++j) c += T(m, j) * T(q, j);
      f += W[m + (size_t)q * K] * c;
    }
  *fx = f;
  for (int j = 0; j < J; ++j)
    for (int i = 0; i < K; ++i) {
      double s = 0;
      if (i >= j)
        for (int q = 0; q < K; ++q) s += (W[i + (size_t)q * K] + W[q + (size_t)i * K]) * T(q, j);
      gL[i + (size_t)j * K] = s;
    }
}

void oracle_quad_form_sym(const double* A, const double* B, int M, int N, const double* Win,
                          int sym, double* fx, double* gA, double* gB) {
  // sym: both operands var -> the prim template autodiffs 0.5 (Cd + Cd^T), so
  // the adjoint reaching Cd is sym(W) (prim/mat/fun/quad_form_sym.hpp:11-18)
  std::vector<double> Ws(Win, Win + (size_t)N * N);
  if (sym)
    for (int c = 0; c < N; ++c)
      for (int r = 0; r < N; ++r) Ws[r + (size_t)c * N] = 0.5 * (Win[r + (size_t)c * N] + Win[c + (size_t)r * N]);
  const double* W = Ws.data();
  std::vector<double> AB((size_t)M * N, 0.0), Cd((size_t)N * N, 0.0);
  for (int c = 0; c < N; ++c)
    for (int k2 = 0; k2 < M; ++k2)
      for (int i = 0; i < M; ++i) AB[i + (size_t)c * M] += A[i + (size_t)k2 * M] * B[k2 + (size_t)c * M];
  for (int c = 0; c < N; ++c)
    for (int r = 0; r < N; ++r) {
      double s = 0;
      for (int i = 0; i < M; ++i) s += B[i + (size_t)r * M] * AB[i + (size_t)c * M];
      Cd[r + (size_t)c * N] = s;
    }
  double f = 0;
  for (int c = 0; c < N; ++c)
    for (int r = 0; r < N; ++r)
      f += Win[r + (size_t)c * N] * 0.5 * (Cd[r + (size_t)c * N] + Cd[c + (size_t)r * N]);
  *fx = f;
  // Aadj = B W B^T ; Badj = A B W^T + A^T B W  (quad_form.hpp chainA / chainB)
  std::vector<double> BW((size_t)M * N, 0.0), BWt((size_t)M * N, 0.0);
  for (int c = 0; c < N; ++c)
    for (int q = 0; q < N; ++q)
      for (int i = 0; i < M; ++i) {
        BW[i + (size_t)c * M] += B[i + (size_t)q * M] * W[q + (size_t)c * N];
        BWt[i + (size_t)c * M] += B[i + (size_t)q * M] * W[c + (size_t)q * N];
      }
  for (int j = 0; j < M; ++j)
    for (int i = 0; i < M; ++i) {
      double s = 0;
      for (int c = 0; c < N; ++c) s += BW[i + (size_t)c * M] * B[j + (size_t)c * M];
      gA[i + (size_t)j * M] = s;
    }
  for (int c = 0; c < N; ++c)
    for (int i = 0; i < M; ++i) {
      double s = 0;
      for (int k2 = 0; k2 < M; ++k2)
        s += A[i + (size_t)k2 * M] * BWt[k2 + (size_t)c * M] + A[k2 + (size_t)i * M] * BW[k2 + (size_t)c * M];
      gB[i + (size_t)c * M] = s;
    }
}

void oracle_gp_marginal(const double* x, const double* y, int n,
                        const double* theta, double* fx, double* grad) {
  const double alpha = theta[0], rho = theta[1], sigma = theta[2];
  const size_t nn = (size_t)n * n;
  std::vector<double> K(nn), L(nn), Ladj(nn, 0.0), Aadj(nn, 0.0), gL(nn);
  std::vector<double> mu(n, 0.0);
  oracle_gp_cov(x, n, alpha, rho, K.data());
  const double s2 = sigma * sigma;
  for (int i = 0; i < n; ++i) K[(size_t)i * n + i] += s2;  // add_diag
  oracle_cholesky(K.data(), n, L.data());
  double lp;
  oracle_mvn_cholesky(y, mu.data(), L.data(), n, &lp, nullptr, nullptr, gL.data());
  *fx = lp;
  // only the lower triangle of L carries vars (upper = dummy vari)
  for (int j = 0; j < n; ++j)
    for (int i = j; i < n; ++i) Ladj[(size_t)j * n + i] = gL[(size_t)j * n + i];
  oracle_cholesky_rev(L.data(), Ladj.data(), n, Aadj.data());
  // add_diag: the diagonal varis are K_ii + s2; s2 = square(sigma)
  double adj_s2 = 0;
  for (int i = 0; i < n; ++i) adj_s2 += Aadj[(size_t)i * n + i];
  double ga = 0, gr = 0;
  oracle_gp_cov_rev(x, n, alpha, rho, Aadj.data(), &ga, &gr);
  grad[0] = ga;
  grad[1] = gr;
  grad[2] = adj_s2 * 2 * sigma;
}

void oracle_mulchol(const double* A, int n, double* fx, double* grad) {
  const size_t nn = (size_t)n * n;
  std::vector<double> At(nn), C(nn), L(nn), Ladj(nn, 0.0), Cadj(nn, 0.0);
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) At[(size_t)i * n + j] = A[(size_t)j * n + i];
  oracle_multiply(A, At.data(), n, n, n, C.data());
  for (int i = 0; i < n; ++i) C[(size_t)i * n + i] += n;
  oracle_cholesky(C.data(), n, L.data());
  double s = 0;
  for (size_t i = 0; i < nn; ++i) s += L[i];
  *fx = s;
  for (int j = 0; j < n; ++j)
    for (int i = j; i < n; ++i) Ladj[(size_t)j * n + i] = 1.0;
  oracle_cholesky_rev(L.data(), Ladj.data(), n, Cadj.data());
  // multiply(A, B = A^T): Aadj += Cadj B^T, Badj += A^T Cadj, B's varis are A's
  std::vector<double> gA(nn, 0.0), gB(nn, 0.0);
  oracle_multiply_rev(A, At.data(), Cadj.data(), n, n, n, gA.data(), gB.data());
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i)
      grad[(size_t)j * n + i] = gA[(size_t)j * n + i] + gB[(size_t)i * n + j];
}

}  // extern "C"
