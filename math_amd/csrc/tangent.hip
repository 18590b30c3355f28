// Tangent (fvar<var>) pieces for the fwd-over-rev functors of
// include/stan/math/mix/fvar_functors.hpp:
//
//   copy_tril           Y(lower) = X(lower) (the Murray reverse's work copy of
//                       a Cholesky factor's adjoint: its strict upper is never read)
//   add_tril            Y(lower) += alpha X(lower): tril() of a tangent
//                       (fwd/mat/fun/mdivide_left_tri_low.hpp:28-33 reads only
//                       A's lower triangle)
//   lse_tangent         t = sum_i softmax(x)_i x'_i, the tangent of
//                       log_sum_exp (fwd/mat/fun/log_sum_exp.hpp), and its
//                       reverse into x and x'
//   glm_tangent         t = sum_i d_i (eta'_i + alpha'), d_i = d logp_i /
//                       d theta_i of bernoulli_logit_glm_lpmf with the
//                       reference's cutoff branches
//                       (prim/mat/prob/bernoulli_logit_glm_lpmf.hpp:95-113),
//                       theta = eta + alpha, and its reverse
//
// The reductions run in ONE 1024-thread workgroup in a fixed order (these
// nodes live on Hessian sweeps over modest sizes; the results are bitwise
// reproducible).
#include "smg_internal.h"

namespace {

constexpr int TT = 1024;

// block-wide sum of v (fixed order: waves' partials summed in wave order)
__device__ double block_sum(double v, double* sh) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0)
    for (int q = 0; q < TT / 64; ++q) s += sh[q];
  __syncthreads();
  if (threadIdx.x == 0) sh[0] = s;
  __syncthreads();
  const double r = sh[0];
  __syncthreads();
  return r;
}

__device__ double block_max(double v, double* sh) {
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_down(v, off));
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double m = sh[0];
    for (int q = 1; q < TT / 64; ++q) m = fmax(m, sh[q]);
    sh[0] = m;
  }
  __syncthreads();
  const double r = sh[0];
  __syncthreads();
  return r;
}

__global__ void k_add_tril(int m, int n, double alpha, const double* __restrict__ X, int ldx, double* __restrict__ Y,
                           int ldy) {
  for (smg_mn it(m, n); it.ok(); it.next())
    if (it.i >= it.j) Y[it.i + (size_t)it.j * ldy] += alpha * X[it.i + (size_t)it.j * ldx];
}

// Y = tril(X): the strict upper triangle of Y is written with zeros (Y is a
// fresh arena buffer whose upper half the Murray reverse reads as stored
// zeros of the work matrix; recycled arena memory may hold NaN / Inf there)
__global__ void k_copy_tril(int m, int n, const double* __restrict__ X, int ldx, double* __restrict__ Y, int ldy) {
  for (smg_mn it(m, n); it.ok(); it.next())
    Y[it.i + (size_t)it.j * ldy] = it.i >= it.j ? X[it.i + (size_t)it.j * ldx] : 0.0;
}

// k_copy_tril over whole columns with 16-byte accesses (even ld, 16-byte
// aligned): row pairs above the diagonal are stored as zeros without a read
__global__ __launch_bounds__(256) void k_copy_tril_col2(int m, int n, const double* __restrict__ X,
                                                        int ldx, double* __restrict__ Y, int ldy) {
  const int mp = m >> 1;
  for (int j = blockIdx.x; j < n; j += gridDim.x) {
    const double2* x = reinterpret_cast<const double2*>(X + (size_t)j * ldx);
    double2* y = reinterpret_cast<double2*>(Y + (size_t)j * ldy);
    const int pz = j >> 1;  // pairs p < pz lie wholly above the diagonal
    for (int p = threadIdx.x; p < (pz < mp ? pz : mp); p += 256) y[p] = make_double2(0.0, 0.0);
    for (int p0 = pz + threadIdx.x; p0 < mp; p0 += 4 * 256) {
      double2 a[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int p = p0 + 256 * k;
        if (p < mp) a[k] = x[p];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int p = p0 + 256 * k;
        if (p < mp) {
          if (2 * p < j) a[k].x = 0.0;  // the pair straddles the diagonal: row 2p + 1 == j only
          y[p] = a[k];
        }
      }
    }
  }
}

// out = [lse(x), sum_i exp(x_i - lse) x'_i]
__global__ __launch_bounds__(TT) void k_lse_tangent_fwd(const double* __restrict__ x, const double* __restrict__ xd,
                                                       long long n, double* __restrict__ out) {
  __shared__ double sh[TT / 64];
  double m = -INFINITY;
  for (long long i = threadIdx.x; i < n; i += TT) m = fmax(m, x[i]);
  m = block_max(m, sh);
  double s = 0.0, u = 0.0;
  if (m > -INFINITY)
    for (long long i = threadIdx.x; i < n; i += TT) {
      const double e = exp(x[i] - m);
      s += e;
      u += e * xd[i];
    }
  s = block_sum(s, sh);
  u = block_sum(u, sh);
  if (threadIdx.x == 0) {
    out[0] = m > -INFINITY ? m + log(s) : -INFINITY;
    out[1] = m > -INFINITY ? u / s : 0.0;
  }
}

// p_i = exp(x_i - lse): xadj += adj p (x' - t), xdadj += adj p
__global__ void k_lse_tangent_rev(const double* __restrict__ x, const double* __restrict__ xd, long long n, double lse,
                                  double t, double adj, double* __restrict__ xa, double* __restrict__ xda) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const double p = exp(x[i] - lse);
    if (xa) xa[i] += adj * p * (xd[i] - t);
    if (xda) xda[i] += adj * p;
  }
}

// The reference's theta_derivative d of one bernoulli logit term (y in
// {0, 1}, s = 2y - 1, e = exp(-s theta); cutoff 20,
// prim/mat/prob/bernoulli_logit_glm_lpmf.hpp:117-123) and dd = d d / d theta
// of that expression as written (the reference's tangent is sum_i d_i
// (eta'_i + alpha') with d a var: its reverse differentiates d itself):
//   s theta > 20 : d = -e           dd = s e
//   s theta < -20: d = s            dd = 0
//   else         : d = s e/(1+e)    dd = -e/(1+e)^2
__device__ __forceinline__ void glm_term(int y, double theta, double& d, double& dd) {
  const double s = 2.0 * y - 1.0;
  const double yt = s * theta;
  const double e = exp(-yt);
  if (yt > 20.0) {
    d = -e;
    dd = s * e;
  } else if (yt < -20.0) {
    d = s;
    dd = 0.0;
  } else {
    const double q = 1.0 / (1.0 + e);
    d = s * e * q;
    dd = -e * q * q;
  }
}

__global__ __launch_bounds__(TT) void k_glm_tangent_fwd(const double* __restrict__ eta, double alpha,
                                                       const double* __restrict__ etad, double alphad,
                                                       const int* __restrict__ y, long long n, double* __restrict__ out) {
  __shared__ double sh[TT / 64];
  double t = 0.0;
  for (long long i = threadIdx.x; i < n; i += TT) {
    double d, dd;
    glm_term(y[i], eta[i] + alpha, d, dd);
    t += d * (etad[i] + alphad);
  }
  t = block_sum(t, sh);
  if (threadIdx.x == 0) out[0] = t;
}

// eta_adj += adj d'(theta) (eta' + alpha'), etad_adj += adj d(theta);
// out = [sum of the first (alpha's adjoint), sum of the second (alpha''s)]
__global__ __launch_bounds__(TT) void k_glm_tangent_rev(const double* __restrict__ eta, double alpha,
                                                       const double* __restrict__ etad, double alphad,
                                                       const int* __restrict__ y, long long n, double adj,
                                                       double* __restrict__ eta_adj, double* __restrict__ etad_adj,
                                                       double* __restrict__ out) {
  __shared__ double sh[TT / 64];
  double sa = 0.0, sd = 0.0;
  for (long long i = threadIdx.x; i < n; i += TT) {
    double d, dd;
    glm_term(y[i], eta[i] + alpha, d, dd);
    const double ga = adj * dd * (etad[i] + alphad), gd = adj * d;
    if (eta_adj) eta_adj[i] += ga;
    if (etad_adj) etad_adj[i] += gd;
    sa += ga;
    sd += gd;
  }
  sa = block_sum(sa, sh);
  sd = block_sum(sd, sh);
  if (threadIdx.x == 0) {
    out[0] = sa;
    out[1] = sd;
  }
}

inline int grid_for(long long tot) {
  long long g = (tot + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

extern "C" {

int smg_add_tril(smg_ctx* ctx, int m, int n, double alpha, const double* X, int ldx, double* Y, int ldy) {
  if (!ctx || m < 0 || n < 0) return SMG_ERR_ARG;
  if (m == 0 || n == 0) return SMG_OK;
  if (!X || !Y || ldx < m || ldy < m) return SMG_ERR_ARG;
  hipLaunchKernelGGL(k_add_tril, dim3(grid_for((long long)m * n)), dim3(256), 0, ctx->stream, m, n, alpha, X, ldx, Y,
                     ldy);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_copy_tril(smg_ctx* ctx, int m, int n, const double* X, int ldx, double* Y, int ldy) {
  if (!ctx || m < 0 || n < 0) return SMG_ERR_ARG;
  if (m == 0 || n == 0) return SMG_OK;
  if (!X || !Y || ldx < m || ldy < m) return SMG_ERR_ARG;
  if (m % 2 == 0 && ldx % 2 == 0 && ldy % 2 == 0 &&
      ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(Y)) & 15) == 0)
    hipLaunchKernelGGL(k_copy_tril_col2, dim3(n < 2048 ? n : 2048), dim3(256), 0, ctx->stream, m, n,
                       X, ldx, Y, ldy);
  else
    hipLaunchKernelGGL(k_copy_tril, dim3(grid_for((long long)m * n)), dim3(256), 0, ctx->stream, m, n,
                       X, ldx, Y, ldy);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_lse_tangent_fwd(smg_ctx* ctx, const double* x, const double* xd, long long n, double* out) {
  if (!ctx || n < 0 || !out || (n > 0 && (!x || !xd))) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_ELEMWISE);
  hipLaunchKernelGGL(k_lse_tangent_fwd, dim3(1), dim3(TT), 0, ctx->stream, x, xd, n, out);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_lse_tangent_rev(smg_ctx* ctx, const double* x, const double* xd, long long n, double lse, double t,
                        double adj, double* xadj, double* xdadj) {
  if (!ctx || n < 0) return SMG_ERR_ARG;
  if (n == 0 || adj == 0.0) return SMG_OK;
  if (!x || !xd) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_ELEMWISE);
  hipLaunchKernelGGL(k_lse_tangent_rev, dim3(grid_for(n)), dim3(256), 0, ctx->stream, x, xd, n, lse, t, adj, xadj,
                     xdadj);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_glm_tangent_fwd(smg_ctx* ctx, const double* eta, double alpha, const double* etad, double alphad,
                        const int* y, long long n, double* out) {
  if (!ctx || n < 0 || !out || (n > 0 && (!eta || !etad || !y))) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_ELEMWISE);
  hipLaunchKernelGGL(k_glm_tangent_fwd, dim3(1), dim3(TT), 0, ctx->stream, eta, alpha, etad, alphad, y, n, out);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_glm_tangent_rev(smg_ctx* ctx, const double* eta, double alpha, const double* etad, double alphad,
                        const int* y, long long n, double adj, double* eta_adj, double* etad_adj, double* out) {
  if (!ctx || n < 0 || !out || (n > 0 && (!eta || !etad || !y))) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_ELEMWISE);
  hipLaunchKernelGGL(k_glm_tangent_rev, dim3(1), dim3(TT), 0, ctx->stream, eta, alpha, etad, alphad, y, n, adj,
                     eta_adj, etad_adj, out);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

}  // extern "C"
