// The GLM reducers over rows, each in ONE pass over x (scalar intercept):
//   KIND 0  bernoulli_logit_glm_lpmf  (y int in {0,1})
//   KIND 1  normal_id_glm_lpdf        (y double, scalar sigma)
//   KIND 2  poisson_log_glm_lpmf      (y int >= 0)
// They differ only in the per-row function of the linear predictor; the
// x-streaming, the x^T theta' product and the deterministic reductions are
// shared.
//
// KIND 1: prim/mat/prob/normal_id_glm_lpdf.hpp:84-150
//   y_scaled = (y - x beta - alpha) / sigma;  mu' = y_scaled / sigma
//   partials: beta' = x^T mu', alpha' = sum mu', sigma' = (sum y_scaled^2 - N)/sigma
//   logp = -N log sqrt(2 pi) - N log sigma - sum y_scaled^2 / 2
//   (device: out = [sum y_scaled^2, sum mu', x^T mu'])
// KIND 2: prim/mat/prob/poisson_log_glm_lpmf.hpp:81-123
//   theta = x beta + alpha;  theta' = y - exp(theta)
//   logp = -sum lgamma(y + 1) + sum(y theta - exp(theta))
//   (device: out = [sum(y theta - exp theta), sum theta', x^T theta', sum lgamma(y + 1)])
//
// KIND 0:
// Reference: prim/mat/prob/bernoulli_logit_glm_lpmf.hpp:46-138
//   ytheta = sign .* (x beta + alpha), sign = 2y - 1            (:92-94)
//   logp   = sum( ytheta > 20 ? -exp(-ytheta)
//               : ytheta < -20 ? ytheta : -log1p(exp(-ytheta)) )  (:99-104)
//   theta' = ytheta > 20 ? -exp(-ytheta) : ytheta < -20 ? sign
//               : sign exp(-ytheta) / (exp(-ytheta) + 1)         (:115-121)
//   d/dbeta = x^T theta',  d/dalpha = sum theta'                  (:123, :133)
// The reference makes two GEMV passes over x (HBM-bound).  Here persistent
// workgroups stream 32-row tiles of x (column-major) through LDS once: the
// tile yields eta for its rows, then theta', then its contribution to x^T
// theta' while it is still on chip.  Each workgroup keeps per-column
// accumulators in registers and writes one [logp, alpha', beta'(M)] partial;
// a fixed-order second pass sums the partials (deterministic).
#include <cmath>

#include "smg_internal.h"

namespace {

constexpr int MMAX = 256;         // fused path: M <= 256

// zero page (global address space) for out-of-range loads: the address is
// redirected, no select on the loaded value
__device__ double g_glm_zero[2] = {0.0, 0.0};

template <int RB, int KIND>
__global__ __launch_bounds__(256) void k_glm_fused(const void* __restrict__ yv,
                                                   const double* __restrict__ x, long long R,
                                                   int M, long long ldx,
                                                   const double* __restrict__ ab,
                                                   double* __restrict__ part) {
  const int* __restrict__ y = static_cast<const int*>(yv);
  const double* __restrict__ yd = static_cast<const double*>(yv);
  constexpr int XS = RB + 1;  // LDS column stride (bank-conflict free)
  constexpr int PER = RB * MMAX / 256;
  constexpr int G = 256 / RB;  // column groups of the eta pass
  __shared__ double X[MMAX * XS];
  __shared__ double beta[MMAX];
  __shared__ double etap[G * RB];
  __shared__ double thd[RB];
  __shared__ double lds[16];
  const int t = threadIdx.x;
  if (t < M) beta[t] = ab[1 + t];
  const double alpha = ab[0];
  const double inv_sigma = KIND == 1 ? 1.0 / ab[1 + M] : 0.0;  // ab = [alpha, beta(M), sigma]
  const long long ntiles = (R + RB - 1) / RB;
  double gacc = 0.0;                 // column t's beta' accumulator (t < M)
  double lp_acc = 0.0, ga_acc = 0.0; // rows' logp / alpha' (threads < RB)
  double c_acc = 0.0;                // KIND 2: rows' lgamma(y + 1)
  double reg[PER];

  auto load = [&](long long tile) {
    const long long r0 = tile * RB;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int e = t + 256 * q;
      const int r = e % RB, c = e / RB;
      const long long gr = r0 + r;
      reg[q] = (c < M && gr < R) ? x[gr + (size_t)c * ldx] : 0.0;
    }
  };

  long long tile = blockIdx.x;
  if (tile < ntiles) load(tile);
  for (; tile < ntiles; tile += gridDim.x) {
    __syncthreads();  // previous tile fully consumed
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int e = t + 256 * q;
      X[(e / RB) * XS + (e % RB)] = reg[q];
    }
    __syncthreads();
    const long long next = tile + gridDim.x;
    if (next < ntiles) load(next);  // in flight during the compute below
    // eta: thread (r, g) sums columns c = g, g + G, ...
    {
      const int r = t % RB, g = t / RB;
      double s = 0.0;
      for (int c = g; c < M; c += G) s += X[c * XS + r] * beta[c];
      etap[g * RB + r] = s;
    }
    __syncthreads();
    if (t < RB) {
      const long long gr = tile * RB + t;
      double th = 0.0;
      if (gr < R) {
        double eta = 0.0;
#pragma unroll
        for (int g = 0; g < G; ++g) eta += etap[g * RB + t];
        if (KIND == 0) {
          const double sgn = 2.0 * y[gr] - 1.0;
          const double yt = sgn * (eta + alpha);
          const double e = exp(-yt);
          lp_acc += yt > 20.0 ? -e : (yt < -20.0 ? yt : -log1p(e));
          th = yt > 20.0 ? -e : (yt < -20.0 ? sgn : sgn * e / (e + 1));
        } else if (KIND == 1) {
          const double ys = (yd[gr] - eta - alpha) * inv_sigma;
          lp_acc += ys * ys;
          th = ys * inv_sigma;
        } else {
          const double yi = (double)y[gr];
          const double theta = eta + alpha;
          const double e = exp(theta);
          lp_acc += yi * theta - e;
          th = yi - e;
          c_acc += lgamma(yi + 1.0);
        }
        ga_acc += th;
      }
      thd[t] = th;
    }
    __syncthreads();
    if (t < M) {
      double s = 0.0;
#pragma unroll
      for (int r = 0; r < RB; ++r) s += X[t * XS + r] * thd[r];
      gacc += s;
    }
  }
  // per-block partial [logp, alpha', beta'(M) (, lgamma sum)]
  const int W = M + 2 + (KIND == 2);
  double* p = part + (size_t)blockIdx.x * W;
  __syncthreads();
  const double lp = block_sum(lp_acc, lds);
  __syncthreads();
  const double ga = block_sum(ga_acc, lds);
  double cs = 0.0;
  if (KIND == 2) {
    __syncthreads();
    cs = block_sum(c_acc, lds);
  }
  if (t == 0) {
    p[0] = lp;
    p[1] = ga;
    if (KIND == 2) p[M + 2] = cs;
  }
  if (t < M) p[2 + t] = gacc;
}

// rows per tile (measured on MI355X: 16 rows 4.3 TB/s, 32 rows 5.1, 64 rows 4.0).
// Also measured and rejected: 16-byte loads (two rows per lane) 4.8 TB/s vs
// 5.0 for 8-byte loads; contiguous per-workgroup tile ranges 3.9 TB/s (the
// interleaved order keeps concurrently running workgroups on adjacent
// segments of every column)
constexpr int GLM_RB = 32;

int glm_blocks(long long R) {
  const long long ntiles = (R + GLM_RB - 1) / GLM_RB;
  // LDS-limited workgroups per CU x 256 CUs (32 rows: 67.6 KB, 2 per CU; 16 rows: 34.8 KB, 4 per CU)
  long long nb = GLM_RB == 16 ? 1024 : (GLM_RB == 32 ? 512 : 256);
  if (nb > ntiles) nb = ntiles;
  if (nb < 1) nb = 1;
  return (int)nb;
}

// ------------------------------------------------ categorical_logit_glm_lpmf
// prim/mat/prob/categorical_logit_glm_lpmf.hpp:38-146 (x an N x M matrix,
// alpha C, beta M x C, y in 1..C), ONE pass over x in 16-row tiles:
//   lin = x beta + alpha;  logp = sum_i lin(i, y_i - 1) - max_i - log sum exp(lin_i - max_i)
//   theta'(i, c) = [c == y_i - 1] - softmax(lin_i)_c
//   alpha' = sum_i theta'(i, :),  beta' = x^T theta'
// (the reference's neg_softmax_lin plus the one-hot terms, :117-143).
// Per-workgroup partial [logp, alpha'(C), beta'(M x C col-major)], reduced in
// fixed order.  M <= 256, C <= CAT_CMAX.
constexpr int CAT_RB = 16;
constexpr int CAT_CMAX = 16;

__global__ __launch_bounds__(256) void k_glm_categorical(const int* __restrict__ y,
                                                         const double* __restrict__ x, long long R,
                                                         int M, long long ldx, int C,
                                                         const double* __restrict__ ab,
                                                         double* __restrict__ part) {
  constexpr int RB = CAT_RB, XS = RB + 1;
  constexpr int PER = RB * MMAX / 256;
  __shared__ double X[MMAX * XS];
  __shared__ double beta[MMAX * CAT_CMAX];  // beta[m * CAT_CMAX + c]
  __shared__ double alpha[CAT_CMAX];
  __shared__ double lin[RB * CAT_CMAX];     // then theta'
  __shared__ double lds[16];
  const int t = threadIdx.x;
  for (int e = t; e < M * C; e += 256) beta[(e % M) * CAT_CMAX + e / M] = ab[C + e];  // ab = [alpha(C), beta(M x C)]
  if (t < C) alpha[t] = ab[t];
  const long long ntiles = (R + RB - 1) / RB;
  double gacc[CAT_CMAX];  // column t of beta': one accumulator per class
#pragma unroll
  for (int c = 0; c < CAT_CMAX; ++c) gacc[c] = 0.0;
  double lp_acc = 0.0, ga_acc = 0.0;  // rows' logp (t < RB) / class t's alpha' (t < C)
  double reg[PER];
  auto load = [&](long long tile) {
    const long long r0 = tile * RB;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int e = t + 256 * q;
      const int r = e % RB, c = e / RB;
      const long long gr = r0 + r;
      reg[q] = *((c < M && gr < R) ? x + gr + (size_t)c * ldx : g_glm_zero);
    }
  };
  long long tile = blockIdx.x;
  if (tile < ntiles) load(tile);
  for (; tile < ntiles; tile += gridDim.x) {
    __syncthreads();  // previous tile fully consumed
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int e = t + 256 * q;
      X[(e / RB) * XS + (e % RB)] = reg[q];
    }
    __syncthreads();
    const long long next = tile + gridDim.x;
    if (next < ntiles) load(next);  // in flight during the compute below
    if (t < RB * C) {  // lin(r, c)
      const int r = t % RB, c = t / RB;
      double s = 0.0;
      for (int m = 0; m < M; ++m) s += X[m * XS + r] * beta[m * CAT_CMAX + c];
      lin[r * CAT_CMAX + c] = s + alpha[c];
    }
    __syncthreads();
    if (t < RB) {  // the row's softmax, logp and theta'
      const long long gr = tile * RB + t;
      if (gr < R) {
        double mx = lin[t * CAT_CMAX];
        for (int c = 1; c < C; ++c) mx = fmax(mx, lin[t * CAT_CMAX + c]);
        double se = 0.0;
        for (int c = 0; c < C; ++c) se += exp(lin[t * CAT_CMAX + c] - mx);
        const double inv = 1.0 / se;
        const int yc = y[gr] - 1;
        lp_acc += log(inv) - mx + lin[t * CAT_CMAX + yc];
        for (int c = 0; c < C; ++c)
          lin[t * CAT_CMAX + c] = (c == yc ? 1.0 : 0.0) - exp(lin[t * CAT_CMAX + c] - mx) * inv;
      } else {
        for (int c = 0; c < C; ++c) lin[t * CAT_CMAX + c] = 0.0;
      }
    }
    __syncthreads();
    if (t < C) {
      double s = 0.0;
#pragma unroll
      for (int r = 0; r < RB; ++r) s += lin[r * CAT_CMAX + t];
      ga_acc += s;
    }
    if (t < M) {
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const double xv = X[t * XS + r];
#pragma unroll
        for (int c = 0; c < CAT_CMAX; ++c)
          if (c < C) gacc[c] += xv * lin[r * CAT_CMAX + c];
      }
    }
  }
  const int W = 1 + C + M * C;
  double* p = part + (size_t)blockIdx.x * W;
  __syncthreads();
  const double lp = block_sum(lp_acc, lds);
  if (t == 0) p[0] = lp;
  if (t < C) p[1 + t] = ga_acc;
  if (t < M)
#pragma unroll
    for (int c = 0; c < CAT_CMAX; ++c)
      if (c < C) p[1 + C + (size_t)c * M + t] = gacc[c];
}

int glm_cat_blocks(long long R) {
  const long long ntiles = (R + CAT_RB - 1) / CAT_RB;
  long long nb = 512;
  if (nb > ntiles) nb = ntiles;
  if (nb < 1) nb = 1;
  return (int)nb;
}

// ------------------------------------------------ generic path (M > 256)
__global__ void k_glm_rows(const int* __restrict__ y, const double* __restrict__ eta, long long R,
                           double alpha, double* __restrict__ th, double* part) {
  __shared__ double lds[16];
  double lp = 0.0, ga = 0.0;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < R;
       i += (long long)gridDim.x * blockDim.x) {
    const double sgn = 2.0 * y[i] - 1.0;
    const double yt = sgn * (eta[i] + alpha);
    const double e = exp(-yt);
    lp += yt > 20.0 ? -e : (yt < -20.0 ? yt : -log1p(e));
    const double d = yt > 20.0 ? -e : (yt < -20.0 ? sgn : sgn * e / (e + 1));
    th[i] = d;
    ga += d;
  }
  lp = block_sum(lp, lds);
  __syncthreads();
  ga = block_sum(ga, lds);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = lp;
    part[2 * blockIdx.x + 1] = ga;
  }
}

// categorical generic path (M > 256 or C > 16): lin = x beta by GEMM, then one
// thread per row turns lin(i, :) (column-major, ld R) into theta'(i, :) in
// place and accumulates the row's logp; alpha' and beta' by GEMM.
__global__ void k_glm_cat_rows(const int* __restrict__ y, double* __restrict__ lin, long long R, int C,
                               const double* __restrict__ alpha, double* __restrict__ ones,
                               double* __restrict__ part) {
  __shared__ double lds[16];
  double lp = 0.0;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < R;
       i += (long long)gridDim.x * blockDim.x) {
    double mx = -INFINITY;
    for (int c = 0; c < C; ++c) {
      const double v = lin[i + (size_t)c * R] + alpha[c];
      lin[i + (size_t)c * R] = v;
      mx = fmax(mx, v);
    }
    double se = 0.0;
    for (int c = 0; c < C; ++c) se += exp(lin[i + (size_t)c * R] - mx);
    const double inv = 1.0 / se;
    const int yc = y[i] - 1;
    lp += log(inv) - mx + lin[i + (size_t)yc * R];
    for (int c = 0; c < C; ++c) {
      const double v = lin[i + (size_t)c * R];
      lin[i + (size_t)c * R] = (c == yc ? 1.0 : 0.0) - exp(v - mx) * inv;
    }
    ones[i] = 1.0;
  }
  lp = block_sum(lp, lds);
  if (threadIdx.x == 0) part[blockIdx.x] = lp;
}

}  // namespace

extern "C" {

long long smg_glm_ws_doubles(long long R, int M) {
  if (M <= MMAX) return (long long)glm_blocks(R) * (M + 3);
  return 2 * R + 2 * 1024;
}

int smg_bernoulli_logit_glm(smg_ctx* ctx, const int* y, const double* x, long long R, int M,
                            long long ldx, const double* ab, double* ws, double* out) {
  if (!ctx || R < 0 || M < 0 || !ab || !ws || !out) return SMG_ERR_ARG;
  if (R > 0 && (!y || (M > 0 && (!x || ldx < R)))) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_GLM);
  if (M <= MMAX) {
    const int nb = glm_blocks(R);
    hipLaunchKernelGGL((k_glm_fused<GLM_RB, 0>), dim3(nb), dim3(256), 0, ctx->stream, y, x, R, M, ldx,
                       ab, ws);
    smg_reduce_partials(ctx, ws, nb, M + 2, out, 0);
    SMG_LAUNCH_CHECK();
    return SMG_OK;
  }
  // eta = x beta (GEMM n = 1), theta' per row, beta' = x^T theta'
  double* eta = ws;
  double* th = ws + R;
  double* part = ws + 2 * R;
  int rc = smg_gemm_impl(ctx, 0, 0, 0, (int)R, 1, M, 1.0, x, (int)ldx, ab + 1, M, 0.0, eta, (int)R);
  if (rc) return rc;
  double alpha_h;
  rc = smg_memcpy_d2h(ctx, &alpha_h, ab, sizeof(double));
  if (rc) return rc;
  rc = smg_sync(ctx);
  if (rc) return rc;
  hipLaunchKernelGGL(k_glm_rows, dim3(1024), dim3(256), 0, ctx->stream, y, eta, R, alpha_h, th, part);
  smg_reduce_partials(ctx, part, 1024, 2, out, 0);
  rc = smg_gemm_impl(ctx, 1, 0, 0, M, 1, (int)R, 1.0, x, (int)ldx, th, (int)R, 0.0, out + 2, M);
  SMG_LAUNCH_CHECK();
  return rc;
}

long long smg_glm_categorical_ws_doubles(long long R, int M, int C) {
  if (M <= MMAX && C <= CAT_CMAX) return (long long)glm_cat_blocks(R) * (1 + C + (long long)M * C);
  return R * ((long long)C + 1) + 1024;
}

int smg_categorical_logit_glm(smg_ctx* ctx, const int* y, const double* x, long long R, int M,
                              long long ldx, int C, const double* alpha_beta, double* ws,
                              double* out) {
  if (!ctx || R < 0 || M < 0 || C < 1 || !alpha_beta || !ws || !out) return SMG_ERR_ARG;
  if (R > 0 && (!y || (M > 0 && (!x || ldx < R)))) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_GLM);
  if (M <= MMAX && C <= CAT_CMAX) {
    const int nb = glm_cat_blocks(R);
    hipLaunchKernelGGL(k_glm_categorical, dim3(nb), dim3(256), 0, ctx->stream, y, x, R, M, ldx, C,
                       alpha_beta, ws);
    smg_reduce_partials(ctx, ws, nb, 1 + C + M * C, out, 0);
    SMG_LAUNCH_CHECK();
    return SMG_OK;
  }
  if (R > INT_MAX || (long long)M * C > INT_MAX) return SMG_ERR_ARG;  // GEMM dimensions
  if (R == 0) return smg_memset(ctx, out, 0, sizeof(double) * (1 + C + (size_t)M * C));
  double* lin = ws;                         // R x C
  double* ones = ws + R * (long long)C;     // R
  double* part = ones + R;                  // 1024
  int rc = smg_gemm_impl(ctx, 0, 0, 0, (int)R, C, M, 1.0, x, (int)ldx, alpha_beta + C, M > 0 ? M : 1,
                         0.0, lin, (int)R);
  if (rc) return rc;
  hipLaunchKernelGGL(k_glm_cat_rows, dim3(1024), dim3(256), 0, ctx->stream, y, lin, R, C, alpha_beta,
                     ones, part);
  smg_reduce_partials(ctx, part, 1024, 1, out, 0);
  rc = smg_gemm_impl(ctx, 1, 0, 0, C, 1, (int)R, 1.0, lin, (int)R, ones, (int)R, 0.0, out + 1, C);
  if (rc) return rc;
  if (M > 0) rc = smg_gemm_impl(ctx, 1, 0, 0, M, C, (int)R, 1.0, x, (int)ldx, lin, (int)R, 0.0, out + 1 + C, M);
  SMG_LAUNCH_CHECK();
  return rc;
}

// normal_id_glm_lpdf / poisson_log_glm_lpmf: the fused pass (M <= 256)
int smg_normal_id_glm(smg_ctx* ctx, const double* y, const double* x, long long R, int M,
                      long long ldx, const double* abs, double* ws, double* out) {
  if (!ctx || R < 0 || M < 0 || M > MMAX || !abs || !ws || !out) return SMG_ERR_ARG;
  if (R > 0 && (!y || (M > 0 && (!x || ldx < R)))) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_GLM);
  const int nb = glm_blocks(R);
  hipLaunchKernelGGL((k_glm_fused<GLM_RB, 1>), dim3(nb), dim3(256), 0, ctx->stream, y, x, R, M, ldx,
                     abs, ws);
  smg_reduce_partials(ctx, ws, nb, M + 2, out, 0);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_poisson_log_glm(smg_ctx* ctx, const int* y, const double* x, long long R, int M,
                        long long ldx, const double* ab, double* ws, double* out) {
  if (!ctx || R < 0 || M < 0 || M > MMAX || !ab || !ws || !out) return SMG_ERR_ARG;
  if (R > 0 && (!y || (M > 0 && (!x || ldx < R)))) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_GLM);
  const int nb = glm_blocks(R);
  hipLaunchKernelGGL((k_glm_fused<GLM_RB, 2>), dim3(nb), dim3(256), 0, ctx->stream, y, x, R, M, ldx,
                     ab, ws);
  smg_reduce_partials(ctx, ws, nb, M + 3, out, 0);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

}  // extern "C"
