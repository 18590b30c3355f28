// gp_exp_quad_cov and add_diag, forward and reverse.
//
// gp_exp_quad_cov(std::vector<double> x, var sigma, var l)
//   rev/mat/fun/gp_exp_quad_cov.hpp:64-94 (forward), :96-112 (chain)
// The reference stores the N(N-1)/2 lower entries once and aliases the upper
// triangle to them (:233-238), so the adjoint of each lower vari is the sum of
// the adjoints of positions (i,j) and (j,i).  Here the node keeps the full
// N x N adjoint and the reverse kernel sweeps every position once (coalesced),
// which sums exactly those pairs:
//   d/dl     = sum_{i != j} Kadj_ij K_ij d_ij^2 / l^3
//   d/dsigma = 2/sigma (sum_{i != j} Kadj_ij K_ij + sum_i Kadj_ii sigma^2)
// K_ij is recomputed from x instead of re-read (HBM: one read of Kadj).
// Reductions are fixed-order (per-block partials + one ordered pass).
//
// add_diag: prim/mat/fun/add_diag.hpp:20-55.
#include "smg_internal.h"

namespace {

constexpr int GP_BLOCKS = 2048;

__global__ __launch_bounds__(256) void k_gp_fwd(const double* __restrict__ x, int n, double s2,
                                                double inv_half_sq_l, double* __restrict__ K,
                                                int ldk) {
  // 2D: blockIdx.y over columns j, x-dim over rows i (coalesced stores)
  const int j = blockIdx.y;
  const double xj = x[j];
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    double v;
    if (i == j) {
      v = s2;
    } else {
      const double d = (i > j) ? x[i] - xj : xj - x[i];
      v = s2 * exp(-(d * d) * inv_half_sq_l);
    }
    K[i + (size_t)j * ldk] = v;
  }
}

__global__ __launch_bounds__(256) void k_gp_rev_partials(const double* __restrict__ x, int n,
                                                         double s2, double inv_half_sq_l,
                                                         const double* __restrict__ Ka, int lda,
                                                         double* __restrict__ part) {
  __shared__ double lds[16];
  double al = 0.0, as = 0.0;
  for (smg_mn it(n, n); it.ok(); it.next()) {
    const long long e = it.e;
    const int i = it.i, j = it.j;
    const double a = Ka[i + (size_t)j * lda];
    if (i == j) {
      as += a * s2;
    } else {
      const double d = (i > j) ? x[i] - x[j] : x[j] - x[i];
      const double dist = d * d;
      const double prod = a * (s2 * exp(-dist * inv_half_sq_l));
      al += prod * dist;
      as += prod;
    }
  }
  const double sl = block_sum(al, lds);
  __syncthreads();
  const double ss = block_sum(as, lds);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x + 0] = ss;
    part[2 * blockIdx.x + 1] = sl;
  }
}

// k_gp_rev_partials in the column form (16-byte reads of Kadj and x; a
// workgroup walks whole columns); the same per-element terms, fixed order.
__global__ __launch_bounds__(256) void k_gp_rev_partials_col2(const double* __restrict__ x, int n,
                                                              double s2, double inv_half_sq_l,
                                                              const double* __restrict__ Ka,
                                                              int lda, double* __restrict__ part) {
  __shared__ double lds[16];
  const int np = n >> 1;
  const double2* x2 = reinterpret_cast<const double2*>(x);
  double al = 0.0, as = 0.0;
  for (int j = blockIdx.x; j < n; j += gridDim.x) {
    const double xj = x[j];
    const double2* col = reinterpret_cast<const double2*>(Ka + (size_t)j * lda);
    for (int p0 = threadIdx.x; p0 < np; p0 += 4 * 256) {
      double2 a[4], xi[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int p = p0 + 256 * k;
        if (p < np) {
          a[k] = col[p];
          xi[k] = x2[p];
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int p = p0 + 256 * k;
        if (p < np) {
          const int i = 2 * p;
          const double av[2] = {a[k].x, a[k].y}, xv[2] = {xi[k].x, xi[k].y};
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            if (i + h == j) {
              as += av[h] * s2;
            } else {
              const double d = (i + h > j) ? xv[h] - xj : xj - xv[h];
              const double dist = d * d;
              const double prod = av[h] * (s2 * exp(-dist * inv_half_sq_l));
              al += prod * dist;
              as += prod;
            }
          }
        }
      }
    }
  }
  const double sl = block_sum(al, lds);
  __syncthreads();
  const double ss = block_sum(as, lds);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x + 0] = ss;
    part[2 * blockIdx.x + 1] = sl;
  }
}

__global__ void k_gp_rev_final(const double* __restrict__ part, int nparts, double sigma, double l,
                               double* out2) {
  __shared__ double lds[16];
  double ss = 0.0, sl = 0.0;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) {
    ss += part[2 * i];
    sl += part[2 * i + 1];
  }
  ss = block_sum(ss, lds);
  __syncthreads();
  sl = block_sum(sl, lds);
  if (threadIdx.x == 0) {
    out2[0] += ss * 2 / sigma;     // :110
    out2[1] += sl / (l * l * l);   // :109
  }
}

__global__ void k_add_diag_fwd(const double* __restrict__ A, int lda, int n, double d,
                               const double* __restrict__ dv, double* __restrict__ B, int ldb) {
  for (smg_mn it(n, n); it.ok(); it.next()) {
    const long long e = it.e;
    const int i = it.i, j = it.j;
    double v = A[i + (size_t)j * lda];
    if (i == j) v += dv ? dv[i] : d;
    B[i + (size_t)j * ldb] = v;
  }
}

// Column forms of k_gp_fwd / k_add_diag_fwd for 16-byte aligned operands with
// even n and leading dimensions (the N=4096 GP): a workgroup walks whole
// columns, each lane moves two rows with one 16-byte access, four accesses in
// flight per lane.  Same per-element expressions as above (the same bits).
__global__ __launch_bounds__(256) void k_gp_fwd_col2(const double* __restrict__ x, int n, double s2,
                                                     double inv_half_sq_l, double* __restrict__ K,
                                                     int ldk) {
  const int np = n >> 1;
  const double2* x2 = reinterpret_cast<const double2*>(x);
  for (int j = blockIdx.x; j < n; j += gridDim.x) {
    const double xj = x[j];
    double2* col = reinterpret_cast<double2*>(K + (size_t)j * ldk);
    for (int p0 = threadIdx.x; p0 < np; p0 += 4 * 256) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int p = p0 + 256 * k;
        if (p < np) {
          const double2 xi = x2[p];
          const int i = 2 * p;
          double2 v;
          if (i == j) {
            v.x = s2;
          } else {
            const double d = (i > j) ? xi.x - xj : xj - xi.x;
            v.x = s2 * exp(-(d * d) * inv_half_sq_l);
          }
          if (i + 1 == j) {
            v.y = s2;
          } else {
            const double d = (i + 1 > j) ? xi.y - xj : xj - xi.y;
            v.y = s2 * exp(-(d * d) * inv_half_sq_l);
          }
          col[p] = v;
        }
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_add_diag_fwd_col2(const double* __restrict__ A, int lda,
                                                           int n, double d,
                                                           const double* __restrict__ dv,
                                                           double* __restrict__ B, int ldb) {
  const int np = n >> 1;
  for (int j = blockIdx.x; j < n; j += gridDim.x) {
    const double2* a = reinterpret_cast<const double2*>(A + (size_t)j * lda);
    double2* b = reinterpret_cast<double2*>(B + (size_t)j * ldb);
    const double dj = dv ? dv[j] : d;
    for (int p0 = threadIdx.x; p0 < np; p0 += 4 * 256) {
      double2 v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int p = p0 + 256 * k;
        if (p < np) v[k] = a[p];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int p = p0 + 256 * k;
        if (p < np) {
          if (2 * p == j) v[k].x += dj;
          if (2 * p + 1 == j) v[k].y += dj;
          b[p] = v[k];
        }
      }
    }
  }
}

// Both column forms need 16-byte aligned columns.
inline bool col2_ok(const void* p, int ld, int n) {
  return ((reinterpret_cast<uintptr_t>(p) & 15) == 0) && (ld % 2 == 0) && (n % 2 == 0);
}

// Y += X over whole columns, 16-byte accesses (add_diag's reverse, A's adjoint)
__global__ __launch_bounds__(256) void k_add_full_col2(const double* __restrict__ X, int ldx, int n,
                                                       double* __restrict__ Y, int ldy) {
  const int np = n >> 1;
  for (int j = blockIdx.x; j < n; j += gridDim.x) {
    const double2* x = reinterpret_cast<const double2*>(X + (size_t)j * ldx);
    double2* y = reinterpret_cast<double2*>(Y + (size_t)j * ldy);
    for (int p0 = threadIdx.x; p0 < np; p0 += 4 * 256) {
      double2 a[4], b[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int p = p0 + 256 * k;
        if (p < np) {
          a[k] = x[p];
          b[k] = y[p];
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int p = p0 + 256 * k;
        if (p < np) {
          b[k].x += a[k].x;
          b[k].y += a[k].y;
          y[p] = b[k];
        }
      }
    }
  }
}

__global__ void k_add_full(const double* __restrict__ X, int ldx, int n, double* __restrict__ Y,
                           int ldy) {
  for (smg_mn it(n, n); it.ok(); it.next()) {
    const long long e = it.e;
    const int i = it.i, j = it.j;
    Y[i + (size_t)j * ldy] += X[i + (size_t)j * ldx];
  }
}

__global__ void k_diag_adj(const double* __restrict__ Ba, int ldb, int n, double* dadj, int vec) {
  __shared__ double lds[16];
  if (vec) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) dadj[i] += Ba[i + (size_t)i * ldb];
    return;
  }
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += Ba[i + (size_t)i * ldb];
  s = block_sum(s, lds);
  if (threadIdx.x == 0) dadj[0] += s;
}

// Tangent of K along (sigma', l') -- the fvar<var> instantiation of the same
// covariance (prim/mat/fun/gp_exp_quad_cov.hpp:40-59 over fvar, used by
// hessian_times_vector):  Kd_ij = 2 sigma sigma' e + sigma^2 l' d^2 e / l^3,
// e = exp(-d^2 / (2 l^2)); Kd_ii = 2 sigma sigma'.
__global__ __launch_bounds__(256) void k_gp_tan_fwd(const double* __restrict__ x, int n, double a,
                                                    double b, double inv_half_sq_l,
                                                    double* __restrict__ K, int ldk) {
  // a = 2 sigma sigma', b = sigma^2 l' / l^3
  const int j = blockIdx.y;
  const double xj = x[j];
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    double v;
    if (i == j) {
      v = a;
    } else {
      const double d = (i > j) ? x[i] - xj : xj - x[i];
      const double d2 = d * d;
      const double e = exp(-d2 * inv_half_sq_l);
      v = a * e + b * d2 * e;
    }
    K[i + (size_t)j * ldk] = v;
  }
}

// per-block partials of S_e = sum A e, S_2 = sum A e d^2, S_4 = sum A e d^4 (all positions)
__global__ __launch_bounds__(256) void k_gp_tan_partials(const double* __restrict__ x, int n,
                                                         double inv_half_sq_l,
                                                         const double* __restrict__ Ka, int lda,
                                                         double* __restrict__ part) {
  __shared__ double lds[16];
  double se = 0.0, s2 = 0.0, s4 = 0.0;
  const long long tot = (long long)n * n;
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < tot;
       q += (long long)gridDim.x * blockDim.x) {
    const int j = (int)(q / n), i = (int)(q % n);
    const double a = Ka[i + (size_t)j * lda];
    if (i == j) {
      se += a;
    } else {
      const double d = (i > j) ? x[i] - x[j] : x[j] - x[i];
      const double d2 = d * d;
      const double ae = a * exp(-d2 * inv_half_sq_l);
      se += ae;
      s2 += ae * d2;
      s4 += ae * d2 * d2;
    }
  }
  se = block_sum(se, lds);
  __syncthreads();
  s2 = block_sum(s2, lds);
  __syncthreads();
  s4 = block_sum(s4, lds);
  if (threadIdx.x == 0) {
    part[3 * blockIdx.x + 0] = se;
    part[3 * blockIdx.x + 1] = s2;
    part[3 * blockIdx.x + 2] = s4;
  }
}

__global__ void k_gp_tan_final(const double* __restrict__ part, int nparts, double sigma, double l,
                               double ds, double dl, double* out4) {
  __shared__ double lds[16];
  double se = 0.0, s2 = 0.0, s4 = 0.0;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) {
    se += part[3 * i];
    s2 += part[3 * i + 1];
    s4 += part[3 * i + 2];
  }
  se = block_sum(se, lds);
  __syncthreads();
  s2 = block_sum(s2, lds);
  __syncthreads();
  s4 = block_sum(s4, lds);
  if (threadIdx.x == 0) {
    const double l3 = l * l * l, l4 = l3 * l, l6 = l3 * l3;
    out4[0] += 2 * ds * se + 2 * sigma * dl * s2 / l3;                                  // d/dsigma
    out4[1] += 2 * sigma * ds * s2 / l3 + sigma * sigma * dl * (s4 / l6 - 3 * s2 / l4);  // d/dl
    out4[2] += 2 * sigma * se;                                                          // d/dsigma'
    out4[3] += sigma * sigma * s2 / l3;                                                 // d/dl'
  }
}


// D-dimensional inputs (gp_exp_quad_cov(std::vector<T_x> x, ...) with T_x an
// Eigen vector, rev/mat/fun/gp_exp_quad_cov.hpp:158-184,211-242): x is D x n
// column-major (point i at x + i D), d_ij^2 = squared_distance(x_i, x_j)
// summed over the D coordinates in order.  A workgroup walks whole columns j;
// x_j is staged in LDS, the row points are read from L2 (x is n D doubles).
__global__ __launch_bounds__(256) void k_gp_nd_fwd(const double* __restrict__ x, int D, int n, double s2,
                                                   double inv_half_sq_l, double* __restrict__ K, int ldk) {
  extern __shared__ double xj[];
  for (int j = blockIdx.x; j < n; j += gridDim.x) {
    __syncthreads();
    for (int d = threadIdx.x; d < D; d += blockDim.x) xj[d] = x[(size_t)j * D + d];
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      double v = s2;
      if (i != j) {
        const double* xi = x + (size_t)i * D;
        double d2 = 0.0;
        for (int d = 0; d < D; ++d) {
          const double t = xi[d] - xj[d];
          d2 += t * t;
        }
        v = s2 * exp(-d2 * inv_half_sq_l);
      }
      K[i + (size_t)j * ldk] = v;
    }
  }
}

__global__ __launch_bounds__(256) void k_gp_nd_rev_partials(const double* __restrict__ x, int D, int n, double s2,
                                                            double inv_half_sq_l, const double* __restrict__ Ka,
                                                            int lda, double* __restrict__ part) {
  extern __shared__ double xj[];
  __shared__ double lds[16];
  double al = 0.0, as = 0.0;
  for (int j = blockIdx.x; j < n; j += gridDim.x) {
    __syncthreads();
    for (int d = threadIdx.x; d < D; d += blockDim.x) xj[d] = x[(size_t)j * D + d];
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const double a = Ka[i + (size_t)j * lda];
      if (i == j) {
        as += a * s2;
      } else {
        const double* xi = x + (size_t)i * D;
        double d2 = 0.0;
        for (int d = 0; d < D; ++d) {
          const double t = xi[d] - xj[d];
          d2 += t * t;
        }
        const double prod = a * (s2 * exp(-d2 * inv_half_sq_l));
        al += prod * d2;
        as += prod;
      }
    }
  }
  const double sl = block_sum(al, lds);
  __syncthreads();
  const double ss = block_sum(as, lds);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x + 0] = ss;
    part[2 * blockIdx.x + 1] = sl;
  }
}

inline int grid_for(long long tot) {
  long long g = (tot + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

extern "C" {

int smg_gp_exp_quad_cov_fwd(smg_ctx* ctx, const double* x, int n, double sigma, double l,
                            double* K, int ldk) {
  if (!ctx || n < 0 || (n > 0 && (!x || !K || ldk < n))) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  smg_prof_scope prof(ctx, SMG_FAM_GP);
  const double s2 = sigma * sigma;
  const double ihl = 0.5 / (l * l);
  if (col2_ok(x, 2, n) && col2_ok(K, ldk, n)) {
    hipLaunchKernelGGL(k_gp_fwd_col2, dim3(n < 2048 ? n : 2048), dim3(256), 0, ctx->stream, x, n,
                       s2, ihl, K, ldk);
    SMG_LAUNCH_CHECK();
    return SMG_OK;
  }
  dim3 grid(smg_ceil_div(n, 256) > 16 ? 16 : smg_ceil_div(n, 256), n);
  hipLaunchKernelGGL(k_gp_fwd, grid, dim3(256), 0, ctx->stream, x, n, s2, ihl, K, ldk);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_gp_exp_quad_cov_rev(smg_ctx* ctx, const double* x, int n, double sigma, double l,
                            const double* Kadj, int ldka, double* out2) {
  if (!ctx || n < 0 || (n > 0 && (!x || !Kadj || !out2 || ldka < n))) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  smg_prof_scope prof(ctx, SMG_FAM_GP);
  const long long tot = (long long)n * n;
  const bool col2 = col2_ok(x, 2, n) && col2_ok(Kadj, ldka, n);
  int nb = col2 ? n : grid_for(tot);
  if (nb > GP_BLOCKS) nb = GP_BLOCKS;
  double* part = smg_ws(ctx, SMG_WS_RED, 2 * (size_t)nb);
  if (!part) return SMG_ERR_OOM;
  if (col2) {
    hipLaunchKernelGGL(k_gp_rev_partials_col2, dim3(nb), dim3(256), 0, ctx->stream, x, n,
                       sigma * sigma, 0.5 / (l * l), Kadj, ldka, part);
  } else {
    hipLaunchKernelGGL(k_gp_rev_partials, dim3(nb), dim3(256), 0, ctx->stream, x, n, sigma * sigma,
                       0.5 / (l * l), Kadj, ldka, part);
  }
  hipLaunchKernelGGL(k_gp_rev_final, dim3(1), dim3(1024), 0, ctx->stream, part, nb, sigma, l, out2);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_gp_exp_quad_cov_nd_fwd(smg_ctx* ctx, const double* x, int D, int n, double sigma, double l, double* K,
                               int ldk) {
  if (!ctx || n < 0 || D < 1 || D > 8192 || (n > 0 && (!x || !K || ldk < n))) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  if (D == 1) return smg_gp_exp_quad_cov_fwd(ctx, x, n, sigma, l, K, ldk);
  smg_prof_scope prof(ctx, SMG_FAM_GP);
  hipLaunchKernelGGL(k_gp_nd_fwd, dim3(n < 2048 ? n : 2048), dim3(256), D * sizeof(double), ctx->stream, x, D, n,
                     sigma * sigma, 0.5 / (l * l), K, ldk);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_gp_exp_quad_cov_nd_rev(smg_ctx* ctx, const double* x, int D, int n, double sigma, double l,
                               const double* Kadj, int ldka, double* out2) {
  if (!ctx || n < 0 || D < 1 || D > 8192 || (n > 0 && (!x || !Kadj || !out2 || ldka < n))) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  if (D == 1) return smg_gp_exp_quad_cov_rev(ctx, x, n, sigma, l, Kadj, ldka, out2);
  smg_prof_scope prof(ctx, SMG_FAM_GP);
  const int nb = n < GP_BLOCKS ? n : GP_BLOCKS;
  double* part = smg_ws(ctx, SMG_WS_RED, 2 * (size_t)nb);
  if (!part) return SMG_ERR_OOM;
  hipLaunchKernelGGL(k_gp_nd_rev_partials, dim3(nb), dim3(256), D * sizeof(double), ctx->stream, x, D, n,
                     sigma * sigma, 0.5 / (l * l), Kadj, ldka, part);
  hipLaunchKernelGGL(k_gp_rev_final, dim3(1), dim3(1024), 0, ctx->stream, part, nb, sigma, l, out2);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_gp_exp_quad_cov_tangent_fwd(smg_ctx* ctx, const double* x, int n, double sigma, double l,
                                    double dsigma, double dl, double* Kd, int ldk) {
  if (!ctx || n < 0 || (n > 0 && (!x || !Kd || ldk < n))) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  smg_prof_scope prof(ctx, SMG_FAM_GP);
  dim3 grid(smg_ceil_div(n, 256) > 16 ? 16 : smg_ceil_div(n, 256), n);
  hipLaunchKernelGGL(k_gp_tan_fwd, grid, dim3(256), 0, ctx->stream, x, n, 2 * sigma * dsigma,
                     sigma * sigma * dl / (l * l * l), 0.5 / (l * l), Kd, ldk);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_gp_exp_quad_cov_tangent_rev(smg_ctx* ctx, const double* x, int n, double sigma, double l,
                                    double dsigma, double dl, const double* Kdadj, int ldka,
                                    double* out4) {
  if (!ctx || n < 0 || (n > 0 && (!x || !Kdadj || !out4 || ldka < n))) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  smg_prof_scope prof(ctx, SMG_FAM_GP);
  int nb = grid_for((long long)n * n);
  if (nb > GP_BLOCKS) nb = GP_BLOCKS;
  double* part = smg_ws(ctx, SMG_WS_RED, 3 * (size_t)nb);
  if (!part) return SMG_ERR_OOM;
  hipLaunchKernelGGL(k_gp_tan_partials, dim3(nb), dim3(256), 0, ctx->stream, x, n, 0.5 / (l * l),
                     Kdadj, ldka, part);
  hipLaunchKernelGGL(k_gp_tan_final, dim3(1), dim3(1024), 0, ctx->stream, part, nb, sigma, l,
                     dsigma, dl, out4);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_add_diag_fwd(smg_ctx* ctx, const double* A, int lda, int n, double d, const double* dv,
                     double* B, int ldb) {
  if (!ctx || n < 0 || (n > 0 && (!A || !B || lda < n || ldb < n))) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  if (col2_ok(A, lda, n) && col2_ok(B, ldb, n)) {
    hipLaunchKernelGGL(k_add_diag_fwd_col2, dim3(n < 2048 ? n : 2048), dim3(256), 0, ctx->stream,
                       A, lda, n, d, dv, B, ldb);
    SMG_LAUNCH_CHECK();
    return SMG_OK;
  }
  hipLaunchKernelGGL(k_add_diag_fwd, dim3(grid_for((long long)n * n)), dim3(256), 0, ctx->stream, A,
                     lda, n, d, dv, B, ldb);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_add_diag_rev(smg_ctx* ctx, const double* Ba, int ldb, int n, double* Aa, int ldaa,
                     double* dadj, int vec) {
  if (!ctx || n < 0 || (n > 0 && !Ba)) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  if (Aa && col2_ok(Ba, ldb, n) && col2_ok(Aa, ldaa, n))
    hipLaunchKernelGGL(k_add_full_col2, dim3(n < 2048 ? n : 2048), dim3(256), 0, ctx->stream, Ba,
                       ldb, n, Aa, ldaa);
  else if (Aa)
    hipLaunchKernelGGL(k_add_full, dim3(grid_for((long long)n * n)), dim3(256), 0, ctx->stream, Ba,
                       ldb, n, Aa, ldaa);
  if (dadj)
    hipLaunchKernelGGL(k_diag_adj, dim3(1), dim3(1024), 0, ctx->stream, Ba, ldb, n, dadj, vec);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

}  // extern "C"
