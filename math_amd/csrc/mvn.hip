// multi_normal_cholesky_lpdf<false>(y | mu, L), forward value and reverse.
//
// Reference: prim/mat/prob/multi_normal_cholesky_lpdf.hpp:40-160.  The
// reference forms the explicit inverse inv_L (:117-118) and then
//   half = inv_L (y - mu),  scaled_diff = inv_L^T half,
//   logp = -n log(sqrt(2 pi)) - half.half/2 + sum log(diag(inv_L)),
//   dlogp/dL = scaled_diff half^T - inv_L^T  (all n^2 entries, :147,155).
// Here the two triangular solves w = L^{-1}(y-mu), sd = L^{-T} w replace the
// inverse (O(n^2) instead of O(n^3)); diag(inv_L) = 1/L_ii.  When L is the
// output of cholesky_decompose its strict upper triangle aliases a dummy vari
// (rev/mat/fun/cholesky_decompose.hpp:34-48) whose adjoint is never read, and
// inv_L^T is upper triangular, so on the lower triangle the partial is
// tril(sd w^T) - diag(1/L_ii): no inverse is needed (lower_only mode).  The
// full n^2 partials (lower_only == 0) form inv_L^T explicitly.
#include <cmath>

#include "smg_internal.h"
#include "tri_small.h"

namespace {

__global__ void k_residual(const double* __restrict__ y, const double* __restrict__ mu, int n,
                           double* __restrict__ r) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    r[i] = mu ? y[i] - mu[i] : y[i];
}

// lp = n * NEG_LOG_SQRT_TWO_PI - 0.5 w.w + sum log(1/L_ii), one block, fixed order
// the value: part[2 b] = sum w_i^2, part[2 b + 1] = sum log(1 / L_ii) over
// workgroup b's strided rows (MVN_LP_PARTS workgroups: the diagonal's
// scattered loads and the logs spread over CUs), then one fixed-order sum
constexpr int MVN_LP_PARTS = 32;
__global__ __launch_bounds__(256) void k_mvn_lp_part(const double* __restrict__ w, const double* __restrict__ L,
                                                     int ldl, int n, double* __restrict__ part) {
  __shared__ double lds[16];
  double q = 0.0, ld = 0.0;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += MVN_LP_PARTS * 256) {
    q += w[i] * w[i];
    ld += log(1.0 / L[i + (size_t)i * ldl]);
  }
  q = block_sum(q, lds);
  __syncthreads();
  ld = block_sum(ld, lds);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = q;
    part[2 * blockIdx.x + 1] = ld;
  }
}
__global__ void k_mvn_lp_final(const double* __restrict__ part, int n, double* out) {
  if (threadIdx.x != 0) return;
  double q = 0.0, ld = 0.0;
  for (int b = 0; b < MVN_LP_PARTS; ++b) {
    q += part[2 * b];
    ld += part[2 * b + 1];
  }
  const double neg_log_sqrt_two_pi = -log(sqrt(2.0 * M_PI));
  double logp = neg_log_sqrt_two_pi * n;
  logp -= 0.5 * q;
  logp += ld;
  out[0] = logp;
}

// Ladj(i,j) += adj*(sd_i w_j) for i >= j;  Ladj(i,i) -= adj / L_ii
__global__ void k_mvn_rev_lower(const double* __restrict__ L, int ldl, int n,
                                const double* __restrict__ w, const double* __restrict__ sd,
                                double adj, double* __restrict__ La, int ldla) {
  for (smg_mn it(n, n); it.ok(); it.next()) {
    const long long e = it.e;
    const int i = it.i, j = it.j;
    if (i < j) continue;
    double g = sd[i] * w[j];
    if (i == j) g -= 1.0 / L[i + (size_t)i * ldl];
    La[i + (size_t)j * ldla] += adj * g;
  }
}

// k_mvn_rev_lower over whole columns with 16-byte accesses (even n and ldla,
// 16-byte aligned La and sd); the same per-element expression
__global__ __launch_bounds__(256) void k_mvn_rev_lower_col2(const double* __restrict__ L, int ldl,
                                                            int n, const double* __restrict__ w,
                                                            const double* __restrict__ sd,
                                                            double adj, double* __restrict__ La,
                                                            int ldla) {
  const int np = n >> 1;
  const double2* sd2 = reinterpret_cast<const double2*>(sd);
  for (int j = blockIdx.x; j < n; j += gridDim.x) {
    const double wj = w[j];
    double2* col = reinterpret_cast<double2*>(La + (size_t)j * ldla);
    for (int p0 = (j >> 1) + threadIdx.x; p0 < np; p0 += 4 * 256) {
      double2 a[4], s[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int p = p0 + 256 * k;
        if (p < np) {
          a[k] = col[p];
          s[k] = sd2[p];
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int p = p0 + 256 * k;
        if (p < np) {
          const int i = 2 * p;
          if (i >= j) {
            double g = s[k].x * wj;
            if (i == j) g -= 1.0 / L[i + (size_t)i * ldl];
            a[k].x += adj * g;
          }
          double g = s[k].y * wj;
          if (i + 1 == j) g -= 1.0 / L[(i + 1) + (size_t)(i + 1) * ldl];
          a[k].y += adj * g;
          col[p] = a[k];
        }
      }
    }
  }
}

// Ladj += adj*(sd w^T - Linv^T) over every entry; Linv given (lower, dense)
__global__ void k_mvn_rev_full(const double* __restrict__ Linv, int n, const double* __restrict__ w,
                               const double* __restrict__ sd, double adj, double* __restrict__ La,
                               int ldla) {
  for (smg_mn it(n, n); it.ok(); it.next()) {
    const long long e = it.e;
    const int i = it.i, j = it.j;
    const double g = sd[i] * w[j] - Linv[j + (size_t)i * n];
    La[i + (size_t)j * ldla] += adj * g;
  }
}

__global__ void k_axpy_vec(int n, double a, const double* __restrict__ x, double* __restrict__ y) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    y[i] += a * x[i];
}

__global__ void k_identity(int n, double* I) {
  const long long tot = (long long)n * n;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < tot;
       e += (long long)gridDim.x * blockDim.x)
    I[e] = (e % n == e / n) ? 1.0 : 0.0;
}

inline int grid_for(long long tot) {
  long long g = (tot + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

extern "C" {

int smg_mvn_cholesky_fwd(smg_ctx* ctx, const double* y, const double* mu, const double* L, int ldl,
                         const double* Dinv, int n, double* ws, double* out_lp) {
  if (!ctx || n < 0 || (n > 0 && (!y || !L || !ws || !out_lp || ldl < n))) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  smg_prof_scope prof(ctx, SMG_FAM_MVN);
  double* w = ws;
  double* sd = ws + n;
  double* r = smg_ws(ctx, SMG_WS_RED, 2 * (size_t)n + 2 * MVN_LP_PARTS);
  if (!r) return SMG_ERR_OOM;
  double* res = r + n;
  double* part = r + 2 * (size_t)n;
  int rc;
  // the Cholesky forward's aux holds the 64- and 256-row diagonal-block
  // inverses (smg_cholesky_aux_doubles); without it, build the 64-row level
  const double* W256 = nullptr;
  const double* W512 = nullptr;
  if (!Dinv) {
    double* W = smg_ws(ctx, SMG_WS_TMP2, (size_t)n * SMG_NB);
    if (!W) return SMG_ERR_OOM;
    rc = smg_trtri_blocks_impl(ctx, L, ldl, n, W);
    if (rc) return rc;
    Dinv = W;
  } else {
    W256 = Dinv + (size_t)n * SMG_AUX_W256;
    W512 = Dinv + (size_t)n * SMG_AUX_W512;
  }
  hipLaunchKernelGGL(k_residual, dim3(grid_for(n)), dim3(256), 0, ctx->stream, y, mu, n, res);
  rc = smg_trsv_lower_impl(ctx, 0, L, ldl, Dinv, W256, W512, n, res, w, r, n);  // w = L^{-1}(y - mu)
  if (rc) return rc;
  rc = smg_trsv_lower_impl(ctx, 1, L, ldl, Dinv, W256, W512, n, w, sd, r, n);  // sd = L^{-T} w
  if (rc) return rc;
  hipLaunchKernelGGL(k_mvn_lp_part, dim3(MVN_LP_PARTS), dim3(256), 0, ctx->stream, w, L, ldl, n, part);
  hipLaunchKernelGGL(k_mvn_lp_final, dim3(1), dim3(64), 0, ctx->stream, part, n, out_lp);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_mvn_cholesky_rev(smg_ctx* ctx, const double* L, int ldl, const double* Dinv, int n,
                         const double* ws, double adj, int lower_only, double* yadj, double* muadj,
                         double* Ladj, int ldla) {
  if (!ctx || n < 0 || (n > 0 && (!L || !ws))) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  smg_prof_scope prof(ctx, SMG_FAM_MVN);
  const double* w = ws;
  const double* sd = ws + n;
  if (yadj) hipLaunchKernelGGL(k_axpy_vec, dim3(grid_for(n)), dim3(256), 0, ctx->stream, n, -adj, sd, yadj);
  if (muadj) hipLaunchKernelGGL(k_axpy_vec, dim3(grid_for(n)), dim3(256), 0, ctx->stream, n, adj, sd, muadj);
  if (Ladj) {
    if (lower_only) {
      if (n % 2 == 0 && ldla % 2 == 0 &&
          ((reinterpret_cast<uintptr_t>(Ladj) | reinterpret_cast<uintptr_t>(sd)) & 15) == 0)
        hipLaunchKernelGGL(k_mvn_rev_lower_col2, dim3(n < 2048 ? n : 2048), dim3(256), 0,
                           ctx->stream, L, ldl, n, w, sd, adj, Ladj, ldla);
      else
        hipLaunchKernelGGL(k_mvn_rev_lower, dim3(grid_for((long long)n * n)), dim3(256), 0,
                           ctx->stream, L, ldl, n, w, sd, adj, Ladj, ldla);
    } else {
      double* Linv = smg_ws(ctx, SMG_WS_TMP, (size_t)n * n);
      if (!Linv) return SMG_ERR_OOM;
      hipLaunchKernelGGL(k_identity, dim3(grid_for((long long)n * n)), dim3(256), 0, ctx->stream, n,
                         Linv);
      int rc = smg_trsm_impl(ctx, 1, 0, L, ldl, Dinv, n, Linv, n, n, n);
      if (rc) return rc;
      hipLaunchKernelGGL(k_mvn_rev_full, dim3(grid_for((long long)n * n)), dim3(256), 0,
                         ctx->stream, Linv, n, w, sd, adj, Ladj, ldla);
    }
  }
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

}  // extern "C"
