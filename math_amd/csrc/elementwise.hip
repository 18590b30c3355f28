// Vectorised scalar functors and reducers: log_sum_exp, lgamma / digamma /
// trigamma, normal_lpdf, plus axpy / sum helpers for the reverse sweep.
// All reductions are two-stage with fixed order (deterministic).
#include <cmath>

#include "smg_internal.h"

namespace {

constexpr int RED_BLOCKS = 1024;

inline int grid_for(long long tot, int cap = 8192) {
  long long g = (tot + 255) / 256;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

// ------------------------------------------------------ special functions
// digamma: boost::math::digamma, 53-bit path, policy errno_on_error -> NaN
// at poles (boost/math/special_functions/digamma.hpp:108-128, 300-347, 381-449;
// stan/math/prim/scal/fun/digamma.hpp:46-48, boost_policy.hpp)
__device__ double dev_digamma_large(double x) {
  const double P0 = 0.083333333333333333333333333333333333333333333333333,
               P1 = -0.0083333333333333333333333333333333333333333333333333,
               P2 = 0.003968253968253968253968253968253968253968253968254,
               P3 = -0.0041666666666666666666666666666666666666666666666667,
               P4 = 0.0075757575757575757575757575757575757575757575757576,
               P5 = -0.021092796092796092796092796092796092796092796092796,
               P6 = 0.083333333333333333333333333333333333333333333333333,
               P7 = -0.44325980392156862745098039215686274509803921568627;
  x -= 1;
  double result = log(x);
  result += 1 / (2 * x);
  const double z = 1 / (x * x);
  const double p = P0 + z * (P1 + z * (P2 + z * (P3 + z * (P4 + z * (P5 + z * (P6 + z * P7))))));
  result -= z * p;
  return result;
}

__device__ double dev_digamma_1_2(double x) {
  const double Y = (double)0.99558162689208984F;
  const double root1 = 1569415565.0 / 1073741824.0;
  const double root2 = (381566830.0 / 1073741824.0) / 1073741824.0;
  const double root3 = 0.9016312093258695918615325266959189453125e-19;
  double g = x - root1;
  g -= root2;
  g -= root3;
  const double t = x - 1;
  const double p = 0.25479851061131551 +
                   t * (-0.32555031186804491 +
                        t * (-0.65031853770896507 +
                             t * (-0.28919126444774784 +
                                  t * (-0.045251321448739056 + t * -0.0020713321167745952))));
  const double q =
      1.0 + t * (2.0767117023730469 +
                 t * (1.4606242909763515 +
                      t * (0.43593529692665969 +
                           t * (0.054151797245674225 +
                                t * (0.0021284987017821144 + t * -0.55789841321675513e-6)))));
  return g * Y + g * (p / q);
}

__device__ double dev_digamma(double x) {
  double result = 0;
  if (x <= -1) {
    x = 1 - x;
    double rem = x - floor(x);
    if (rem > 0.5) rem -= 1;
    if (rem == 0) return __longlong_as_double(0x7ff8000000000000LL);
    result = M_PI / tan(M_PI * rem);
  }
  if (x == 0) return __longlong_as_double(0x7ff8000000000000LL);
  if (isnan(x)) return x;
  if (x >= 10) {
    result += dev_digamma_large(x);
  } else {
    while (x > 2) {
      x -= 1;
      result += 1 / x;
    }
    while (x < 1) {
      result -= 1 / x;
      x += 1;
    }
    result += dev_digamma_1_2(x);
  }
  return result;
}

// trigamma: stan/math/prim/scal/fun/trigamma.hpp:33-80 (reflection unrolled)
__device__ double dev_trigamma_pos(double x) {
  const double small = 0.0001, large = 5.0;
  const double b2 = 1.0 / 6.0, b4 = -1.0 / 30.0, b6 = 1.0 / 42.0, b8 = -1.0 / 30.0;
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

__device__ double dev_trigamma(double x) {
  if (isnan(x)) return x;
  if (x <= 0.0 && floor(x) == x) return __longlong_as_double(0x7ff0000000000000LL);
  if (x <= 0) {
    const double s = M_PI / sin(-M_PI * x);
    return -dev_trigamma_pos(-x + 1.0) + s * s;
  }
  return dev_trigamma_pos(x);
}

// lgamma: the reference calls glibc lgamma_r (prim/scal/fun/lgamma.hpp:62-71);
// the device uses the ROCm libm lgamma (same function, <= a few ulp apart).
__device__ double dev_lgamma(double x) { return lgamma(x); }

template <int F>
__global__ void k_unary(const double* __restrict__ x, long long n, double* __restrict__ y) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const double v = x[i];
    y[i] = F == 0 ? dev_lgamma(v) : (F == 1 ? dev_digamma(v) : dev_trigamma(v));
  }
}

// xadj += yadj * f'(x):  F = 0 lgamma -> digamma, F = 1 digamma -> trigamma
template <int F>
__global__ void k_unary_rev(const double* __restrict__ x, long long n,
                            const double* __restrict__ ya, double* __restrict__ xa) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const double v = x[i];
    xa[i] += ya[i] * (F == 0 ? dev_digamma(v) : dev_trigamma(v));
  }
}

// --------------------------------------------------------- log_sum_exp
__global__ void k_max_part(const double* __restrict__ x, long long n, double* part) {
  __shared__ double lds[16];
  double m = -INFINITY;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    m = fmax(m, x[i]);
  m = wave_max(m);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) lds[w] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    double r = -INFINITY;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) r = fmax(r, lds[i]);
    part[blockIdx.x] = r;
  }
}

__global__ void k_sumexp_part(const double* __restrict__ x, long long n, const double* maxp,
                              int nmax, double* part) {
  __shared__ double lds[16];
  __shared__ double smax;
  if (threadIdx.x == 0) {
    double r = -INFINITY;
    for (int i = 0; i < nmax; ++i) r = fmax(r, maxp[i]);
    smax = r;
  }
  __syncthreads();
  const double mx = smax;
  double s = 0.0;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    s += exp(x[i] - mx);
  s = block_sum(s, lds);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ void k_lse_final(const double* maxp, const double* sump, int np, double* out) {
  __shared__ double lds[16];
  double s = 0.0;
  for (int i = threadIdx.x; i < np; i += blockDim.x) s += sump[i];
  s = block_sum(s, lds);
  if (threadIdx.x == 0) {
    double mx = -INFINITY;
    for (int i = 0; i < np; ++i) mx = fmax(mx, maxp[i]);
    // rev/mat/fun/log_sum_exp.hpp:24-31
    out[0] = isfinite(mx) ? mx + log(s) : mx;
  }
}

__global__ void k_lse_rev(const double* __restrict__ x, long long n, double lse, double adj,
                          double* __restrict__ xa) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    xa[i] += adj * exp(x[i] - lse);
}

// -------------------------------------------------------------- normal
// per-block partials: [logp, sum gy, sum gmu, sum gsigma]
__global__ void k_normal(const double* __restrict__ y, int sy, const double* __restrict__ mu,
                         int smu, const double* __restrict__ sg, int ssg, long long n, int inc,
                         double* gy, double* gmu, double* gs, int red_y, int red_mu, int red_s,
                         double* part) {
  __shared__ double lds[16];
  const double neg_log_sqrt_two_pi = -log(sqrt(2.0 * M_PI));
  double lp = 0, sy_ = 0, smu_ = 0, ss_ = 0;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const double s = sg[i * ssg];
    const double inv_s = 1.0 / s;
    const double z = (y[i * sy] - mu[i * smu]) * inv_s;
    const double z2 = z * z;
    if (inc & 1) lp += neg_log_sqrt_two_pi;
    if (inc & 2) lp -= log(s);
    if (inc & 4) lp += -0.5 * z2;
    const double sc = inv_s * z;
    const double gsv = -inv_s + inv_s * z2;
    if (gy) {
      if (red_y) sy_ -= sc; else gy[i] -= sc;
    }
    if (gmu) {
      if (red_mu) smu_ += sc; else gmu[i] += sc;
    }
    if (gs) {
      if (red_s) ss_ += gsv; else gs[i] += gsv;
    }
  }
  lp = block_sum(lp, lds);
  __syncthreads();
  sy_ = block_sum(sy_, lds);
  __syncthreads();
  smu_ = block_sum(smu_, lds);
  __syncthreads();
  ss_ = block_sum(ss_, lds);
  if (threadIdx.x == 0) {
    part[4 * blockIdx.x + 0] = lp;
    part[4 * blockIdx.x + 1] = sy_;
    part[4 * blockIdx.x + 2] = smu_;
    part[4 * blockIdx.x + 3] = ss_;
  }
}

__global__ void k_normal_final(const double* part, int np, double* out, double* gy, double* gmu,
                               double* gs, int red_y, int red_mu, int red_s) {
  __shared__ double lds[16];
  double v[4];
  for (int c = 0; c < 4; ++c) {
    double s = 0.0;
    for (int i = threadIdx.x; i < np; i += blockDim.x) s += part[4 * i + c];
    s = block_sum(s, lds);
    __syncthreads();
    v[c] = s;
  }
  if (threadIdx.x == 0) {
    out[0] = v[0];
    if (gy && red_y) gy[0] += v[1];
    if (gmu && red_mu) gmu[0] += v[2];
    if (gs && red_s) gs[0] += v[3];
  }
}

// fused normal_lpdf: domain checks, value and partials in ONE launch; every
// operand / output pointer may be device memory or pinned host memory
// (zero-copy: the latency-bound small calls on host vars read and write the
// host directly).  Per-block [lp, bad_y, bad_mu, bad_s, sum gy, sum gmu,
// sum gs]; with several blocks the last to arrive (self-resetting ticket)
// sums them in block order (deterministic).  Publication: plain stores (the
// pinned staging is coarse-grained, so partials leave the L2 as whole lines
// at the release, not one PCIe write per 8-B store: write-through stores
// measured 1.5 us slower at N = 1024), ONE system-scope release per block
// (an L2 write-back), drained, then ONE system-scope store of seq to the host
// completion word.
__global__ void __launch_bounds__(1024) k_normal_fused(
    const double* __restrict__ y, const double* __restrict__ mu, const double* __restrict__ sg, double y0,
    double mu0, double s0, long long n, int inc, double* gy, double* gmu, double* gs,
    int red_y, int red_mu, int red_s, double* part, unsigned int* counter, double* res,
    long long* done, long long seq) {
  __shared__ double lds[7][16];
  __shared__ int last;
  const double neg_log_sqrt_two_pi = -0.91893853320467274178;  // -log(sqrt(2 pi))
  double v[7] = {0, 0, 0, 0, 0, 0, 0};
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const double yv = y ? y[i] : y0, mv = mu ? mu[i] : mu0, s = sg ? sg[i] : s0;
    if (yv != yv) v[1] = 1.0;                               // check_not_nan(y)
    if (!(fabs(mv) <= 1.7976931348623157e308)) v[2] = 1.0;  // check_finite(mu)
    if (!(s > 0.0)) v[3] = 1.0;                             // check_positive(sigma)
    const double inv_s = 1.0 / s;
    const double z = (yv - mv) * inv_s;
    const double z2 = z * z;
    if (inc & 1) v[0] += neg_log_sqrt_two_pi;
    if (inc & 2) v[0] -= log(s);
    if (inc & 4) v[0] += -0.5 * z2;
    const double sc = inv_s * z;
    const double gsv = -inv_s + inv_s * z2;
    if (gy) {
      if (red_y) v[4] -= sc; else gy[i] = -sc;
    }
    if (gmu) {
      if (red_mu) v[5] += sc; else gmu[i] = sc;
    }
    if (gs) {
      if (red_s) v[6] += gsv; else gs[i] = gsv;
    }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  // flags by ballot; shuffle reductions (ds_bpermute round trips, the bulk
  // of a small call's kernel time) only for the sums that are used
  const bool any_y = __any(v[1] != 0.0), any_mu = __any(v[2] != 0.0), any_s = __any(v[3] != 0.0);
  const double t0 = wave_sum(v[0]);
  const double t4 = (gy && red_y) ? wave_sum(v[4]) : 0.0;
  const double t5 = (gmu && red_mu) ? wave_sum(v[5]) : 0.0;
  const double t6 = (gs && red_s) ? wave_sum(v[6]) : 0.0;
  if (lane == 0) {
    lds[0][w] = t0;
    lds[1][w] = any_y ? 1.0 : 0.0;
    lds[2][w] = any_mu ? 1.0 : 0.0;
    lds[3][w] = any_s ? 1.0 : 0.0;
    lds[4][w] = t4;
    lds[5][w] = t5;
    lds[6][w] = t6;
  }
  __syncthreads();
  double tot = 0.0;  // thread c < 7: column c summed over the block's waves in order
  if (threadIdx.x < 7)
    for (int k = 0; k < nw; ++k) tot += lds[threadIdx.x][k];
  if (gridDim.x > 1) {
    if (threadIdx.x < 7)
      __hip_atomic_store(part + 7 * blockIdx.x + threadIdx.x, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // every wave's partial-vector (gy / gmu / gs) and part stores have left
    // it before the barrier; then ONE system-scope release by thread 0 makes
    // them all visible (pinned host memory included) ahead of the ticket, and
    // the ticket's acquire orders the last block's reads of every part
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      last = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    if (threadIdx.x < 7) {
      tot = 0.0;
      for (unsigned int b = 0; b < gridDim.x; ++b)
        tot += __hip_atomic_load(part + 7 * b + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (threadIdx.x == 0) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (threadIdx.x < 7) res[threadIdx.x] = tot;
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: the L2 lines of every output
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(done, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ------------------------------------------------------------- helpers
__global__ void k_axpy(long long n, double a, const double* __restrict__ x, int incx,
                       double* __restrict__ y, int incy) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    y[i * incy] += a * x[i * incx];
}

__global__ void k_axpy_dev(long long n, const double* a, const double* __restrict__ x,
                           double* __restrict__ y) {
  const double av = *a;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    y[i] += av * x[i];
}

__global__ void k_sum_part(const double* __restrict__ x, long long n, double* part) {
  __shared__ double lds[16];
  double s = 0.0;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    s += x[i];
  s = block_sum(s, lds);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

}  // namespace

extern "C" {

int smg_lgamma_fwd(smg_ctx* ctx, const double* x, long long n, double* y) {
  if (!ctx || n < 0) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  smg_prof_scope prof(ctx, SMG_FAM_ELEMWISE);
  hipLaunchKernelGGL(k_unary<0>, dim3(grid_for(n)), dim3(256), 0, ctx->stream, x, n, y);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}
int smg_digamma_fwd(smg_ctx* ctx, const double* x, long long n, double* y) {
  if (!ctx || n < 0) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  smg_prof_scope prof(ctx, SMG_FAM_ELEMWISE);
  hipLaunchKernelGGL(k_unary<1>, dim3(grid_for(n)), dim3(256), 0, ctx->stream, x, n, y);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}
int smg_trigamma_fwd(smg_ctx* ctx, const double* x, long long n, double* y) {
  if (!ctx || n < 0) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  smg_prof_scope prof(ctx, SMG_FAM_ELEMWISE);
  hipLaunchKernelGGL(k_unary<2>, dim3(grid_for(n)), dim3(256), 0, ctx->stream, x, n, y);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}
int smg_lgamma_rev(smg_ctx* ctx, const double* x, long long n, const double* ya, double* xa) {
  if (!ctx || n < 0) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  smg_prof_scope prof(ctx, SMG_FAM_ELEMWISE);
  hipLaunchKernelGGL(k_unary_rev<0>, dim3(grid_for(n)), dim3(256), 0, ctx->stream, x, n, ya, xa);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}
int smg_digamma_rev(smg_ctx* ctx, const double* x, long long n, const double* ya, double* xa) {
  if (!ctx || n < 0) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  smg_prof_scope prof(ctx, SMG_FAM_ELEMWISE);
  hipLaunchKernelGGL(k_unary_rev<1>, dim3(grid_for(n)), dim3(256), 0, ctx->stream, x, n, ya, xa);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_log_sum_exp_fwd(smg_ctx* ctx, const double* x, long long n, double* out) {
  if (!ctx || n < 0 || !out) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_ELEMWISE);
  if (n == 0) {  // empty -> -inf (rev/mat/fun/log_sum_exp.hpp:21-23)
    const double ninf = -INFINITY;
    double* h = (double*)smg_host_scratch(ctx, 8);
    h[0] = ninf;
    int rc = smg_memcpy_h2d(ctx, out, h, 8);
    if (rc) return rc;
    return smg_sync(ctx);
  }
  const int nb = grid_for(n, RED_BLOCKS);
  double* part = smg_ws(ctx, SMG_WS_RED, 2 * (size_t)nb);
  if (!part) return SMG_ERR_OOM;
  hipLaunchKernelGGL(k_max_part, dim3(nb), dim3(256), 0, ctx->stream, x, n, part);
  hipLaunchKernelGGL(k_sumexp_part, dim3(nb), dim3(256), 0, ctx->stream, x, n, part, nb, part + nb);
  hipLaunchKernelGGL(k_lse_final, dim3(1), dim3(1024), 0, ctx->stream, part, part + nb, nb, out);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_log_sum_exp_rev(smg_ctx* ctx, const double* x, long long n, double lse, double adj,
                        double* xa) {
  if (!ctx || n < 0) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  smg_prof_scope prof(ctx, SMG_FAM_ELEMWISE);
  hipLaunchKernelGGL(k_lse_rev, dim3(grid_for(n)), dim3(256), 0, ctx->stream, x, n, lse, adj, xa);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_normal_lpdf(smg_ctx* ctx, const double* y, int sy, const double* mu, int smu,
                    const double* sigma, int ssig, long long n, int include, double* out, double* gy,
                    double* gmu, double* gsigma) {
  if (!ctx || n < 0 || !out || !y || !mu || !sigma) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_ELEMWISE);
  const int nb = n == 0 ? 1 : grid_for(n, RED_BLOCKS);
  double* part = smg_ws(ctx, SMG_WS_RED, 4 * (size_t)nb);
  if (!part) return SMG_ERR_OOM;
  const int ry = sy == 0, rmu = smu == 0, rs = ssig == 0;
  hipLaunchKernelGGL(k_normal, dim3(nb), dim3(256), 0, ctx->stream, y, sy, mu, smu, sigma, ssig, n,
                     include, gy, gmu, gsigma, ry, rmu, rs, part);
  hipLaunchKernelGGL(k_normal_final, dim3(1), dim3(1024), 0, ctx->stream, part, nb, out, gy, gmu,
                     gsigma, ry, rmu, rs);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_normal_lpdf_fused(smg_ctx* ctx, const double* y, const double* mu, const double* sigma, double y0,
                          double mu0, double sigma0, long long n, int include, double* res, double* gy,
                          double* gmu, double* gsigma) {
  if (!ctx || n < 0 || !res) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_ELEMWISE);
  const int nb = n <= 4096 ? 1 : (int)(n / 4096 < 512 ? (n + 4095) / 4096 : 512);
  double* part = nb > 1 ? smg_ws(ctx, SMG_WS_RED, 7 * (size_t)nb) : nullptr;
  if (nb > 1 && !part) return SMG_ERR_OOM;
  const long long seq = ++ctx->done_seq;
  const int ry = y == nullptr, rmu = mu == nullptr, rs = sigma == nullptr;
  hipLaunchKernelGGL(k_normal_fused, dim3(nb), dim3(1024), 0, ctx->stream, y, mu, sigma, y0, mu0, sigma0, n,
                     include, gy, gmu, gsigma, ry, rmu, rs, part, ctx->red_counter_d, res, ctx->done_h, seq);
  SMG_LAUNCH_CHECK();
  return smg_wait_done(ctx, seq);
}

int smg_axpy(smg_ctx* ctx, long long n, double a, const double* x, int incx, double* y, int incy) {
  if (!ctx || n < 0) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  hipLaunchKernelGGL(k_axpy, dim3(grid_for(n)), dim3(256), 0, ctx->stream, n, a, x, incx, y, incy);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_axpy_dev(smg_ctx* ctx, long long n, const double* a, const double* x, double* y) {
  if (!ctx || n < 0) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  hipLaunchKernelGGL(k_axpy_dev, dim3(grid_for(n)), dim3(256), 0, ctx->stream, n, a, x, y);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_sum(smg_ctx* ctx, const double* x, long long n, double* out) {
  if (!ctx || n < 0 || !out) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  const int nb = grid_for(n, RED_BLOCKS);
  double* part = smg_ws(ctx, SMG_WS_RED, (size_t)nb);
  if (!part) return SMG_ERR_OOM;
  hipLaunchKernelGGL(k_sum_part, dim3(nb), dim3(256), 0, ctx->stream, x, n, part);
  smg_reduce_partials(ctx, part, nb, 1, out, 1);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

}  // extern "C"
