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
// workgroups stream 32-row tiles of x (column-major) once: the tile yields
// eta for its rows, then theta', then its contribution to x^T theta' while it
// is still on chip.  Each workgroup keeps per-column accumulators in
// registers and writes one [logp, alpha', beta'(M)] partial; a fixed-order
// second pass sums the partials (deterministic).  The default kernel is
// k_glm_reg (the tile stays in registers); the LDS-staged form measured
// slower (below) and lives in git history.
//
// Measured at 1e7 x 256 on MI355X (bench.py --workload glm, same box):
//   k_glm_fused 32 rows x 256 threads, 512 WGs   5.08 TB/s
//   k_glm_reg   32 rows x 512 threads            5.67-5.74 TB/s (256 or 512 WGs)
//   k_glm_reg   16 rows x 256 threads            4.75 TB/s (128-byte column segments)
//   k_glm_reg   16 rows x 512 threads            4.04 TB/s
//   k_glm_reg   32 x 512 with two tiles in flight (3 register buffers): no gain
//   k_glm_reg   32 x 512, x read with nontemporal loads (x is streamed once,
//               it should not displace other lines): 5.61-5.73 -> 5.81 TB/s
// The first k_glm_reg build ran at 1.7 TB/s: a branch or a select next to a
// load, a loop-carried register copy and a y load issued after x each made
// the compiler wait for the loads within the tile that issued them.
#include <cmath>
#include <cstdlib>

#include "smg_internal.h"

namespace {

constexpr int MMAX = 256;         // fused path: M <= 256

// zero page (global address space) for out-of-range loads: the address is
// redirected, no select on the loaded value
__device__ double g_glm_zero[2] = {0.0, 0.0};


// Register-resident variant: the tile never goes through LDS.  512 threads:
// thread t holds row r = t & 31 of the tile and the 16 columns c = g + 16q
// (g = t >> 5, q = 0..15): eta_r is 16 FMAs per thread plus one 16-way sum through a small
// LDS array (double-buffered: one barrier per tile), every thread forms
// theta'_r for its own row, and x^T theta' accumulates in 16 registers per
// thread (summed over the 32 rows of a column group once, at the end, by
// lane shuffles).  A load instruction still covers two 256-byte column
// segments per wave.
// check_y (KIND 0): also count the rows whose y is outside {0, 1} (the
// reference's check_bounded(y, 0, 1), prim/mat/prob/bernoulli_logit_glm_lpmf.hpp:75)
// into partial slot M + 2 -- the pass reads y anyway, so the check costs no
// extra launch and no extra pass over y.
template <int KIND, int RB, int NT, bool NTL>
__device__ __forceinline__ void glm_reg_body(const void* __restrict__ yv, const double* __restrict__ x, long long R,
                                             int M, long long ldx, const double* __restrict__ ab,
                                             double* __restrict__ part, int check_y) {
  constexpr int G = NT / RB, Q = MMAX / G;
  const int* __restrict__ y = static_cast<const int*>(yv);
  const double* __restrict__ yd = static_cast<const double*>(yv);
  __shared__ double beta[MMAX];
  __shared__ double red[2][G][RB];
  __shared__ double lds[16];
  const int t = threadIdx.x, r = t % RB, g = t / RB;
  for (int c = t; c < MMAX; c += NT) beta[c] = c < M ? ab[1 + c] : 0.0;
  const double alpha = ab[0];
  const double inv_sigma = KIND == 1 ? 1.0 / ab[1 + M] : 0.0;
  const long long ntiles = (R + RB - 1) / RB;
  double gacc[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) gacc[q] = 0.0;
  double lp_acc = 0.0, ga_acc = 0.0, c_acc = 0.0;
  double xc[Q], xn[Q];
  double yc = 0.0, yn = 0.0;  // the row's y (as double), loaded one tile ahead with x
  // Loads are straight-line code: addresses are clamped into x and the
  // values masked where they are consumed (a branch or a select next to a
  // load makes the compiler wait for it there), and y is issued before x so
  // that waiting for it leaves the x loads in flight (vmcnt counts in order).
  auto load = [&](double (&v)[Q], double& yv_, long long tile) {
    const long long gr = tile * RB + r;
    const size_t rc = (size_t)(gr < R ? gr : R - 1);
    yv_ = KIND == 1 ? yd[rc] : (double)y[rc];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int c = g + G * q;
      const int cc = c < M ? c : M - 1;
      const double* px = x + rc + (size_t)cc * ldx;
      v[q] = NTL ? __builtin_nontemporal_load(px) : *px;
    }
  };
  // one tile's work on the registers cur / cy (the other buffer's loads
  // stay in flight meanwhile); ping-pong buffers instead of a copy, which
  // would wait for the loads
  auto work = [&](double (&cur)[Q], double cy, long long tile, int buf) {
    const long long gr = tile * RB + r;
#pragma unroll
    for (int q = 0; q < Q; ++q) cur[q] = (gr < R && g + G * q < M) ? cur[q] : 0.0;
    double e = 0.0;
#pragma unroll
    for (int q = 0; q < Q; ++q) e += cur[q] * beta[g + G * q];
    red[buf][g][r] = e;
    __syncthreads();
    double th = 0.0;
    if (gr < R) {
      double eta = 0.0;
#pragma unroll
      for (int k = 0; k < G; ++k) eta += red[buf][k][r];
      double lp;
      if (KIND == 0) {
        const double sgn = 2.0 * cy - 1.0;
        const double yt = sgn * (eta + alpha);
        const double ex = exp(-yt);
        lp = yt > 20.0 ? -ex : (yt < -20.0 ? yt : -log1p(ex));
        th = yt > 20.0 ? -ex : (yt < -20.0 ? sgn : sgn * ex / (ex + 1));
      } else if (KIND == 1) {
        const double ys = (cy - eta - alpha) * inv_sigma;
        lp = ys * ys;
        th = ys * inv_sigma;
      } else {
        const double yi = cy;
        const double theta = eta + alpha;
        const double ex = exp(theta);
        lp = yi * theta - ex;
        th = yi - ex;
      }
      if (g == 0) {  // one thread per row accumulates the row's terms
        lp_acc += lp;
        ga_acc += th;
        if (KIND == 0) c_acc += (cy != 0.0 && cy != 1.0) ? 1.0 : 0.0;
      }
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) gacc[q] += th * cur[q];
  };
  __syncthreads();  // beta
  long long tile = blockIdx.x;
  const long long gs = gridDim.x;
  auto clampt = [&](long long tt) { return tt < ntiles ? tt : tile; };
  {
    if (tile < ntiles) load(xc, yc, tile);
    for (;;) {
      if (tile >= ntiles) break;
      load(xn, yn, clampt(tile + gs));
      work(xc, yc, tile, 0);
      tile += gs;
      if (tile >= ntiles) break;
      load(xc, yc, clampt(tile + gs));
      work(xn, yn, tile, 1);
      tile += gs;
    }
  }
  if (KIND == 2)  // sum of lgamma(y + 1) over this workgroup's rows, off the streaming loop
    for (long long k = t / RB;; k += NT / RB) {
      const long long tl2 = blockIdx.x + k * gridDim.x;
      if (tl2 >= ntiles) break;
      const long long gr = tl2 * RB + r;
      if (gr < R) c_acc += lgamma((double)y[gr] + 1.0);
    }
  // column sums over the RB rows of each column group: RB adjacent lanes
#pragma unroll
  for (int q = 0; q < Q; ++q)
    for (int off = RB / 2; off > 0; off >>= 1) gacc[q] += __shfl_xor(gacc[q], off, RB);
  const bool extra = KIND == 2 || (KIND == 0 && check_y);
  const int W = M + 2 + (extra ? 1 : 0);
  double* p = part + (size_t)blockIdx.x * W;
  __syncthreads();
  const double lp = block_sum(lp_acc, lds);
  __syncthreads();
  const double ga = block_sum(ga_acc, lds);
  double cs = 0.0;
  if (extra) {
    __syncthreads();
    cs = block_sum(c_acc, lds);
  }
  if (t == 0) {
    p[0] = lp;
    p[1] = ga;
    if (extra) p[M + 2] = cs;
  }
  if (r == 0)
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int c = g + G * q;
      if (c < M) p[2 + c] = gacc[q];
    }
}

template <int KIND, int RB, int NT, bool NTL = false>
__global__ __launch_bounds__(NT) void k_glm_reg(const void* __restrict__ yv, const double* __restrict__ x,
                                                long long R, int M, long long ldx, const double* __restrict__ ab,
                                                double* __restrict__ part, int check_y = 0) {
  glm_reg_body<KIND, RB, NT, NTL>(yv, x, R, M, ldx, ab, part, check_y);
}

// [alpha, beta(M)] as a kernel argument: the launch carries the parameters,
// no host-to-device copy ahead of it
struct glm_ab_arg {
  double v[MMAX + 1];
};

// The latency-bound form of k_glm_reg (KIND 0, y-bounds count on) takes the
// parameters from the kernel arguments of a one-workgroup copy ahead of it
// (no host-to-device copy).  The kernel arguments live in host memory: the
// streaming kernel reading them directly (every workgroup, 8 B at a time
// over the bus) measured 0.44 -> 0.53 ms at 1.25e6 rows.
__global__ __launch_bounds__(256) void k_glm_params(glm_ab_arg a, int n, double* __restrict__ dst) {
  for (int i = threadIdx.x; i < n; i += 256) dst[i] = a.v[i];
}

// ...and its finish: one workgroup per output column c sums column c of the
// per-workgroup partials (the order of k_reduce_partials: the same bits as
// the staged path), writes out[c] (device) and out_h[c] (pinned host), and
// takes a ticket; the last workgroup publishes seq to the host completion
// word, so the host spins on it instead of a copy back and a stream
// synchronisation.  (One workgroup summing all M + 3 columns measured 84 us
// at M = 256 -- 1 MB of partials through one CU -- against 4.7 us here.)
__global__ __launch_bounds__(256) void k_glm_io_final(const double* __restrict__ part, int nb, int W, double* out,
                                                      double* out_h, unsigned int* counter, long long* done,
                                                      long long seq) {
  __shared__ double lds[16];
  const int c = blockIdx.x;
  double s = 0.0;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) s += part[(size_t)i * W + c];
  s = block_sum(s, lds);
  if (threadIdx.x != 0) return;
  out[c] = s;
  if (!out_h) return;
  // a system-scope store goes to host memory directly; the ticket's
  // system-scope release orders it (and out[c]) before this workgroup's
  // arrival, the last arrival's acquire orders every column before done
  __hip_atomic_store(out_h + c, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (__hip_atomic_fetch_add(counter, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM) != gridDim.x - 1) return;
  __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
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

template <int KIND>
int glm_launch(hipStream_t st, const void* y, const double* x, long long R, int M, long long ldx,
               const double* ab, double* ws, int check_y = 0) {
  const int nb = glm_blocks(R);
  hipLaunchKernelGGL((k_glm_reg<KIND, 32, 512, true>), dim3(nb), dim3(512), 0, st, y, x, R, M, ldx, ab, ws, check_y);
  return nb;
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
    const int nb = glm_launch<0>(ctx->stream, y, x, R, M, ldx, ab, ws);
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

int smg_bernoulli_logit_glm_checked(smg_ctx* ctx, const int* y, const double* x, long long R, int M,
                                    long long ldx, const double* ab, double* ws, double* out) {
  if (!ctx || R < 0 || M < 0 || !ab || !ws || !out) return SMG_ERR_ARG;
  if (R > 0 && (!y || (M > 0 && (!x || ldx < R)))) return SMG_ERR_ARG;
  if (M > MMAX || R == 0) {  // the general path: a separate bound check
    int rc = smg_memset(ctx, out + M + 2, 0, sizeof(double));
    if (!rc) rc = smg_check_bounded_int(ctx, y, R, 0, 1, out + M + 2);
    if (!rc) rc = R > 0 ? smg_bernoulli_logit_glm(ctx, y, x, R, M, ldx, ab, ws, out)
                        : smg_memset(ctx, out, 0, sizeof(double) * (M + 2));
    return rc;
  }
  smg_prof_scope prof(ctx, SMG_FAM_GLM);
  const int nb = glm_launch<0>(ctx->stream, y, x, R, M, ldx, ab, ws, 1);
  smg_reduce_partials(ctx, ws, nb, M + 3, out, 0);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_bernoulli_logit_glm_io(smg_ctx* ctx, const int* y, const double* x, long long R, int M, long long ldx,
                               double alpha, const double* beta, double* ws, double* out, double* out_h) {
  if (!ctx || R < 0 || M < 0 || !ws || !out || (M > 0 && !beta)) return SMG_ERR_ARG;
  if (R > 0 && (!y || (M > 0 && (!x || ldx < R)))) return SMG_ERR_ARG;
  if (M > MMAX || R == 0) {  // the general path, then one copy back and a synchronisation
    double* ab = smg_ws(ctx, SMG_WS_GLM, (size_t)M + 1);
    double* h = (double*)smg_host_scratch(ctx, sizeof(double) * (M + 1));
    if (!ab || !h) return SMG_ERR_OOM;
    h[0] = alpha;
    for (int j = 0; j < M; ++j) h[1 + j] = beta[j];
    int rc = smg_memcpy_h2d(ctx, ab, h, sizeof(double) * (M + 1));
    if (!rc) rc = smg_bernoulli_logit_glm_checked(ctx, y, x, R, M, ldx, ab, ws, out);
    if (!rc && out_h) rc = smg_memcpy_d2h(ctx, out_h, out, sizeof(double) * (M + 3));
    if (!rc) rc = smg_sync(ctx);  // the scratch upload has been read
    return rc;
  }
  glm_ab_arg a;
  a.v[0] = alpha;
  for (int j = 0; j < M; ++j) a.v[1 + j] = beta[j];
  const int nb = glm_blocks(R);
  const long long seq = out_h ? ++ctx->done_seq : 0;
  {  // (the profiling scope closes before the host waits)
    smg_prof_scope prof(ctx, SMG_FAM_GLM);
    double* ab = smg_ws(ctx, SMG_WS_GLM, MMAX + 1);
    if (!ab) return SMG_ERR_OOM;
    hipLaunchKernelGGL(k_glm_params, dim3(1), dim3(256), 0, ctx->stream, a, M + 1, ab);
    hipLaunchKernelGGL((k_glm_reg<0, GLM_RB, 512, true>), dim3(nb), dim3(512), 0, ctx->stream, y, x, R, M, ldx, ab, ws, 1);
    hipLaunchKernelGGL(k_glm_io_final, dim3(M + 3), dim3(256), 0, ctx->stream, ws, nb, M + 3, out, out_h,
                       ctx->red_counter_d + 1, out_h ? ctx->done_h : nullptr, seq);
    SMG_LAUNCH_CHECK();
  }
  return out_h ? smg_wait_done(ctx, seq) : SMG_OK;
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
  const int nb = glm_launch<1>(ctx->stream, y, x, R, M, ldx, abs, ws);
  smg_reduce_partials(ctx, ws, nb, M + 2, out, 0);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_poisson_log_glm(smg_ctx* ctx, const int* y, const double* x, long long R, int M,
                        long long ldx, const double* ab, double* ws, double* out) {
  if (!ctx || R < 0 || M < 0 || M > MMAX || !ab || !ws || !out) return SMG_ERR_ARG;
  if (R > 0 && (!y || (M > 0 && (!x || ldx < R)))) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_GLM);
  const int nb = glm_launch<2>(ctx->stream, y, x, R, M, ldx, ab, ws);
  smg_reduce_partials(ctx, ws, nb, M + 3, out, 0);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

}  // extern "C"
