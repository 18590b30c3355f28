// The reverse of cholesky_decompose when the factor's whole adjoint comes from
// multi_normal_cholesky_lpdf(y | mu, L) (the GP marginal, config 3).
//
// The MVN's partials for a lower-structured L are
//   Lbar = adj (tril(s w^T) - diag(1/L_ii)),  w = L^{-1}(y - mu),  s = L^{-T} w
// (prim/mat/prob/multi_normal_cholesky_lpdf.hpp:139-155, upper half on the
// dummy vari), and pushing exactly that Lbar through the Cholesky adjoint
// (rev/mat/fun/cholesky_decompose.hpp:118-166, Murray's blocked algorithm,
// 2 N^3 / 3 in ~N/64 dependent GEMM rounds) has the closed form
//   Abar (lower) += adj Phi(s s^T - K^{-1}),  K = L L^T,
// Phi = strict lower triangle + half the diagonal (the reference's lower-entry
// convention: an off-diagonal A_ij stands for both K_ij and K_ji).  K^{-1} =
// V V^T with V = L^{-T}: V by recursive doubling from the factorisation's
// 512-row block inverses (N^3 / 3), V V^T lower (N^3 / 3) -- the same
// 2 N^3 / 3 as Murray's, in 16 large triangular-operand GEMMs instead of
// ~40 dependent rounds of small ones.  The host layer takes this path only
// when it can prove no other node wrote the factor's adjoint
// (stan/math/rev/fun/cholesky_decompose.hpp).
#include "smg_internal.h"
#include "tri_small.h"

#include <vector>

namespace {

// V[lo:hi, lo:hi] = L[lo:hi, lo:hi]^{-T} (upper) from the 512-row block
// inverses W_b (aux level SMG_AUX_W512, ld n; lower with stored zeros above):
//   leaves V_bb = W_b^T;  V12 = -V11 (L21^T V22)  -- as T = V11 L21^T (NT),
//   V12 = -T V22 (NN), T a workspace of ld n.
// Only the upper triangle and the strict-lower zeros inside the 512 leaves
// are written: every later product reads V through triangular K-range cuts
// whose tiles never leave a leaf below the diagonal.
// (the leaves and, with `pairs`, the 1024-row nodes are formed beforehand in
// batched launches: inv_t_leaves)
int inv_t_rec(smg_ctx* ctx, const double* L, int ldl, const double* w512, int n, double* V, int ldv, double* T,
              int lo, int hi, bool pairs) {
  if (hi - lo == SMG_NBR || (pairs && hi - lo == 2 * SMG_NBR)) return SMG_OK;
  const int mid = lo + ((hi - lo) / SMG_NBR / 2) * SMG_NBR;
  int rc = inv_t_rec(ctx, L, ldl, w512, n, V, ldv, T, lo, mid, pairs);
  if (!rc) rc = inv_t_rec(ctx, L, ldl, w512, n, V, ldv, T, mid, hi, pairs);
  if (rc) return rc;
  const int b = mid - lo, a = hi - mid;
  // T (b x a) = V11 L21^T: op(A) = V11 upper
  rc = smg_gemm_impl(ctx, 0, 1, 0, b, a, b, 1.0, V + lo + (size_t)lo * ldv, ldv, L + mid + (size_t)lo * ldl, ldl, 0.0,
                     T, n, SMG_TRI_A_UPPER);
  if (rc) return rc;
  // V12 (b x a) = -T V22: op(B) = V22 upper
  return smg_gemm_impl(ctx, 0, 0, 0, b, a, a, -1.0, T, n, V + mid + (size_t)mid * ldv, ldv, 0.0,
                       V + lo + (size_t)mid * ldv, ldv, SMG_TRI_B_UPPER);
}

// V_bb = W_b^T for every 512-row leaf b from b0 (one launch: blockIdx.z =
// leaf, 64 x 64 tiles through LDS)
__global__ __launch_bounds__(256) void k_leaf_transpose(const double* __restrict__ w512, int n, int lo,
                                                       double* __restrict__ V, int ldv) {
  __shared__ double t[64][65];
  const int b0 = lo + blockIdx.z * SMG_NBR;
  const int i0 = blockIdx.x * 64, j0 = blockIdx.y * 64;  // tile of W_b (rows i, cols j)
  const int r = threadIdx.x & 63, c4 = threadIdx.x >> 6;
#pragma unroll 4
  for (int c = c4; c < 64; c += 4) t[c][r] = w512[b0 + i0 + r + (size_t)(j0 + c) * n];
  __syncthreads();
#pragma unroll 4
  for (int c = c4; c < 64; c += 4)  // V(b0 + j0 + r, b0 + i0 + c) = W_b(i0 + c, j0 + r)
    V[b0 + j0 + r + (size_t)(b0 + i0 + c) * ldv] = t[r][c];
}

// the leaves of V[lo:hi, lo:hi] and, when (hi - lo) / 512 is a power of two
// (the recursion's 1024-row nodes are then the aligned leaf pairs), every
// pair's V12 = -V11 L21^T V22 as two strided-batched products (T: ld n);
// returns whether the pairs were formed
int inv_t_leaves(smg_ctx* ctx, const double* L, int ldl, const double* w512, int n, int lo, int hi, double* V,
                 int ldv, double* T, bool* pairs) {
  const int nl = (hi - lo) / SMG_NBR;
  hipLaunchKernelGGL(k_leaf_transpose, dim3(SMG_NBR / 64, SMG_NBR / 64, nl), dim3(256), 0, ctx->stream, w512, n, lo,
                     V, ldv);
  SMG_LAUNCH_CHECK();
  *pairs = (nl & (nl - 1)) == 0 && nl >= 2;
  if (!*pairs) return SMG_OK;
  const int np = nl / 2, b = SMG_NBR;
  const long long sv = 2LL * b * (1 + (long long)ldv), sl = 2LL * b * (1 + (long long)ldl);
  const double* V0 = V + lo + (size_t)lo * ldv;
  const double* L0 = L + lo + (size_t)lo * ldl;
  // T_p (b x b, rows p b of T, ld n) = V11_p L21_p^T
  int rc = smg_gemm_batched_impl(ctx, 0, 1, b, b, b, 1.0, V0, ldv, sv, L0 + b, ldl, sl, 0.0, T, n, b, np);
  if (rc) return rc;
  // V12_p = -T_p V22_p
  return smg_gemm_batched_impl(ctx, 0, 0, b, b, b, -1.0, T, n, b, V0 + b + (size_t)b * ldv, ldv, sv, 0.0,
                               V + lo + (size_t)(lo + b) * ldv, ldv, sv, np);
}

// Abar(i, j) += adj ((sum_o s_oi s_oj - k C_ij) * (i == j ? 1/2 : 1)), i >= j,
// C lower; s_o = s + o * ss (k observations); the column form of
// k_add_lower_col2 (16-byte accesses, whole columns per workgroup, only the
// row pairs at or below the diagonal touched)
__global__ __launch_bounds__(256) void k_chol_mvn_adj_col2(const double* __restrict__ C, int ldc, int n,
                                                          const double* __restrict__ s, int k, long long ss,
                                                          double adj, double* __restrict__ A, int lda) {
  const int np = n >> 1;
  const double kc = adj * k;
  for (int j = blockIdx.x; j < n; j += gridDim.x) {
    const double2* c = reinterpret_cast<const double2*>(C + (size_t)j * ldc);
    double2* a = reinterpret_cast<double2*>(A + (size_t)j * lda);
    const int p1 = j >> 1;  // first pair holding a row >= j
    for (int p0 = p1 + threadIdx.x; p0 < np; p0 += 4 * 256) {
      double2 cv[4], av[4], gv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int p = p0 + 256 * q;
        gv[q] = double2{0.0, 0.0};
        if (p < np) {
          cv[q] = c[p];
          av[q] = a[p];
        }
      }
      for (int o = 0; o < k; ++o) {
        const double* so = s + o * ss;
        const double2* s2 = reinterpret_cast<const double2*>(so);
        const double sj = adj * so[j];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int p = p0 + 256 * q;
          if (p < np) {
            const double2 sv = s2[p];
            gv[q].x += sv.x * sj;
            gv[q].y += sv.y * sj;
          }
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int p = p0 + 256 * q;
        if (p < np) {
          const int r = 2 * p;
          const double gx = gv[q].x - kc * cv[q].x;
          const double gy = gv[q].y - kc * cv[q].y;
          if (r > j) av[q].x += gx;
          else if (r == j) av[q].x += 0.5 * gx;
          if (r + 1 > j) av[q].y += gy;  // row 2p + 1 >= j for every p >= j / 2
          else av[q].y += 0.5 * gy;
          a[p] = av[q];
        }
      }
    }
  }
}

__global__ void k_chol_mvn_adj(const double* __restrict__ C, int ldc, int n, const double* __restrict__ s, int k,
                               long long ss, double adj, double* __restrict__ A, int lda) {
  for (smg_mn it(n, n); it.ok(); it.next()) {
    const int i = it.i, j = it.j;
    if (i < j) continue;
    double g = 0.0;
    for (int o = 0; o < k; ++o) g += s[o * ss + i] * s[o * ss + j];
    g = adj * (g - k * C[i + (size_t)j * ldc]);
    A[i + (size_t)j * lda] += (i == j) ? 0.5 * g : g;
  }
}

// The GP marginal's three reverses in one pass (gp_inverse_adjoint below):
// per workgroup partials [sum_i g_ii, sum_{i>=j} g_ij K0_ij, sum_{i>j} g_ij
// K0_ij d2_ij] with g = Phi(sum_o s_o s_o^T - k C) (adj factored out).  A
// workgroup takes the column pair (j, n - 1 - j) (balanced: n + 1 rows), its
// threads the rows at or below the diagonal; PAIRS: two rows per thread with
// 16-byte loads (even n, 16-byte aligned operands, D == 1).
template <bool PAIRS>
__global__ __launch_bounds__(256) void k_gp_inv_reduce(const double* __restrict__ C, int ldc, int n,
                                                      const double* __restrict__ s, int k, long long ss,
                                                      const double* __restrict__ K0, int ldk,
                                                      const double* __restrict__ x, int D,
                                                      double* __restrict__ part) {
  __shared__ double lds[16];
  double sd = 0.0, sa = 0.0, sl = 0.0;
  const int half = (n + 1) / 2;
  for (int b = blockIdx.x; b < half; b += gridDim.x) {
    for (int h = 0; h < 2; ++h) {
      const int j = h == 0 ? b : n - 1 - b;
      if (h == 1 && j == b) break;
      const double* c = C + (size_t)j * ldc;
      const double* kc = K0 + (size_t)j * ldk;
      if (PAIRS) {
        const double xj = x[j];
        double sjs[4];
        for (int o = 0; o < k && o < 4; ++o) sjs[o] = s[o * ss + j];
        const double2* c2 = reinterpret_cast<const double2*>(c);
        const double2* k2 = reinterpret_cast<const double2*>(kc);
        const double2* x2 = reinterpret_cast<const double2*>(x);
        for (int p = (j >> 1) + threadIdx.x; p < (n >> 1); p += 256) {
          const double2 cv = c2[p], kv = k2[p], xv = x2[p];
          double g0 = 0.0, g1 = 0.0;
          for (int o = 0; o < k; ++o) {
            const double2 sv = reinterpret_cast<const double2*>(s + o * ss)[p];
            const double sj = o < 4 ? sjs[o] : s[o * ss + j];
            g0 += sv.x * sj;
            g1 += sv.y * sj;
          }
          g0 -= k * cv.x;
          g1 -= k * cv.y;
          const int i = 2 * p;
          if (i > j) {
            const double d = xv.x - xj;
            const double t = g0 * kv.x;
            sa += t;
            sl += t * (d * d);
          } else if (i == j) {
            sd += 0.5 * g0;
            sa += 0.5 * g0 * kv.x;
          }
          if (i + 1 > j) {
            const double d = xv.y - xj;
            const double t = g1 * kv.y;
            sa += t;
            sl += t * (d * d);
          } else {  // i + 1 == j
            sd += 0.5 * g1;
            sa += 0.5 * g1 * kv.y;
          }
        }
      } else {
        for (int i = j + threadIdx.x; i < n; i += 256) {
          double g = 0.0;
          for (int o = 0; o < k; ++o) g += s[o * ss + i] * s[o * ss + j];
          g -= k * c[i];
          if (i == j) {
            sd += 0.5 * g;
            sa += 0.5 * g * kc[i];
          } else {
            double d2 = 0.0;
            for (int d = 0; d < D; ++d) {
              const double t = x[(size_t)i * D + d] - x[(size_t)j * D + d];
              d2 += t * t;
            }
            const double t = g * kc[i];
            sa += t;
            sl += t * d2;
          }
        }
      }
    }
  }
  sd = block_sum(sd, lds);
  __syncthreads();
  sa = block_sum(sa, lds);
  __syncthreads();
  sl = block_sum(sl, lds);
  if (threadIdx.x == 0) {
    part[3 * blockIdx.x + 0] = sd;
    part[3 * blockIdx.x + 1] = sa;
    part[3 * blockIdx.x + 2] = sl;
  }
}

// the fixed-order sum of k_gp_inv_reduce's partials: dadj = adj sum g_ii
// (add_diag's d'), out2 = [2 adj sa / sigma, adj sl / l^3]
// (rev/mat/fun/gp_exp_quad_cov.hpp:109-110)
__global__ void k_gp_inv_final(const double* __restrict__ part, int nparts, double adj, double sigma, double l,
                               double* dadj, double* out2) {
  __shared__ double lds[16];
  double sd = 0.0, sa = 0.0, sl = 0.0;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) {
    sd += part[3 * i];
    sa += part[3 * i + 1];
    sl += part[3 * i + 2];
  }
  sd = block_sum(sd, lds);
  __syncthreads();
  sa = block_sum(sa, lds);
  __syncthreads();
  sl = block_sum(sl, lds);
  if (threadIdx.x == 0) {
    if (dadj) dadj[0] = adj * sd;
    if (out2) {
      out2[0] = adj * sa * 2 / sigma;
      out2[1] = adj * sl / (l * l * l);
    }
  }
}

// Aadj (lower) += G + G^T below the diagonal and G_ii on it: one 64 x 64
// tile of the lower triangle per workgroup, the mirror tile G(j0.., i0..)
// read column-coalesced and transposed through LDS
__global__ __launch_bounds__(256) void k_add_lower_sym(const double* __restrict__ G, int ldg, int n,
                                                      double* __restrict__ A, int lda) {
  const int bx = blockIdx.x, by = blockIdx.y;  // tile rows bx, cols by
  if (bx < by) return;
  __shared__ double t[64][65];
  const int i0 = bx * 64, j0 = by * 64;
  const int r = threadIdx.x & 63, c4 = threadIdx.x >> 6;
#pragma unroll 4
  for (int c = c4; c < 64; c += 4) {  // t[r][c] = G(j0 + r, i0 + c) = G^T(i0 + c, j0 + r)
    const int i = j0 + r, j = i0 + c;
    t[r][c] = (i < n && j < n) ? G[i + (size_t)j * ldg] : 0.0;
  }
  __syncthreads();
#pragma unroll 4
  for (int c = c4; c < 64; c += 4) {
    const int i = i0 + r, j = j0 + c;
    if (i < n && j < n && i >= j) {
      double v = G[i + (size_t)j * ldg];
      if (i != j) v += t[c][r];
      A[i + (size_t)j * lda] += v;
    }
  }
}

// P = Phi(P) in place over a lower-output product: the diagonal halved, the
// strict upper (never written by the product: stale workspace) zeroed, since
// the next product's triangular K cut still reads whole diagonal tiles
__global__ void k_phi_upper(double* __restrict__ P, int ldp, int n) {
  for (int j = blockIdx.x; j < n; j += gridDim.x) {
    double* c = P + (size_t)j * ldp;
    for (int i = threadIdx.x; i <= j; i += blockDim.x) c[i] = i == j ? 0.5 * c[i] : 0.0;
  }
}

inline int grid_for(long long tot) {
  long long g = (tot + 255) / 256;
  return (int)(g < 4096 ? (g < 1 ? 1 : g) : 4096);
}

// V = L^{-T} (n % 512 == 0, n >= 1024, with the factorisation's aux)
// (V[lo:hi, lo:hi] only: the diagonal block of rows lo..hi)
int form_v(smg_ctx* ctx, const double* L, int ldl, const double* aux, int n, double* V, double* T, int lo = 0,
           int hi = -1) {
  if (hi < 0) hi = n;
  const double* w512 = aux + (size_t)n * SMG_AUX_W512;
  bool pairs = false;
  int rc = inv_t_leaves(ctx, L, ldl, w512, n, lo, hi, V, n, T, &pairs);
  if (!rc) rc = inv_t_rec(ctx, L, ldl, w512, n, V, n, T, lo, hi, pairs);
  return rc;
}

bool v_by_doubling(int n, const double* aux) { return n % SMG_NBR == 0 && n >= 2 * SMG_NBR && aux; }

// Abar (lower) += adj Phi(sum_o s_o s_o^T - k C), C = K^{-1} lower
int mvn_adj_epilogue(smg_ctx* ctx, const double* C, int n, const double* s, int k, long long ss, double adj,
                     double* Aadj, int ldaa) {
  if (n % 2 == 0 && ldaa % 2 == 0 && ss % 2 == 0 &&
      ((reinterpret_cast<uintptr_t>(Aadj) | reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(C)) & 15) ==
          0)
    hipLaunchKernelGGL(k_chol_mvn_adj_col2, dim3(n < 2048 ? n : 2048), dim3(256), 0, ctx->stream, C, n, n, s, k, ss,
                       adj, Aadj, ldaa);
  else
    hipLaunchKernelGGL(k_chol_mvn_adj, dim3(grid_for((long long)n * n)), dim3(256), 0, ctx->stream, C, n, n, s, k, ss,
                       adj, Aadj, ldaa);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

}  // namespace

// K^{-1} formed progressively during the factorisation (cholesky.hip
// chol_fwd), one 512-row block row k of W = L^{-1} at a time, once panel k is
// final:
//   W_kk = L_kk^{-1}                        (the block inverses of rows k P.., P = 512)
//   W_{k,0:k} = -W_kk Y_k,  Y_k = L_{k,0:k} W_{0:k,0:k}
//   C(0:(k+1)P, 0:(k+1)P) += W_k^T W_k      (C = K^{-1} = W^T W = sum_k W_k^T W_k, lower)
// Y is accumulated right-looking, like the factorisation's trailing updates:
// once W_k is formed, its contribution L_{r,k} W_{k,0:k+1} is added to every
// later row's Y_r -- the next row's (r = k + 1, small: on the latency chain)
// and the rest (r >= k + 2, the bulk: off it) as separate parts -- so that
// after the last panel only its own block row remains (its inverse, -W_77 Y_7
// and one rank-512 share), instead of forming Y_7 = L_{7,0:7} W_{0:7,0:7}
// (6.6 GFLOP at n = 4096) there.
// Parts of block row k: 0 W_kk; 1 W_{k,0:k}; 2 its K^{-1} share; 3 Y_{k+1} +=
// L_{k+1,k} W_k; 4 Y_{k+2:} += L_{k+2:,k} W_k (part 1 of row r needs parts 3
// of row r - 1 and 4 of rows <= r - 2).
// ws: [W (n x n, ld n) | C (n x n, lower) | Y (n x n, ld n; block row r's
// columns 0 .. r P) | T (P/2 x 256)]; W's strict upper is never read outside
// its diagonal blocks (the triangular K cuts stay inside a tile band), whose
// copies from aux carry stored zeros.
bool smg_inv_prog_ok(int n) { return n % SMG_NBR == 0 && n >= 2 * SMG_NBR; }

// C and Y accumulate without a zeroing beforehand: C's rows k P .. (k+1) P
// (lower) first receive row k's share, Y's column block k (every row r > k)
// first receives row k's parts 3 / 4, so those products take beta = 0 from
// that row / column on (smg_gemm_bz_impl) and beta = 1 before it.  Zeroing
// the 2 n^2 doubles instead put 268 MB of stores beside the first panel
// (GP 356-362 -> 365-368 evals/s without it).
int smg_inv_prog_init(smg_ctx* ctx, int n, double* ws) {
  (void)ctx;
  (void)n;
  (void)ws;
  return SMG_OK;
}

// the accumulated products of the parts: beta = 1 before the boundary bz
// (rows bz > 0 / columns -bz < 0), 0 from it on; k = 0 has no earlier terms
static int prog_acc(smg_ctx* ctx, int ta, int uplo, int m, int nc, int kk, const double* A, int lda,
                    const double* B, int ldb, double* C, int ldc, int bz, bool first) {
  if (first) return smg_gemm_impl(ctx, ta, 0, uplo, m, nc, kk, 1.0, A, lda, B, ldb, 0.0, C, ldc);
  return smg_gemm_bz_impl(ctx, ta, 0, uplo, m, nc, kk, 1.0, A, lda, B, ldb, 1.0, C, ldc, 0, bz);
}

int smg_inv_prog_row(smg_ctx* ctx, const double* L, int ldl, double* aux, int n, double* ws, int k, int part,
                     bool inverses_here) {
  constexpr int P = SMG_NBR;
  const size_t nn = (size_t)n * n;
  double* W = ws;
  double* C = ws + nn;
  double* Y = C + nn;
  double* T = Y + nn;
  const int r0 = k * P, r1 = r0 + P;
  const double* Wkk = aux + (size_t)n * SMG_AUX_W512 + r0;  // ld n, stored zeros above
  int rc;
  switch (part) {
    case 0:  // W_kk (the block row's 128/256/512 inverses first when asked)
      if (inverses_here) {  // (the solves after the factorisation wait for them: inv_ev_aux)
        bool wrote = false;  // (the one-launch inverse writes W_kk into W itself)
        if ((rc = smg_block_inverses_rows(ctx, L, ldl, aux, n, r0, P, T, W + r0 + (size_t)r0 * n, &wrote)))
          return rc;
        SMG_HIP_TRY(hipEventRecord(ctx->inv_ev_aux, ctx->stream));
        if (wrote) return SMG_OK;
      }
      return smg_copy_impl(ctx, P, P, Wkk, n, W + r0 + (size_t)r0 * n, n, 1.0, 0);
    case 1:  // W_{k,0:k} = -W_kk Y_k
      if (k == 0) return SMG_OK;
      return smg_gemm_impl(ctx, 0, 0, 0, P, r0, P, -1.0, Wkk, n, Y + r0, n, 0.0, W + r0, n, SMG_TRI_A_LOWER);
    case 2:  // C (lower, leading r1 x r1) += W_k^T W_k (rows r0.. first written here)
      return prog_acc(ctx, 1, 1, r1, r1, P, W + r0, n, W + r0, n, C, n, r0, k == 0);
    case 3:  // Y_{k+1}[:, 0:r1] (+)= L_{k+1,k} W_{k,0:r1}
      if (r1 >= n) return SMG_OK;
      return prog_acc(ctx, 0, 0, P, r1, P, L + r1 + (size_t)r0 * ldl, ldl, W + r0, n, Y + r1, n, -r0, k == 0);
    default:  // Y_{k+2:}[:, 0:r1] (+)= L_{k+2:,k} W_{k,0:r1}
      if (r1 + P >= n) return SMG_OK;
      return prog_acc(ctx, 0, 0, n - r1 - P, r1, P, L + r1 + P + (size_t)r0 * ldl, ldl, W + r0, n, Y + r1 + P, n, -r0,
                      k == 0);
  }
}

// device time of part `part` of block row k, us: flops at the rate these
// products reach beside the panels (~30 TF/s; tools/ubench_gemm's shapes
// run at 33-46 alone) plus ~6 us per launch
double smg_inv_prog_cost(int n, int k, int part, bool inverses_here) {
  constexpr double P = SMG_NBR, rate = 30e6;  // flop per us
  const double r0 = k * P, r1 = r0 + P;
  switch (part) {
    case 0: return inverses_here ? 60.0 : 6.0;
    case 1: return k == 0 ? 0.0 : 6.0 + P * r0 * P / rate;
    case 2: return 6.0 + r1 * r1 * P / rate;
    case 3: return r1 >= n ? 0.0 : 6.0 + 2.0 * P * r1 * P / rate;
    default: return r1 + P >= n ? 0.0 : 6.0 + 2.0 * (n - r1 - P) * r1 * P / rate;
  }
}

extern "C" {

size_t smg_cholesky_mvn_rev_ws_doubles(int n) {
  return n > 0 ? 3 * (size_t)n * n + SMG_NBR / 2 * 256 : 0;
}

int smg_cholesky_mvn_rev(smg_ctx* ctx, const double* L, int ldl, const double* aux, int n, const double* s, int k,
                         long long s_stride, double adj, double* Aadj, int ldaa, double* ws) {
  if (!ctx || n < 0 || k < 1 || (k > 1 && s_stride < n)) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  if (!L || !ws || ldl < n || (Aadj && (!s || ldaa < n))) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_CHOL_REV);
  const size_t nn = (size_t)n * n;
  double* V = ws;       // L^{-T} (upper), or W = L^{-1} on the general path
  double* C = ws + nn;  // K^{-1} (lower); the doubling's T before that
  int rc;
  if (v_by_doubling(n, aux)) {
    if ((rc = form_v(ctx, L, ldl, aux, n, V, C))) return rc;
    // C = V V^T, lower: op(A) = V upper, op(B) = V^T lower
    rc = smg_gemm_impl(ctx, 0, 1, 1, n, n, n, 1.0, V, n, V, n, 0.0, C, n, SMG_TRI_A_UPPER | SMG_TRI_B_LOWER);
  } else {  // any n: W = L^{-1} by the blocked solve, C = W^T W
    if ((rc = smg_memset(ctx, V, 0, sizeof(double) * nn))) return rc;
    if ((rc = smg_add_diag_fwd(ctx, V, n, n, 1.0, nullptr, V, n))) return rc;  // W = I
    if ((rc = smg_trsm_impl(ctx, 1, 0, L, ldl, nullptr, 0, V, n, n, n, nullptr, 0, aux))) return rc;
    rc = smg_gemm_impl(ctx, 1, 0, 1, n, n, n, 1.0, V, n, V, n, 0.0, C, n, SMG_TRI_A_UPPER | SMG_TRI_B_LOWER);
  }
  if (rc) return rc;
  if (!Aadj) return SMG_OK;  // K^{-1} only (the GP's fused reverse reads it)
  return mvn_adj_epilogue(ctx, C, n, s, k, s_stride, adj, Aadj, ldaa);
}

// cholesky_decompose's reverse for ANY factor adjoint Lbar in closed form on
// the factor's inverse W = L^{-1} (rev/mat/fun/cholesky_decompose.hpp:118-166
// computes the same by Murray's blocked algorithm):
//   P = Phi(L^T tril(Lbar)),  G = W^T P W,  Abar (lower) += tril(G + G^T)
//   with G_ii on the diagonal
// from <Lbar, dL> = <Phi(L^T Lbar), L^{-1} dA L^{-T}> (dL = L Phi(L^{-1} dA
// L^{-T})).  4 n^3 / 3 flops in three large triangular-operand products
// (P: n^3/3, T = P W: n^3/3, G = W^T T: 2 n^3/3) instead of Murray's 2 n^3 / 3
// in ~n/64 dependent rounds.  ws: 2 n^2 doubles.
int smg_cholesky_rev_inverse(smg_ctx* ctx, const double* L, int ldl, const double* W, const double* Wt, int ldw,
                             const double* La, int ldla, int n, double* Aadj, int ldaa, double* ws) {
  if (!ctx || n < 0) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  if (!L || !W || !Wt || !La || !Aadj || !ws || ldl < n || ldw < n || ldla < n || ldaa < n) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_CHOL_REV);
  const size_t nn = (size_t)n * n;
  double* P = ws;
  double* T = ws + nn;
  int rc;
  // T = tril(Lbar) (stored zeros above: the products' triangular K cuts read whole tiles)
  if ((rc = smg_copy_tril(ctx, n, n, La, ldla, T, n))) return rc;
  // P = Phi(L^T T) (lower): op(A) = L^T upper, op(B) = T lower
  if ((rc = smg_gemm_impl(ctx, 1, 0, 1, n, n, n, 1.0, L, ldl, T, n, 0.0, P, n, SMG_TRI_A_UPPER | SMG_TRI_B_LOWER)))
    return rc;
  hipLaunchKernelGGL(k_phi_upper, dim3(n < 2048 ? n : 2048), dim3(256), 0, ctx->stream, P, n, n);
  SMG_LAUNCH_CHECK();
  // T = P W (lower x lower: lower; T's strict upper keeps tril's zeros)
  if ((rc = smg_gemm_impl(ctx, 0, 0, 1, n, n, n, 1.0, P, n, W, ldw, 0.0, T, n, SMG_TRI_A_LOWER | SMG_TRI_B_LOWER)))
    return rc;
  // G = W^T T (upper x lower: full) into P
  if ((rc = smg_gemm_impl(ctx, 0, 0, 0, n, n, n, 1.0, Wt, ldw, T, n, 0.0, P, n, SMG_TRI_A_UPPER | SMG_TRI_B_LOWER)))
    return rc;
  const int tb = smg_ceil_div(n, 64);
  hipLaunchKernelGGL(k_add_lower_sym, dim3(tb, tb), dim3(256), 0, ctx->stream, P, n, n, Aadj, ldaa);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_cholesky_inverse_adjoint(smg_ctx* ctx, const double* C, int ldc, int n, const double* s, int k,
                                 long long s_stride, double adj, double* Aadj, int ldaa) {
  if (!ctx || n < 0 || k < 1 || (k > 1 && s_stride < n)) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  if (!C || !s || !Aadj || ldc != n || ldaa < n) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_CHOL_REV);
  return mvn_adj_epilogue(ctx, C, n, s, k, s_stride, adj, Aadj, ldaa);
}

int smg_gp_inverse_adjoint(smg_ctx* ctx, const double* C, int ldc, int n, const double* s, int k,
                           long long s_stride, double adj, const double* K0, int ldk, const double* x, int D,
                           double sigma, double l, double* dadj, double* out2) {
  if (!ctx || n < 0 || k < 1 || (k > 1 && s_stride < n) || D < 1) return SMG_ERR_ARG;
  if (n == 0) {
    if (dadj || out2) {
      const double z[2] = {0.0, 0.0};
      if (dadj) SMG_HIP_TRY(hipMemcpyAsync(dadj, z, sizeof(double), hipMemcpyHostToDevice, ctx->stream));
      if (out2) SMG_HIP_TRY(hipMemcpyAsync(out2, z, 2 * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
      SMG_HIP_TRY(hipStreamSynchronize(ctx->stream));
    }
    return SMG_OK;
  }
  if (!out2) {  // the diagonal sum alone: K0 and x unused (any readable n x n / n operands)
    if (!K0) K0 = C, ldk = ldc;
    if (!x) x = s, D = 1;
  }
  if (!C || !s || !K0 || !x || ldc < n || ldk < n || (out2 && !(sigma > 0 && l > 0))) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_GP);
  const int half = (n + 1) / 2;
  const int nb = half < 2048 ? half : 2048;
  double* part = smg_ws(ctx, SMG_WS_RED, 3 * (size_t)nb);
  if (!part) return SMG_ERR_OOM;
  const bool pairs = D == 1 && n % 2 == 0 && ldc % 2 == 0 && ldk % 2 == 0 && (k == 1 || s_stride % 2 == 0) &&
                     ((reinterpret_cast<uintptr_t>(C) | reinterpret_cast<uintptr_t>(s) |
                       reinterpret_cast<uintptr_t>(K0) | reinterpret_cast<uintptr_t>(x)) & 15) == 0;
  if (pairs)
    hipLaunchKernelGGL(k_gp_inv_reduce<true>, dim3(nb), dim3(256), 0, ctx->stream, C, ldc, n, s, k, s_stride, K0, ldk,
                       x, D, part);
  else
    hipLaunchKernelGGL(k_gp_inv_reduce<false>, dim3(nb), dim3(256), 0, ctx->stream, C, ldc, n, s, k, s_stride, K0,
                       ldk, x, D, part);
  hipLaunchKernelGGL(k_gp_inv_final, dim3(1), dim3(1024), 0, ctx->stream, part, nb, adj, sigma, l, dadj, out2);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_cholesky_inv_t_async(smg_ctx* ctx, const double* L, int ldl, const double* aux, int n, double* ws,
                             int early_done, int* started) {
  if (!ctx || n < 0 || !started) return SMG_ERR_ARG;
  *started = 0;
  if (n == 0 || !v_by_doubling(n, aux)) return SMG_OK;
  if (early_done) {  // K^{-1} already queued by the factorisation (its inv_ev joins it)
    *started = 1;
    return SMG_OK;
  }
  if (!L || !ws || ldl < n) return SMG_ERR_ARG;
  if (int rc = smg_side_begin(ctx)) return rc;
  if (int rc = smg_inv_events(ctx)) return rc;
  // L and its block inverses are complete once the main stream's queued work is
  SMG_HIP_TRY(hipEventRecord(ctx->inv_ev_main, ctx->stream));
  SMG_HIP_TRY(hipStreamWaitEvent(ctx->side, ctx->inv_ev_main, 0));
  int rc;
  {
    smg_on_side on(ctx);  // V only: K^{-1} in the reverse (formed here it measured no faster)
    rc = form_v(ctx, L, ldl, aux, n, ws, ws + (size_t)n * n);
  }
  if (rc) return rc;
  SMG_HIP_TRY(hipEventRecord(ctx->inv_ev, ctx->side));
  ctx->inv_pending = 1;
  *started = 1;
  return SMG_OK;
}

int smg_cholesky_mvn_rev_v(smg_ctx* ctx, int n, const double* s, int k, long long s_stride, double adj, double* Aadj,
                           int ldaa, double* ws, int c_formed) {
  if (!ctx || n < 0 || k < 1 || (k > 1 && s_stride < n)) return SMG_ERR_ARG;
  if (n == 0) return SMG_OK;
  if (!ws || (Aadj && (!s || ldaa < n))) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_CHOL_REV);
  if (ctx->inv_pending) {
    SMG_HIP_TRY(hipStreamWaitEvent(ctx->stream, ctx->inv_ev, 0));
    ctx->inv_pending = 0;
  }
  const size_t nn = (size_t)n * n;
  double* C = ws + nn;
  if (!c_formed) {
    int rc = smg_gemm_impl(ctx, 0, 1, 1, n, n, n, 1.0, ws, n, ws, n, 0.0, C, n, SMG_TRI_A_UPPER | SMG_TRI_B_LOWER);
    if (rc) return rc;
  }
  if (!Aadj) return SMG_OK;  // K^{-1} only
  return mvn_adj_epilogue(ctx, C, n, s, k, s_stride, adj, Aadj, ldaa);
}

}  // extern "C"
