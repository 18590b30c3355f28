// Dense kernels on ONE 64 x 64 diagonal block held in LDS by one 256-thread
// workgroup (4 waves).  Shared by the Cholesky forward / reverse and the
// blocked triangular solves.
//
// Layout: row-major [r][c] with stride SMG_NBP = 65 doubles.
// Latency structure (the block is on the critical path of every blocked
// algorithm, so latency, not throughput, is what matters here):
//   * 16 x 16 leaves live in the registers of ONE wave (lane i = row i or
//     column i); broadcasts are v_readlane_b32 pairs, no LDS round trips;
//   * everything between leaves is a 64 x 64 (or smaller) product on the
//     fp64 matrix cores (v_mfma_f64_16x16x4_f64), 4 waves x 4 tiles.
#pragma once
#include "smg_internal.h"

constexpr int SMG_NB = 64;           // diagonal block size of every blocked kernel
constexpr int SMG_NB2 = 256;         // outer block of the blocked triangular solves
constexpr int SMG_NBR = 512;         // outer block of the two-level Cholesky reverse
#ifndef SMG_NBF_COLS
#define SMG_NBF_COLS 512
#endif
constexpr int SMG_NBF = SMG_NBF_COLS;  // panel width of the two-level Cholesky forward
// cholesky aux layout (n rows each, ld n): inverses of the 64-, 128-, 256-
// and 512-row diagonal blocks of L
constexpr int SMG_AUX_W128 = SMG_NB;
constexpr int SMG_AUX_W256 = SMG_NB + 128;
constexpr int SMG_AUX_W512 = SMG_NB + 128 + 256;
constexpr int SMG_AUX_COLS = SMG_NB + 128 + 256 + 512;
constexpr int SMG_NBP = SMG_NB + 1;  // padded LDS row stride
constexpr int SMG_DIAG_THREADS = 512;  // threads of the fused diagonal-block kernels

__device__ __forceinline__ double bcast(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

// C (64x64) = alpha * op(A) op(B) + beta * C, all LDS [r][c] stride 65.
// Safe when C aliases A or B (barrier between the MFMA loop and the store).
// Every thread of the workgroup must call it.
template <bool TA, bool TB>
__device__ inline void lds_mma64(double* C, const double* A, const double* B, double alpha,
                                 double beta) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int fr = l & 15, fk = l >> 4;
  d4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
  for (int k0 = 0; k0 < SMG_NB; k0 += 4) {
    const int kk = k0 + fk;
    const int i = 16 * w + fr;
    const double a = TA ? A[kk * SMG_NBP + i] : A[i * SMG_NBP + kk];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int j = 16 * t + fr;
      const double b = TB ? B[j * SMG_NBP + kk] : B[kk * SMG_NBP + j];
      acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[t], 0, 0, 0);
    }
  }
  __syncthreads();
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 16 * w + fk + 4 * r, j = 16 * t + fr;
      double* c = &C[i * SMG_NBP + j];
      *c = beta == 0.0 ? alpha * acc[t][r] : alpha * acc[t][r] + beta * *c;
    }
  __syncthreads();
}

// C (64x64) = alpha op(A) op(B) + beta C with NW = 8 waves: wave w owns row
// stripe w & 3 and column tiles 2 (w >> 2) .. +1.  Safe when C aliases A or B.
template <bool TA, bool TB, typename P = double*, typename CP = const double*>
__device__ inline void lds_mma64_8w(P C, CP A, CP B, double alpha = 1.0, double beta = 0.0) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int fr = l & 15, fk = l >> 4;
  const int i = 16 * (w & 3) + fr, t0 = 2 * (w >> 2);
  d4 acc[2];
  acc[0] = d4{0.0, 0.0, 0.0, 0.0};
  acc[1] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
  for (int k0 = 0; k0 < SMG_NB; k0 += 4) {
    const int kk = k0 + fk;
    const double a = TA ? A[kk * SMG_NBP + i] : A[i * SMG_NBP + kk];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int j = 16 * (t0 + t) + fr;
      const double b = TB ? B[j * SMG_NBP + kk] : B[kk * SMG_NBP + j];
      acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[t], 0, 0, 0);
    }
  }
  __syncthreads();
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      auto c = &C[(16 * (w & 3) + fk + 4 * r) * SMG_NBP + 16 * (t0 + t) + fr];
      *c = beta == 0.0 ? alpha * acc[t][r] : alpha * acc[t][r] + beta * *c;
    }
  __syncthreads();
}

// The 32-row tiles below a panel: C = alpha A B^T + beta C with A, C 32 x 64
// (rows 0 .. 31 of the 64-row LDS layout), B 64 x 64.  8 waves: wave w owns
// row stripe w & 1 and column tile w >> 1 (one accumulator; the SIMD's two
// waves interleave).  Each element's k order is lds_mma64_8w's.  Safe when C
// aliases A.
template <typename P, typename CP>
__device__ inline void lds_mma32_8w(P C, CP A, CP B, double alpha = 1.0, double beta = 0.0) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int fr = l & 15, fk = l >> 4;
  const int i = 16 * (w & 1) + fr, j = 16 * (w >> 1) + fr;
  d4 acc = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
  for (int k0 = 0; k0 < SMG_NB; k0 += 4) {
    const int kk = k0 + fk;
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[i * SMG_NBP + kk], B[j * SMG_NBP + kk], acc, 0, 0, 0);
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    auto c = &C[(16 * (w & 1) + fk + 4 * r) * SMG_NBP + 16 * (w >> 1) + fr];
    *c = beta == 0.0 ? alpha * acc[r] : alpha * acc[r] + beta * *c;
  }
  __syncthreads();
}

// This wave's 16 x 16 tile of the 32 x 64 product A B^T (A: 32 x 64, B:
// 64 x 64 in LDS), returned in the accumulator layout lds_mma32_8w stores:
// lane l of wave w holds rows 16 (w & 1) + (l >> 4) + 4 r, column
// 16 (w >> 1) + (l & 15).  No barrier: the caller owns the ordering.
template <typename CP>
__device__ inline d4 lds_mma32_8w_acc(CP A, CP B) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int fr = l & 15, fk = l >> 4;
  const int i = 16 * (w & 1) + fr, j = 16 * (w >> 1) + fr;
  d4 acc = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
  for (int k0 = 0; k0 < SMG_NB; k0 += 4) {
    const int kk = k0 + fk;
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[i * SMG_NBP + kk], B[j * SMG_NBP + kk], acc, 0, 0, 0);
  }
  return acc;
}

// The panel chain's next diagonal block: C = C - A A^T (A, C: 64 x 64 in
// LDS), written straight in the factorisation's input form -- lower triangle,
// zero strict upper, identity padding beyond row / column b -- so no separate
// pass over C follows
template <typename P, typename CP>
__device__ inline void lds_syrk64_8w_next(P C, CP A, int b) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int fr = l & 15, fk = l >> 4;
  const int i = 16 * (w & 3) + fr, t0 = 2 * (w >> 2);
  d4 acc[2];
  acc[0] = d4{0.0, 0.0, 0.0, 0.0};
  acc[1] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
  for (int k0 = 0; k0 < SMG_NB; k0 += 4) {
    const int kk = k0 + fk;
    const double a = A[i * SMG_NBP + kk];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int j = 16 * (t0 + t) + fr;
      acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, A[j * SMG_NBP + kk], acc[t], 0, 0, 0);
    }
  }
  __syncthreads();
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * (w & 3) + fk + 4 * r, col = 16 * (t0 + t) + fr;
      auto c = &C[row * SMG_NBP + col];
      *c = col > row ? 0.0 : (row == col && row >= b ? 1.0 : *c - acc[t][r]);
    }
  __syncthreads();
}

// One wave: Cholesky of the 16x16 leaf p of D (lower), then its inverse into X.
// Latches SMG_ERR_NOT_PD (check_pos_definite, prim/mat/err/check_pos_definite.hpp:77-81).
__device__ inline void wave_leaf_potrf_inv(double* D, double* X, int p, int* status) {
  const int l = threadIdx.x & 63;
  const int r0 = 16 * p;
  const int lr = l < 16 ? l : 15;
  double a[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) a[c] = D[(r0 + lr) * SMG_NBP + r0 + c];
  bool bad = false;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const double piv = bcast(a[j], j);
    const bool ok = piv > 0.0 && isfinite(piv);
    bad |= !ok;
    const double ljj = ok ? sqrt(piv) : 1.0;
    const double inv = 1.0 / ljj;
    const double lij = (l == j) ? ljj : a[j] * inv;
    a[j] = lij;
#pragma unroll
    for (int c = j + 1; c < 16; ++c) a[c] -= lij * bcast(lij, c);
  }
  if (bad && l == 0) atomicOr(status, (int)SMG_ERR_NOT_PD);
  // inverse: lane l owns column l of X (forward substitution on e_l)
  double x[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    double s = (l == r) ? 1.0 : 0.0;
#pragma unroll
    for (int t = 0; t < r; ++t) s -= bcast(a[t], r) * x[t];
    x[r] = s / bcast(a[r], r);
  }
  if (l < 16) {
#pragma unroll
    for (int c = 0; c < 16; ++c) D[(r0 + l) * SMG_NBP + r0 + c] = c <= l ? a[c] : 0.0;
#pragma unroll
    for (int r = 0; r < 16; ++r) X[(r0 + r) * SMG_NBP + r0 + l] = x[r];
  }
}

// One wave: inverse of the (already lower-triangular) 16x16 leaf p of D into X.
__device__ inline void wave_leaf_inv(const double* D, double* X, int p) {
  const int l = threadIdx.x & 63;
  const int r0 = 16 * p;
  const int lr = l < 16 ? l : 15;
  double a[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) a[c] = D[(r0 + lr) * SMG_NBP + r0 + c];
  double x[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    double s = (l == r) ? 1.0 : 0.0;
#pragma unroll
    for (int t = 0; t < r; ++t) s -= bcast(a[t], r) * x[t];
    x[r] = s / bcast(a[r], r);
  }
  if (l < 16)
#pragma unroll
    for (int r = 0; r < 16; ++r) X[(r0 + r) * SMG_NBP + r0 + l] = x[r];
}

// Off-diagonal 16x16 blocks of X = L^{-1} given the diagonal leaf inverses:
//   X_ij = -X_ii sum_{k=j}^{i-1} L_ik X_kj   (i > j), by diagonals s = i - j.
// T: LDS scratch (>= 3 * 256 doubles).  All threads call.
__device__ inline void lds_trtri_offdiag(const double* L, double* X, double* T) {
  for (int s = 1; s < 4; ++s) {
    const int nb = 4 - s;  // blocks (j + s, j), j = 0..nb-1
    for (int e = threadIdx.x; e < nb * 256; e += blockDim.x) {
      const int j = e >> 8, r = (e >> 4) & 15, c = e & 15;
      const int i = j + s;
      double acc = 0.0;
      for (int k = j; k < i; ++k)
#pragma unroll 4
        for (int t = 0; t < 16; ++t)
          acc += L[(16 * i + r) * SMG_NBP + 16 * k + t] * X[(16 * k + t) * SMG_NBP + 16 * j + c];
      T[e] = acc;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < nb * 256; e += blockDim.x) {
      const int j = e >> 8, r = (e >> 4) & 15, c = e & 15;
      const int i = j + s;
      double acc = 0.0;
#pragma unroll 4
      for (int t = 0; t <= r; ++t) acc += X[(16 * i + r) * SMG_NBP + 16 * i + t] * T[(j << 8) + t * 16 + c];
      X[(16 * i + r) * SMG_NBP + 16 * j + c] = -acc;
    }
    __syncthreads();
  }
}

// In-LDS Cholesky of the lower triangle of D (64x64, padded with identity
// beyond b) AND X = L^{-1}.  Blocked right-looking with 16-wide panels.
// T: LDS scratch (>= 3 * 256 doubles).  All threads call.
__device__ inline void lds_potrf_inv64(double* D, double* X, double* T, int* status) {
  const int w = threadIdx.x >> 6;
  for (int e = threadIdx.x; e < SMG_NB * SMG_NBP; e += blockDim.x) X[e] = 0.0;
  __syncthreads();
  for (int p = 0; p < 4; ++p) {
    if (w == 0) wave_leaf_potrf_inv(D, X, p, status);
    __syncthreads();
    const int r1 = 16 * (p + 1), m = SMG_NB - r1;
    if (m == 0) break;
    // panel L21 = A21 X_pp^T : L(i, 16p+c) = sum_{t<=c} A(i, 16p+t) X(16p+c, 16p+t)
    double v[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int e = threadIdx.x + 256 * q;
      v[q] = 0.0;
      if (e < m * 16) {
        const int i = r1 + (e >> 4), c = e & 15;
        double acc = 0.0;
        for (int t = 0; t <= c; ++t) acc += D[i * SMG_NBP + 16 * p + t] * X[(16 * p + c) * SMG_NBP + 16 * p + t];
        v[q] = acc;
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int e = threadIdx.x + 256 * q;
      if (e < m * 16) D[(r1 + (e >> 4)) * SMG_NBP + 16 * p + (e & 15)] = v[q];
    }
    __syncthreads();
    // trailing lower triangle: A22(i, c) -= sum_t L(i, 16p+t) L(c, 16p+t)
    for (int e = threadIdx.x; e < m * m; e += blockDim.x) {
      const int i = r1 + e % m, c = r1 + e / m;
      if (i < c) continue;
      double acc = 0.0;
#pragma unroll
      for (int t = 0; t < 16; ++t) acc += D[i * SMG_NBP + 16 * p + t] * D[c * SMG_NBP + 16 * p + t];
      D[i * SMG_NBP + c] -= acc;
    }
    __syncthreads();
  }
  // strict upper of D: leaves wrote zeros in their blocks; panels never touch upper
  lds_trtri_offdiag(D, X, T);
}

// X = L^{-1} for a lower-triangular L in LDS (64x64, identity-padded).
__device__ inline void lds_trtri64(const double* D, double* X, double* T) {
  const int w = threadIdx.x >> 6;
  for (int e = threadIdx.x; e < SMG_NB * SMG_NBP; e += blockDim.x) X[e] = 0.0;
  __syncthreads();
  wave_leaf_inv(D, X, w);  // four leaves, one per wave
  __syncthreads();
  lds_trtri_offdiag(D, X, T);
}

// ---------------------------------------------------------------------------
// Single-wave 64x64 Cholesky, register resident (one wave = 64 lanes).
// Lane i holds row i of the block.  Step j: pivot = a[j] of lane j
// (v_readlane); l_jj = sqrt(pivot); lanes i > j divide a[j] by l_jj (Eigen
// LLT's column scaling); the new column goes to LDS with ONE ds_write per lane
// and is read back as broadcast LDS reads, 8 at a time (sched_barrier bounds
// the live registers), for the rank-1 update of the trailing columns.
// upper: load the block as the lower-triangular U^T of an upper-stored U.
// Writes L row-major into Lrow (LDS [64][SMG_NBP], strict upper zeroed) and,
// if Lout, col-major to global.  col: LDS >= 64 doubles.
__device__ __forceinline__ void wave_potrf64_reg(const double* __restrict__ A, int lda, int b, bool upper,
                                        double* Lout, int ldl, double* col, double* Lrow,
                                        int* status, bool factor) {
  const int l = threadIdx.x & 63;
  // stage through LDS (runtime loop: no per-element address registers)
#pragma unroll 4
  for (int c = 0; c < 64; ++c) {
    double v = (l == c) ? 1.0 : 0.0;  // identity padding beyond b
    if (l < b && c < b && c <= l) v = upper ? A[c + (size_t)l * lda] : A[l + (size_t)c * lda];
    Lrow[l * SMG_NBP + c] = v;
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  double a[64];
#pragma unroll
  for (int c = 0; c < 64; ++c) a[c] = Lrow[l * SMG_NBP + c];
  if (factor) {
    // lanes l < j only touch their (unused) strict-upper entries; a non-PD
    // pivot propagates NaN and is latched below.  Constant trip counts keep
    // a[] in VGPRs once fully unrolled.
    double minpiv = 1.0;
#pragma unroll
    for (int j = 0; j < 64; ++j) {
      const double piv = bcast(a[j], j);
      minpiv = fmin(minpiv, piv > 0.0 && piv < INFINITY ? 1.0 : -1.0);
      const double ljj = sqrt(piv);
      const double lij = (l == j) ? ljj : a[j] / ljj;
      a[j] = lij;
      col[l] = lij;
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's write is visible
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int c = 0; c < 64; ++c)
        if (c > j) a[c] -= lij * col[c];
      __builtin_amdgcn_wave_barrier();
    }
    if (!(minpiv > 0.0) && l == 0) atomicOr(status, (int)SMG_ERR_NOT_PD);
  }
#pragma unroll
  for (int c = 0; c < 64; ++c) Lrow[l * SMG_NBP + c] = (c <= l) ? a[c] : 0.0;
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  if (Lout && l < b) {
#pragma unroll 4
    for (int c = 0; c < b; ++c) Lout[l + (size_t)c * ldl] = Lrow[l * SMG_NBP + c];
  }
}

// X = L^{-1} from Lrow (LDS, lower, row-major stride SMG_NBP), one wave:
// lane c owns column c; the column lives in LDS (Xcol, same layout) so no
// register array is indexed at run time.  Four partial sums per entry.
__device__ inline void wave_trtri64_lds(const double* Lrow, double* Xcol, double* Xout, int ldx,
                                        int b) {
  const int c = threadIdx.x & 63;
  for (int r = 0; r < 64; ++r) {
    double s0 = (r == c) ? 1.0 : 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    int t = c;  // X(t, c) = 0 for t < c
    for (; t + 3 < r; t += 4) {
      s0 -= Lrow[r * SMG_NBP + t] * Xcol[t * SMG_NBP + c];
      s1 -= Lrow[r * SMG_NBP + t + 1] * Xcol[(t + 1) * SMG_NBP + c];
      s2 -= Lrow[r * SMG_NBP + t + 2] * Xcol[(t + 2) * SMG_NBP + c];
      s3 -= Lrow[r * SMG_NBP + t + 3] * Xcol[(t + 3) * SMG_NBP + c];
    }
    for (; t < r; ++t) s0 -= Lrow[r * SMG_NBP + t] * Xcol[t * SMG_NBP + c];
    const double xv = (r < c) ? 0.0 : ((s0 + s1) + (s2 + s3)) / Lrow[r * SMG_NBP + r];
    Xcol[r * SMG_NBP + c] = xv;
    if (Xout && r < b && c < b) Xout[r + (size_t)c * ldx] = xv;
  }
}

// ---------------------------------------------------------------------------
// Fused 64x64 Cholesky + inverse by right-looking elimination, all waves of
// the workgroup (blockDim.x = 64 * G), ONE barrier per column.
// Thread (i = lane, g = wave) owns row i and the column class c = g (mod G).
// Step j (all threads compute l_jj = sqrt(D[j][j]) redundantly -- no
// broadcast, no extra barrier):
//   l_ij = D[i][j] / l_jj                        (Eigen LLT column scaling)
//   D[i][c] -= l_ij * (D[c][j] / l_jj)  j < c <= i   (trailing update)
//   X[i][c] -= l_ij * (X[j][c] / l_jj)  c <= j, i > j (same row ops on I)
//   X_final[j][:] = X[j][:] / l_jj,  L[:, j] final
// D's column j and X's row j are only READ during step j; every write goes
// to a different row/column, so no intra-step hazard.  With factor == false
// D already holds L and l_ij = D[i][j] (no scaling): X = L^{-1} only.
// D, X: LDS [64][SMG_NBP]; X must hold the identity on entry.
// Lout / Xout: col-major global destinations (b x b; Lout may be null).
__device__ inline void lds_potrf_inv64_v2(double* D, double* X, int b, double* Lout, int ldl,
                                          double* Xout, int ldx, int* status, bool factor) {
  constexpr int GC = SMG_DIAG_THREADS / 64;  // column classes (waves)
  const int i = threadIdx.x & 63;
  const int g = threadIdx.x >> 6;
  bool bad = false;
  double li_prev = 0.0, inv_prev = 1.0;
  for (int j = 0; j < 64; ++j) {
    // deferred finalisation of step j-1 (column j-1 of D / row j-1 of X are
    // not read in step j): l_{i,j-1} into D, row j-1 of X scaled in place
    if (j > 0) {
      if (factor && g == 0 && i >= j - 1) D[i * SMG_NBP + j - 1] = li_prev;
      if (i == j - 1)
#pragma unroll
        for (int q = 0; q < 64 / GC; ++q) {
          const int c = g + q * GC;
          if (c <= i) X[i * SMG_NBP + c] *= inv_prev;
        }
    }
    const double piv = D[j * SMG_NBP + j];
    double ljj, inv, li;
    // the pivot chain is the kernel's critical path: v_rsq_f64 + two Newton
    // steps (~1 ulp, vs ~360 cycles for IEEE sqrt + divide on gfx950)
    if (factor) {
      bad |= !(piv > 0.0 && piv < INFINITY);
      double r = __builtin_amdgcn_rsq(piv);
      r = r * (1.5 - 0.5 * piv * r * r);
      r = r * (1.5 - 0.5 * piv * r * r);
      inv = r;
      ljj = piv * r;
      li = (i > j) ? D[i * SMG_NBP + j] * inv : (i == j ? ljj : 0.0);
    } else {
      ljj = piv;
      double r = __builtin_amdgcn_rcp(piv);
      r = r * (2.0 - piv * r);
      inv = r * (2.0 - piv * r);
      li = (i >= j) ? D[i * SMG_NBP + j] : 0.0;
    }
    if (i > j) {
      // fixed trip counts (64 / GC per loop), predicated: all loads of a
      // loop issue back to back instead of one LDS round trip per element
      if (factor) {
        double lc[64 / GC], dv[64 / GC];
#pragma unroll
        for (int q = 0; q < 64 / GC; ++q) {
          const int c = g + q * GC;
          lc[q] = D[c * SMG_NBP + j];
          dv[q] = D[i * SMG_NBP + c];
        }
#pragma unroll
        for (int q = 0; q < 64 / GC; ++q) {
          const int c = g + q * GC;
          if (c > j && c <= i) D[i * SMG_NBP + c] = dv[q] - li * (lc[q] * inv);
        }
      }
      const double lx = li * inv;
      double xj[64 / GC], xi[64 / GC];
#pragma unroll
      for (int q = 0; q < 64 / GC; ++q) {
        const int c = g + q * GC;
        xj[q] = X[j * SMG_NBP + c];
        xi[q] = X[i * SMG_NBP + c];
      }
#pragma unroll
      for (int q = 0; q < 64 / GC; ++q) {
        const int c = g + q * GC;
        if (c <= j) X[i * SMG_NBP + c] = xi[q] - lx * xj[q];
      }
    }
    li_prev = li;
    inv_prev = inv;
    __syncthreads();
  }
  // finalisation of step 63
  if (factor && g == 0 && i == 63) D[63 * SMG_NBP + 63] = li_prev;
  if (i == 63)
#pragma unroll
    for (int q = 0; q < 64 / GC; ++q) X[63 * SMG_NBP + g + q * GC] *= inv_prev;
  __syncthreads();
  if (bad && threadIdx.x == 0) atomicOr(status, (int)SMG_ERR_NOT_PD);
  // one coalesced write of L (lower, upper zeroed) and X (dense, upper zeros)
  for (int e = threadIdx.x; e < b * b; e += blockDim.x) {
    const int c = e / b, r = e % b;
    if (Lout) Lout[r + (size_t)c * ldl] = (r >= c) ? D[r * SMG_NBP + c] : 0.0;
    if (Xout) Xout[r + (size_t)c * ldx] = (r >= c) ? X[r * SMG_NBP + c] : 0.0;
  }
}

// ---------------------------------------------------------------------------
// Blocked 64x64 Cholesky in LDS (512 threads = 8 waves), 8-wide panels.
//   panel p (columns j0 = 8p .. j0+7): wave 0, lane i = row i holds the 8
//     panel values in registers; 8 pivot steps with v_readlane broadcasts;
//     l_jj = sqrt(pivot) via v_rsq_f64 + 2 Newton steps (~1 ulp), the
//     column scaled by the reciprocal (Eigen LLT divides; same to ~1 ulp).
//   trailing rank-8 update of the lower triangle below the panel: thread
//     (row i = lane, column class g = wave) keeps row i's panel in registers
//     and walks columns c = g (mod 8): 8 FMAs per loaded D[i][c].
// D: LDS [64][SMG_NBP], lower triangle holds A (identity padded); on exit the
// lower triangle holds L (strict upper untouched).
__device__ inline void lds_potrf64_blocked(double* D, int* status) {
  const int i = threadIdx.x & 63;
  const int g = threadIdx.x >> 6;
  bool bad = false;
  for (int p = 0; p < 8; ++p) {
    const int j0 = 8 * p;
    if (g == 0) {
      double a[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) a[t] = (i >= j0) ? D[i * SMG_NBP + j0 + t] : 0.0;
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const double piv = bcast(a[t], j0 + t);
        bad |= !(piv > 0.0 && piv < INFINITY);
        double r = __builtin_amdgcn_rsq(piv);
        r = r * (1.5 - 0.5 * piv * r * r);
        r = r * (1.5 - 0.5 * piv * r * r);
        const double li = (i == j0 + t) ? piv * r : a[t] * r;
        a[t] = li;
#pragma unroll
        for (int c = t + 1; c < 8; ++c) a[c] -= li * bcast(li, j0 + c);
      }
      if (i >= j0)
#pragma unroll
        for (int t = 0; t < 8; ++t)
          if (i >= j0 + t) D[i * SMG_NBP + j0 + t] = a[t];
    }
    __syncthreads();
    const int c1 = j0 + 8;
    if (c1 < 64 && i >= c1) {
      double li[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) li[t] = D[i * SMG_NBP + j0 + t];
      // columns c = c1 + g + 8q (q = 0..6), c <= i
#pragma unroll
      for (int q = 0; q < 7; ++q) {
        const int c = c1 + g + 8 * q;
        if (c <= i) {
          double s = D[i * SMG_NBP + c];
#pragma unroll
          for (int t = 0; t < 8; ++t) s -= li[t] * D[c * SMG_NBP + j0 + t];
          D[i * SMG_NBP + c] = s;
        }
      }
    }
    __syncthreads();
  }
  if (bad && threadIdx.x == 0) atomicOr(status, (int)SMG_ERR_NOT_PD);
}

// X = L^{-1} (64x64, LDS) for L lower in D (LDS), 512 threads, 8x8 blocks.
//   leaves: wave w inverts the 8x8 diagonal block w (lane c < 8 owns column c)
//   block rows p = 1..7 in order: T = -sum_{k<p} L_pk X_k (all columns c < 8p),
//   then X_p = X_pp T (thread (row r = wave, column c = lane)).
// X: LDS [64][SMG_NBP] (fully written, upper zeros); T: LDS >= 8*64 doubles.
__device__ inline void lds_trtri64_blocked(const double* D, double* X, double* T) {
  const int l = threadIdx.x & 63;
  const int g = threadIdx.x >> 6;
  for (int e = threadIdx.x; e < 64 * SMG_NBP; e += blockDim.x) X[e] = 0.0;
  __syncthreads();
  {  // diagonal leaf g
    const int j0 = 8 * g;
    double x[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      double s = (l == r) ? 1.0 : 0.0;
#pragma unroll
      for (int t = 0; t < r; ++t) s -= D[(j0 + r) * SMG_NBP + j0 + t] * x[t];
      double rr = __builtin_amdgcn_rcp(D[(j0 + r) * SMG_NBP + j0 + r]);
      const double dd = D[(j0 + r) * SMG_NBP + j0 + r];
      rr = rr * (2.0 - dd * rr);
      rr = rr * (2.0 - dd * rr);
      x[r] = s * rr;
    }
    if (l < 8)
#pragma unroll
      for (int r = 0; r < 8; ++r) X[(j0 + r) * SMG_NBP + j0 + l] = x[r];
  }
  __syncthreads();
  for (int p = 1; p < 8; ++p) {
    const int j0 = 8 * p;
    // T[r][c] = -sum_{t < j0} L[j0+r][t] X[t][c], c < j0 ; thread (r = g, c = l)
    if (l < j0) {
      double s[4] = {0.0, 0.0, 0.0, 0.0};
      for (int t0 = 0; t0 < j0; t0 += 8) {  // 16 independent LDS reads per trip
        double dl[8], xl[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          dl[t] = D[(j0 + g) * SMG_NBP + t0 + t];
          xl[t] = X[(t0 + t) * SMG_NBP + l];
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) s[t & 3] -= dl[t] * xl[t];
      }
      T[g * 64 + l] = (s[0] + s[1]) + (s[2] + s[3]);
    }
    __syncthreads();
    // X[j0+r][c] = sum_{t <= r} Xpp[r][t] T[t][c]
    if (l < j0) {
      double s = 0.0;
#pragma unroll
      for (int t = 0; t < 8; ++t)
        if (t <= g) s += X[(j0 + g) * SMG_NBP + j0 + t] * T[t * 64 + l];
      X[(j0 + g) * SMG_NBP + l] = s;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Look-ahead variant of lds_potrf64_blocked (same panels, same arithmetic per
// element): in iteration p, wave 0 applies panel p's rank-8 update to panel
// p+1 and factors it, WHILE waves 1..7 apply panel p's update to the columns
// right of panel p+1.  The serial pivot chain (wave 0) overlaps the bulk of
// the trailing work; one barrier per panel.
// wave 0: factor the 8 columns held in a[] (lane i = row i, rows < j0 hold 0)
// The column's entries of rows j0+c are broadcast BEFORE the pivot's
// reciprocal root and scaled by it on every lane (the same product lane j0+c
// forms, so the same bits as broadcasting l_{j0+c}): one readlane less on
// the pivot chain
__device__ __forceinline__ void wave_factor8_reg(double (&a)[8], int j0, bool& bad) {
  const int i = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    double sc[8];
#pragma unroll
    for (int c = t + 1; c < 8; ++c) sc[c] = bcast(a[t], j0 + c);
    const double piv = bcast(a[t], j0 + t);
    bad |= !(piv > 0.0 && piv < INFINITY);
    double r = __builtin_amdgcn_rsq(piv);
    r = r * (1.5 - 0.5 * piv * r * r);
    r = r * (1.5 - 0.5 * piv * r * r);
    const double li = (i == j0 + t) ? piv * r : a[t] * r;
    a[t] = li;
#pragma unroll
    for (int c = t + 1; c < 8; ++c) a[c] -= li * (sc[c] * r);
  }
}

// The same 8 columns two pivots at a time: for the 2x2 diagonal block
// [[A, B], [B, C]] both reciprocal roots come from values known before
// either is taken -- r1 = A^{-1/2} and rp = (AC - B^2)^{-1/2}, the second
// pivot's l22^{-1} = sqrt(A) rp = A r1 rp -- so the two rsq + Newton chains
// run side by side and the pivot chain is one root deep per PAIR of columns.
// The rows' entries are pre-broadcast before the roots and scaled locally
// (as in wave_factor8_reg).  Not bit-identical to wave_factor8_reg (l22 from
// det / A instead of C - l21^2), same accuracy class.
__device__ __forceinline__ void wave_factor8_pair(double (&a)[8], int j0, bool& bad) {
  const int i = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < 8; t += 2) {
    double s0[8], s1[8];
#pragma unroll
    for (int c = t + 2; c < 8; ++c) {
      s0[c] = bcast(a[t], j0 + c);
      s1[c] = bcast(a[t + 1], j0 + c);
    }
    const double A = bcast(a[t], j0 + t);
    const double B = bcast(a[t], j0 + t + 1);
    const double C = bcast(a[t + 1], j0 + t + 1);
    const double det = __builtin_fma(A, C, -(B * B));
    bad |= !(A > 0.0 && A < INFINITY) || !(det > 0.0 && det < INFINITY);
    double r1 = __builtin_amdgcn_rsq(A);
    double rp = __builtin_amdgcn_rsq(det);
    r1 = r1 * (1.5 - 0.5 * A * r1 * r1);
    rp = rp * (1.5 - 0.5 * det * rp * rp);
    r1 = r1 * (1.5 - 0.5 * A * r1 * r1);
    rp = rp * (1.5 - 0.5 * det * rp * rp);
    const double r2 = (A * r1) * rp;  // (C - l21^2)^{-1/2}
    const double l21 = B * r1;
    const double li0 = a[t] * r1;
    const double li1 = (a[t + 1] - li0 * l21) * r2;
    a[t] = li0;
    a[t + 1] = li1;
#pragma unroll
    for (int c = t + 2; c < 8; ++c) {
      const double lc0 = s0[c] * r1;
      const double lc1 = (s1[c] - lc0 * l21) * r2;
      a[c] = a[c] - li0 * lc0 - li1 * lc1;
    }
  }
  (void)i;
}

// wave 0: factor panel columns j0..j0+7 (rows >= j0) of D in place, with NO
// cross-lane traffic on the pivot chain: every lane factors the 8x8 diagonal
// block redundantly in registers (left-looking), then solves its own row
// against it: x_t = (a_t - sum_{s<t} x_s L_ts) / L_tt.
__device__ __forceinline__ void wave_panel8_local(double* D, int j0, bool& bad) {
  const int i = threadIdx.x & 63;
  double Ld[8][8], inv[8];
#pragma unroll
  for (int r = 0; r < 8; ++r)
#pragma unroll
    for (int c = 0; c <= r; ++c) Ld[r][c] = D[(j0 + r) * SMG_NBP + j0 + c];  // LDS broadcast
  double a[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) a[t] = (i >= j0 + 8) ? D[i * SMG_NBP + j0 + t] : 0.0;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    double piv = Ld[t][t];
#pragma unroll
    for (int q = 0; q < t; ++q) piv -= Ld[t][q] * Ld[t][q];
    bad |= !(piv > 0.0 && piv < INFINITY);
    double r = __builtin_amdgcn_rsq(piv);
    r = r * (1.5 - 0.5 * piv * r * r);
    r = r * (1.5 - 0.5 * piv * r * r);
    inv[t] = r;
    Ld[t][t] = piv * r;
#pragma unroll
    for (int c = t + 1; c < 8; ++c) {
      double v = Ld[c][t];
#pragma unroll
      for (int q = 0; q < t; ++q) v -= Ld[c][q] * Ld[t][q];
      Ld[c][t] = v * r;
    }
  }
  // own row below the diagonal block: x = a L_dd^{-T}
  double x[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    double v = a[t];
#pragma unroll
    for (int q = 0; q < t; ++q) v -= x[q] * Ld[t][q];
    x[t] = v * inv[t];
  }
  if (i >= j0 + 8) {
#pragma unroll
    for (int t = 0; t < 8; ++t) D[i * SMG_NBP + j0 + t] = x[t];
  } else if (i >= j0) {
    const int r = i - j0;
#pragma unroll
    for (int t = 0; t < 8; ++t)
      if (t <= r) {
        double v = 0.0;
#pragma unroll
        for (int rr = 0; rr < 8; ++rr)
          if (rr == r) v = Ld[rr][t];
        D[i * SMG_NBP + j0 + t] = v;
      }
  }
}

template <typename P>
__device__ __forceinline__ void wave_store8(P D, const double (&a)[8], int j0) {
  const int i = threadIdx.x & 63;
  if (i >= j0)
#pragma unroll
    for (int t = 0; t < 8; ++t)
      if (i >= j0 + t) D[i * SMG_NBP + j0 + t] = a[t];
}

// wave 0: load, factor (v_readlane broadcasts), store panel j0..j0+7
template <bool PAIR = false, typename P>
__device__ __forceinline__ void wave_panel8_rl(P D, int j0, bool& bad) {
  const int i = threadIdx.x & 63;
  double a[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) a[t] = (i >= j0) ? D[i * SMG_NBP + j0 + t] : 0.0;
  if (PAIR)
    wave_factor8_pair(a, j0, bad);
  else
    wave_factor8_reg(a, j0, bad);
  wave_store8(D, a, j0);
}

// (templated on the pointer type: double* when inlined into a kernel, an
// address_space(3) pointer when called out of line)
template <bool PAIR = false, typename P>
__device__ inline void lds_potrf64_lookahead(P D, int* status) {
  const int i = threadIdx.x & 63;
  const int g = threadIdx.x >> 6;
  bool bad = false;
  if (g == 0) wave_panel8_rl<PAIR>(D, 0, bad);
  __syncthreads();
  for (int p = 0; p < 7; ++p) {
    const int j0 = 8 * p, c1 = j0 + 8, c2 = j0 + 16;
    // (A) waves 1..7: panel p+1 (rows >= c1, 8 columns) -= panel p's rank-8
    //     update, one element per thread
    if (g > 0) {
      const int e = threadIdx.x - 64;
      const int r = c1 + (e >> 3), c = c1 + (e & 7);
      if (r < 64 && r >= c) {
        double v = D[r * SMG_NBP + c];
#pragma unroll
        for (int t = 0; t < 8; ++t) v -= D[r * SMG_NBP + j0 + t] * D[c * SMG_NBP + j0 + t];
        D[r * SMG_NBP + c] = v;
      }
    }
    __syncthreads();
    // (B) wave 0 factors panel p+1 while waves 1..7 update columns >= c2
    if (g == 0) {
      wave_panel8_rl<PAIR>(D, c1, bad);
    } else if (c2 < 64) {
      // rank-8 trailing update of rows/cols >= c2 on the matrix cores: 16x16
      // tiles (ti >= tj) from 16-tile t0 = c2/16, 2 MFMAs each (K = 8); only
      // entries with col >= c2 and row >= col are written back
      const int t0 = c2 >> 4, nt = 4 - t0, ntiles = nt * (nt + 1) / 2;
      const int fr = i & 15, fk = i >> 4;
      for (int q = g - 1; q < ntiles; q += 7) {
        int ti = 0, rem = q;
        while (rem > ti) {
          rem -= ti + 1;
          ++ti;
        }
        const int tj = rem + t0;
        ti += t0;
        d4 acc = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k0 = 0; k0 < 8; k0 += 4) {
          const double av = D[(16 * ti + fr) * SMG_NBP + j0 + k0 + fk];
          const double bv = D[(16 * tj + fr) * SMG_NBP + j0 + k0 + fk];
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
        }
        const int col = 16 * tj + fr;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * ti + fk + 4 * r;
          if (col >= c2 && row >= col) D[row * SMG_NBP + col] -= acc[r];
        }
      }
    }
    __syncthreads();
  }
  if (bad) atomicOr(status, (int)SMG_ERR_NOT_PD);
}

// ---------------------------------------------------------------------------
// x^{-1/2} to ~1 ulp: v_rsq_f64 (about 2^-22 relative) and ONE third-order
// (Halley-type) correction r (1 + e/2 + 3 e^2 / 8), e = 1 - x r^2 -- four
// dependent operations instead of two Newton steps' eight
__device__ __forceinline__ double rsq_h(double x) {
  const double r = __builtin_amdgcn_rsq(x);
  const double t = x * r;
  const double e = __builtin_fma(-t, r, 1.0);
  const double s = r * e;
  const double p = __builtin_fma(0.375, e, 0.5);
  return __builtin_fma(s, p, r);
}

// wave_factor8_pair with rsq_h roots
__device__ __forceinline__ void wave_factor8_pair_h(double (&a)[8], int j0, bool& bad) {
#pragma unroll
  for (int t = 0; t < 8; t += 2) {
    double s0[8], s1[8];
#pragma unroll
    for (int c = t + 2; c < 8; ++c) {
      s0[c] = bcast(a[t], j0 + c);
      s1[c] = bcast(a[t + 1], j0 + c);
    }
    const double A = bcast(a[t], j0 + t);
    const double B = bcast(a[t], j0 + t + 1);
    const double C = bcast(a[t + 1], j0 + t + 1);
    const double det = __builtin_fma(A, C, -(B * B));
    bad |= !(A > 0.0 && A < INFINITY) || !(det > 0.0 && det < INFINITY);
    const double r1 = rsq_h(A);
    const double rp = rsq_h(det);
    const double r2 = (A * r1) * rp;
    const double l21 = B * r1;
    const double li0 = a[t] * r1;
    const double li1 = (a[t + 1] - li0 * l21) * r2;
    a[t] = li0;
    a[t + 1] = li1;
#pragma unroll
    for (int c = t + 2; c < 8; ++c) {
      const double lc0 = s0[c] * r1;
      const double lc1 = (s1[c] - lc0 * l21) * r2;
      a[c] = a[c] - li0 * lc0 - li1 * lc1;
    }
  }
}

// The pairs with the fewest operations: rsq_h roots, and the later columns
// updated with the factor's own entries broadcast from the lanes that form
// them (li0 / li1 of lane j0 + c are L[c][t] / L[c][t+1]): per column and pair
// two FMAs (wave_factor8_pair recomputes both entries on every lane from
// pre-broadcast raw values: five operations).  PRE: the next pair's two
// columns' entries are broadcast first, the rest after their update.
template <bool PRE = true>
__device__ __forceinline__ void wave_factor8_pair2(double (&a)[8], int j0, bool& bad) {
#pragma unroll
  for (int t = 0; t < 8; t += 2) {
    const double A = bcast(a[t], j0 + t);
    const double B = bcast(a[t], j0 + t + 1);
    const double C = bcast(a[t + 1], j0 + t + 1);
    const double det = __builtin_fma(A, C, -(B * B));
    bad |= !(A > 0.0 && A < INFINITY) || !(det > 0.0 && det < INFINITY);
    const double r1 = rsq_h(A);
    const double rp = rsq_h(det);
    const double r2 = (A * r1) * rp;
    const double l21 = B * r1;
    const double li0 = a[t] * r1;
    const double li1 = (a[t + 1] - li0 * l21) * r2;
    a[t] = li0;
    a[t + 1] = li1;
    if (PRE && t + 2 < 8) {  // the next pair's columns first (its pivots' chain)
#pragma unroll
      for (int c = t + 2; c < t + 4; ++c) a[c] = a[c] - li0 * bcast(li0, j0 + c) - li1 * bcast(li1, j0 + c);
#pragma unroll
      for (int c = t + 4; c < 8; ++c) a[c] = a[c] - li0 * bcast(li0, j0 + c) - li1 * bcast(li1, j0 + c);
    } else {
#pragma unroll
      for (int c = t + 2; c < 8; ++c) a[c] = a[c] - li0 * bcast(li0, j0 + c) - li1 * bcast(li1, j0 + c);
    }
  }
}

// wave 0: panel j0..j0+7 with the 8 x 8 diagonal block factored UNIFORMLY
// (every lane the same values, read as LDS broadcasts: no cross-lane traffic
// on the pivot chain), pivots in pairs (wave_factor8_pair's 2 x 2 leading
// minors) with rsq_h roots, then each lane solves its own row against it:
// x_t = (a_t - sum_{q<t} x_q L_tq) / L_tt.  The diagonal rows store the
// uniform factor.  Same accuracy class as wave_factor8_pair.
template <typename P>
__device__ __forceinline__ void wave_panel8_uniform(P D, int j0, bool& bad) {
  const int i = threadIdx.x & 63;
  double a[8], d[8][8];
#pragma unroll
  for (int t = 0; t < 8; ++t) a[t] = D[i * SMG_NBP + j0 + t];
#pragma unroll
  for (int r = 0; r < 8; ++r)
#pragma unroll
    for (int c = 0; c <= r; ++c) d[r][c] = D[(j0 + r) * SMG_NBP + j0 + c];  // (broadcast)
  double rinv[8];
#pragma unroll
  for (int t = 0; t < 8; t += 2) {
    const double A = d[t][t], B = d[t + 1][t], C = d[t + 1][t + 1];
    const double det = __builtin_fma(A, C, -(B * B));
    bad |= !(A > 0.0 && A < INFINITY) || !(det > 0.0 && det < INFINITY);
    const double r1 = rsq_h(A);
    const double rp = rsq_h(det);
    const double r2 = (A * r1) * rp;  // (C - l21^2)^{-1/2}
    const double l21 = B * r1;
    d[t][t] = A * r1;
    d[t + 1][t] = l21;
    d[t + 1][t + 1] = (det * rp) * r1;  // sqrt(det / A)
    rinv[t] = r1;
    rinv[t + 1] = r2;
#pragma unroll
    for (int c = t + 2; c < 8; ++c) {
      const double lc0 = d[c][t] * r1;
      d[c][t] = lc0;
      d[c][t + 1] = (d[c][t + 1] - lc0 * l21) * r2;
    }
#pragma unroll
    for (int c = t + 2; c < 8; ++c)
#pragma unroll
      for (int c2 = t + 2; c2 <= c; ++c2) d[c][c2] = d[c][c2] - d[c][t] * d[c2][t] - d[c][t + 1] * d[c2][t + 1];
  }
  double x[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    double v = a[t];
#pragma unroll
    for (int q = 0; q < t; ++q) v -= x[q] * d[t][q];
    x[t] = v * rinv[t];
  }
  if (i >= j0 + 8) {
#pragma unroll
    for (int t = 0; t < 8; ++t) D[i * SMG_NBP + j0 + t] = x[t];
  } else if (i >= j0) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
      if (i == j0 + r)
#pragma unroll
        for (int t = 0; t <= r; ++t) D[i * SMG_NBP + j0 + t] = d[r][t];
  }
}

// The look-ahead factor with selectable pieces (tools/ubench_factor):
//   PANEL 0: wave_factor8_pair (readlane broadcasts, Newton roots)
//         1: wave_factor8_pair_h (readlane broadcasts, rsq_h roots)
//         2: wave_panel8_uniform (uniform diagonal block, rsq_h roots)
//         3: wave_factor8_pair2 (the factor's own entries broadcast, rsq_h roots)
//   AMFMA:  the next panel's rank-8 update (A) on the matrix cores (waves
//           1..4, one 16-row tile each, 2 MFMAs) instead of one element per
//           thread of waves 1..7 (17 LDS loads each)
template <int PANEL, bool AMFMA, typename P>
__device__ inline void lds_potrf64_v3(P D, int* status) {
  const int i = threadIdx.x & 63;
  const int g = threadIdx.x >> 6;
  bool bad = false;
  auto panel = [&](int j0) {
    if (PANEL == 2) {
      wave_panel8_uniform(D, j0, bad);
    } else {
      double a[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) a[t] = (i >= j0) ? D[i * SMG_NBP + j0 + t] : 0.0;
      if (PANEL == 1)
        wave_factor8_pair_h(a, j0, bad);
      else if (PANEL == 3)
        wave_factor8_pair2(a, j0, bad);
      else
        wave_factor8_pair(a, j0, bad);
      wave_store8(D, a, j0);
    }
  };
  if (g == 0) panel(0);
  __syncthreads();
  for (int p = 0; p < 7; ++p) {
    const int j0 = 8 * p, c1 = j0 + 8, c2 = j0 + 16;
    if (AMFMA) {
      // (A): rows >= c1 of columns c1..c1+7 -= L[:, j0:j0+8] L[c1:c1+8, j0:j0+8]^T,
      // 16-row tiles ti = (c1 >> 4) + g - 1 on waves g = 1..; B's columns past
      // c1 + 7 are clamped rows (their outputs are dropped)
      const int ti = (c1 >> 4) + g - 1;
      if (g >= 1 && ti < 4) {
        const int fr = i & 15, fk = i >> 4;
        const int brow = min(c1 + fr, 63);
        d4 acc = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k0 = 0; k0 < 8; k0 += 4) {
          const double av = D[(16 * ti + fr) * SMG_NBP + j0 + k0 + fk];
          const double bv = D[brow * SMG_NBP + j0 + k0 + fk];
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
        }
        const int col = c1 + fr;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * ti + fk + 4 * r;
          if (fr < 8 && row >= col) D[row * SMG_NBP + col] -= acc[r];
        }
      }
    } else if (g > 0) {
      const int e = threadIdx.x - 64;
      const int r = c1 + (e >> 3), c = c1 + (e & 7);
      if (r < 64 && r >= c) {
        double v = D[r * SMG_NBP + c];
#pragma unroll
        for (int t = 0; t < 8; ++t) v -= D[r * SMG_NBP + j0 + t] * D[c * SMG_NBP + j0 + t];
        D[r * SMG_NBP + c] = v;
      }
    }
    __syncthreads();
    // (B) wave 0 factors panel p+1 while waves 1..7 update columns >= c2
    if (g == 0) {
      panel(c1);
    } else if (c2 < 64) {
      const int t0 = c2 >> 4, nt = 4 - t0, ntiles = nt * (nt + 1) / 2;
      const int fr = i & 15, fk = i >> 4;
      for (int q = g - 1; q < ntiles; q += 7) {
        int ti = 0, rem = q;
        while (rem > ti) {
          rem -= ti + 1;
          ++ti;
        }
        const int tj = rem + t0;
        ti += t0;
        d4 acc = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k0 = 0; k0 < 8; k0 += 4) {
          const double av = D[(16 * ti + fr) * SMG_NBP + j0 + k0 + fk];
          const double bv = D[(16 * tj + fr) * SMG_NBP + j0 + k0 + fk];
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
        }
        const int col = 16 * tj + fr;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * ti + fk + 4 * r;
          if (col >= c2 && row >= col) D[row * SMG_NBP + col] -= acc[r];
        }
      }
    }
    __syncthreads();
  }
  if (bad) atomicOr(status, (int)SMG_ERR_NOT_PD);
}

// A wave's 16 x 16 leaf inverse k (the diagonal block of X written by
// trtri_leaf16) stored (sc1) into G (ld ldg; rows / columns < b): 4 values
// per lane, rows fastest (128-byte column runs), read back from LDS after the
// wave's own writes
template <typename P>
__device__ __forceinline__ void leaf16_store(const P X, double* G, int ldg, int b, int k);

// Pieces of X = L^{-1} (64x64) on 16x16 blocks, shared by lds_trtri64_mfma
// and the fused lds_potrf_trtri64 (same arithmetic, same order: same bits).
// Leaf k (one wave, lane c < 16 owns column c): X_kk = L_kk^{-1} by
// right-looking elimination -- each x[q] still accumulates its terms in
// ascending order, but only one FMA per row sits on the dependency chain.
template <typename CP, typename P>
__device__ __forceinline__ void trtri_leaf16(CP D, P X, int k) {
  const int l = threadIdx.x & 63;
  const int r0 = 16 * k;
  double x[16], rv[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    x[r] = (l == r) ? 1.0 : 0.0;
    const double dd = D[(r0 + r) * SMG_NBP + r0 + r];
    double rr = __builtin_amdgcn_rcp(dd);
    rr = rr * (2.0 - dd * rr);
    rv[r] = rr * (2.0 - dd * rr);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    x[r] = x[r] * rv[r];
#pragma unroll
    for (int q = r + 1; q < 16; ++q) x[q] -= D[(r0 + q) * SMG_NBP + r0 + r] * x[r];
  }
  if (l < 16)
#pragma unroll
    for (int r = 0; r < 16; ++r) X[(r0 + r) * SMG_NBP + r0 + l] = x[r];
}
// T_q = -L[p, q:p] X[q:p, q] accumulated over k in [kb, ke) (multiples of 8,
// from 16q): two MFMA chains (even / odd k-steps of 4), summed at the store
template <typename CP, typename XP>
__device__ __forceinline__ void trtri_t_acc(CP D, XP X, int p, int q, int kb, int ke, d4& acc,
                                            d4& acc2) {
  const int l = threadIdx.x & 63;
  const int fr = l & 15, fk = l >> 4;
  for (int k0 = kb; k0 < ke; k0 += 8) {
    const double a = D[(16 * p + fr) * SMG_NBP + k0 + fk];
    const double b = X[(k0 + fk) * SMG_NBP + 16 * q + fr];
    const double a2 = D[(16 * p + fr) * SMG_NBP + k0 + 4 + fk];
    const double b2 = X[(k0 + 4 + fk) * SMG_NBP + 16 * q + fr];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a2, b2, acc2, 0, 0, 0);
  }
}
template <typename P>
__device__ __forceinline__ void trtri_t_store(P T, int q, const d4& acc, const d4& acc2) {
  const int l = threadIdx.x & 63;
  const int fr = l & 15, fk = l >> 4;
#pragma unroll
  for (int r = 0; r < 4; ++r) T[q * 256 + (fk + 4 * r) * 16 + fr] = -(acc[r] + acc2[r]);
}
// X[p, q] = X_pp T_q
template <typename P>
__device__ __forceinline__ void trtri_x_tile(P X, P T, int p, int q) {
  const int l = threadIdx.x & 63;
  const int fr = l & 15, fk = l >> 4;
  d4 acc = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int k0 = 0; k0 < 16; k0 += 4) {
    const double a = X[(16 * p + fr) * SMG_NBP + 16 * p + k0 + fk];
    const double b = T[q * 256 + (k0 + fk) * 16 + fr];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) X[(16 * p + fk + 4 * r) * SMG_NBP + 16 * q + fr] = acc[r];
}

// X = L^{-1} (64x64) with 16x16 blocks on the fp64 matrix cores:
//   leaves: wave w < 4 inverts diagonal block w (trtri_leaf16)
//   block rows p = 1..3:  T = -L[p, 0:p] X[0:p, 0:p]  (wave q < p: tile (p, q)),
//                         X[p, 0:p] = X_pp T          (wave q < p)
// X: LDS [64][SMG_NBP], fully written (upper zeros); T: LDS >= 3 * 256 doubles.
template <typename CP, typename P>
__device__ inline void lds_trtri64_mfma(CP D, P X, P T) {
  const int w = threadIdx.x >> 6;
  for (int e = threadIdx.x; e < 64 * SMG_NBP; e += blockDim.x) X[e] = 0.0;
  __syncthreads();
  if (w < 4) trtri_leaf16(D, X, w);
  __syncthreads();
  for (int p = 1; p < 4; ++p) {
    if (w < p) {
      d4 acc = d4{0.0, 0.0, 0.0, 0.0}, acc2 = acc;
      trtri_t_acc(D, X, p, w, 16 * w, 16 * p, acc, acc2);
      trtri_t_store(T, w, acc, acc2);
    }
    __syncthreads();
    if (w < p) trtri_x_tile(X, T, p, w);
    __syncthreads();
  }
}

template <typename P>
__device__ __forceinline__ void leaf16_store(const P X, double* G, int ldg, int b, int k) {
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int e = l + 64 * q, r = 16 * k + (e & 15), c = 16 * k + (e >> 4);
    if (r < b && c < b)
      __hip_atomic_store(&G[r + (size_t)c * ldg], (double)X[r * SMG_NBP + c], __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Y <- Y L^{-T} in place (Y: 64 x 64, L: 64 x 64 lower, both LDS [r][c]
// stride SMG_NBP), given the 16 x 16 leaf inverses Li_pp = L_pp^{-1} on the
// diagonal blocks of Li (trtri_leaf16).  Wave w < 4 solves row tile w alone,
// column blocks p = 0..3 in order:
//   Z = Y[w, p] - sum_{q < p} X[w, q] L[p, q]^T,   X[w, p] = Z Li_pp^T
// (40 MFMAs on one dependency chain per wave; no barrier inside: a wave's
// LDS accesses complete in order).  Waves >= row_tiles return at once (Y's
// first 16 row_tiles rows are solved).
template <typename P, typename CP>
__device__ inline void lds_trsm64_rt(P Y, CP L, CP Li, int row_tiles = 4) {
  const int w = threadIdx.x >> 6;
  if (w >= row_tiles) return;
  const int l = threadIdx.x & 63, fr = l & 15, fk = l >> 4;
  const int r0 = 16 * w;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    d4 acc = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < p; ++q)
#pragma unroll
      for (int k0 = 0; k0 < 16; k0 += 4) {
        const double a = Y[(r0 + fr) * SMG_NBP + 16 * q + k0 + fk];  // X[w, q](fr, k)
        const double b = L[(16 * p + fr) * SMG_NBP + 16 * q + k0 + fk];  // L[p, q]^T(k, fr)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
      }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      auto y = &Y[(r0 + fk + 4 * r) * SMG_NBP + 16 * p + fr];
      *y = *y - acc[r];
    }
    d4 x = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int k0 = 0; k0 < 16; k0 += 4) {
      const double a = Y[(r0 + fr) * SMG_NBP + 16 * p + k0 + fk];        // Z(fr, k)
      const double b = Li[(16 * p + fr) * SMG_NBP + 16 * p + k0 + fk];   // Li_pp^T(k, fr)
      x = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, x, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) Y[(r0 + fk + 4 * r) * SMG_NBP + 16 * p + fr] = x[r];
  }
}

// Drop-in for lds_potrf_inv64_v2 built from the blocked pieces: factor (if
// asked) then invert, then one coalesced write of L (lower) and X = L^{-1}.
__device__ __forceinline__ void lds_potrf_inv64_blk(double* D, double* X, int b, double* Lout, int ldl,
                                           double* Xout, int ldx, int* status, bool factor) {
  __shared__ double T[3 * 256];
  if (factor) lds_potrf64_lookahead(D, status);
  lds_trtri64_mfma(D, X, T);
  for (int e = threadIdx.x; e < b * b; e += blockDim.x) {
    const int c = e / b, r = e % b;
    if (Lout) Lout[r + (size_t)c * ldl] = (r >= c) ? D[r * SMG_NBP + c] : 0.0;
    if (Xout) Xout[r + (size_t)c * ldx] = (r >= c) ? X[r * SMG_NBP + c] : 0.0;
  }
}

// load a b x b block (col-major, ld) into LDS [r][c]; lower_only zeroes the
// strict upper triangle; rows/cols >= b are identity padding
__device__ inline void lds_load_block(double* D, const double* A, int ld, int b, bool lower_only) {
  constexpr int PER = SMG_NB * SMG_NB / SMG_DIAG_THREADS;
  if (blockDim.x == SMG_DIAG_THREADS) {  // all global loads in flight at once
    double v[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int e = threadIdx.x + q * SMG_DIAG_THREADS;
      const int c = e / SMG_NB, r = e % SMG_NB;
      v[q] = (r < b && c < b && (!lower_only || r >= c)) ? A[r + (size_t)c * ld] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int e = threadIdx.x + q * SMG_DIAG_THREADS;
      const int c = e / SMG_NB, r = e % SMG_NB;
      D[r * SMG_NBP + c] = (r < b && c < b) ? v[q] : (r == c ? 1.0 : 0.0);
    }
    return;
  }
  for (int e = threadIdx.x; e < SMG_NB * SMG_NB; e += blockDim.x) {
    const int c = e / SMG_NB, r = e % SMG_NB;
    double v;
    if (r < b && c < b)
      v = (!lower_only || r >= c) ? A[r + (size_t)c * ld] : 0.0;
    else
      v = (r == c) ? 1.0 : 0.0;
    D[r * SMG_NBP + c] = v;
  }
}

// zero-padded load (no identity): for adjoint blocks
__device__ inline void lds_load_block0(double* D, const double* A, int ld, int b, bool lower_only) {
  constexpr int PER = SMG_NB * SMG_NB / SMG_DIAG_THREADS;
  if (blockDim.x == SMG_DIAG_THREADS) {  // all global loads in flight at once
    double v[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int e = threadIdx.x + q * SMG_DIAG_THREADS;
      const int c = e / SMG_NB, r = e % SMG_NB;
      v[q] = (r < b && c < b && (!lower_only || r >= c)) ? A[r + (size_t)c * ld] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int e = threadIdx.x + q * SMG_DIAG_THREADS;
      D[(e % SMG_NB) * SMG_NBP + e / SMG_NB] = v[q];
    }
    return;
  }
  for (int e = threadIdx.x; e < SMG_NB * SMG_NB; e += blockDim.x) {
    const int c = e / SMG_NB, r = e % SMG_NB;
    double v = 0.0;
    if (r < b && c < b && (!lower_only || r >= c)) v = A[r + (size_t)c * ld];
    D[r * SMG_NBP + c] = v;
  }
}

__device__ inline void lds_store_block(const double* D, double* A, int ld, int b, bool lower_only) {
  for (int e = threadIdx.x; e < b * b; e += blockDim.x) {
    const int c = e / b, r = e % b;
    if (lower_only && r < c) continue;
    A[r + (size_t)c * ld] = D[r * SMG_NBP + c];
  }
}
