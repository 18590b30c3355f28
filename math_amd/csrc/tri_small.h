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
constexpr int SMG_NBP = SMG_NB + 1;  // padded LDS row stride

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

// load a b x b block (col-major, ld) into LDS [r][c]; lower_only zeroes the
// strict upper triangle; rows/cols >= b are identity padding
__device__ inline void lds_load_block(double* D, const double* A, int ld, int b, bool lower_only) {
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
