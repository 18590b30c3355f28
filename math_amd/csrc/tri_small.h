// Small dense triangular kernels on one diagonal block (<= 64 x 64) held in
// LDS by one 256-thread workgroup.  Shared by the Cholesky forward/reverse and
// the blocked triangular solves.
#pragma once
#include "smg_internal.h"

constexpr int SMG_NB = 64;        // diagonal block size of every blocked kernel
constexpr int SMG_NBP = SMG_NB + 1;  // padded LDS row stride

// X (lower, b x b in LDS, stride SMG_NBP) <- inverse of lower-triangular D
// (LDS, same layout).  Row-sequential forward substitution; threads over the
// columns c <= r of row r.  X and D must not alias.
__device__ inline void lds_tri_inverse_lower(const double* D, double* X, int b) {
  for (int e = threadIdx.x; e < SMG_NB * SMG_NBP; e += blockDim.x) X[e] = 0.0;
  __syncthreads();
  for (int r = 0; r < b; ++r) {
    const double inv_rr = 1.0 / D[r * SMG_NBP + r];
    for (int c = threadIdx.x; c <= r; c += blockDim.x) {
      double s = (r == c) ? 1.0 : 0.0;
      for (int t = c; t < r; ++t) s -= D[r * SMG_NBP + t] * X[t * SMG_NBP + c];
      X[r * SMG_NBP + c] = s * inv_rr;
    }
    __syncthreads();
  }
}

// In-LDS right-looking Cholesky of the lower triangle of D (b x b).
// Latches SMG_ERR_NOT_PD in *status when a pivot is not > 0 / not finite
// (check_pos_definite, prim/mat/err/check_pos_definite.hpp:77-81).
__device__ inline void lds_potrf_lower(double* D, int b, int* status) {
  for (int j = 0; j < b; ++j) {
    const double piv = D[j * SMG_NBP + j];
    const bool ok = piv > 0.0 && isfinite(piv);
    if (!ok && threadIdx.x == 0) atomicOr(status, (int)SMG_ERR_NOT_PD);
    const double ljj = ok ? sqrt(piv) : 1.0;
    const double inv = 1.0 / ljj;
    __syncthreads();
    for (int i = j + 1 + threadIdx.x; i < b; i += blockDim.x) D[i * SMG_NBP + j] *= inv;
    if (threadIdx.x == 0) D[j * SMG_NBP + j] = ljj;
    __syncthreads();
    const int m = b - j - 1;
    // trailing lower triangle (i >= c > j)
    for (int e = threadIdx.x; e < m * m; e += blockDim.x) {
      const int c = j + 1 + e / m, i = j + 1 + e % m;
      if (i >= c) D[i * SMG_NBP + c] -= D[i * SMG_NBP + j] * D[c * SMG_NBP + j];
    }
    __syncthreads();
  }
}

// load a b x b block (col-major, ld) into LDS (row-major [r][c], stride SMG_NBP);
// lower_only zeroes the strict upper triangle
__device__ inline void lds_load_block(double* D, const double* A, int ld, int b, bool lower_only) {
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
