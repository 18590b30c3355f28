// Dev microbenchmarks: the GEMM shapes of one GP N = 4096 gradient evaluation
// (two-level Cholesky forward with 512-column panels, Murray reverse with
// 512-column blocks), shared by tools/ubench_gemm.cpp (the hand-written GEMM)
// and tools/ubench_rocblas.cpp (rocBLAS, a reference point only).
#pragma once
struct ub_shape {
  const char* name;
  int ta, tb, uplo, m, n, k;
  int tri;  // SMG_TRI_* (smg_gemm_tri), 0: dense
  double fl;  // useful flops when the formula below does not apply (0: use it)
};
static const ub_shape ub_shapes[] = {
    // forward: (a) next panel's columns (lower trapezoid), (b) the rest (SYRK)
    {"fwd (a) NT lower (3584,512,512)", 0, 1, 1, 3584, 512, 512},
    {"fwd (a) NT lower (2048,512,512)", 0, 1, 1, 2048, 512, 512},
    {"fwd (b) SYRK (3072,3072,512)", 0, 1, 1, 3072, 3072, 512},
    {"fwd (b) SYRK (2048,2048,512)", 0, 1, 1, 2048, 2048, 512},
    {"fwd (b) SYRK (1024,1024,512)", 0, 1, 1, 1024, 1024, 512},
    // reverse, block P (J = 512 P, K = J + 512, m = 4096 - K)
    {"rev C*W NN (3072,512,512)", 0, 0, 0, 3072, 512, 512},
    {"rev C*W NN (1536,512,512)", 0, 0, 0, 1536, 512, 512},
    {"rev B_adj NN (2048,1536,512)", 0, 0, 0, 2048, 1536, 512},
    {"rev B_adj NN (1024,2560,512)", 0, 0, 0, 1024, 2560, 512},
    {"rev B_adj NN (3072,512,512)", 0, 0, 0, 3072, 512, 512},
    {"rev [R|D] TN (512,2048,2048)", 1, 0, 0, 512, 2048, 2048},
    {"rev [R|D] TN (512,1024,3072)", 1, 0, 0, 512, 1024, 3072},
    {"rev [R|D] TN (512,3584,512)", 1, 0, 0, 512, 3584, 512},
    {"rev sym TN (512,512,512)", 1, 0, 0, 512, 512, 512},
    {"rev sym NN (512,512,512)", 0, 0, 0, 512, 512, 512},
    {"rev P*R NN (512,2048,512)", 0, 0, 0, 512, 2048, 512},
    {"rev P*R NN (512,3584,512)", 0, 0, 0, 512, 3584, 512},
    {"big NN (4096,4096,4096)", 0, 0, 0, 4096, 4096, 4096},
    // progressive K^{-1} (chol_mvn.hip smg_inv_prog_row), block row k = 7 / 6
    {"prog share TN lower (4096,4096,512)", 1, 0, 1, 4096, 4096, 512},
    {"prog share NT lower (4096,4096,512)", 0, 1, 1, 4096, 4096, 512},
    {"prog share TN lower (3584,3584,512)", 1, 0, 1, 3584, 3584, 512},
    {"prog Y NN triB (512,3584,3584)", 0, 0, 0, 512, 3584, 3584, 4},
    {"prog Y NN dense (512,3584,3584)", 0, 0, 0, 512, 3584, 3584},
    {"prog W NN triA (512,3584,512)", 0, 0, 0, 512, 3584, 512, 1},
    // the HVP's Cholesky tangent node at N = 4096 (chol_tangent.hip); flops
    // counted over the cut K ranges (N^3 = 68.7 GFLOP)
    {"hvp T=tril(W A') NT lower triA", 0, 1, 1, 4096, 4096, 4096, 1, 2.0 / 3.0 * 68719476736.0},
    {"hvp Y=T W^T NT sym triB_up", 0, 1, 3, 4096, 4096, 4096, 8, 1.0 / 3.0 * 68719476736.0},
    {"hvp M=W^T S NN triA_up", 0, 0, 0, 4096, 4096, 4096, 2, 68719476736.0},
    {"hvp tril(M Y) NT lower", 0, 1, 1, 4096, 4096, 4096, 0, 68719476736.0},
    {"hvp (1/2)M W NT upper triB_lo", 0, 1, 2, 4096, 4096, 4096, 4, 1.0 / 3.0 * 68719476736.0},
    {"hvp L P NN lower triA_lo triB_lo", 0, 0, 1, 4096, 4096, 4096, 5, 1.0 / 3.0 * 68719476736.0},
    {"hvp T P^T NT lower triA_lo triB_up", 0, 1, 1, 4096, 4096, 4096, 9, 1.0 / 3.0 * 68719476736.0},
    {"hvp L^T T TN lower triA_up triB_lo", 1, 0, 1, 4096, 4096, 4096, 6, 1.0 / 3.0 * 68719476736.0},
};
static const int ub_nshapes = sizeof(ub_shapes) / sizeof(ub_shapes[0]);
static inline double ub_flops(const ub_shape& s) {
  if (s.fl > 0) return s.fl;
  if (s.uplo) {  // lower trapezoid of an m x n product (n <= m): n (n + 1) / 2 + (m - n) n entries
    const double e = (double)s.n * (s.n + 1) / 2 + (double)(s.m - s.n) * s.n;
    return 2.0 * e * s.k;
  }
  return (s.tri ? 1.0 : 2.0) * s.m * s.n * s.k;  // a triangular operand: ~half the products
}
