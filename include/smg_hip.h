/*
 * smg_hip.h — the C-ABI of libsmg_hip.so, the MI355X (gfx950) device side of
 * the Stan-Math-compatible reverse-mode hot path.
 *
 * The reference (Stan Math 3.0.0) is header-only C++ with no FFI; its device
 * offload boundary is the set of `#ifdef STAN_OPENCL` hooks inside the rev
 * functors' constructors (forward) and chain() (reverse).  Each entry point
 * below replaces one such forward or chain() body and is called only by the
 * header-only host layer in math_amd/include/stan/math/ (vari subclasses) or,
 * in tests, through ctypes.  The replaced reference code is cited per entry.
 *
 * Conventions
 *  - every matrix is column-major fp64 with an explicit leading dimension;
 *  - every pointer argument is a DEVICE pointer unless named *_host;
 *  - work is enqueued on the context's HIP stream and is asynchronous; the
 *    only synchronising calls are smg_sync / smg_status / smg_memcpy_d2h_sync;
 *  - adjoint outputs ACCUMULATE (+=), like vari::adj_ in the reference
 *    (rev/core/vari.hpp:30-143): callers zero them once per sweep;
 *  - nothing throws across this boundary: every function returns SMG_OK or an
 *    error code; device-detected domain errors (not positive definite,
 *    not symmetric, non-finite) are latched in the context status word and
 *    read with smg_status(), which the C++ layer turns into the reference's
 *    std::domain_error (prim/scal/err/domain_error.hpp:28-33).
 */
#ifndef SMG_HIP_H
#define SMG_HIP_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

enum smg_status_code {
  SMG_OK = 0,
  SMG_ERR_HIP = 1,            /* a HIP runtime call failed */
  SMG_ERR_NOT_PD = 2,         /* check_pos_definite (prim/mat/err/check_pos_definite.hpp:77-81) */
  SMG_ERR_NOT_SYMMETRIC = 4,  /* check_symmetric, abs tol 1e-8 (prim/mat/err/check_symmetric.hpp:43-44) */
  SMG_ERR_NONFINITE = 8,      /* check_finite / not_nan family */
  SMG_ERR_ARG = 16,           /* bad sizes / null pointers (host-side check) */
  SMG_ERR_OOM = 32,           /* device arena exhausted */
  SMG_ERR_NOT_POSITIVE = 64,  /* check_positive */
  SMG_ERR_SYNC = 128          /* a cross-workgroup wait of a device kernel timed out */
};

typedef struct smg_ctx smg_ctx;

/* ------------------------------------------------------------ context ---
 * One context per host thread = one HIP stream + one device bump arena.
 * Mirrors the per-thread AutodiffStackSingleton tape
 * (rev/core/autodiffstackstorage.hpp:88-143) and its stack_alloc arena
 * (memory/stack_alloc.hpp:72-287): blocks double in size, nested marks,
 * bulk release only. */
int smg_device_count(int* n_host);
int smg_ctx_create(int device, size_t initial_arena_bytes, smg_ctx** out_host);
int smg_ctx_destroy(smg_ctx* ctx);
int smg_ctx_device(const smg_ctx* ctx);
void* smg_ctx_stream(smg_ctx* ctx); /* hipStream_t */

/* stack_alloc::alloc (:169-178); 256-byte aligned; NULL + SMG_ERR_OOM latched on failure */
void* smg_arena_alloc(smg_ctx* ctx, size_t bytes);
/* stack_alloc::start_nested / recover_nested (:209-231) as explicit marks */
size_t smg_arena_mark(smg_ctx* ctx);
int smg_arena_rewind(smg_ctx* ctx, size_t mark);
/* stack_alloc::recover_all (:199) and bytes_allocated (:251) */
int smg_arena_recover_all(smg_ctx* ctx);
size_t smg_arena_used(const smg_ctx* ctx);
size_t smg_arena_reserved(const smg_ctx* ctx);
/* pinned host staging buffer (lifetime of the context) */
void* smg_host_scratch(smg_ctx* ctx, size_t bytes);
/* pinned host memory mapped into the device (zero-copy operands and outputs
 * of the *_fused entries; coarse-grained: the kernels publish it with one
 * system-scope release); grown on demand, reused by the next call */
void* smg_pinned_io(smg_ctx* ctx, size_t bytes);
/* pinned host memory mapped into the device, fine-grained (coherent): every
 * kernel store reaches the host without relying on a cache write-back, so
 * the host may read it as soon as the completion word moves.  For small
 * results published by the zero-copy reducer steps (the GLM's M + 3 sums);
 * grown on demand, reused by the next call. */
void* smg_pinned_result(smg_ctx* ctx, size_t bytes);
/* dst (pinned host memory from smg_pinned_io) <- n device doubles of src, in
 * stream order, written by a one-workgroup kernel that then publishes a
 * completion word; returns once they have landed (no copy-engine transfer,
 * no stream synchronisation).  For small results read right after the work
 * that produced them (the row-sharded reducers after their all-reduce). */
int smg_publish_to_host(smg_ctx* ctx, const double* src, long long n, double* dst);
/* dst[i] <- *src[i] for n device scalars (src a host array of device
 * pointers), in stream order, written to fine-grained pinned memory (dst from
 * smg_pinned_result) by one kernel that then publishes the completion word;
 * returns once they have landed -- the reverse sweep's device->host scalar
 * adjoints (the reference's vari::adj_ of scalar operands) in one launch and
 * one host wait instead of a copy and a stream synchronisation each.
 * status_out != NULL: the device status word as well (smg_status_enqueue). */
int smg_gather_scalars(smg_ctx* ctx, const double* const* src, int n, double* dst, int* status_out);

int smg_memcpy_h2d(smg_ctx* ctx, void* dst, const void* src_host, size_t bytes);
int smg_memcpy_d2h(smg_ctx* ctx, void* dst_host, const void* src, size_t bytes);
int smg_memcpy_d2d(smg_ctx* ctx, void* dst, const void* src, size_t bytes);
int smg_memset(smg_ctx* ctx, void* dst, int value, size_t bytes);
/* Zero `bytes` at dst on the context's zeroing stream, after everything
 * already enqueued on the main stream, overlapping what is enqueued there
 * next; smg_join_async makes the main stream wait for every such zeroing
 * (the tape zeroes large adjoint buffers this way and joins before the
 * reverse sweep, grad.hpp).  The zeroing may be issued later than the call:
 * at the next latency-bound entry (Cholesky panels, persistent solves), at
 * smg_join_async or at an arena rewind / recover, whichever comes first; the
 * buffer must not be touched on the main stream before smg_join_async. */
int smg_memset_async(smg_ctx* ctx, void* dst, size_t bytes);
int smg_join_async(smg_ctx* ctx);
int smg_sync(smg_ctx* ctx);
/* Block the host until every stream of the context (main, side, zeroing) is
 * idle: work queued on a speculation that is then discarded (the Eigen
 * boundary's cholesky_decompose of a block that turns out modified). */
int smg_sync_all(smg_ctx* ctx);
/* Host-side pipelining: record marker `slot` (0..63) on the context stream
 * after the work enqueued so far; smg_marker_wait blocks the host until the
 * stream reaches it (e.g. a large device->host copy issued in chunks whose
 * host-side consumption overlaps the next chunk's transfer). */
int smg_marker_record(smg_ctx* ctx, int slot);
int smg_marker_wait(smg_ctx* ctx, int slot);
/* synchronise, return the latched status bits (0 = ok) and clear them */
int smg_status(smg_ctx* ctx, int* status_host);
/* 1 when a launch that can latch the status word asynchronously (a persistent
 * solve or panel: SMG_ERR_SYNC on a timed-out hand-off) was enqueued since the
 * status was last read; the reverse sweep reads it then (stan::math::grad) */
int smg_status_armed(smg_ctx* ctx, int* armed);
/* enqueue (no sync) the copy of the status word into pinned host_dst (the
 * word stays latched: smg_status reads and clears it); the caller reads
 * host_dst after its next smg_sync */
int smg_status_enqueue(smg_ctx* ctx, int* host_dst);
/* test hook: OR `bits` into the device status word (arms it) */
int smg_status_inject(smg_ctx* ctx, int bits);
/* test hook: the 256/512-level block inverses of a progressive block row by
 * mode 0: one launch (k_inv_block512, 64 workgroups behind grid-wide counters)
 *         when the device holds them beside a panel launch (occupancy, checked
 *         once per context), else the six-launch chain;
 * mode 1: always the six-launch chain */
int smg_set_inv_block_mode(smg_ctx* ctx, int mode);
/* 1 when mode 0 takes the one-launch form for an n x n factorisation on this
 * device, 0 if not, -1 on a null ctx or n <= 0 */
int smg_inv_block_fused(smg_ctx* ctx, int n);

/* ------------------------------------------------------- instrumentation ---
 * HIP-event timing of the kernel families on the context stream (used by
 * bench.py to report the dominant kernel's average launch duration). */
enum smg_family {
  SMG_FAM_GEMM = 0, SMG_FAM_CHOL_FWD = 1, SMG_FAM_CHOL_REV = 2,
  SMG_FAM_GP = 3, SMG_FAM_MVN = 4, SMG_FAM_TRSV = 5, SMG_FAM_GLM = 6,
  SMG_FAM_ELEMWISE = 7,
  SMG_FAM_PANEL = 8,  /* each k_chol_panel launch alone (flops: its in-panel work m b^2 - 2 b^3 / 3) */
  SMG_FAM_COMM = 9,   /* each RCCL all-reduce (smg_comm_allreduce_sum) */
  SMG_FAM_COUNT = 10
};
int smg_profile_enable(smg_ctx* ctx, int on);
/* total milliseconds and number of timed regions per family since enable */
int smg_profile_read(smg_ctx* ctx, int family, double* total_ms_host, long long* count_host);
/* algorithmic flops issued per family since enable (GEMM: 2mnk per call) */
int smg_profile_flops(smg_ctx* ctx, int family, double* flops_host);

/* deterministic synthetic data on the device (SplitMix64, oracle/gen.h):
 * out[i] = a + (b - a) * u_i  /  out[i] = (u_i < p) */
int smg_fill_unif(smg_ctx* ctx, double* out, long long n, unsigned long long seed,
                  double a, double b, double scale);
int smg_fill_bernoulli(smg_ctx* ctx, int* out, long long n, unsigned long long seed, double p);

/* --------------------------------------------------------------- BLAS-3 ---
 * C = alpha op(A) op(B) + beta C  (op = transpose when trans != 0), fp64 MFMA
 * (v_mfma_f64_16x16x4_f64).  uplo: 0 = full C, 1 = only the lower triangle of
 * C (i >= j) is computed and written (SYRK-style), 2 = only the upper, 3 = the
 * lower triangle computed and written to both triangles (a symmetric C).  Replaces the Eigen GEMMs
 * in multiply_mat_vari (rev/mat/fun/multiply.hpp:65-135) and
 * cholesky_block::chain (rev/mat/fun/cholesky_decompose.hpp:135-158). */
int smg_gemm(smg_ctx* ctx, int transA, int transB, int uplo, int m, int n, int k,
             double alpha, const double* A, int lda, const double* B, int ldb,
             double beta, double* C, int ldc);
/* smg_gemm with triangular operands: tri = OR of SMG_TRI_A_LOWER (op(A)(i,k)
 * = 0 for k > i), SMG_TRI_A_UPPER (= 0 for k < i), SMG_TRI_B_LOWER (op(B)(k,j)
 * = 0 for k < j), SMG_TRI_B_UPPER (= 0 for k > j).  Every output tile's K
 * loop covers only the k where both operands can be nonzero (a lower x lower
 * product with lower output: 1/6 of the dense multiply-adds); the zeros must
 * be stored.  Used by the tangent L' = L Phi and its reverse, and by the
 * triangular solves' diagonal-block products. */
#define SMG_TRI_A_LOWER 1
#define SMG_TRI_A_UPPER 2
#define SMG_TRI_B_LOWER 4
#define SMG_TRI_B_UPPER 8
int smg_gemm_tri(smg_ctx* ctx, int transA, int transB, int uplo, int tri, int m, int n, int k, double alpha,
                 const double* A, int lda, const double* B, int ldb, double beta, double* C, int ldc);

/* ---------------------------------------------------------- functors ---- */

/* gp_exp_quad_cov(std::vector<double> x, var sigma, var l)
 *   fwd: rev/mat/fun/gp_exp_quad_cov.hpp:64-94   K (n x n full, symmetric)
 *   rev: :96-112  out[0] += d/dsigma, out[1] += d/dl given the full adjoint
 *        Kadj (entries (i,j),(j,i) alias one vari in the reference, :233-238). */
int smg_gp_exp_quad_cov_fwd(smg_ctx* ctx, const double* x, int n, double sigma,
                            double l, double* K, int ldk);
int smg_gp_exp_quad_cov_rev(smg_ctx* ctx, const double* x, int n, double sigma,
                            double l, const double* Kadj, int ldka, double* out2);

/* gp_exp_quad_cov(std::vector<VectorXd> x, var|double sigma, var l) with
 * D-dimensional points (rev/mat/fun/gp_exp_quad_cov.hpp:158-184 forward via
 * squared_distance, :96-112 chain, :211-286 the overloads): x is D x n
 * column-major (point i at x + i D), K_ij = sigma^2 exp(-|x_i - x_j|^2 / (2 l^2)).
 * Same outputs as the scalar-x pair above (D == 1 is that pair); D x n
 * doubles of one point are staged in LDS (D <= 8192). */
int smg_gp_exp_quad_cov_nd_fwd(smg_ctx* ctx, const double* x, int D, int n, double sigma,
                               double l, double* K, int ldk);
int smg_gp_exp_quad_cov_nd_rev(smg_ctx* ctx, const double* x, int D, int n, double sigma,
                               double l, const double* Kadj, int ldka, double* out2);

/* Tangent of the same covariance along (sigma', l') -- what the fvar<var>
 * instantiation of gp_exp_quad_cov computes inside hessian_times_vector
 * (mix/mat/functor/hessian_times_vector.hpp:13-40):
 *   Kd_ij = 2 sigma sigma' e_ij + sigma^2 l' d_ij^2 e_ij / l^3,  e = exp(-d^2/(2 l^2))
 * rev: out4 += [d/dsigma, d/dl, d/dsigma', d/dl'] of sum(Kdadj .* Kd). */
int smg_gp_exp_quad_cov_tangent_fwd(smg_ctx* ctx, const double* x, int n, double sigma,
                                    double l, double dsigma, double dl, double* Kd, int ldk);
int smg_gp_exp_quad_cov_tangent_rev(smg_ctx* ctx, const double* x, int n, double sigma,
                                    double l, double dsigma, double dl, const double* Kdadj,
                                    int ldka, double* out4);

/* add_diag(A, d) (prim/mat/fun/add_diag.hpp:20-55): B = A + diag(d) where d is
 * the host scalar d_scalar (d_vec == NULL) or the device vector d_vec.
 * rev: Aadj += Badj (NULL skips); dadj (device) += diag(Badj), summed into
 * dadj[0] when d_is_vec == 0 (NULL skips). */
int smg_add_diag_fwd(smg_ctx* ctx, const double* A, int lda, int n,
                     double d_scalar, const double* d_vec, double* B, int ldb);
int smg_add_diag_rev(smg_ctx* ctx, const double* Badj, int ldb, int n,
                     double* Aadj, int ldaa, double* dadj, int d_is_vec);

/* cholesky_decompose(Matrix<var>) (rev/mat/fun/cholesky_decompose.hpp:378-427)
 *   check: latches SMG_ERR_NOT_SYMMETRIC when |A_ij - A_ji| > 1e-8 (:383)
 *   fwd:   L = lower Cholesky factor (upper zeroed); latches SMG_ERR_NOT_PD.
 *          aux (smg_cholesky_aux_doubles(n) doubles, may be NULL) receives the
 *          inverses of L's diagonal blocks at 64, 128, 256 and 512
 *          granularity (n x 64 | n x 128 | n x 256 | n x 512, each leading
 *          dimension n), reused by the reverse pass and by the triangular
 *          solves (TRSV / MVN / TRSM).
 *   rev:   Murray's blocked adjoint (:118-165): Aadj(lower) += f(L, Ladj);
 *          Ladj (lower) is used as workspace and overwritten; aux as written
 *          by the forward, or NULL (recomputed). */
long long smg_cholesky_aux_doubles(int n);
int smg_cholesky_block_size(int n);
int smg_check_symmetric(smg_ctx* ctx, const double* A, int lda, int n);
int smg_cholesky_fwd(smg_ctx* ctx, const double* A, int lda, int n, double* L,
                     int ldl, double* aux);
/* check_symmetric(A) (tolerance 1e-8, prim/mat/err/check_symmetric.hpp:37-52)
 * fused with smg_cholesky_fwd's copy of A into L -- one pass over A; the
 * status latches SMG_ERR_NOT_SYMMETRIC and / or SMG_ERR_NOT_PD.  Replaces
 * smg_check_symmetric followed by smg_cholesky_fwd. */
int smg_cholesky_fwd_checked(smg_ctx* ctx, const double* A, int lda, int n, double* L, int ldl,
                             double* Dinv);
/* smg_cholesky_fwd_checked with a status mark after the last launch that can
 * latch the status (before the block inverses): smg_status_mark_wait then
 * returns the symmetric / not-PD bits (and resets them) without waiting for
 * the rest of the entry, so the host enqueues the next node's work while the
 * device finishes it.  Same throw points as the reference
 * (rev/mat/fun/cholesky_decompose.hpp:380-406: the check fails the call). */
int smg_cholesky_fwd_checked_mark(smg_ctx* ctx, const double* A, int lda, int n, double* L, int ldl,
                                  double* Dinv);
/* Wait for the latest status mark and read (and reset) the status it copied;
 * with no mark pending this is smg_status. */
int smg_status_mark_wait(smg_ctx* ctx, int* status);
int smg_cholesky_rev(smg_ctx* ctx, const double* L, int ldl, const double* aux,
                     double* Ladj, int ldla, int n, double* Aadj, int ldaa);

/* mdivide_left_tri<TriView>(A, B) (rev/mat/fun/mdivide_left_tri.hpp:16-373)
 *   fwd: C = tri(A)^{-1} B              (lower != 0: Eigen::Lower, else Upper)
 *   rev: Badj += tri(A)^{-T} Cadj ; Aadj(tri) -= (tri(A)^{-T} Cadj) C^T
 * Aadj / Badj may be NULL (double operands).  ws: >= m*n doubles workspace. */
int smg_mdivide_left_tri_fwd(smg_ctx* ctx, int lower, const double* A, int lda,
                             const double* B, int ldb, int m, int n, double* C,
                             int ldc);
int smg_mdivide_left_tri_rev(smg_ctx* ctx, int lower, const double* A, int lda,
                             const double* C, int ldc, const double* Cadj,
                             int ldca, int m, int n, double* Aadj, int ldaa,
                             double* Badj, int ldba, double* ws);
/* The same with A = a Cholesky factor and aux its smg_cholesky_fwd block
 * inverses (n x SMG_AUX_COLS doubles, ld m; NULL: computed per call, as
 * above): the solves reuse them instead of rebuilding them from A (lower
 * only; upper ignores aux).  The fvar<var> MVN tangent's solves against L. */
int smg_mdivide_left_tri_aux_fwd(smg_ctx* ctx, int lower, const double* A, int lda, const double* aux,
                                 const double* B, int ldb, int m, int n, double* C, int ldc);
int smg_mdivide_left_tri_aux_rev(smg_ctx* ctx, int lower, const double* A, int lda, const double* aux,
                                 const double* C, int ldc, const double* Cadj, int ldca, int m, int n, double* Aadj,
                                 int ldaa, double* Badj, int ldba, double* ws);

/* mdivide_left_spd(A, B) (rev/mat/fun/mdivide_left_spd.hpp:20-150)
 *   fwd: L = chol(lower(A)) into L (m x m, ld m) and aux
 *        (smg_cholesky_aux_doubles(m)); C = A^{-1} B via two blocked TRSMs.
 *        Latches SMG_ERR_NOT_PD.
 *   rev: W = A^{-1} Cadj; Aadj -= W C^T (every entry); Badj += W.
 *        Aadj / Badj may be NULL.  ws: >= m*n doubles. */
int smg_mdivide_left_spd_fwd(smg_ctx* ctx, const double* A, int lda,
                             const double* B, int ldb, int m, int n, double* L,
                             double* aux, double* C, int ldc);
int smg_mdivide_left_spd_rev(smg_ctx* ctx, const double* L, const double* aux,
                             int m, int n, const double* C, int ldc,
                             const double* Cadj, int ldca, double* Aadj,
                             int ldaa, double* Badj, int ldba, double* ws);

/* log_determinant_spd(A) (rev/mat/fun/log_determinant_spd.hpp:16-57)
 *   fwd: L = chol(lower(A)) (+aux), out[0] = 2 sum log L_ii; latches
 *        SMG_ERR_NOT_PD.
 *   rev: Aadj += adj * A^{-1} (every entry).  ws: >= n*n doubles. */
int smg_log_determinant_spd_fwd(smg_ctx* ctx, const double* A, int lda, int n,
                                double* L, double* aux, double* out);
int smg_log_determinant_spd_rev(smg_ctx* ctx, const double* L,
                                const double* aux, int n, double adj,
                                double* Aadj, int ldaa, double* ws);

/* log_determinant(A) of a general square A (rev/mat/fun/log_determinant.hpp:14-37;
 * the reference factors with a full-pivoting Householder QR, this with a
 * blocked LU with partial pivoting: the same |det| and A^{-T})
 *   fwd: LU (n x n, ld n) = P A's unit-lower L and U, piv (n ints) = the row
 *        swaps (LAPACK ipiv, 0-based), out[0] = sum_i log|u_ii| (-inf for a
 *        singular A).  ws: >= 64*64 doubles.
 *   rev: Aadj += adj * A^{-T}.  ws: >= 3*n*n doubles, iws: >= n ints. */
int smg_log_determinant_fwd(smg_ctx* ctx, const double* A, int lda, int n,
                            double* LU, int* piv, double* ws, double* out);
int smg_log_determinant_rev(smg_ctx* ctx, const double* LU, const int* piv,
                            int n, double adj, double* Aadj, int ldaa,
                            double* ws, int* iws);

/* Tangent pieces of the fvar<var> (fwd-over-rev) functors (SURVEY.md 8(f)
 * row 4; mix/fvar_functors.hpp):
 *   smg_add_tril: Y(i >= j) += alpha X(i >= j) (m x n).
 *   smg_lse_tangent_fwd: out[0] = log_sum_exp(x), out[1] = sum_i
 *     exp(x_i - out[0]) xd_i (fwd/mat/fun/log_sum_exp.hpp).  rev: xadj +=
 *     adj p (xd - t), xdadj += adj p, p = exp(x - lse) (either may be NULL).
 *   smg_glm_tangent_fwd: out[0] = sum_i d_i (etad_i + alphad), d_i = the
 *     reference's theta_derivative of bernoulli_logit_glm_lpmf at theta_i =
 *     eta_i + alpha (prim/mat/prob/bernoulli_logit_glm_lpmf.hpp:117-123).
 *     rev: eta_adj += adj d'(theta) (etad + alphad), etad_adj += adj d;
 *     out[0], out[1] = their sums (alpha's and alphad's adjoints). */
/* Y = tril(X) (m x n): Y(i >= j) = X(i >= j), Y's strict upper triangle is
 * stored as zeros (write-only).  The work copy of L's adjoint that
 * smg_cholesky_rev overwrites: it reads the lower triangle of X only, and the
 * Murray reverse may read the work matrix's strict upper as stored zeros. */
int smg_copy_tril(smg_ctx* ctx, int m, int n, const double* X, int ldx, double* Y, int ldy);
int smg_add_tril(smg_ctx* ctx, int m, int n, double alpha, const double* X,
                 int ldx, double* Y, int ldy);
int smg_lse_tangent_fwd(smg_ctx* ctx, const double* x, const double* xd,
                        long long n, double* out);
int smg_lse_tangent_rev(smg_ctx* ctx, const double* x, const double* xd,
                        long long n, double lse, double t, double adj,
                        double* xadj, double* xdadj);
int smg_glm_tangent_fwd(smg_ctx* ctx, const double* eta, double alpha,
                        const double* etad, double alphad, const int* y,
                        long long n, double* out);
int smg_glm_tangent_rev(smg_ctx* ctx, const double* eta, double alpha,
                        const double* etad, double alphad, const int* y,
                        long long n, double adj, double* eta_adj,
                        double* etad_adj, double* out);

/* multiply_lower_tri_self_transpose(L), L: K x J
 * (rev/mat/fun/multiply_lower_tri_self_transpose.hpp:14-44)
 *   fwd: C (K x K) = T T^T, T = lower trapezoid of L.  ws: >= K*J.
 *   rev: Ladj (lower trapezoid) += (Cadj + Cadj^T) T.  ws: >= 2 K*J + K*K. */
int smg_multiply_lower_tri_self_transpose_fwd(smg_ctx* ctx, const double* L,
                                              int ldl, int K, int J, double* C,
                                              int ldc, double* ws);
int smg_multiply_lower_tri_self_transpose_rev(smg_ctx* ctx, const double* L,
                                              int ldl, int K, int J,
                                              const double* Cadj, int ldca,
                                              double* Ladj, int ldla, double* ws);

/* quad_form_sym(A, B), A: M x M symmetric, B: M x N
 * (rev/mat/fun/quad_form_sym.hpp:15-40, quad_form.hpp:17-100)
 *   fwd: C (N x N) = (Cd + Cd^T)/2, Cd = B^T A B.  ws: >= M*N + N*N.
 *   rev: Aadj += B S B^T; Badj += A B S^T + A^T B S (NULL skips), with
 *        S = Cadj, or (Cadj + Cadj^T)/2 when sym_adj (A and B both var: the
 *        prim template, prim/mat/fun/quad_form_sym.hpp:11-18).
 *        ws: >= M*N + N*N. */
int smg_quad_form_sym_fwd(smg_ctx* ctx, const double* A, int lda,
                          const double* B, int ldb, int M, int N, double* C,
                          int ldc, double* ws);
int smg_quad_form_sym_rev(smg_ctx* ctx, const double* A, int lda,
                          const double* B, int ldb, int M, int N,
                          const double* Cadj, int ldca, int sym_adj, double* Aadj,
                          int ldaa, double* Badj, int ldba, double* ws);

/* multiply(A, B) (rev/mat/fun/multiply.hpp:65-135): fwd C = A B;
 * rev Aadj += Cadj B^T, Badj += A^T Cadj (NULL skips an operand). */
/* C = L P for lower-triangular L, P (the Cholesky tangent L' = L Phi(Y) of
 * the fvar<var> functors): lower output, every tile's K range cut to the
 * triangles (N^3/3 flops instead of 2 N^3); the reverse accumulates the
 * lower triangles of L_adj += tril(C_adj) P^T and P_adj += L^T tril(C_adj)
 * (ws: n x n doubles). */
int smg_multiply_lower_fwd(smg_ctx* ctx, const double* L, int ldl, const double* P, int ldp, int n, double* C,
                           int ldc);
/* The tangent of a Cholesky factor, L' = L Phi(L^{-1} A' L^{-T}), as one
 * node (the fvar<var> cholesky_decompose of mix/fvar_functors.hpp; the
 * reference forms the same L' through Eigen's LLT on fvar<var> scalars,
 * prim/mat/fun/cholesky_decompose.hpp).  aux: smg_cholesky_fwd's block
 * inverses of L (NULL: rebuilt).  fwd: W = L^{-1} (lower, zeros
 * above), Wt = W^T, Y = W A' W^T (symmetric, full), P = Phi(Y) (its strict
 * upper zeroed only inside the diagonal tiles: the node's own products read
 * no other part of it), Ld = L P (lower); W, Wt, Y, P: n x n, ld.  rev
 * (Ld_adj lower): Ladj += tril(Ld_adj P^T) - tril(W^T S Y), A'adj +=
 * (1/2) W^T S W (symmetric, both triangles), with S = Phi(Padj) + Phi(Padj)^T,
 * Padj = tril(L^T tril(Ld_adj)); NULL Ladj / Adadj skip.  ws: 2 n^2 doubles.
 * ~5.3 n^3 flops for both against 7 n^3 through two N-column triangular
 * solves.  Independent products run on the context's side stream and are
 * joined before return: the outputs are ordered on the context stream. */
int smg_chol_tangent_fwd(smg_ctx* ctx, const double* L, int ldl, const double* aux, const double* Ad, int ldad, int n,
                         double* W, double* Wt, double* Y, double* P, double* Ld, int ld);
/* smg_chol_tangent_fwd on a given W = L^{-1} (ld, lower; its strict upper
 * is read only inside the 512-row diagonal blocks, as the progressive
 * factorisation leaves it: smg_cholesky_fwd_checked_mark_winv): Wt, Y, P, Ld
 * as above, W itself not written. */
int smg_chol_tangent_fwd_w(smg_ctx* ctx, const double* L, int ldl, const double* W, const double* Ad, int ldad, int n,
                           double* Wt, double* Y, double* P, double* Ld, int ld);
int smg_chol_tangent_rev(smg_ctx* ctx, const double* L, int ldl, const double* W, const double* Wt, const double* Y,
                         const double* P, int ld, const double* Ldadj, int ldla, int n, double* Ladj, int ldladj,
                         double* Adadj, int ldaa, double* ws);
int smg_multiply_lower_rev(smg_ctx* ctx, const double* L, int ldl, const double* P, int ldp, const double* Cadj,
                           int ldca, int n, double* Ladj, int ldla, double* Padj, int ldpa, double* ws);
int smg_multiply_fwd(smg_ctx* ctx, const double* A, int lda, const double* B,
                     int ldb, int m, int k, int n, double* C, int ldc);
int smg_multiply_rev(smg_ctx* ctx, const double* A, int lda, const double* B,
                     int ldb, const double* Cadj, int ldca, int m, int k, int n,
                     double* Aadj, int ldaa, double* Badj, int ldba);

/* multi_normal_cholesky_lpdf<false>(y | mu, L)
 * (prim/mat/prob/multi_normal_cholesky_lpdf.hpp:40-160).
 *   fwd: out3 = [lp, -, -]; w = L^{-1}(y - mu), sd = L^{-T} w kept in ws
 *        (ws >= 2n doubles); aux optional (smg_cholesky_fwd's block inverses).
 *   rev: with adj = d(root)/d(lp) (host scalar):
 *        yadj -= adj sd, muadj += adj sd  (NULL skips)
 *        lower_only != 0: Ladj(lower) += adj (tril(sd w^T) - diag(1/L_ii))
 *          (exact when L's upper triangle is structurally zero, as the output
 *           of cholesky_decompose is: those entries alias a dummy vari, :34-48)
 *        lower_only == 0: Ladj += adj (sd w^T - L^{-T}) over all n^2 entries,
 *          the reference's full partials (:147,155). */
int smg_mvn_cholesky_fwd(smg_ctx* ctx, const double* y, const double* mu,
                         const double* L, int ldl, const double* aux, int n,
                         double* ws, double* out_lp);
int smg_mvn_cholesky_rev(smg_ctx* ctx, const double* L, int ldl,
                         const double* aux, int n, const double* ws, double adj,
                         int lower_only, double* yadj, double* muadj,
                         double* Ladj, int ldla);
/* The same forward on the factor's explicit inverse W = L^{-1} (lower, n x n,
 * ld ldw; n % 64 == 0; W's strict upper is read only inside its diagonal
 * 64 x 64 tiles, which must hold stored zeros there): w = W (y - mu),
 * sd = W^T w as two passes over W's lower triangle -- the reference's own
 * arithmetic, half = inv_L (y - mu), scaled_diff = half inv_L
 * (prim/mat/prob/multi_normal_cholesky_lpdf.hpp:117-131) -- then the same
 * out_lp and ws [w, sd] as smg_mvn_cholesky_fwd. */
int smg_mvn_cholesky_fwd_inv(smg_ctx* ctx, const double* y, const double* mu,
                             const double* L, int ldl, const double* W, int ldw, int n,
                             double* ws, double* out_lp);
/* The context's stream waits until W = L^{-1} of the latest factorisation
 * that formed it progressively (smg_cholesky_fwd_checked_mark_inv with
 * *started == 2, the first n^2 doubles of its ws) is complete, and every
 * earlier one's.  SMG_ERR_ARG when no factorisation has formed one. */
int smg_cholesky_inverse_wait(smg_ctx* ctx);
/* cholesky_decompose's reverse (rev/mat/fun/cholesky_decompose.hpp:118-166)
 * for the one adjoint multi_normal_cholesky_lpdf gives a lower-structured
 * factor (the Ladj above with lower_only = 1: adj (tril(s w^T) - diag(1/L_ii)),
 * s = ws + n of smg_mvn_cholesky_fwd), in closed form:
 *   Aadj (lower) += adj Phi(s s^T - K^{-1}),  K^{-1} = L^{-T} L^{-1}
 * (Phi: strict lower + half diagonal); k observations sharing L (the array
 * form, s_o = s + o s_stride): adj Phi(sum_o s_o s_o^T - k K^{-1}).  aux: the
 * factor's smg_cholesky_fwd
 * block inverses (NULL: a blocked solve forms L^{-1}).  ws: at least
 * smg_cholesky_mvn_rev_ws_doubles(n) doubles. */
size_t smg_cholesky_mvn_rev_ws_doubles(int n);
int smg_cholesky_mvn_rev(smg_ctx* ctx, const double* L, int ldl, const double* aux, int n,
                         const double* s, int k, long long s_stride, double adj, double* Aadj, int ldaa,
                         double* ws);
/* The same in two parts, the first overlapping the MVN's forward solves:
 * smg_cholesky_inv_t_async forms V = L^{-T} in ws (with aux, n % 512 == 0,
 * n >= 1024; else *started = 0 and nothing is queued) on the context's side
 * stream after the work queued so far; smg_cholesky_mvn_rev_v (the same ws,
 * c_formed = 0) joins it, forms K^{-1} and applies the closed form.  With
 * early_done (after smg_cholesky_fwd_checked_mark_inv) it forms the rest of V
 * and K^{-1} itself (then c_formed = 1).  smg_join_async and arena rewinds
 * also join it. */
int smg_cholesky_inv_t_async(smg_ctx* ctx, const double* L, int ldl, const double* aux, int n,
                             double* ws, int early_done, int* started);
/* cholesky_decompose's reverse (rev/mat/fun/cholesky_decompose.hpp:118-166)
 * for any factor adjoint Lbar (its lower triangle is read) in closed form on
 * the factor's inverse W = L^{-1} (lower, zeros above; Wt = W^T, both ld ldw):
 *   Abar (lower) += tril(G + G^T) - diag(G),  G = W^T Phi(L^T tril(Lbar)) W
 * (Phi: lower triangle, half the diagonal): the same adjoint as
 * smg_cholesky_rev's blocked (Murray) algorithm, in three large products.
 * ws: 2 n^2 doubles. */
int smg_cholesky_rev_inverse(smg_ctx* ctx, const double* L, int ldl, const double* W, const double* Wt, int ldw,
                             const double* Ladj, int ldla, int n, double* Aadj, int ldaa, double* ws);
/* (smg_cholesky_mvn_rev / smg_cholesky_mvn_rev_v with Aadj == NULL only form
 * K^{-1} (lower) into ws + n^2; s may then be NULL.)  The closed form's
 * adjoint from that K^{-1} = C (ld n):
 *   Aadj (lower) += adj Phi(sum_o s_o s_o^T - k C)   (the epilogue alone). */
int smg_cholesky_inverse_adjoint(smg_ctx* ctx, const double* C, int ldc, int n, const double* s, int k,
                                 long long s_stride, double adj, double* Aadj, int ldaa);
/* The GP marginal's reverse through add_diag and gp_exp_quad_cov in one pass
 * over K^{-1}'s lower triangle, when that closed-form adjoint
 * G = adj Phi(sum_o s_o s_o^T - k C) is the only adjoint of add_diag(K0, d)
 * and of K0 = gp_exp_quad_cov(x, sigma, l) (values K0, ld ldk; x D x n):
 *   dadj (NULL skips) = sum_i G_ii                   (prim/mat/fun/add_diag.hpp:25-27)
 *   out2 (NULL skips) = [2 sum_{i>=j} G_ij K0_ij / sigma,
 *                        sum_{i>j} G_ij K0_ij d2_ij / l^3]
 *                                                   (rev/mat/fun/gp_exp_quad_cov.hpp:96-112)
 * written (not accumulated); fixed-order sums. */
int smg_gp_inverse_adjoint(smg_ctx* ctx, const double* C, int ldc, int n, const double* s, int k,
                           long long s_stride, double adj, const double* K0, int ldk, const double* x, int D,
                           double sigma, double l, double* dadj, double* out2);
int smg_cholesky_mvn_rev_v(smg_ctx* ctx, int n, const double* s, int k, long long s_stride, double adj,
                           double* Aadj, int ldaa, double* ws, int c_formed);
/* smg_cholesky_fwd_checked_mark that also queues the top half's part of
 * V = L^{-T} (V11, V11 L21^T, with the top half's block inverses) into ws
 * (smg_cholesky_mvn_rev_ws_doubles(n)) on the side stream as soon as the
 * first n/2 columns are factored, in steps behind the remaining trailing
 * updates; *started = 1 when queued (n / 512 a power of two >= 2).  Then
 * smg_cholesky_inv_t_async(..., early_done = 1) queues the rest of V and
 * K^{-1} = V V^T, and smg_cholesky_mvn_rev_v(..., c_formed = 1) applies the
 * closed form.  For a factor whose reverse is predicted to take the closed
 * form (the host layer's history per tape position). */
int smg_cholesky_fwd_checked_mark_inv(smg_ctx* ctx, const double* A, int lda, int n, double* L, int ldl,
                                      double* aux, double* ws, int* started);
/* smg_cholesky_fwd_checked_mark_inv forming W = L^{-1} alone (no K^{-1}
 * shares): the block rows of W progressively beside the panels, W in ws's
 * first n^2 doubles (ld n; lower, its strict upper written inside the 512-row
 * diagonal blocks only) once smg_cholesky_inverse_wait returns; *started = 3
 * when queued (n % 512 == 0, n >= 1024), 0 when not (the plain
 * factorisation ran).  For the HVP's value factor, whose W the Cholesky
 * tangent node reuses (mix/fvar_functors.hpp) instead of forming it after
 * the factorisation; the reference's fvar<var> cholesky_decompose has no
 * inverse at all (prim/mat/fun/cholesky_decompose.hpp:31-39, Eigen LLT). */
/* y = W x (trans 0) or W^T x (trans 1) for the lower triangle of W (n x n,
 * ld ldw, n % 64 == 0; W's strict upper never read): one HBM pass over the
 * lower tiles plus a deterministic in-order sum of the tile partials.  x and
 * y must not alias.  mdivide_left_tri<Lower>(L, b) = L^{-1} b on a factor
 * that carries W = L^{-1} (rev/mat/fun/mdivide_left_tri.hpp:16-130 solves
 * instead) and its reverse's L^{-T} Cadj; multiply(L, b) and its reverse on a
 * structurally lower L (rev/mat/fun/multiply.hpp:65-135). */
int smg_trmv_inv(smg_ctx* ctx, int trans, const double* W, int ldw, int n, const double* x, double* y);
/* A(i, j) += alpha x_i y_j for i >= j (A n x n, ld lda): the lower-triangle
 * adjoint of a structurally lower matrix times a vector, and of
 * mdivide_left_tri's A (rev/mat/fun/mdivide_left_tri.hpp:108-123), one pass */
int smg_rank1_lower(smg_ctx* ctx, int n, double alpha, const double* x, const double* y, double* A, int lda);
int smg_cholesky_fwd_checked_mark_winv(smg_ctx* ctx, const double* A, int lda, int n, double* L, int ldl,
                                       double* aux, double* ws, int* started);
/* smg_cholesky_fwd_checked_mark_inv (ws may be NULL: no K^{-1}) that also
 * streams the factor to the host while it is formed: once panel p (columns
 * [512 p, min(512 (p + 1), n)); one panel when n <= 512) is final, its columns
 * of the packed lower triangle (column-major, column j's rows j..n-1 from
 * j n - j (j - 1) / 2) are packed into `packed` (device, n (n + 1) / 2
 * doubles) and copied into host_dst (pinned host memory of the same size)
 * on the context's zeroing stream, and marker marker_base + p is recorded
 * behind the copy (smg_marker_wait).  smg_cholesky_stream_panels(n) markers;
 * marker_base + that count <= 64.  The Eigen boundary's cholesky_decompose
 * builds the factor's host varis panel by panel while the later panels are
 * factored (the reference's cholesky_decompose returns an Eigen matrix of
 * varis, rev/mat/fun/cholesky_decompose.hpp:378-427). */
int smg_cholesky_stream_panels(int n);
/* The columns [*j0, *j1) panel p of the streamed factor covers (the packed
 * triangle's offsets j n - j (j - 1) / 2 of those columns are what marker
 * marker_base + p covers); SMG_ERR_ARG outside 0 <= p < smg_cholesky_stream_panels(n). */
int smg_cholesky_stream_panel_cols(int n, int p, int* j0, int* j1);
int smg_cholesky_fwd_checked_mark_stream(smg_ctx* ctx, const double* A, int lda, int n, double* L, int ldl,
                                         double* aux, double* ws, int* started, double* packed, double* host_dst,
                                         int marker_base);

/* log_sum_exp(vector<var>) (rev/mat/fun/log_sum_exp.hpp:20-53):
 *   fwd: out = max + log(sum exp(x - max)); empty -> -inf; non-finite max -> max
 *   rev: xadj_i += adj * exp(x_i - lse)   (lse, adj: host values of the vari) */
int smg_log_sum_exp_fwd(smg_ctx* ctx, const double* x, long long n, double* out);
int smg_log_sum_exp_rev(smg_ctx* ctx, const double* x, long long n,
                        double lse, double adj, double* xadj);

/* vectorised lgamma / digamma / trigamma (apply_scalar_unary,
 * rev/mat/vectorize/apply_scalar_unary.hpp:18-32):
 *   lgamma rev: xadj += yadj * digamma(x)   (rev/scal/fun/lgamma.hpp:13-32)
 *   digamma rev: xadj += yadj * trigamma(x) (rev/scal/fun/digamma.hpp:13-22) */
int smg_lgamma_fwd(smg_ctx* ctx, const double* x, long long n, double* y);
int smg_lgamma_rev(smg_ctx* ctx, const double* x, long long n, const double* yadj, double* xadj);
int smg_digamma_fwd(smg_ctx* ctx, const double* x, long long n, double* y);
int smg_digamma_rev(smg_ctx* ctx, const double* x, long long n, const double* yadj, double* xadj);
int smg_trigamma_fwd(smg_ctx* ctx, const double* x, long long n, double* y);

/* normal_lpdf<propto>(y | mu, sigma) (prim/scal/prob/normal_lpdf.hpp:36-119):
 * each operand is a device vector (stride 1) or scalar (stride 0) of n
 * broadcast elements.  include bits: 1 = NEG_LOG_SQRT_TWO_PI term,
 * 2 = -log(sigma) term, 4 = -z^2/2 term (include_summand<propto, ...>).
 * Writes out[0] = logp and per-element partials (NULL skips; scalar operands
 * get their partial summed into element 0). */
int smg_normal_lpdf(smg_ctx* ctx, const double* y, int sy, const double* mu,
                    int smu, const double* sigma, int ssig, long long n,
                    int include, double* out, double* gy, double* gmu,
                    double* gsigma);
/* The same reduction fused with the three domain checks in ONE launch that
 * completes before returning (latency-bound calls, e.g. config 1's 1024 host
 * vars).  A vector operand is a pointer (device memory, or pinned host memory
 * from smg_pinned_io: zero-copy, no separate copies); a NULL pointer selects
 * the scalar value y0 / mu0 / sigma0 (a kernel argument: no memory read).
 * res = [lp, bad_y, bad_mu, bad_sigma, gy, gmu, gsigma (the reduced partials
 * of scalar operands)]; vector partials are WRITTEN (not accumulated).
 * Replaces the body of prim/scal/prob/normal_lpdf.hpp:36-119. */
int smg_normal_lpdf_fused(smg_ctx* ctx, const double* y, const double* mu, const double* sigma, double y0,
                          double mu0, double sigma0, long long n, int include, double* res, double* gy,
                          double* gmu, double* gsigma);

/* bernoulli_logit_glm_lpmf<false>(y | x, alpha, beta), scalar alpha
 * (prim/mat/prob/bernoulli_logit_glm_lpmf.hpp:46-138) in ONE fused pass over
 * x (R x M column-major, leading dimension ldx):
 *   out[0] = logp, out[1] = sum theta', out[2..M+1] = x^T theta'.
 * Deterministic (fixed-order two-stage reduction).  ws: >= smg_glm_ws_doubles. */
long long smg_glm_ws_doubles(long long R, int M);
int smg_bernoulli_logit_glm(smg_ctx* ctx, const int* y, const double* x,
                            long long R, int M, long long ldx,
                            const double* alpha_beta, double* ws, double* out);

/* smg_bernoulli_logit_glm with the reference's check_bounded(y, 0, 1)
 * (prim/mat/prob/bernoulli_logit_glm_lpmf.hpp:75) fused into the same pass:
 * out (M + 3 doubles) = [logp, sum theta', x^T theta' (M), number of y
 * outside {0, 1}].  Replaces smg_check_bounded_int + smg_bernoulli_logit_glm
 * (one launch and one pass over y fewer per evaluation). */
int smg_bernoulli_logit_glm_checked(smg_ctx* ctx, const int* y, const double* x,
                                    long long R, int M, long long ldx,
                                    const double* alpha_beta, double* ws, double* out);
/* The latency-bound form: alpha and beta (M doubles, host memory) are passed
 * in the launch's kernel arguments (no upload), and the pass's last
 * workgroup writes out (device, M + 3 doubles: [logp, alpha', beta'(M),
 * count of y outside {0, 1}]) and, when out_h is non-null (pinned host
 * memory from smg_pinned_io), the same values to out_h, then returns once
 * they have landed (the host spins on a completion word, no stream
 * synchronisation).  With out_h null the call returns without waiting.
 * ws: smg_glm_ws_doubles(R, M) doubles.  Other variants / M > 256 / R == 0
 * take the general path (upload, smg_bernoulli_logit_glm_checked, copy back). */
int smg_bernoulli_logit_glm_io(smg_ctx* ctx, const int* y, const double* x, long long R, int M, long long ldx,
                               double alpha, const double* beta, double* ws, double* out, double* out_h);

/* normal_id_glm_lpdf<false>(y | x, alpha, beta, sigma), scalar alpha and
 * sigma (prim/mat/prob/normal_id_glm_lpdf.hpp:40-150), ONE fused pass over x:
 *   abs = [alpha, beta(M), sigma] (device);
 *   out[0] = sum y_scaled^2, out[1] = sum mu', out[2..M+1] = x^T mu'
 *   with y_scaled = (y - x beta - alpha)/sigma, mu' = y_scaled/sigma.
 * M <= 256.  ws: >= smg_glm_ws_doubles(R, M). */
int smg_normal_id_glm(smg_ctx* ctx, const double* y, const double* x,
                      long long R, int M, long long ldx,
                      const double* alpha_beta_sigma, double* ws, double* out);

/* poisson_log_glm_lpmf<false>(y | x, alpha, beta), scalar alpha
 * (prim/mat/prob/poisson_log_glm_lpmf.hpp:37-123), ONE fused pass over x:
 *   out[0] = sum(y theta - exp theta), out[1] = sum theta',
 *   out[2..M+1] = x^T theta', out[M+2] = sum lgamma(y + 1)
 *   with theta = x beta + alpha, theta' = y - exp(theta).
 * M <= 256.  ws: >= smg_glm_ws_doubles(R, M).  y >= 0 is checked by the
 * caller (smg_check_bounded_int). */
int smg_poisson_log_glm(smg_ctx* ctx, const int* y, const double* x,
                        long long R, int M, long long ldx,
                        const double* alpha_beta, double* ws, double* out);

/* categorical_logit_glm_lpmf<false>(y | x, alpha, beta)
 * (prim/mat/prob/categorical_logit_glm_lpmf.hpp:38-146): x R x M
 * (column-major, ld ldx), alpha_beta = [alpha(C), beta(M x C column-major)],
 * y in 1..C (checked by the caller), ONE fused pass over x:
 *   out[0] = logp, out[1..C] = alpha', out[C+1 ..] = beta' (M x C).
 * M <= 256 and C <= 16: one fused pass; otherwise lin = x beta by GEMM, a
 * row softmax pass, alpha' / beta' by GEMM (R, M C < 2^31).
 * ws: >= smg_glm_categorical_ws_doubles(R, M, C). */
long long smg_glm_categorical_ws_doubles(long long R, int M, int C);
int smg_categorical_logit_glm(smg_ctx* ctx, const int* y, const double* x,
                              long long R, int M, long long ldx, int C,
                              const double* alpha_beta, double* ws, double* out);

/* generic helpers used by the host layer's reverse sweep */
/* y[i*incy] += alpha * x[i*incx] with alpha read from host */
int smg_axpy(smg_ctx* ctx, long long n, double alpha, const double* x, int incx,
             double* y, int incy);
/* y[i] += (*alpha_d) * x[i], alpha read from device */
int smg_axpy_dev(smg_ctx* ctx, long long n, const double* alpha_d, const double* x, double* y);
/* out += sum(x) (deterministic) */
int smg_sum(smg_ctx* ctx, const double* x, long long n, double* out);
/* B(i,j) = A(j,i) style copy helpers */
int smg_copy_matrix(smg_ctx* ctx, int m, int n, const double* A, int lda,
                    double* B, int ldb, int trans, int uplo_zero_upper);
/* A (n x n, in place): strict upper triangle <- the transpose of the strict
 * lower one (multiply(A, transpose(A)) forms the lower half of the Gram
 * product on the GEMM, then mirrors it). */
int smg_sym_from_lower(smg_ctx* ctx, int n, double* A, int lda);
/* The Eigen boundary's packed lower triangle (column-major: column j's rows
 * j..n-1 at offset j n - j (j - 1) / 2; n (n + 1) / 2 doubles), the layout of
 * the host varis of a cholesky_decompose factor (its strict upper triangle is
 * one dummy vari, rev/mat/fun/cholesky_decompose.hpp:34-48) and of a
 * gp_exp_quad_cov matrix (K(i, j) and K(j, i) share one vari,
 * rev/mat/fun/gp_exp_quad_cov.hpp:235).  pack: mode 0 dst <- tril(A);
 * mode 1 dst <- tril(A) + strict tril(A^T) (the shared vari's adjoint);
 * mode 2 dst[i] <- A_ii (n doubles: add_diag's own varis,
 * prim/mat/fun/add_diag.hpp:25-27).  unpack_tril_add: modes 0 / 1
 * tril(A) += unpack(src), mode 2 A_ii += src[i]. */
int smg_pack_tril(smg_ctx* ctx, int mode, int n, const double* A, int lda, double* dst);
/* out[0] = the sum of A's strict upper triangle (fixed order): what a
 * cholesky_decompose factor's one dummy vari accumulates from every
 * upper-element adjoint (rev/mat/fun/cholesky_decompose.hpp:34-48). */
int smg_sum_strict_upper(smg_ctx* ctx, int n, const double* A, int lda, double* out);
int smg_unpack_tril_add(smg_ctx* ctx, int mode, int n, const double* src, double* A, int lda);
/* B (n x m) = A^T + beta B, A m x n (transpose(Matrix<var>): forward copy and
 * the reverse Aadj += Badj^T) */
int smg_transpose(smg_ctx* ctx, int m, int n, const double* A, int lda,
                  double* B, int ldb, double beta);
/* Y += c on every entry (uplo == 1: lower triangle only); the reverse of
 * sum(Matrix<var>) (rev/mat/fun/sum.hpp:18-60) */
int smg_shift(smg_ctx* ctx, int m, int n, double c, double* Y, int ldy, int uplo);
/* out += sum_i x_i y_i (deterministic) */
int smg_dot(smg_ctx* ctx, const double* x, const double* y, long long n, double* out);
/* Y = Phi(X) (accumulate: Y += Phi(X)): strict lower triangle of X, halved
 * diagonal, zero upper -- the tangent map of a Cholesky factor; Phi is its own
 * adjoint, so the reverse is the same call with accumulate = 1 */
int smg_phi(smg_ctx* ctx, int n, const double* X, int ldx, double* Y, int ldy, int accumulate);
/* out += sum_i A_ii / B_ii; rev Aadj_ii += adj / B_ii, Badj_ii -= adj A_ii / B_ii^2
 * (the log-determinant tangent term of multi_normal_cholesky_lpdf) */
int smg_diag_ratio_fwd(smg_ctx* ctx, int n, const double* A, int lda, const double* B, int ldb,
                       double* out);
int smg_diag_ratio_rev(smg_ctx* ctx, int n, const double* A, int lda, const double* B, int ldb,
                       double adj, double* Aadj, int ldaa, double* Badj, int ldba);
/* argument checks of the lpdf reducers (prim/scal/err/check_*.hpp): *flag (a
 * device double the caller zeroes) becomes 1.0 if any x_i fails.  kind 0:
 * check_not_nan, 1: check_finite, 2: check_positive, 3: check_positive_finite.
 * The host layer reads the flags back with the value and throws the
 * reference's std::domain_error for the first failing argument. */
int smg_check_domain(smg_ctx* ctx, const double* x, long long n, int kind, double* flag);
/* *flag = 1.0 if any y_i is outside [lo, hi] (check_bounded) */
int smg_check_bounded_int(smg_ctx* ctx, const int* y, long long n, int lo, int hi, double* flag);

/* ------------------------------------------------------ multi-GPU ------
 * One RCCL communicator per process/device; a single fp64 sum all-reduce of
 * [logp, alpha_adj, beta_adj...] per gradient (replaces the Boost.MPI
 * gather/reduce of map_rect, prim/mat/functor/mpi_parallel_call.hpp:332-392). */
int smg_comm_unique_id(char* id_host /* 128 bytes */);
int smg_comm_init(smg_ctx* ctx, int nranks, int rank, const char* id_host);
int smg_comm_allreduce_sum(smg_ctx* ctx, double* buf, long long count);
/* recv (device, nranks * count doubles) <- every rank's count doubles of send
 * (device), rank order; the distributed map_rect executor's exchange of
 * per-job [value; partials] columns (replaces the gatherv of
 * prim/mat/functor/mpi_parallel_call.hpp:374-382). */
int smg_comm_allgather(smg_ctx* ctx, const double* send, long long count, double* recv);
/* recv (device, counts[my rank] doubles) <- my block of the root's send
 * (device, the blocks of ranks 0, 1, ... back to back; read on the root
 * only): the distributed map_rect's one-time scatter of each rank's job data
 * per call_id (replaces boost::mpi::scatterv in
 * prim/mat/functor/mpi_parallel_call.hpp:423-450). counts: nranks entries,
 * the same on every rank. */
int smg_comm_scatterv(smg_ctx* ctx, const double* send, const long long* counts, double* recv, int root);
int smg_comm_destroy(smg_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif
