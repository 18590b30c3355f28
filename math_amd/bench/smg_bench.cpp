// libsmg_bench.so — BASELINE workloads written against the drop-in
// stan::math API (header-only layer + libsmg_hip.so), exported with a C ABI
// for bench.py / __graft_entry__.smoke().  One "step" = one
// stan::math::gradient() call (stan/math/rev/mat/functor/gradient.hpp:41-57).
#include <stan/math.hpp>

#include <malloc.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <cmath>
#include <cstdio>
#include <exception>
#include <vector>

namespace {

using stan::math::dev_data;
using stan::math::var;

// config 3: multi_normal_cholesky_lpdf(y | 0, cholesky_decompose(add_diag(
//           gp_exp_quad_cov(x, alpha, rho), sigma^2)))
// (T = var for gradient(), T = fvar<var> for hessian_times_vector(), config 5)
struct gp_functor {
  const dev_data<double>& x;
  const dev_data<double>& y;
  template <typename T>
  T operator()(const std::vector<T>& th) const {
    using namespace stan::math;
    auto K = gp_exp_quad_cov(x, th[0], th[1]);
    auto Kd = add_diag(K, square(th[2]));
    auto L = cholesky_decompose(Kd);
    return multi_normal_cholesky_lpdf(y, mu0, L);
  }
  const dev_data<double>& mu0;
};

// the same with the reference's input types (the harness's gp_functor
// arguments: std::vector<double> x, Eigen y and mu -- uploaded per
// evaluation) and device-typed intermediates (`auto`)
struct gp_reftypes_functor {
  const std::vector<double>& x;
  const Eigen::VectorXd& y;
  template <typename T>
  T operator()(const std::vector<T>& th) const {
    using namespace stan::math;
    auto K = gp_exp_quad_cov(x, th[0], th[1]);
    auto Kd = add_diag(K, square(th[2]));
    auto L = cholesky_decompose(Kd);
    const Eigen::VectorXd mu = Eigen::VectorXd::Zero(y.size());
    return multi_normal_cholesky_lpdf(y, mu, L);
  }
};

// config 3 exactly as Stan-generated code declares it (and as the reference
// harness times it, oracle/ref_harness.cpp gp_functor): host std::vector x,
// Eigen y / mu, and `matrix[N,N] K = ...` as Eigen::Matrix<var,-1,-1>, so
// every stage crosses the Eigen boundary (materialised host blocks,
// recognised again by the next functor).
struct gp_eigen_functor {
  const std::vector<double>& x;
  const Eigen::VectorXd& y;
  template <typename T>
  T operator()(const Eigen::Matrix<T, -1, 1>& th) const {
    using namespace stan::math;
    const int N = int(x.size());
    Eigen::Matrix<T, -1, -1> K = gp_exp_quad_cov(x, th(0), th(1));
    Eigen::Matrix<T, -1, -1> Kd = add_diag(K, square(th(2)));
    Eigen::Matrix<T, -1, -1> L = cholesky_decompose(Kd);
    Eigen::VectorXd mu = Eigen::VectorXd::Zero(N);
    return multi_normal_cholesky_lpdf(y, mu, L);
  }
};

dev_data<double> g_x, g_y, g_mu0;
std::vector<double> g_xh;
Eigen::VectorXd g_yh;
int g_n = 0;
char g_err[512];

// config 4: bernoulli_logit_glm_lpmf over this rank's row block, one RCCL
// all-reduce of [logp, alpha', beta'] when world > 1
stan::math::glm_shard g_shard;

// config 2: sum(cholesky_decompose(add_diag(multiply(A, A^T), N))), A device-resident
double* g_A = nullptr;
double* g_G = nullptr;
double* g_R = nullptr;  // [sum, sum of squares] of the config-2 gradient
int g_N2 = 0;

constexpr unsigned long long SEED = 20260101ull;
constexpr unsigned long long GOLDEN = 0x9E3779B97F4A7C15ull;  // SplitMix64 increment (oracle/gen.h)

int fail(const std::exception& e) {
  std::snprintf(g_err, sizeof g_err, "%s", e.what());
  return -1;
}

}  // namespace

extern "C" {

const char* smg_bench_error() { return g_err; }

void* smg_bench_ctx() { return stan::math::amd::ctx(); }

int smg_bench_gp_init(int device, int n, const double* x, const double* y) {
  try {
    stan::math::amd::set_device(device);
    // data resident in HBM before the timed region (outer arena level, so the
    // nested gradient() scopes never rewind it)
    g_x = stan::math::to_dev_data(x, size_t(n));
    g_y = stan::math::to_dev_data(y, size_t(n));
    const std::vector<double> zeros(size_t(n), 0.0);
    g_mu0 = stan::math::to_dev_data(zeros);
    g_xh.assign(x, x + n);
    g_yh = Eigen::Map<const Eigen::VectorXd>(y, n);
    g_n = n;
    return 0;
  } catch (const std::exception& e) {
    return fail(e);
  }
}

int smg_bench_gp_step(const double* theta, double* fx, double* grad) {
  try {
    std::vector<double> th(theta, theta + 3), g;
    stan::math::gradient(gp_functor{g_x, g_y, g_mu0}, th, *fx, g);
    for (int i = 0; i < 3; ++i) grad[i] = g[i];
    return 0;
  } catch (const std::exception& e) {
    return fail(e);
  }
}

/* config 3 with the reference's argument types (gp_reftypes_functor). */
int smg_bench_gp_step_reftypes(const double* theta, double* fx, double* grad) {
  try {
    std::vector<double> th(theta, theta + 3), g;
    stan::math::gradient(gp_reftypes_functor{g_xh, g_yh}, th, *fx, g);
    for (int i = 0; i < 3; ++i) grad[i] = g[i];
    return 0;
  } catch (const std::exception& e) {
    return fail(e);
  }
}

/* config 3 through the Eigen-typed boundary (gp_eigen_functor); data from
 * smg_bench_gp_init.  malloc_tuning != 0 keeps Eigen's N^2 heap buffers in
 * the brk heap (M_MMAP_MAX = 0, no trimming) so they are reused without page
 * faults: the application's allocator choice, reported with the bench line. */
int smg_bench_gp_eigen_step(const double* theta, double* fx, double* grad) {
  try {
    Eigen::VectorXd th = Eigen::Map<const Eigen::VectorXd>(theta, 3), g;
    stan::math::gradient(gp_eigen_functor{g_xh, g_yh}, th, *fx, g);
    for (int i = 0; i < 3; ++i) grad[i] = g(i);
    return 0;
  } catch (const std::exception& e) {
    return fail(e);
  }
}
/* Where one gp_eigen evaluation's host time goes (seconds): out[0] the
 * functor's forward pass (three crossings), out[1] the reverse sweep of a
 * top-level grad() (with the host blocks' adjoints published), out[2]
 * recover_memory, out[3] the whole evaluation (gradient()), out[4..7] the
 * forward's statements: K = gp_exp_quad_cov, Kd = add_diag, L =
 * cholesky_decompose, the MVN; out[8..31] the L statement's host timeline
 * from its start (amd::phase_mark: 0 the factorisation enqueued, 1 the
 * pointer array filled, 2 + 2p / 3 + 2p panel p's values arrived / its varis
 * built, 18 the output matrix allocated, 19 the input's candidate block
 * found, 20 the host staging buffer ready, 21 the speculative input verified,
 * 30 the status read; 0 where a point was not reached). */
int smg_bench_gp_eigen_phases(const double* theta, double* out) {
  try {
    using namespace stan::math;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto sec = [](auto a, auto b) { return std::chrono::duration<double>(b - a).count(); };
    Eigen::VectorXd th = Eigen::Map<const Eigen::VectorXd>(theta, 3);
    auto t0 = now();
    Eigen::Matrix<var, -1, 1> tv(3);
    for (int i = 0; i < 3; ++i) tv(i) = th(i);
    var f = gp_eigen_functor{g_xh, g_yh}(tv);
    auto t1 = now();
    grad(f.vi_);
    amd::check(smg_sync(amd::ctx()), "phases");
    auto t2 = now();
    recover_memory();
    auto t3 = now();
    double fx;
    Eigen::VectorXd g;
    auto t4 = now();
    gradient(gp_eigen_functor{g_xh, g_yh}, th, fx, g);
    auto t5 = now();
    out[0] = sec(t0, t1);
    out[1] = sec(t1, t2);
    out[2] = sec(t2, t3);
    out[3] = sec(t4, t5);
    {  // the forward statement by statement (each ends where the host has its result)
      start_nested();
      Eigen::Matrix<var, -1, 1> tv2(3);
      for (int i = 0; i < 3; ++i) tv2(i) = th(i);
      auto s0 = now();
      Eigen::Matrix<var, -1, -1> K = gp_exp_quad_cov(g_xh, tv2(0), tv2(1));
      auto s1 = now();
      Eigen::Matrix<var, -1, -1> Kd = add_diag(K, square(tv2(2)));
      auto s2 = now();
      amd::phase_log_t& pl = amd::phase_log();
      for (double& t : pl.t) t = 0.0;
      pl.on = true;
      Eigen::Matrix<var, -1, -1> L = cholesky_decompose(Kd);
      pl.on = false;
      auto s3 = now();
      const double base = std::chrono::duration<double>(s2.time_since_epoch()).count();
      for (int k = 0; k < 24; ++k) {
        const int src = k < 23 ? k : 30;
        out[8 + k] = src >= 0 && pl.t[src] > 0 ? pl.t[src] - base : 0.0;
      }
      Eigen::VectorXd mu = Eigen::VectorXd::Zero(g_n);
      var lp = multi_normal_cholesky_lpdf(g_yh, mu, L);
      auto s4 = now();
      out[4] = sec(s0, s1);
      out[5] = sec(s1, s2);
      out[6] = sec(s2, s3);
      out[7] = sec(s3, s4);
      (void)lp;
      recover_memory_nested();
    }
    return 0;
  } catch (const std::exception& e) {
    return fail(e);
  }
}

/* The host pool's memory bandwidth on the cores the Eigen boundary's
 * crossings use (the same persistent pool, the same partition): out[0] GB/s
 * of a write-only pass laid out like a crossing (24-byte vari records, then
 * an 8-byte pointer array), out[1] GB/s of a read + write pass; best of
 * `reps` over a `bytes` buffer whose pages are faulted in first; out[2] the
 * pool's thread count, out[3] sizeof(vari). */
int smg_bench_host_bw(long long bytes, int reps, double* out) {
  try {
    using namespace stan::math;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto sec = [](auto a, auto b) { return std::chrono::duration<double>(b - a).count(); };
    const size_t nrec = size_t(bytes) / 32;  // 24 + 8 bytes per element, as a crossing writes
    std::vector<char> buf(nrec * 32);
    std::memset(buf.data(), 0, buf.size());
    struct rec {
      void* vt;
      double val, adj;
    };
    rec* R = reinterpret_cast<rec*>(buf.data());
    void** P = reinterpret_cast<void**>(buf.data() + nrec * sizeof(rec));
    static_assert(sizeof(rec) == 24, "record");
    double wbest = 1e30, cbest = 1e30;
    for (int r = 0; r < reps; ++r) {
      auto t0 = now();
      internal::host_parallel_for(nrec, [&](size_t b, size_t e) {
        for (size_t i = b; i < e; ++i) R[i] = rec{&R[0], double(i), 0.0};
      });
      internal::host_parallel_for(nrec, [&](size_t b, size_t e) {
        for (size_t i = b; i < e; ++i) P[i] = &R[i];
      });
      auto t1 = now();
      internal::host_parallel_for(nrec, [&](size_t b, size_t e) {
        for (size_t i = b; i < e; ++i) R[i].adj = R[i].val + 1.0;
      });
      auto t2 = now();
      wbest = std::min(wbest, sec(t0, t1));
      cbest = std::min(cbest, sec(t1, t2));
    }
    out[0] = double(nrec) * 32 / wbest * 1e-9;
    out[1] = double(nrec) * sizeof(rec) * 2 / cbest * 1e-9;
    out[2] = internal::host_threads();
    out[3] = sizeof(vari);
    return 0;
  } catch (const std::exception& e) {
    return fail(e);
  }
}

void smg_bench_malloc_tuning(int on) {
  if (on) {
    mallopt(M_MMAP_MAX, 0);
    mallopt(M_TRIM_THRESHOLD, 1 << 30);
    mallopt(M_TOP_PAD, 64 << 20);
  } else {
    mallopt(M_MMAP_MAX, 65536);
  }
}

/* The Eigen boundary's cost per crossing of an n x n device matrix (seconds,
 * best of `reps`): out[0] to_host_matrix (one D2H of the values, n^2 varis
 * constructed in one arena block, the Eigen pointer array), out[1] to_dev of
 * that matrix (recognised: a parallel pointer check), out[2] to_dev of a copy
 * with one element replaced (gathered and uploaded), out[3] the reverse
 * sweep's gather of the block's host adjoints (a host node touched it),
 * out[4] the same sweep when nothing touched it (skipped). */
int smg_bench_bridge_cost(int n, int reps, double* out) {
  try {
    using namespace stan::math;
    const size_t nn = size_t(n) * n;
    for (int k = 0; k < 5; ++k) out[k] = 1e30;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto sec = [](auto a, auto b) { return std::chrono::duration<double>(b - a).count(); };
    for (int r = 0; r < reps; ++r) {
      for (int touch = 0; touch < 2; ++touch) {
        start_nested();
        auto* node = new dev_matrix_vari(n, n);
        amd::check(smg_fill_unif(amd::ctx(), node->val_, (long long)nn, SEED + 7, -1.0, 1.0, 1.0), "bridge");
        dev_var_matrix A(node);
        var f0 = sum(A);  // a device consumer below the block (the sweep's common part)
        auto t0 = now();
        Eigen::Matrix<var, -1, -1> M = to_host_matrix(A);
        auto t1 = now();
        dev_var_matrix B = to_dev(M);
        auto t2 = now();
        if (B.vi_ != A.vi_) throw std::runtime_error("bridge: the round trip did not recognise its block");
        var f = f0 + sum(B);
        if (touch) f += 2.0 * M(1, 1);
        amd::check(smg_sync(amd::ctx()), "bridge");
        auto t4 = now();
        {
          no_publish_scope quiet;  // (the bridge's own cost: the blocks' adjoints are not published)
          f.grad();  // the block's bridge runs inside: gathers when touched, skips otherwise
        }
        auto t5 = now();
        out[0] = std::min(out[0], sec(t0, t1));
        out[1] = std::min(out[1], sec(t1, t2));
        out[touch ? 3 : 4] = std::min(out[touch ? 3 : 4], sec(t4, t5));
        recover_memory_nested();
      }
      start_nested();  // a copy with one element replaced is not the block: gathered and uploaded
      auto* node = new dev_matrix_vari(n, n);
      amd::check(smg_fill_unif(amd::ctx(), node->val_, (long long)nn, SEED + 7, -1.0, 1.0, 1.0), "bridge");
      Eigen::Matrix<var, -1, -1> M2 = to_host_matrix(dev_var_matrix(node));
      M2(0, 0) = var(1.0);
      auto t3 = now();
      dev_var_matrix C = to_dev(M2);
      auto t4 = now();
      out[2] = std::min(out[2], sec(t3, t4));
      recover_memory_nested();
    }
    return 0;
  } catch (const std::exception& e) {
    return fail(e);
  }
}

/* Allocate and fill this rank's rows [b0, b1) of the config-4 data directly in
 * HBM: x(i, j) = unif(SEED+41)[i + j R] * sqrt(3), y(i) = bern(SEED+42)[i], the
 * same streams as oracle/gen.h (a SplitMix64 stream started k elements later
 * is the stream of seed + k * GOLDEN). */
int smg_bench_glm_init(int device, long long R, int M, int rank, int world, const char* comm_id) {
  try {
    using namespace stan::math;
    amd::set_device(device);
    smg_ctx* c = amd::ctx();
    // world == 1 with an id: a one-rank RCCL communicator, so the sharded
    // path (all-reduce, zero-copy read of the sums) runs as on each of W ranks
    if (world > 1 || comm_id) amd::comm_init(world, rank, comm_id);
    long long b0, b1;
    row_partition(R, world, rank, &b0, &b1);
    const long long rows = b1 - b0;
    double* x = amd::alloc_doubles(size_t(rows > 0 ? rows : 1) * M);
    int* y = amd::alloc_ints(size_t(rows > 0 ? rows : 1));
    for (int j = 0; j < M && rows > 0; ++j)
      amd::check(smg_fill_unif(c, x + size_t(j) * rows, rows,
                               SEED + 41 + (unsigned long long)(b0 + (long long)j * R) * GOLDEN, -1.0,
                               1.0, std::sqrt(3.0)),
                 "glm_init");
    if (rows > 0)
      amd::check(smg_fill_bernoulli(c, y, rows, SEED + 42 + (unsigned long long)b0 * GOLDEN, 0.5),
                 "glm_init");
    amd::check(smg_sync(c), "glm_init");
    g_shard = glm_shard{};
    g_shard.y = y;
    g_shard.x = x;
    g_shard.rows = rows;
    g_shard.M = M;
    g_shard.ldx = rows > 0 ? rows : 1;
    g_shard.row0 = b0;
    g_shard.total_rows = R;
    g_shard.distributed = world > 1 || comm_id;
    return 0;
  } catch (const std::exception& e) {
    return fail(e);
  }
}

int smg_bench_glm_step(const double* theta, double* fx, double* grad) {
  try {
    using namespace stan::math;
    const int M = g_shard.M;
    std::vector<double> th(theta, theta + M + 1), g;
    gradient(
        [](const std::vector<var>& t) {
          std::vector<var> beta(t.begin() + 1, t.end());
          return reduce_sum_bernoulli_logit_glm(g_shard, t[0], beta);
        },
        th, *fx, g);
    for (int i = 0; i <= M; ++i) grad[i] = g[i];
    return 0;
  } catch (const std::exception& e) {
    return fail(e);
  }
}

/* config 5: H v of the same GP marginal (fwd-over-rev), data from smg_bench_gp_init */
int smg_bench_hvp_step(const double* theta, const double* v, double* fx, double* hv) {
  try {
    std::vector<double> th(theta, theta + 3), vv(v, v + 3), h;
    stan::math::hessian_times_vector(gp_functor{g_x, g_y, g_mu0}, th, vv, *fx, h);
    for (int i = 0; i < 3; ++i) hv[i] = h[i];
    return 0;
  } catch (const std::exception& e) {
    return fail(e);
  }
}

/* config 1: gradient of normal_lpdf(theta | 0, 1) wrt the n entries of theta
 * (host std::vector<var> operand, as the reference's normal_functor) */
int smg_bench_normal_step(int n, const double* theta, double* fx, double* grad) {
  try {
    std::vector<double> th(theta, theta + n), g;
    stan::math::gradient(
        [](const std::vector<var>& t) { return stan::math::normal_lpdf(t, 0.0, 1.0); }, th, *fx, g);
    for (int i = 0; i < n; ++i) grad[i] = g[i];
    return 0;
  } catch (const std::exception& e) {
    return fail(e);
  }
}

/* k config-1 evaluations back to back (the timed loop without a host-language
 * call per evaluation, as the reference harness times its own loop) */
int smg_bench_normal_run(int k, int n, const double* theta, double* fx, double* grad) {
  try {  // the reference harness's loop: one x and one gradient vector, reused
    std::vector<double> th(theta, theta + n), g;
    for (int r = 0; r < k; ++r)
      stan::math::gradient(
          [](const std::vector<var>& t) { return stan::math::normal_lpdf(t, 0.0, 1.0); }, th, *fx, g);
    for (int i = 0; i < n; ++i) grad[i] = g[i];
    return 0;
  } catch (const std::exception& e) {
    return fail(e);
  }
}

/* the normal_lpdf host gate (elements; 0: every call on the device) */
void smg_bench_normal_gate(long long n) { stan::math::amd::set_normal_host_max(size_t(n)); }

int smg_bench_device_init(int device) {
  try {
    stan::math::amd::set_device(device);
    return 0;
  } catch (const std::exception& e) {
    return fail(e);
  }
}

long long smg_bench_glm_local_rows() { return g_shard.rows; }

/* the row partition every sharded reducer uses (stan::math::row_partition) */
void smg_bench_row_partition(long long R, int world, int rank, long long* b0, long long* b1) {
  stan::math::row_partition(R, world, rank, b0, b1);
}

int smg_bench_mulchol_init(int device, int N) {
  try {
    using namespace stan::math;
    amd::set_device(device);
    smg_ctx* c = amd::ctx();
    const size_t nn = size_t(N) * N;
    g_A = amd::alloc_doubles(nn);
    g_G = amd::alloc_doubles(nn);
    g_R = amd::alloc_doubles(2);
    amd::check(smg_fill_unif(c, g_A, (long long)nn, SEED + 2, -1.0, 1.0, std::sqrt(3.0 / N)),
               "mulchol_init");
    g_N2 = N;
    return 0;
  } catch (const std::exception& e) {
    return fail(e);
  }
}

/* one gradient of config 2 wrt all N^2 entries; the gradient stays in HBM
 * (g_G); grad_sum_l2 = [sum, l2] of it for the parity guard when requested */
int smg_bench_mulchol_step(double* fx, double* grad_sum_l2) {
  try {
    using namespace stan::math;
    const int N = g_N2;
    const size_t nn = size_t(N) * N;
    gradient(
        [N](const dev_var_matrix& a) {
          return sum(cholesky_decompose(add_diag(multiply(a, transpose(a)), double(N))));
        },
        dev_data<double>(g_A, nn, N, N), *fx, g_G);
    if (grad_sum_l2) {
      smg_ctx* c = amd::ctx();
      double* r = g_R;
      amd::check(smg_memset(c, r, 0, 2 * sizeof(double)), "mulchol");
      amd::check(smg_sum(c, g_G, (long long)nn, r), "mulchol");
      amd::check(smg_dot(c, g_G, g_G, (long long)nn, r + 1), "mulchol");
      amd::to_host(grad_sum_l2, r, 2);
      grad_sum_l2[1] = std::sqrt(grad_sum_l2[1]);
    }
    return 0;
  } catch (const std::exception& e) {
    return fail(e);
  }
}

}  // extern "C"
