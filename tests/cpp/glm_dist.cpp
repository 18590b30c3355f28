// Test shim (shared library, loaded by tests/test_sharding.py through ctypes):
// the product's row-sharded GLM reducers (reduce_sum_bernoulli_logit_glm and
// the poisson_log_glm shard overload) driven by a host collective, so W
// processes joined by torch.distributed gloo -- each holding its row block on
// the GPU -- run exactly the code the RCCL path runs on W GPUs: the same
// partition, the same device pass, ONE sum all-reduce of
// [logp, alpha', beta' | y flag] (amd::allreduce_sum), the same node.
#include <stan/math.hpp>

#include <cstring>
#include <stdexcept>
#include <vector>

using namespace stan::math;

extern "C" {

/* kind 0: bernoulli_logit_glm_lpmf, 1: poisson_log_glm_lpmf.  This rank holds
 * rows [row0, row0 + rows) of R: x (rows x M, column-major), y.  theta =
 * (alpha, beta(M)).  Returns 0, 1 (domain_error; message in err) or 2 (other). */
int glm_dist_eval(int nranks, int rank, amd::allgather_fn ag, amd::allreduce_fn ar, void* user, int kind,
                  long long R, long long row0, long long rows, int M, const double* x, const int* y,
                  const double* theta, double* fx, double* grad, char* err, int errlen) {
  amd::set_host_collective(nranks, rank, ag, user, ar);
  int rc = 0;
  start_nested();
  try {
    std::vector<int> yv(y, y + rows);
    dev_data<int> yd = to_dev_data(yv);
    dev_data<double> xd = to_dev_data(x, size_t(rows) * M, int(rows), M);
    glm_shard s;
    s.y = yd.data();
    s.x = xd.data();
    s.rows = rows;
    s.M = M;
    s.ldx = rows > 0 ? rows : 1;
    s.row0 = row0;
    s.total_rows = R;
    s.distributed = true;
    std::vector<double> th(theta, theta + M + 1), g;
    gradient(
        [&](const std::vector<var>& t) {
          std::vector<var> beta(t.begin() + 1, t.end());
          if (kind == 0) return reduce_sum_bernoulli_logit_glm(s, t[0], beta);
          return poisson_log_glm_lpmf<false>(s, t[0], beta);
        },
        th, *fx, g);
    for (int i = 0; i <= M; ++i) grad[i] = g[size_t(i)];
  } catch (const std::domain_error& e) {
    std::strncpy(err, e.what(), size_t(errlen - 1));
    err[errlen - 1] = 0;
    rc = 1;
  } catch (const std::exception& e) {
    std::strncpy(err, e.what(), size_t(errlen - 1));
    err[errlen - 1] = 0;
    rc = 2;
  }
  recover_memory_nested();
  amd::set_host_collective(1, 0, nullptr, nullptr);
  return rc;
}

/* stan::math::row_partition, from this library (a process that has
 * dlopen'ed it need not load a second one) */
void glm_dist_row_partition(long long R, int world, int rank, long long* b0, long long* b1) {
  stan::math::row_partition(R, world, rank, b0, b1);
}

}  // extern "C"
