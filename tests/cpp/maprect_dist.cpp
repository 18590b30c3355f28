// Test shim (shared library, loaded by tests/test_sharding.py through ctypes):
// the multi-rank map_rect executor (rev/functor/map_rect.hpp) driven by a
// host collective, so a world of W CPU processes joined by torch.distributed
// gloo exercises the same partition / exchange / combine code the RCCL path
// runs on W GPUs.  The user functor is host scalar arithmetic only (no device
// op), the one oracle/ref_harness.cpp fix_maprect runs through the real
// reference's map_rect.
#include <stan/math.hpp>

#include <cstring>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

using namespace stan::math;

namespace {

template <typename T1, typename T2>
using ret_t = typename std::conditional<std::is_same<T1, double>::value && std::is_same<T2, double>::value,
                                        double, var>::type;

// outputs: x_i[0] of them; x_i[1] == 1 makes the job throw
struct hier_job {
  template <typename T1, typename T2>
  Eigen::Matrix<ret_t<T1, T2>, Eigen::Dynamic, 1> operator()(const Eigen::Matrix<T1, Eigen::Dynamic, 1>& phi,
                                                             const Eigen::Matrix<T2, Eigen::Dynamic, 1>& theta,
                                                             const std::vector<double>& x_r,
                                                             const std::vector<int>& x_i, std::ostream*) const {
    using std::exp;
    using std::log;
    if (x_i[1] == 1) throw std::domain_error("hier_job: job failed");
    const int nout = x_i[0];
    Eigen::Matrix<ret_t<T1, T2>, Eigen::Dynamic, 1> out(nout);
    const T1 sigma = exp(phi(1));
    for (int k = 0; k < nout; ++k) {
      ret_t<T1, T2> acc = 0.0;
      for (size_t i = size_t(k); i < x_r.size(); i += size_t(nout)) {
        const ret_t<T1, T2> z = (x_r[i] - (phi(0) + theta(0))) / sigma;
        acc += -0.5 * (z * z) - log(sigma);
      }
      out(k) = acc;
    }
    return out;
  }
};

int g_ragged = 0;  // rank 0's last job gets one real datum fewer (maprect_set_ragged)

}  // namespace

extern "C" {

/* Make rank 0's x_r ragged in the following calls (the argument-check
 * agreement test: every rank must throw rank 0's invalid_argument). */
void maprect_set_ragged(int on) { g_ragged = on; }

/* mode 0: phi and theta var; 1: phi var, theta data; 2: phi data, theta var;
 * 3: all data.  f = sum_i (1 + 0.1 i) out_i.  grad: (phi(2), theta(J)) (zeros
 * for data).  vals: the concatenated outputs; *nvals their count.
 * fresh: forget the cached job data first (map_rect_clear_cache); root_only:
 * ranks other than 0 pass empty x_r / x_i (their blocks come from rank 0's
 * scatter, sc: the scatterv hook or null).
 * Returns 0, 1 (domain_error; message in err) or 2 (other exception). */
int maprect_hier_ex(int nranks, int rank, amd::allgather_fn fn, amd::scatterv_fn sc, void* user, int J,
                    const double* xr_flat, int nr, const int* xi_flat, const double* th, int mode, int fresh,
                    int root_only, double* fx, double* grad, double* vals, int* nvals, char* err, int errlen) {
  amd::set_host_collective(nranks, rank, nranks > 1 ? fn : nullptr, user, nullptr, sc);
  if (fresh) map_rect_clear_cache();
  const bool hold = !(root_only && rank != 0);
  std::vector<std::vector<double>> xr(hold ? static_cast<size_t>(J) : 0);
  std::vector<std::vector<int>> xi(hold ? static_cast<size_t>(J) : 0);
  for (int j = 0; hold && j < J; ++j) {
    xr[size_t(j)].assign(xr_flat + size_t(j) * nr, xr_flat + size_t(j + 1) * nr);
    xi[size_t(j)].assign(xi_flat + 2 * j, xi_flat + 2 * j + 2);
  }
  if (g_ragged && rank == 0 && J > 1) xr[size_t(J - 1)].pop_back();
  int rc = 0;
  start_nested();
  try {
    auto weigh = [](const auto& out) {
      typename std::decay<decltype(out(0))>::type f = 0.0;
      for (Eigen::Index i = 0; i < out.size(); ++i) f += (1.0 + 0.1 * double(i)) * out(i);
      return f;
    };
    auto emit = [&](const auto& out) {
      *nvals = int(out.size());
      for (Eigen::Index i = 0; i < out.size(); ++i) vals[i] = value_of(out(i));
    };
    for (int k = 0; k < 2 + J; ++k) grad[k] = 0.0;
    using VV = Eigen::Matrix<var, Eigen::Dynamic, 1>;
    Eigen::VectorXd phid(2);
    phid << th[0], th[1];
    std::vector<Eigen::VectorXd> jobd(size_t(J), Eigen::VectorXd(1));
    for (int j = 0; j < J; ++j) jobd[size_t(j)](0) = th[2 + j];
    if (mode == 3) {
      Eigen::VectorXd out = map_rect<1, hier_job>(phid, jobd, xr, xi);
      emit(out);
      *fx = weigh(out);
    } else {
      VV phi(2);
      phi(0) = th[0];
      phi(1) = th[1];
      std::vector<VV> jobv(size_t(J), VV(1));
      for (int j = 0; j < J; ++j) jobv[size_t(j)](0) = th[2 + j];
      VV out;
      if (mode == 0) out = map_rect<2, hier_job>(phi, jobv, xr, xi);
      if (mode == 1) out = map_rect<3, hier_job>(phi, jobd, xr, xi);
      if (mode == 2) out = map_rect<4, hier_job>(phid, jobv, xr, xi);
      emit(out);
      var f = weigh(out);
      *fx = f.val();
      f.grad();
      if (mode != 2)
        for (int k = 0; k < 2; ++k) grad[k] = phi(k).adj();
      if (mode != 1)
        for (int j = 0; j < J; ++j) grad[2 + j] = jobv[size_t(j)](0).adj();
    }
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

/* Every rank holds the data; the job data cache is cleared before the call. */
int maprect_hier(int nranks, int rank, amd::allgather_fn fn, void* user, int J, const double* xr_flat, int nr,
                 const int* xi_flat, const double* th, int mode, double* fx, double* grad, double* vals, int* nvals,
                 char* err, int errlen) {
  return maprect_hier_ex(nranks, rank, fn, nullptr, user, J, xr_flat, nr, xi_flat, th, mode, 1, 0, fx, grad, vals,
                         nvals, err, errlen);
}

/* The same call over RCCL: joins a one-rank communicator on this process's
 * GPU (so the executor's two exchanges are real ncclAllGather calls), runs
 * maprect_hier, leaves the communicator. */
int maprect_hier_rccl(int J, const double* xr_flat, int nr, const int* xi_flat, const double* th, int mode,
                      double* fx, double* grad, double* vals, int* nvals, char* err, int errlen) {
  char id[128];
  if (smg_comm_unique_id(id) != SMG_OK) return 3;
  amd::comm_init(1, 0, id);
  const int rc = maprect_hier(1, 0, nullptr, nullptr, J, xr_flat, nr, xi_flat, th, mode, fx, grad, vals, nvals,
                              err, errlen);
  amd::comm_destroy();
  return rc;
}

}  // extern "C"
