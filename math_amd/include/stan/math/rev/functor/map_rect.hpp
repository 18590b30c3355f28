#ifndef STAN_MATH_REV_FUNCTOR_MAP_RECT_HPP
#define STAN_MATH_REV_FUNCTOR_MAP_RECT_HPP

// map_rect<call_id, F>(shared_params, job_params, x_r, x_i, msgs)
// (prim/mat/functor/map_rect.hpp:120-177) with the reference's semantics:
//   * the same argument checks (:133-167), an empty result for no jobs;
//   * per job, a nested tape: F()(shared, job, x_r[j], x_i[j], msgs) and, for
//     each output i, set_zero_all_adjoints_nested + grad, collecting
//     [value, d/d shared, d/d job] (map_rect_reduce, rev/mat/functor/
//     map_rect_reduce.hpp:17-134);
//   * one precomputed-gradients var per output over the outer operands
//     (map_rect_combine, prim/mat/functor/map_rect_combine.hpp:36-92).
// Jobs run in order on this thread's tape and device stream; F may use any
// device functor (e.g. bernoulli_logit_glm_lpmf over the job's rows).
//
// Multi-GPU (replaces the reference's MPI executor,
// prim/mat/functor/mpi_parallel_call.hpp:268-392): once the process has joined
// an RCCL job (amd::comm_init, one process per GPU, W >= 1) or W > 1 ranks of
// a host collective (amd::set_host_collective), every rank calls
// map_rect with the same arguments (SPMD -- there is no listening worker
// loop), evaluates only its chunk of jobs (the reference's mpi_map_chunks
// split, prim/arr/functor/mpi_cluster.hpp:84-100: J / W each, the remainder
// to ranks 1, 2, ...) on its own GPU, and two all-gathers exchange
//   (1) [status, outputs per job] of every rank, then
//   (2) every job's [value; d/d shared; d/d job] columns,
// after which every rank combines the same full result.
//
// Job data cache (prim/mat/functor/mpi_parallel_call.hpp:170-181, 423-450):
// the first distributed call of a call_id fixes each rank's block of x_r /
// x_i -- sliced locally when every rank passed the data, scattered from rank
// 0 (amd::scatterv) when only the root holds it (the other ranks may pass
// empty x_r / x_i) -- and every later call of that call_id uses the cached
// block without exchanging any data, as the reference's workers do (the
// x_r / x_i passed to a later call are then not read for the evaluation:
// the reference's cache semantics).  map_rect_clear_cache() forgets every
// call_id's block.  The per-job values
// and partials are the ones a single process computes, so the result is
// bit-identical to the serial path.  A job that throws on any rank makes
// every rank throw std::domain_error("Error during MPI evaluation."), as the
// reference's root does (:384-389), so no rank is left waiting in a
// collective.  The row-sharded GLM reducers keep their own one all-reduce
// (glm_shard + reduce_sum_bernoulli_logit_glm).

#include <stan/math/amd/comm.hpp>
#include <stan/math/rev/core.hpp>

#include <Eigen/Dense>

#include <algorithm>
#include <ostream>
#include <sstream>
#include <stdexcept>
#include <type_traits>
#include <vector>

namespace stan {
namespace math {

namespace internal {

inline void map_rect_size_match(const char* what1, size_t a, const char* what2, size_t b) {
  if (a != b) {
    std::ostringstream m;
    m << "map_rect: " << what1 << " (" << a << ") and " << what2 << " (" << b
      << ") must match in size";
    throw std::invalid_argument(m.str());
  }
}

/** The outcome of map_rect's argument checks (prim/mat/functor/map_rect.hpp:
 * 133-167, in that order): code 0 = passed, else which check failed and the
 * two sizes it compared.  On a distributed job it travels in the first
 * exchange of the call, so every rank throws the same invalid_argument
 * together (the reference's root checks before it dispatches to its workers;
 * a rank throwing alone would leave the others waiting in a collective). */
struct map_rect_check {
  int code = 0;
  size_t a = 0, b = 0;
};

inline void map_rect_throw(const map_rect_check& c) {
  static const char* const what[6][2] = {
      {"", ""},
      {"job parameters", "real data"},
      {"job parameters", "int data"},
      {"Size of one of the vectors of the job specific parameters",
       "size of another vector of the job specifc parameters"},
      {"Size of one of the arrays of the job specific real data", "size of another array of the job specifc real data"},
      {"Size of one of the arrays of the job specific int data", "size of another array of the job specifc int data"}};
  if (c.code > 0 && c.code < 6) map_rect_size_match(what[c.code][0], c.a, what[c.code][1], c.b);
  if (c.code == 6)
    throw std::invalid_argument(
        "map_rect: every rank must pass the same number of jobs, and a call_id's number of jobs must not change "
        "between calls");
}

/** The checks; data_elsewhere: this rank left the job data to the root. */
template <typename T_job>
map_rect_check map_rect_checks(const std::vector<Eigen::Matrix<T_job, Eigen::Dynamic, 1>>& job_params,
                               const std::vector<std::vector<double>>& x_r, const std::vector<std::vector<int>>& x_i,
                               bool data_elsewhere) {
  const size_t J = job_params.size();
  if (!data_elsewhere && J != x_r.size()) return {1, J, x_r.size()};
  if (!data_elsewhere && J != x_i.size()) return {2, J, x_i.size()};
  for (size_t i = 1; i < J; ++i) {
    if (job_params[i].size() != job_params[0].size())
      return {3, size_t(job_params[i].size()), size_t(job_params[0].size())};
    if (data_elsewhere) continue;
    if (x_r[i].size() != x_r[0].size()) return {4, x_r[i].size(), x_r[0].size()};
    if (x_i[i].size() != x_i[0].size()) return {5, x_i[i].size(), x_i[0].size()};
  }
  return {};
}

/** After an exchange that carried every rank's check outcome at `all + r *
 * stride + off` (code, a, b): throw the first failing rank's (root first). */
inline void map_rect_throw_gathered(const double* all, int W, size_t stride, size_t off) {
  for (int r = 0; r < W; ++r) {
    const double* h = all + size_t(r) * stride + off;
    if (h[0] != 0.0) map_rect_throw({int(h[0]), size_t(h[1]), size_t(h[2])});
  }
}

template <typename T>
inline Eigen::Matrix<double, Eigen::Dynamic, 1> map_rect_values(
    const Eigen::Matrix<T, Eigen::Dynamic, 1>& v) {
  Eigen::Matrix<double, Eigen::Dynamic, 1> out(v.size());
  for (Eigen::Index i = 0; i < v.size(); ++i) out(i) = value_of(v(i));
  return out;
}

/** map_rect_reduce: [value; d/dshared (if var); d/djob (if var)] per output column. */
template <typename F, bool SV, bool JV>
Eigen::MatrixXd map_rect_reduce_job(const Eigen::VectorXd& shared, const Eigen::VectorXd& job,
                                    const std::vector<double>& x_r, const std::vector<int>& x_i,
                                    std::ostream* msgs) {
  using vector_var = Eigen::Matrix<var, Eigen::Dynamic, 1>;
  const Eigen::Index ns = SV ? shared.size() : 0, nj = JV ? job.size() : 0;
  Eigen::MatrixXd out(1 + ns + nj, 0);
  start_nested();
  no_publish_scope quiet;  // (the job reads only its leaves' adjoints)
  try {
    vector_var s_v(shared.size()), j_v(job.size());
    for (Eigen::Index i = 0; i < shared.size(); ++i) s_v(i) = shared(i);
    for (Eigen::Index i = 0; i < job.size(); ++i) j_v(i) = job(i);
    vector_var fx = [&]() -> vector_var {
      if constexpr (SV && JV) {
        return F()(s_v, j_v, x_r, x_i, msgs);
      } else if constexpr (SV) {
        return F()(s_v, job, x_r, x_i, msgs);
      } else {
        return F()(shared, j_v, x_r, x_i, msgs);
      }
    }();
    out.resize(Eigen::NoChange, fx.size());
    for (Eigen::Index i = 0; i < fx.size(); ++i) {
      out(0, i) = fx(i).val();
      set_zero_all_adjoints_nested();
      fx(i).grad();
      for (Eigen::Index k = 0; k < ns; ++k) out(1 + k, i) = s_v(k).adj();
      for (Eigen::Index k = 0; k < nj; ++k) out(1 + ns + k, i) = j_v(k).adj();
    }
  } catch (const std::exception&) {
    recover_memory_nested();
    throw;
  }
  recover_memory_nested();
  return out;
}

/** One call_id's cached job data: this rank's block of jobs (the reference
 * keeps one cache per call_id, mpi_parallel_call_cache<call_id, ...>). */
struct map_rect_data {
  bool valid = false;
  int world = 0;
  size_t J = 0, nr = 0, ni = 0;
  std::vector<std::vector<double>> x_r;
  std::vector<std::vector<int>> x_i;
};
inline std::vector<map_rect_data*>& map_rect_caches() {
  static std::vector<map_rect_data*> all;
  return all;
}
template <int call_id>
map_rect_data& map_rect_cache() {
  static map_rect_data* d = [] {
    auto* p = new map_rect_data();
    map_rect_caches().push_back(p);
    return p;
  }();
  return *d;
}

/** Jobs per rank: J / W each, the remainder one by one to ranks 1, 2, ...
 * (from rank 0 when J < W) -- mpi_map_chunks. */
inline std::vector<int> map_rect_chunks(size_t J, int W) {
  std::vector<int> c(size_t(W), int(J / size_t(W)));
  const size_t delta = c[0] == 0 ? 0 : 1;
  for (size_t r = 0; r != J % size_t(W); ++r) ++c[r + delta];
  return c;
}

/** Fill `c` with this rank's block of the job data: one all-gather of
 * [J, x_r length, x_i length, holds data] per rank, then either a local slice
 * (every rank holds the data) or two scatters from rank 0 (x_r, then x_i as
 * doubles: exact for every int).  The root's sizes are the job's. */
inline void map_rect_fill_cache(map_rect_data& c, size_t J, const std::vector<std::vector<double>>& x_r,
                                const std::vector<std::vector<int>>& x_i, const map_rect_check& chk) {
  const int W = amd::world_size(), rank = amd::world_rank();
  const bool have = x_r.size() == J && x_i.size() == J;
  // [J, x_r length, x_i length, holds data, check code, its two sizes]
  double hdr[7] = {double(J), have && J ? double(x_r[0].size()) : 0.0, have && J ? double(x_i[0].size()) : 0.0,
                   have ? 1.0 : 0.0, double(chk.code), double(chk.a), double(chk.b)};
  std::vector<double> all(size_t(7) * W);
  amd::allgather(hdr, 7, all.data());
  map_rect_throw_gathered(all.data(), W, 7, 4);  // (every rank sees every rank's checks: all of them throw)
  if (all[3] != 1.0)
    throw std::invalid_argument("map_rect: the root (rank 0) must hold the job data");
  const size_t nr = size_t(all[1]), ni = size_t(all[2]);
  bool everyone = true;
  for (int r = 0; r < W; ++r) {
    everyone = everyone && all[size_t(7 * r + 3)] == 1.0;
    if (size_t(all[size_t(7 * r)]) != J)
      throw std::invalid_argument("map_rect: every rank must pass the same number of jobs");
  }
  const std::vector<int> chunks = map_rect_chunks(J, W);
  size_t first = 0;
  for (int r = 0; r < rank; ++r) first += size_t(chunks[size_t(r)]);
  const size_t mine = size_t(chunks[size_t(rank)]);
  c.x_r.assign(mine, std::vector<double>(nr));
  c.x_i.assign(mine, std::vector<int>(ni));
  if (everyone) {
    for (size_t i = 0; i < mine; ++i) {
      c.x_r[i] = x_r[first + i];
      c.x_i[i] = x_i[first + i];
    }
  } else {
    std::vector<long long> cr(static_cast<size_t>(W)), ci(static_cast<size_t>(W));
    for (int r = 0; r < W; ++r) {
      cr[size_t(r)] = (long long)chunks[size_t(r)] * (long long)nr;
      ci[size_t(r)] = (long long)chunks[size_t(r)] * (long long)ni;
    }
    std::vector<double> fr, fi;
    if (rank == 0) {
      fr.reserve(J * nr);
      fi.reserve(J * ni);
      for (size_t j = 0; j < J; ++j) {
        fr.insert(fr.end(), x_r[j].begin(), x_r[j].end());
        for (int v : x_i[j]) fi.push_back(double(v));
      }
    }
    std::vector<double> lr(mine * nr), li(mine * ni);
    amd::scatterv(fr.data(), cr, lr.data());
    amd::scatterv(fi.data(), ci, li.data());
    for (size_t i = 0; i < mine; ++i) {
      std::copy(lr.begin() + i * nr, lr.begin() + (i + 1) * nr, c.x_r[i].begin());
      for (size_t k = 0; k < ni; ++k) c.x_i[i][k] = int(li[i * ni + k]);
    }
  }
  c.J = J;
  c.nr = nr;
  c.ni = ni;
  c.world = W;
  c.valid = true;
}

/** Evaluate this rank's chunk of jobs on its cached block of the job data,
 * then all-gather every job's output columns (rows = 1 + shared partials +
 * job partials, or 1 for values). */
template <typename F, bool SV, bool JV, typename T_job>
std::vector<Eigen::MatrixXd> map_rect_distributed(const Eigen::VectorXd& shared_d,
                                                  const std::vector<Eigen::Matrix<T_job, Eigen::Dynamic, 1>>& job_params,
                                                  const map_rect_data& data, std::ostream* msgs, Eigen::Index rows,
                                                  const map_rect_check& chk) {
  const int W = amd::world_size(), rank = amd::world_rank();
  // the call_id's job count (equal on every rank: map_rect_fill_cache checks
  // it), so that every rank's exchanges have the same size even when this
  // rank was passed a different number of jobs -- that is reported in the
  // first exchange and every rank throws together, instead of the others
  // waiting in it
  const size_t J = data.J;
  map_rect_check c = chk;
  if (!c.code && job_params.size() != J) c = {6, job_params.size(), J};
  const std::vector<int> chunks = map_rect_chunks(J, W);
  int first = 0, maxc = 0;
  for (int r = 0; r < W; ++r) {
    if (r < rank) first += chunks[size_t(r)];
    maxc = std::max(maxc, chunks[size_t(r)]);
  }
  const int mine = chunks[size_t(rank)];
  std::vector<Eigen::MatrixXd> local(static_cast<size_t>(mine));
  double ok = c.code ? 0.0 : 1.0;  // (a failed check: nothing evaluated)
  try {
    for (int i = 0; ok != 0.0 && i < mine; ++i) {
      const size_t j = size_t(first + i);
      const Eigen::VectorXd job_d = map_rect_values(job_params[j]);
      if constexpr (SV || JV) {
        local[size_t(i)] = map_rect_reduce_job<F, SV, JV>(shared_d, job_d, data.x_r[size_t(i)], data.x_i[size_t(i)],
                                                          msgs);
      } else {
        Eigen::VectorXd v = F()(shared_d, job_d, data.x_r[size_t(i)], data.x_i[size_t(i)], msgs);
        local[size_t(i)] = v.transpose();
      }
    }
  } catch (const std::exception&) {
    ok = 0.0;  // flagged, not rethrown: every rank must reach the exchange
  }
  // (1) status, the argument checks (code, a, b) and the number of outputs of each local job
  const long long hn = 4 + maxc;
  std::vector<double> hdr(size_t(hn), 0.0), all_hdr(size_t(hn) * W);
  hdr[0] = ok;
  hdr[1] = double(c.code);
  hdr[2] = double(c.a);
  hdr[3] = double(c.b);
  if (ok != 0.0)
    for (int i = 0; i < mine; ++i) hdr[size_t(4 + i)] = double(local[size_t(i)].cols());
  amd::allgather(hdr.data(), hn, all_hdr.data());
  map_rect_throw_gathered(all_hdr.data(), W, size_t(hn), 1);
  for (int r = 0; r < W; ++r)
    if (all_hdr[size_t(r) * hn] != 1.0) throw std::domain_error("Error during MPI evaluation.");
  long long max_pay = 0;
  for (int r = 0; r < W; ++r) {
    long long p = 0;
    for (int i = 0; i < chunks[size_t(r)]; ++i) p += rows * (long long)all_hdr[size_t(r) * hn + 4 + i];
    max_pay = std::max(max_pay, p);
  }
  // (2) every job's columns, rank r's block at r * max_pay
  std::vector<double> pay(size_t(max_pay), 0.0), all(size_t(max_pay) * W);
  long long off = 0;
  for (int i = 0; i < mine; ++i) {
    const Eigen::MatrixXd& o = local[size_t(i)];
    std::copy(o.data(), o.data() + o.size(), pay.begin() + off);
    off += o.size();
  }
  amd::allgather(pay.data(), max_pay, all.data());
  std::vector<Eigen::MatrixXd> outs(J);
  size_t j = 0;
  for (int r = 0; r < W; ++r) {
    const double* base = all.data() + size_t(r) * max_pay;
    for (int i = 0; i < chunks[size_t(r)]; ++i, ++j) {
      const Eigen::Index cols = Eigen::Index(all_hdr[size_t(r) * hn + 4 + i]);
      outs[j] = Eigen::Map<const Eigen::MatrixXd>(base, rows, cols);
      base += rows * cols;
    }
  }
  return outs;
}

}  // namespace internal

/** Forget every call_id's cached job data (the next distributed map_rect of
 * each call_id distributes its data again). */
inline void map_rect_clear_cache() {
  for (auto* c : internal::map_rect_caches()) *c = internal::map_rect_data{};
}

template <int call_id, typename F, typename T_shared, typename T_job>
Eigen::Matrix<typename std::conditional<std::is_same<T_shared, var>::value ||
                                            std::is_same<T_job, var>::value,
                                        var, double>::type,
              Eigen::Dynamic, 1>
map_rect(const Eigen::Matrix<T_shared, Eigen::Dynamic, 1>& shared_params,
         const std::vector<Eigen::Matrix<T_job, Eigen::Dynamic, 1>>& job_params,
         const std::vector<std::vector<double>>& x_r, const std::vector<std::vector<int>>& x_i,
         std::ostream* msgs = nullptr) {
  constexpr bool SV = std::is_same<T_shared, var>::value;
  constexpr bool JV = std::is_same<T_job, var>::value;
  using R = typename std::conditional<SV || JV, var, double>::type;
  using result_t = Eigen::Matrix<R, Eigen::Dynamic, 1>;
  const size_t J = job_params.size();
  // a non-root rank of a distributed job may leave the job data to the root
  // (empty x_r and x_i; its block then comes from the cache / the scatter)
  const bool dist = amd::distributed();
  const bool data_elsewhere = dist && amd::world_rank() != 0 && x_r.empty() && x_i.empty();
  const internal::map_rect_check chk = internal::map_rect_checks(job_params, x_r, x_i, data_elsewhere);
  if (!dist) internal::map_rect_throw(chk);  // (no exchange follows: throw here)
  if (!dist && J == 0) return result_t();

  const Eigen::VectorXd shared_d = internal::map_rect_values(shared_params);
  std::vector<Eigen::MatrixXd> outs(J);
  if (dist) {
    // every rank enters the exchanges, J == 0 included: a rank returning
    // early would leave the others waiting in them
    internal::map_rect_data& data = internal::map_rect_cache<call_id>();
    if (!data.valid) internal::map_rect_fill_cache(data, J, x_r, x_i, chk);
    if (data.world != amd::world_size())
      throw std::invalid_argument("map_rect: the number of jobs of a call_id must not change between calls");
    const Eigen::Index rows = 1 + (SV ? shared_params.size() : 0) + (JV && J ? job_params[0].size() : 0);
    outs = internal::map_rect_distributed<F, SV, JV>(shared_d, job_params, data, msgs, rows, chk);
    if (J == 0) return result_t();
  } else {
    for (size_t j = 0; j < J; ++j) {
      const Eigen::VectorXd job_d = internal::map_rect_values(job_params[j]);
      if constexpr (SV || JV) {
        outs[j] = internal::map_rect_reduce_job<F, SV, JV>(shared_d, job_d, x_r[j], x_i[j], msgs);
      } else {
        Eigen::VectorXd v = F()(shared_d, job_d, x_r[j], x_i[j], msgs);
        outs[j] = v.transpose();
      }
    }
  }
  size_t total = 0;
  for (size_t j = 0; j < J; ++j) total += size_t(outs[j].cols());

  // map_rect_combine: one precomputed-gradients var per output over the outer operands
  result_t result(total);
  size_t pos = 0;
  for (size_t j = 0; j < J; ++j) {
    const Eigen::MatrixXd& o = outs[j];
    for (Eigen::Index i = 0; i < o.cols(); ++i, ++pos) {
      if constexpr (SV || JV) {
        const size_t ns = SV ? size_t(shared_params.size()) : 0;
        const size_t nj = JV ? size_t(job_params[j].size()) : 0;
        vari** ops = ChainableStack::instance_->memalloc_.alloc_array<vari*>(ns + nj + 1);
        double* g = ChainableStack::instance_->memalloc_.alloc_array<double>(ns + nj + 1);
        size_t k = 0;
        if constexpr (SV)
          for (size_t s = 0; s < ns; ++s, ++k) {
            ops[k] = shared_params(s).vi_;
            g[k] = o(1 + s, i);
          }
        if constexpr (JV)
          for (size_t s = 0; s < nj; ++s, ++k) {
            ops[k] = job_params[j](s).vi_;
            g[k] = o(1 + ns + s, i);
          }
        result(pos) = var(new precomputed_gradients_vari(o(0, i), k, ops, g));
      } else {
        result(pos) = o(0, i);
      }
    }
  }
  return result;
}

}  // namespace math
}  // namespace stan
#endif
