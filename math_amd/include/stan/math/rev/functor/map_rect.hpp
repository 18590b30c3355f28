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
// device functor (e.g. bernoulli_logit_glm_lpmf over the job's rows).  The
// reference's TBB / MPI executors are replaced by one HIP stream per tape; the
// row-sharded multi-GPU form of the GLM reducer is glm_shard +
// reduce_sum_bernoulli_logit_glm (bernoulli_logit_glm_lpmf.hpp).

#include <stan/math/rev/core.hpp>

#include <Eigen/Dense>

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

}  // namespace internal

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
  internal::map_rect_size_match("job parameters", job_params.size(), "real data", x_r.size());
  internal::map_rect_size_match("job parameters", job_params.size(), "int data", x_i.size());
  const size_t J = job_params.size();
  for (size_t i = 1; i < J; ++i) {
    internal::map_rect_size_match("Size of one of the vectors of the job specific parameters",
                                  job_params[i].size(),
                                  "size of another vector of the job specifc parameters",
                                  job_params[0].size());
    internal::map_rect_size_match("Size of one of the arrays of the job specific real data",
                                  x_r[i].size(),
                                  "size of another array of the job specifc real data",
                                  x_r[0].size());
    internal::map_rect_size_match("Size of one of the arrays of the job specific int data",
                                  x_i[i].size(), "size of another array of the job specifc int data",
                                  x_i[0].size());
  }
  if (J == 0) return result_t();

  const Eigen::VectorXd shared_d = internal::map_rect_values(shared_params);
  std::vector<Eigen::MatrixXd> outs(J);
  size_t total = 0;
  for (size_t j = 0; j < J; ++j) {
    const Eigen::VectorXd job_d = internal::map_rect_values(job_params[j]);
    if constexpr (SV || JV) {
      outs[j] = internal::map_rect_reduce_job<F, SV, JV>(shared_d, job_d, x_r[j], x_i[j], msgs);
    } else {
      Eigen::VectorXd v = F()(shared_d, job_d, x_r[j], x_i[j], msgs);
      outs[j] = v.transpose();
    }
    total += size_t(outs[j].cols());
  }

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
