#ifndef STAN_MATH_REV_FUN_NORMAL_LPDF_HPP
#define STAN_MATH_REV_FUN_NORMAL_LPDF_HPP

// normal_lpdf<propto>(y | mu, sigma) (prim/scal/prob/normal_lpdf.hpp:36-119)
// as ONE fused device launch (smg_normal_lpdf_fused): the three domain checks,
// the value sum_i [-1/2 z_i^2 - log sigma_i - log sqrt(2 pi)] and the
// partials dy = -z/sigma, dmu = z/sigma, dsigma = -1/sigma + z^2/sigma
// (:92-104).  The node is built with operands_and_partials, as in the
// reference (:61-62, :117).
//
// Operands: double, var, std::vector<double|var>, Eigen vectors of double|var
// (host values), dev_data<double> and dev_var_matrix (device values).  Host
// operands are staged in pinned, host-coherent memory the kernel reads and
// writes directly (zero-copy): a call over host vars is one launch and one
// completion wait, no separate copies, and its partials land in host memory
// (the node's chain() is then pure host work).  Device operands stay on the
// device and get device partials (a device edge: one axpy in chain()).
//
// Semantics kept: size_zero -> 0 (:45-47); check_not_nan(y),
// check_finite(mu), check_positive(sigma) -- reported in that order -- then
// check_consistent_sizes (:51-55); include_summand<propto, ...> drops the
// constant terms (:56-58, :86-91); all-double propto -> 0.

#include <stan/math/amd/matrix.hpp>
#include <stan/math/rev/core.hpp>
#include <stan/math/rev/meta/operands_and_partials.hpp>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <sstream>
#include <stdexcept>
#include <type_traits>
#include <vector>

namespace stan {
namespace math {

namespace internal {

/** One operand as the fused kernel sees it. */
struct fused_operand {
  size_t n = 1;
  bool vec = false;
  bool host = true;             // values staged in pinned memory
  const double* dev = nullptr;  // device values (host == false)
  double scalar = 0.0;          // value of a scalar operand
};

inline fused_operand fused_of(double x) {
  fused_operand o;
  o.scalar = x;
  return o;
}
inline fused_operand fused_of(const var& x) { return fused_of(x.val()); }
template <typename T>
inline fused_operand fused_vec(size_t n) {
  fused_operand o;
  o.n = n;
  o.vec = true;
  return o;
}
inline fused_operand fused_of(const std::vector<double>& x) { return fused_vec<double>(x.size()); }
inline fused_operand fused_of(const std::vector<var>& x) { return fused_vec<var>(x.size()); }
inline fused_operand fused_of(const dev_data<double>& x) {
  fused_operand o;
  o.n = x.size();
  o.vec = true;
  o.host = false;
  o.dev = x.data();
  return o;
}
inline fused_operand fused_of(const dev_var_matrix& x) {
  fused_operand o;
  o.n = x.size();
  o.vec = true;
  o.host = false;
  o.dev = x.val_ptr();
  return o;
}
#ifdef STAN_MATH_AMD_HAS_EIGEN
template <typename T, int R, int C>
inline fused_operand fused_of(const Eigen::Matrix<T, R, C>& x) {
  return fused_vec<T>(size_t(x.size()));
}
#endif

/** Host values of a host vector operand into dst. */
inline void fused_stage(const std::vector<double>& x, double* dst) {
  if (!x.empty()) std::memcpy(dst, x.data(), x.size() * sizeof(double));
}
inline void fused_stage(const std::vector<var>& x, double* dst) {
  for (size_t i = 0; i < x.size(); ++i) dst[i] = x[i].vi_->val_;
}
#ifdef STAN_MATH_AMD_HAS_EIGEN
template <int R, int C>
inline void fused_stage(const Eigen::Matrix<double, R, C>& x, double* dst) {
  for (Eigen::Index i = 0; i < x.size(); ++i) dst[i] = x(i);
}
template <int R, int C>
inline void fused_stage(const Eigen::Matrix<var, R, C>& x, double* dst) {
  for (Eigen::Index i = 0; i < x.size(); ++i) dst[i] = x(i).vi_->val_;
}
#endif
template <typename T>
inline void fused_stage(const T&, double*) {}  // scalars and device operands

/** Host partials of a host vector edge from the staging area. */
template <typename Edge>
inline void fused_take(Edge& e, const double* src, size_t n) {
  for (size_t i = 0; i < n; ++i) e.partials_[int(i)] = src[i];
}

template <typename T>
struct is_device_operand
    : std::integral_constant<bool, std::is_same<T, dev_var_matrix>::value ||
                                       std::is_same<T, dev_data<double>>::value> {};

/**
 * The reference's domain error for the first offending element of one
 * operand (check_not_nan / check_finite / check_positive,
 * prim/scal/err/check_*.hpp: "name[i] is v, but must ...", 1-based index for
 * a vector, no index for a scalar; v printed with the stream defaults).
 * kind: 0 not nan, 1 finite, 2 positive.  Returns without throwing when no
 * element fails.
 */
inline void normal_throw_first(const char* fn, int kind, const double* v, size_t n, bool vec) {
  static const char* const names[3] = {"Random variable", "Location parameter", "Scale parameter"};
  static const char* const musts[3] = {"not be nan!", "be finite!", "be > 0!"};
  for (size_t i = 0; i < n; ++i) {
    const double x = v[i];
    const bool bad = kind == 0 ? std::isnan(x) : (kind == 1 ? !(std::fabs(x) <= 1.7976931348623157e308) : !(x > 0.0));
    if (!bad) continue;
    std::ostringstream m;
    m << fn << ": " << names[kind];
    if (vec) m << "[" << i + 1 << "]";
    m << " is " << x << ", but must " << musts[kind];
    throw std::domain_error(m.str());
  }
}

/** Element i of a host operand (scalars broadcast). */
inline double host_val(double x, size_t) { return x; }
inline double host_val(const var& x, size_t) { return x.vi_->val_; }
inline double host_val(const std::vector<double>& x, size_t i) { return x[i]; }
inline double host_val(const std::vector<var>& x, size_t i) { return x[i].vi_->val_; }
#ifdef STAN_MATH_AMD_HAS_EIGEN
template <int R, int C>
inline double host_val(const Eigen::Matrix<double, R, C>& x, size_t i) { return x(Eigen::Index(i)); }
template <int R, int C>
inline double host_val(const Eigen::Matrix<var, R, C>& x, size_t i) { return x(Eigen::Index(i)).vi_->val_; }
#endif

/**
 * Largest element count evaluated on the host (the size gate the reference
 * applies before offloading, opencl/opencl_context.hpp:164-182): below it a
 * call over host operands is cheaper than one device round trip (~20 us on
 * MI355X against ~1 ns per element on a host core).  SMG_NORMAL_HOST_MAX
 * overrides it; 0 sends every call to the device.
 */
inline size_t& normal_host_max_ref() {
  static size_t v = [] {
    const char* e = std::getenv("SMG_NORMAL_HOST_MAX");
    return e ? size_t(std::strtoull(e, nullptr, 10)) : size_t(16384);
  }();
  return v;
}
inline size_t normal_host_max() { return normal_host_max_ref(); }

inline void normal_check_sizes(const char* fn, const fused_operand* ops);

}  // namespace internal

namespace amd {
/** Set the normal_lpdf host gate (elements); 0 sends every call to the device. */
inline void set_normal_host_max(size_t n) { internal::normal_host_max_ref() = n; }
}  // namespace amd

namespace internal {

/**
 * Host evaluation of normal_lpdf over host operands (small calls), the
 * reference's own loop (prim/scal/prob/normal_lpdf.hpp:51-117): checks in the
 * same order, value accumulated in element order, partials into the edges.
 */
template <bool propto, typename T_y, typename T_loc, typename T_scale>
inline typename ops_return<T_y, T_loc, T_scale>::type normal_lpdf_host(const T_y& y, const T_loc& mu,
                                                                       const T_scale& sigma,
                                                                       const fused_operand* ops, size_t N,
                                                                       int include) {
  static const char* fn = "normal_lpdf";
  constexpr bool vy = op_is_var<T_y>::value, vmu = op_is_var<T_loc>::value, vs = op_is_var<T_scale>::value;
  // the reference's checks in its order (not NaN y, finite mu, positive
  // sigma, then consistent sizes); the message is built from a copy of the
  // values only when an element fails
  auto check = [&](int kind, const auto& x, const fused_operand& o) {
    bool bad = false;
    for (size_t i = 0; i < o.n; ++i) {
      const double v = host_val(x, i);
      bad |= kind == 0 ? std::isnan(v) : (kind == 1 ? !(std::fabs(v) <= 1.7976931348623157e308) : !(v > 0.0));
    }
    if (!bad) return;
    std::vector<double> v(o.n);
    for (size_t i = 0; i < o.n; ++i) v[i] = host_val(x, i);
    normal_throw_first(fn, kind, v.data(), o.n, o.vec);
  };
  auto check_all = [&] {
    check(0, y, ops[0]);
    check(1, mu, ops[1]);
    check(2, sigma, ops[2]);
  };
  bool sizes_ok = true;
  for (int i = 0; i < 3; ++i)
    if (ops[i].vec && ops[i].n != N) sizes_ok = false;
  if (!sizes_ok) {  // no element loop over ragged operands: the checks, then the sizes error
    check_all();
    normal_check_sizes(fn, ops);
  }
  // scalar operands are checked now; the vector operands' checks ride along
  // in the element loop below (one pass over the values instead of two), and
  // a failure re-runs the ordered checks before anything reaches the tape
  for (int i = 0; i < 3; ++i)
    if (!ops[i].vec) {
      if (i == 0) check(0, y, ops[0]);
      if (i == 1) check(1, mu, ops[1]);
      if (i == 2) check(2, sigma, ops[2]);
    }
  using ret_t = typename ops_return<T_y, T_loc, T_scale>::type;
  if constexpr (!(vy || vmu || vs)) {
    if (propto) {
      check_all();
      return ret_t(0.0);
    }
  }
  operands_and_partials<T_y, T_loc, T_scale> ops_partials(y, mu, sigma);
  const double neg_log_sqrt_two_pi = -0.91893853320467274178;
  // 1 / sigma and log sigma once per element of sigma (:71-77): once for a scalar
  const bool svec = ops[2].vec;
  const double inv_s0 = 1.0 / host_val(sigma, 0);
  const double log_s0 = (include & 2) ? std::log(host_val(sigma, 0)) : 0.0;
  // the three summands accumulated separately, the quadratic one in four
  // interleaved partial sums (no loop-carried add chain through one logp);
  // same terms as the reference's per-element logp updates (:87-97), summed
  // in a different order (round-off only)
  double q[4] = {0.0, 0.0, 0.0, 0.0};
  double sum_log_s = 0.0;
  bool bad = false;
  const bool yvec = ops[0].vec, mvec = ops[1].vec;
  for (size_t n = 0; n < N; ++n) {
    const double yv = host_val(y, n), mv = host_val(mu, n), sv = host_val(sigma, n);
    if (yvec) bad |= std::isnan(yv);
    if (mvec) bad |= !(std::fabs(mv) <= 1.7976931348623157e308);
    if (svec) bad |= !(sv > 0.0);
    const double inv_s = svec ? 1.0 / sv : inv_s0;
    const double z = (yv - mv) * inv_s;
    const double z2 = z * z;
    q[n & 3] += z2;
    if (svec && (include & 2)) sum_log_s += std::log(sv);
    const double sc = inv_s * z;
    if constexpr (vy) ops_partials.edge1_.partials_[int(n)] -= sc;
    if constexpr (vmu) ops_partials.edge2_.partials_[int(n)] += sc;
    if constexpr (vs) ops_partials.edge3_.partials_[int(n)] += -inv_s + inv_s * z2;
  }
  if (bad) check_all();  // throws the reference's first failure
  double logp = 0.0;
  if (include & 1) logp += neg_log_sqrt_two_pi * double(N);
  if (include & 2) logp -= svec ? sum_log_s : log_s0 * double(N);
  if (include & 4) logp += -0.5 * ((q[0] + q[1]) + (q[2] + q[3]));
  if constexpr (vy || vmu || vs) {
    return ops_partials.build(logp);
  } else {
    return logp;
  }
}

inline void normal_check_sizes(const char* fn, const fused_operand* ops) {
  // check_consistent_sizes (prim/scal/err/check_consistent_sizes.hpp): the
  // expected size is the largest vector's; the first vector operand of
  // another size is reported
  static const char* const names[3] = {"Random variable", "Location parameter", "Scale parameter"};
  size_t expect = 0;
  for (int i = 0; i < 3; ++i)
    if (ops[i].vec && ops[i].n > expect) expect = ops[i].n;
  for (int i = 0; i < 3; ++i)
    if (ops[i].vec && ops[i].n != expect) {
      std::ostringstream m;
      m << fn << ": " << names[i] << " has dimension = " << ops[i].n << ", expecting dimension = " << expect
        << "; a function was called with arguments of different scalar, array, vector, or "
           "matrix types, and they were not consistently sized;  all arguments must be "
           "scalars or multidimensional values of the same shape.";
      throw std::invalid_argument(m.str());
    }
}

}  // namespace internal

template <bool propto, typename T_y, typename T_loc, typename T_scale>
inline typename internal::ops_return<T_y, T_loc, T_scale>::type normal_lpdf(const T_y& y, const T_loc& mu,
                                                                            const T_scale& sigma) {
  using internal::fused_operand;
  static const char* fn = "normal_lpdf";
  constexpr bool vy = internal::op_is_var<T_y>::value, vmu = internal::op_is_var<T_loc>::value,
                 vs = internal::op_is_var<T_scale>::value;
  using ret_t = typename internal::ops_return<T_y, T_loc, T_scale>::type;
  fused_operand ops[3] = {internal::fused_of(y), internal::fused_of(mu), internal::fused_of(sigma)};
  for (auto& o : ops)
    if (o.vec && o.n == 0) return ret_t(0.0);
  // include_summand<propto, ...>
  const bool inc_const = !propto;
  const bool inc_logsig = !propto || vs;
  const bool inc_quad = !propto || vy || vmu || vs;
  size_t N = 1;
  bool sizes_ok = true;
  for (auto& o : ops)
    if (o.vec) N = o.n > N ? o.n : N;
  for (auto& o : ops)
    if (o.vec && o.n != N) sizes_ok = false;

  const int include = (inc_const ? 1 : 0) | (inc_logsig ? 2 : 0) | (inc_quad ? 4 : 0);
  if constexpr (!internal::is_device_operand<T_y>::value && !internal::is_device_operand<T_loc>::value
                && !internal::is_device_operand<T_scale>::value) {
    if (N <= internal::normal_host_max())
      return internal::normal_lpdf_host<propto>(y, mu, sigma, ops, N, include);
  }

  smg_ctx* c = amd::ctx();
  // pinned staging: [res(8) | host values of y, mu, sigma | host partials of y, mu, sigma]
  size_t off = 8, val_off[3], g_off[3];
  for (int i = 0; i < 3; ++i) {
    val_off[i] = off;
    if (ops[i].host && ops[i].vec) off += ops[i].n;
  }
  const bool want_g[3] = {vy, vmu, vs};
  for (int i = 0; i < 3; ++i) {
    g_off[i] = off;
    if (want_g[i] && ops[i].vec && ops[i].host) off += ops[i].n;
  }
  double* st = static_cast<double*>(smg_pinned_result(c, off * sizeof(double)));
  if (!st) throw std::bad_alloc();
  for (int i = 0; i < 8; ++i) st[i] = 0.0;
  internal::fused_stage(y, st + val_off[0]);
  internal::fused_stage(mu, st + val_off[1]);
  internal::fused_stage(sigma, st + val_off[2]);
  const double* vals[3];  // vector operands; NULL: the scalar value (a kernel argument)
  for (int i = 0; i < 3; ++i) vals[i] = !ops[i].vec ? nullptr : (ops[i].host ? st + val_off[i] : ops[i].dev);
  operands_and_partials<T_y, T_loc, T_scale> ops_partials(y, mu, sigma);
  // partial outputs: host vectors -> staging, device vars -> the device edge,
  // scalars -> reduced into res[4 + i]
  double* g[3] = {nullptr, nullptr, nullptr};
  if constexpr (vy) {
    if (ops[0].vec) {
      if constexpr (internal::is_device_operand<T_y>::value) g[0] = ops_partials.edge1_.partials_;
      else g[0] = st + g_off[0];
    } else {
      g[0] = st + 4;
    }
  }
  if constexpr (vmu) {
    if (ops[1].vec) {
      if constexpr (internal::is_device_operand<T_loc>::value) g[1] = ops_partials.edge2_.partials_;
      else g[1] = st + g_off[1];
    } else {
      g[1] = st + 5;
    }
  }
  if constexpr (vs) {
    if (ops[2].vec) {
      if constexpr (internal::is_device_operand<T_scale>::value) g[2] = ops_partials.edge3_.partials_;
      else g[2] = st + g_off[2];
    } else {
      g[2] = st + 6;
    }
  }
  if (sizes_ok) {
    amd::check(smg_normal_lpdf_fused(c, vals[0], vals[1], vals[2], ops[0].scalar, ops[1].scalar, ops[2].scalar,
                                     (long long)N, include, st, g[0], g[1], g[2]),
               fn);
  } else {
    // error path: the domain checks over each operand's own length, in order
    for (int i = 0; i < 3; ++i) {
      if (vals[i]) {
        amd::check(smg_check_domain(c, vals[i], (long long)ops[i].n, i, st + 1 + i), fn);
      } else {
        const double x = ops[i].scalar;
        st[1 + i] = (i == 0 ? x != x : i == 1 ? !(std::fabs(x) <= 1.7976931348623157e308) : !(x > 0.0)) ? 1.0 : 0.0;
      }
    }
    amd::check(smg_sync(c), fn);
  }
  for (int i = 0; i < 3; ++i) {
    if (st[1 + i] == 0.0) continue;
    // error path: the operand's values on the host, the first offending one reported
    std::vector<double> hv(ops[i].vec ? ops[i].n : 1);
    if (!ops[i].vec) hv[0] = ops[i].scalar;
    else if (ops[i].host) std::memcpy(hv.data(), st + val_off[i], ops[i].n * sizeof(double));
    else amd::to_host(hv.data(), ops[i].dev, ops[i].n);
    internal::normal_throw_first(fn, i, hv.data(), hv.size(), ops[i].vec);
  }
  internal::normal_check_sizes(fn, ops);
  const double logp = st[0];
  if constexpr (vy || vmu || vs) {
    if constexpr (vy) {
      if (!ops[0].vec) ops_partials.edge1_.partials_[0] = st[4];
      else if constexpr (!internal::is_device_operand<T_y>::value)
        internal::fused_take(ops_partials.edge1_, st + g_off[0], ops[0].n);
    }
    if constexpr (vmu) {
      if (!ops[1].vec) ops_partials.edge2_.partials_[0] = st[5];
      else if constexpr (!internal::is_device_operand<T_loc>::value)
        internal::fused_take(ops_partials.edge2_, st + g_off[1], ops[1].n);
    }
    if constexpr (vs) {
      if (!ops[2].vec) ops_partials.edge3_.partials_[0] = st[6];
      else if constexpr (!internal::is_device_operand<T_scale>::value)
        internal::fused_take(ops_partials.edge3_, st + g_off[2], ops[2].n);
    }
    return ops_partials.build(logp);
  } else {
    return propto ? 0.0 : logp;
  }
}

template <typename T_y, typename T_loc, typename T_scale>
inline auto normal_lpdf(const T_y& y, const T_loc& mu, const T_scale& sigma) {
  return normal_lpdf<false>(y, mu, sigma);
}

}  // namespace math
}  // namespace stan
#endif
