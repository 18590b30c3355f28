#ifndef STAN_MATH_AMD_HOST_PARALLEL_HPP
#define STAN_MATH_AMD_HOST_PARALLEL_HPP

// Host-side data parallelism for the O(N^2) passes at the Eigen boundary
// (materialising a device matrix as N^2 host varis, recognising it again,
// gathering its host adjoints).  These are pure memory passes over disjoint
// index ranges, so they split across threads with no synchronisation beyond
// the join.  Small passes stay on the calling thread.
//   SMG_HOST_THREADS   worker count (default: hardware threads, at most 16)

#include <algorithm>
#include <cstdlib>
#include <thread>
#include <vector>

namespace stan {
namespace math {
namespace internal {

inline int host_threads() {
  static const int t = [] {
    const char* e = std::getenv("SMG_HOST_THREADS");
    int n = e ? std::atoi(e) : int(std::thread::hardware_concurrency());
    return std::max(1, std::min(n, 16));
  }();
  return t;
}

/** f(begin, end) over a partition of [0, n) (in order on one thread below
 * `grain` elements per thread). */
template <typename F>
inline void host_parallel_for(size_t n, F&& f, size_t grain = size_t(1) << 18) {
  const size_t want = n / grain;
  const int t = int(std::min<size_t>(size_t(host_threads()), want));
  if (t <= 1) {
    if (n) f(size_t(0), n);
    return;
  }
  std::vector<std::thread> pool;
  pool.reserve(size_t(t - 1));
  const size_t step = (n + size_t(t) - 1) / size_t(t);
  for (int k = 1; k < t; ++k) {
    const size_t b = size_t(k) * step, e = std::min(n, b + step);
    if (b < e) pool.emplace_back([&f, b, e] { f(b, e); });
  }
  f(size_t(0), std::min(n, step));
  for (auto& th : pool) th.join();
}

/** True when pred(begin, end) holds on every range of the partition. */
template <typename P>
inline bool host_parallel_all(size_t n, P&& pred, size_t grain = size_t(1) << 18) {
  const size_t want = n / grain;
  const int t = int(std::min<size_t>(size_t(host_threads()), want));
  if (t <= 1) return n == 0 || pred(size_t(0), n);
  std::vector<char> ok(size_t(t), 1);
  host_parallel_for(
      size_t(t), [&](size_t b, size_t e) {
        const size_t step = (n + size_t(t) - 1) / size_t(t);
        for (size_t k = b; k < e; ++k) {
          const size_t lo = k * step, hi = std::min(n, lo + step);
          ok[k] = lo >= hi || pred(lo, hi);
        }
      },
      1);
  for (char c : ok)
    if (!c) return false;
  return true;
}

}  // namespace internal
}  // namespace math
}  // namespace stan
#endif
