#ifndef STAN_MATH_AMD_HOST_PARALLEL_HPP
#define STAN_MATH_AMD_HOST_PARALLEL_HPP

// Host-side data parallelism for the O(N^2) passes at the Eigen boundary
// (materialising a device matrix as N^2 host varis, recognising it again,
// gathering its host adjoints).  These are pure memory passes over disjoint
// index ranges, so they split across a small persistent pool of worker
// threads with no synchronisation beyond the join.  Small passes stay on the
// calling thread.
//   SMG_HOST_THREADS   worker count (default: hardware threads, at most 16)

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <mutex>
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

/** A persistent pool: run(f) calls f(0..n-1), f(0) on the caller, and
 * returns when all have finished.  Workers sleep on a condition variable
 * between jobs.  One job at a time (callers from several tape threads take
 * turns). */
class host_pool {
 public:
  explicit host_pool(int n) : n_(n) {
    for (int i = 1; i < n; ++i) th_.emplace_back([this, i] { loop(i); });
  }
  ~host_pool() {
    {
      std::lock_guard<std::mutex> lk(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int size() const { return n_; }
  void run(const std::function<void(int)>& f) {
    std::lock_guard<std::mutex> one(run_m_);
    {
      std::lock_guard<std::mutex> lk(m_);
      job_ = &f;
      left_.store(n_ - 1, std::memory_order_relaxed);
      ++gen_;
    }
    cv_.notify_all();
    f(0);
    while (left_.load(std::memory_order_acquire) > 0) std::this_thread::yield();
  }

 private:
  void loop(int i) {
    long long seen = 0;
    for (;;) {
      const std::function<void(int)>* f;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        f = job_;
      }
      (*f)(i);
      left_.fetch_sub(1, std::memory_order_release);
    }
  }
  int n_;
  std::vector<std::thread> th_;
  std::mutex m_, run_m_;
  std::condition_variable cv_;
  const std::function<void(int)>* job_ = nullptr;
  long long gen_ = 0;
  std::atomic<int> left_{0};
  bool stop_ = false;
};

inline host_pool& the_host_pool() {
  static host_pool p(host_threads());
  return p;
}

/** f(begin, end) over a partition of [0, n) (in order on the calling thread
 * below `grain` elements per thread). */
template <typename F>
inline void host_parallel_for(size_t n, F&& f, size_t grain = size_t(1) << 18) {
  const size_t want = n / grain;
  const int t = int(std::min<size_t>(size_t(host_threads()), want));
  if (t <= 1) {
    if (n) f(size_t(0), n);
    return;
  }
  host_pool& pool = the_host_pool();
  const int parts = pool.size();
  const size_t step = (n + size_t(parts) - 1) / size_t(parts);
  pool.run([&](int k) {
    const size_t b = size_t(k) * step, e = std::min(n, b + step);
    if (b < e) f(b, e);
  });
}

/** True when pred(begin, end) holds on every range of the partition. */
template <typename P>
inline bool host_parallel_all(size_t n, P&& pred, size_t grain = size_t(1) << 18) {
  std::atomic<bool> ok{true};
  host_parallel_for(
      n,
      [&](size_t b, size_t e) {
        if (!pred(b, e)) ok.store(false, std::memory_order_relaxed);
      },
      grain);
  return ok.load();
}

}  // namespace internal
}  // namespace math
}  // namespace stan
#endif
