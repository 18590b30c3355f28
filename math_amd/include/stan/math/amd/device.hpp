#ifndef STAN_MATH_AMD_DEVICE_HPP
#define STAN_MATH_AMD_DEVICE_HPP

// Per-thread device context: the MI355X side of the autodiff tape.
//
// The reference keeps one tape per thread (rev/core/autodiffstackstorage.hpp:
// 11-25, 88-143).  Every tape here owns, lazily, one smg_ctx from the C-ABI
// (include/smg_hip.h): a HIP stream and a device bump arena that start_nested
// / recover_memory(_nested) mark and rewind exactly like the host arena.
// Device selection: set_device(d) before the first device op, else the
// environment variable SMG_DEVICE, else 0.
//
// Error mapping: C-ABI status bits become the reference's exceptions
// (std::domain_error for domain checks, prim/scal/err/domain_error.hpp:28-33;
// std::invalid_argument for size mismatches; std::bad_alloc for OOM;
// std::runtime_error for HIP failures).

#include <chrono>
#include <smg_hip.h>

#include <cmath>
#include <cstdlib>
#include <sys/syscall.h>
#include <unistd.h>
#include <new>
#include <sstream>
#include <stdexcept>
#include <string>

namespace stan {
namespace math {
namespace amd {

struct device_state {
  smg_ctx* ctx = nullptr;
  int device = -1;
  // a worker thread's context is released when the thread ends; the main
  // thread's is left to process teardown: its thread_local destructor runs
  // inside exit(), after the HIP runtime (or a profiler's tool library) may
  // already have torn down the streams it would release
  ~device_state() {
    if (ctx && ::syscall(SYS_gettid) != ::getpid()) smg_ctx_destroy(ctx);
  }
};

inline device_state& state() {
  static thread_local device_state s;
  return s;
}

inline int default_device() {
  const char* e = std::getenv("SMG_DEVICE");
  return e ? std::atoi(e) : 0;
}

/** Select the device for this thread's tape (before its first device op). */
inline void set_device(int d) {
  device_state& s = state();
  if (s.ctx && s.device != d)
    throw std::logic_error("stan::math::amd::set_device: context already created");
  s.device = d;
}

inline void throw_status(int st, const char* function, const char* what = "") {
  if (st == SMG_OK) return;
  std::ostringstream m;
  m << function << ": ";
  if (st & SMG_ERR_NOT_PD) {
    m << "Matrix " << what << " is not positive definite";
    throw std::domain_error(m.str());
  }
  if (st & SMG_ERR_NOT_SYMMETRIC) {
    m << what << " is not symmetric";
    throw std::domain_error(m.str());
  }
  if (st & SMG_ERR_NOT_POSITIVE) {
    m << what << " is not positive";
    throw std::domain_error(m.str());
  }
  if (st & SMG_ERR_NONFINITE) {
    m << what << " is not finite";
    throw std::domain_error(m.str());
  }
  if (st & SMG_ERR_OOM) throw std::bad_alloc();
  if (st & SMG_ERR_SYNC) {
    m << "device synchronisation timed out in " << what;
    throw std::runtime_error(m.str());
  }
  if (st & SMG_ERR_ARG) {
    m << "invalid argument " << what;
    throw std::invalid_argument(m.str());
  }
  m << "HIP runtime failure (status " << st << ")";
  throw std::runtime_error(m.str());
}

/**
 * The reference's check_symmetric message (prim/mat/err/check_symmetric.hpp:
 * 36-55): the first pair (m < n, m outer) with !(|A(m,n) - A(n,m)| <= 1e-8),
 * "<fn>: <name> is not symmetric. <name>[m,n] = a, but <name>[n,m] = b"
 * (1-based).  A: host, column-major n x n.
 */
inline void throw_not_symmetric_host(const char* fn, const char* name, const double* A, int n) {
  for (int m = 0; m < n; ++m)
    for (int q = m + 1; q < n; ++q) {
      const double a = A[m + size_t(q) * n], b = A[q + size_t(m) * n];
      if (!(std::fabs(a - b) <= 1e-8)) {
        std::ostringstream o;
        o << fn << ": " << name << " is not symmetric. " << name << "[" << m + 1 << "," << q + 1 << "] = " << a
          << ", but " << name << "[" << q + 1 << "," << m + 1 << "] = " << b;
        throw std::domain_error(o.str());
      }
    }
  std::ostringstream o;  // (the device flagged it; no pair found on the host copy)
  o << fn << ": " << name << " is not symmetric";
  throw std::domain_error(o.str());
}

/** This thread's device context (created on first use). */
inline smg_ctx* ctx() {
  device_state& s = state();
  if (__builtin_expect(s.ctx == nullptr, 0)) {
    if (s.device < 0) s.device = default_device();
    smg_ctx* c = nullptr;
    const int rc = smg_ctx_create(s.device, size_t(256) << 20, &c);
    if (rc != SMG_OK) throw_status(rc, "stan::math::amd::ctx", "(device context)");
    s.ctx = c;
  }
  return s.ctx;
}

inline bool has_ctx() { return state().ctx != nullptr; }

/** Check a C-ABI return code. */
inline void check(int rc, const char* function, const char* what = "") {
  if (__builtin_expect(rc != SMG_OK, 0)) throw_status(rc, function, what);
}

/** After a status word read with smg_status_enqueue: a timed-out hand-off
 * (SMG_ERR_SYNC) throws here.  smg_status clears the WHOLE latch first, so
 * any domain bits latched with it are dropped: the evaluation is abandoned
 * (its values are not trustworthy after a failed hand-off) and the next one
 * starts from a clean status word. */
inline void throw_if_sync(int st, const char* function, const char* what) {
  if (__builtin_expect(!(st & SMG_ERR_SYNC), 1)) return;
  int cleared = 0;
  smg_status(state().ctx, &cleared);
  throw_status(SMG_ERR_SYNC, function, what);
}

/** Synchronise and translate latched device-side domain errors. */
inline void check_status(const char* function, const char* what = "") {
  int st = 0;
  check(smg_status(ctx(), &st), function);
  throw_status(st, function, what);
}

/** Device arena allocation (recovered with the tape). */
inline double* alloc_doubles(size_t n) {
  void* p = smg_arena_alloc(ctx(), (n ? n : 1) * sizeof(double));
  if (!p) throw std::bad_alloc();
  return static_cast<double*>(p);
}
inline int* alloc_ints(size_t n) {
  void* p = smg_arena_alloc(ctx(), (n ? n : 1) * sizeof(int));
  if (!p) throw std::bad_alloc();
  return static_cast<int*>(p);
}

/** Blocking host -> device copy of a host buffer (safe for pageable memory). */
inline void to_device(double* dst, const double* src, size_t n) {
  if (!n) return;
  smg_ctx* c = ctx();
  void* stage = smg_host_scratch(c, n * sizeof(double));
  if (!stage) throw std::bad_alloc();
  __builtin_memcpy(stage, src, n * sizeof(double));
  check(smg_memcpy_h2d(c, dst, stage, n * sizeof(double)), "to_device");
  check(smg_sync(c), "to_device");
}
inline void to_device_int(int* dst, const int* src, size_t n) {
  if (!n) return;
  smg_ctx* c = ctx();
  void* stage = smg_host_scratch(c, n * sizeof(int));
  if (!stage) throw std::bad_alloc();
  __builtin_memcpy(stage, src, n * sizeof(int));
  check(smg_memcpy_h2d(c, dst, stage, n * sizeof(int)), "to_device");
  check(smg_sync(c), "to_device");
}

/** Blocking device -> host copy.  When a launch that can latch the status
 * word asynchronously is in flight (a persistent solve / panel, whose timed-out
 * hand-off latches SMG_ERR_SYNC), the status is read in the same sync and a
 * latched error throws here instead of returning a wrong value. */
inline void to_host(double* dst, const double* src, size_t n) {
  if (!n) return;
  smg_ctx* c = ctx();
  int armed = 0;
  check(smg_status_armed(c, &armed), "to_host");
  double* stage = static_cast<double*>(smg_host_scratch(c, (n + 1) * sizeof(double)));
  if (!stage) throw std::bad_alloc();
  check(smg_memcpy_d2h(c, stage, src, n * sizeof(double)), "to_host");
  if (armed) check(smg_status_enqueue(c, reinterpret_cast<int*>(stage + n)), "to_host");
  check(smg_sync(c), "to_host");
  if (armed) throw_if_sync(*reinterpret_cast<int*>(stage + n), "to_host", "a persistent solve");
  __builtin_memcpy(dst, stage, n * sizeof(double));
}

/** Dev instrumentation: host timestamps (steady clock, seconds) at numbered
 * points of one evaluation, taken only while phase_log_on() (the bench's
 * phase split sets it around one evaluation). */
struct phase_log_t {
  bool on = false;
  double t[32] = {};
};
inline phase_log_t& phase_log() {
  static phase_log_t p;
  return p;
}
inline void phase_mark(int k) {
  phase_log_t& p = phase_log();
  if (p.on && k >= 0 && k < 32)
    p.t[k] = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

inline void zero(double* p, size_t n) {
  if (n) check(smg_memset(ctx(), p, 0, n * sizeof(double)), "zero");
}

}  // namespace amd
}  // namespace math
}  // namespace stan
#endif
