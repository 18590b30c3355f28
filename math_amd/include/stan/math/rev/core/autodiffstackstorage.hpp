#ifndef STAN_MATH_REV_CORE_AUTODIFFSTACKSTORAGE_HPP
#define STAN_MATH_REV_CORE_AUTODIFFSTACKSTORAGE_HPP

// The per-thread autodiff tape.
//
// Same members and nesting semantics as the reference's AutodiffStackSingleton
// (stan/math/rev/core/autodiffstackstorage.hpp:88-143): var_stack_ (varis
// whose chain() runs in the reverse sweep), var_nochain_stack_ (varis that
// only hold values/adjoints), var_alloc_stack_ (arena objects with
// destructors), the host arena memalloc_, and the nested size stacks.
// The tape is always thread-local here (the reference makes it thread-local
// under STAN_THREADS).
//
// MI355X extension: matrix-valued nodes keep their values and adjoints in the
// thread's device arena (stan/math/amd/device.hpp).  The tape therefore also
// records
//   dev_adj_stack_      device adjoint buffers (zeroed by set_zero_all_adjoints)
//   nested_dev_marks_   device-arena marks per nesting level
//   pending_            device -> host adjoint contributions that must land in
//                       host vari::adj_ before the next host chain() runs.
//   host_blocks_        device nodes materialised as contiguous host varis at
//                       an Eigen boundary (recognised again by to_dev).

#include <stan/math/memory/stack_alloc.hpp>

#include <cstddef>
#include <vector>

namespace stan {
namespace math {

class vari;
class chainable_alloc;

struct dev_buffer {
  double* ptr;
  size_t n;
};
struct pending_adjoint {
  vari* target;       // host vari whose adj_ receives the value
  const double* src;  // device scalar
};
/** A device matrix node materialised as host varis (stan/math/amd/matrix.hpp):
 * the n varis the block owns, contiguous in the arena, registered here
 * instead of on var_nochain_stack_ (zeroed by set_zero_all_adjoints).  Which
 * vari stands at element (i, j) follows the reference's vari identity for the
 * producing function (layout; stan/math/amd/matrix.hpp block_column):
 *   0 dense  every element its own vari, column-major (n = rows cols);
 *   1 lower  a cholesky_decompose factor: the lower triangle packed column by
 *            column (n = rows (rows + 1) / 2), the strict upper one dummy vari
 *            (rev/mat/fun/cholesky_decompose.hpp:34-48);
 *   2 sym    a gp_exp_quad_cov matrix: the lower triangle packed, (i, j) and
 *            (j, i) one vari (rev/mat/fun/gp_exp_quad_cov.hpp:235);
 *   3 diag   add_diag's output: n = min(rows, cols) new diagonal varis, every
 *            other element the input's own vari (prim/mat/fun/add_diag.hpp:25-27)
 *            -- block `base`'s, or base_elems[i + j rows] when the input was
 *            no block. */
struct host_block {
  vari* first;   // the owned varis
  size_t n;
  void* node;    // the dev_matrix_vari it mirrors
  vari* dummy;   // layout 1: the strict upper triangle's one vari, else null
  int rows, cols;
  bool dirty;    // a landed device->host pending adjoint targeted one of its varis
  int layout = 0;
  long base = -1;
  vari* const* base_elems = nullptr;
  // layout 1: the device's strict-upper adjoint sum already published into
  // dummy (a later publish adds only what the device gained since)
  double dummy_dev = 0.0;
  // the sweep in which a node chained after the block's bridge added into
  // one of its varis' host adjoints (grad.hpp log_host_touches)
  size_t touched_sweep = 0;
};
/** A node that may add into some matrix node's DEVICE adjoint
 * (vari::may_write_device_adjoint), with its var_stack_ position: the
 * writers a structured reverse checks are the entries after its own
 * position (a binary search), not the whole rest of the tape. */
struct dev_writer {
  size_t pos;
  vari* v;
};

template <typename ChainableT, typename ChainableAllocT>
struct AutodiffStackSingleton {
  using AutodiffStackSingleton_t = AutodiffStackSingleton<ChainableT, ChainableAllocT>;

  struct AutodiffStackStorage {
    AutodiffStackStorage& operator=(const AutodiffStackStorage&) = delete;

    std::vector<ChainableT*> var_stack_;
    std::vector<ChainableT*> var_nochain_stack_;
    std::vector<ChainableAllocT*> var_alloc_stack_;
    stack_alloc memalloc_;

    std::vector<size_t> nested_var_stack_sizes_;
    std::vector<size_t> nested_var_nochain_stack_sizes_;
    std::vector<size_t> nested_var_alloc_stack_starts_;

    // device side
    std::vector<dev_buffer> dev_adj_stack_;
    std::vector<size_t> nested_dev_adj_sizes_;
    std::vector<size_t> nested_dev_marks_;
    std::vector<pending_adjoint> pending_;
    std::vector<host_block> host_blocks_;
    std::vector<size_t> nested_host_block_sizes_;
    std::vector<dev_writer> dev_writers_;  // in stack order (registered at construction)
    // host_blocks_ indices ordered by address, rebuilt once per sweep that
    // has blocks (the bisection of log_host_touches), and the sweep it is for
    std::vector<size_t> block_order_;
    size_t block_order_sweep_ = 0;
    // reverse sweeps started on this tape (grad()): a structured adjoint a
    // node deposits is valid for the sweep that deposited it only
    size_t sweep_ = 0;
    // after a sweep, publish_ (set once a host block exists: stan/math/amd/
    // matrix.hpp) writes every host block's device adjoint into its varis, so
    // they read what the reference's would; no_publish_ > 0 while a functional
    // that reads only its independent variables runs its sweeps (gradient(),
    // hessian(), hessian_times_vector(), map_rect's jobs, var::grad(x, g))
    void (*publish_)(size_t from) = nullptr;
    int no_publish_ = 0;
  };

  AutodiffStackSingleton() : own_instance_(init()) {}
  ~AutodiffStackSingleton() {
    if (own_instance_) {
      delete instance_;
      instance_ = nullptr;
    }
  }
  AutodiffStackSingleton(const AutodiffStackSingleton_t&) = delete;
  AutodiffStackSingleton& operator=(const AutodiffStackSingleton_t&) = delete;

  // The tape pointer is read on every var construction and every chain() of
  // the sweep.  Executables get the local-exec model by default; a shared
  // library built with STAN_MATH_AMD_TLS_INITIAL_EXEC uses initial-exec, which
  // avoids a __tls_get_addr call per read but draws on glibc's small static
  // TLS surplus (a library dlopen'ed late can then fail with "cannot allocate
  // memory in static TLS block"), so it is opt-in: our bench library, loaded
  // first by bench.py, opts in; other shared builds keep the default model.
#ifdef STAN_MATH_AMD_TLS_INITIAL_EXEC
  static inline thread_local AutodiffStackStorage* instance_ __attribute__((tls_model("initial-exec"))) = nullptr;
#else
  static inline thread_local AutodiffStackStorage* instance_ = nullptr;
#endif

 private:
  static bool init() {
    if (!instance_) {
      instance_ = new AutodiffStackStorage();
      return true;
    }
    return false;
  }
  bool own_instance_;
};

using ChainableStack = AutodiffStackSingleton<vari, chainable_alloc>;

// The main thread's tape (the reference instantiates it in
// rev/core/init_chainablestack.hpp); other threads construct a
// ChainableStack object before touching the AD system.
inline ChainableStack main_thread_tape_owner_;

}  // namespace math
}  // namespace stan
#endif
