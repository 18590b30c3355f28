#ifndef STAN_MATH_REV_FUN_CHOLESKY_DECOMPOSE_HPP
#define STAN_MATH_REV_FUN_CHOLESKY_DECOMPOSE_HPP

// add_diag and cholesky_decompose on device matrices of vars.
//
// add_diag (prim/mat/fun/add_diag.hpp:20-55): the reference builds N scalar
// `+` varis for the diagonal and shares the off-diagonal varis; here the
// output node carries its own value/adjoint columns and chain() folds the
// adjoint back: Aadj += Badj, d' += diag(Badj).
//
// cholesky_decompose (rev/mat/fun/cholesky_decompose.hpp:378-427): the same
// checks in the same order (check_square, check_symmetric at absolute 1e-8,
// check_pos_definite -> std::domain_error) BEFORE the node is pushed; the
// output's strict upper triangle is structurally zero (the reference points
// those entries at a dummy vari, :34-48), which downstream nodes exploit.
// chain() runs Murray's blocked adjoint on the device (smg_cholesky_rev) and
// adds into the LOWER triangle of A's adjoint only, like :159-164 -- or, when
// the factor's only adjoint is a multi_normal_cholesky_lpdf's, the closed
// form of that composition (cholesky_dev_vari below).

#include <stan/math/amd/matrix.hpp>
#include <stan/math/rev/core.hpp>

#include <cstdlib>
#include <sstream>
#include <stdexcept>
#include <utility>
#include <vector>

namespace stan {
namespace math {

namespace internal {

/** B = A + diag(d) over the min(m, n) leading diagonal (prim/mat/fun/add_diag.hpp:20-55):
 * A a device var node or data; d a scalar (var or double) or a device vector
 * (var node or data). */
class add_diag_dev_vari : public device_vari, public structured_adjoint_sink {
 public:
  dev_operand A_;
  dev_matrix_vari* B_;
  vari* d_vi_;    // scalar var diagonal (null otherwise)
  double* dadj_;  // its device adjoint
  dev_operand dv_;  // vector diagonal (dv_.rows == 0 when scalar)
  size_t pos_;      // this node's index in var_stack_
  // B's adjoint in inverse form (a Cholesky factorisation's closed form,
  // cholesky_dev_vari): dep_ deposited in this sweep, exp_ consumed without
  // forming B's dense adjoint (expand_adjoint writes it when read)
  inverse_adjoint dep_, exp_;

  add_diag_dev_vari(const dev_operand& A, double d, vari* d_vi, const dev_operand& dv)
      : device_vari(0.0), A_(A), B_(new dev_matrix_vari(A.rows, A.cols)), d_vi_(d_vi),
        dadj_(d_vi ? amd::alloc_doubles(1) : nullptr), dv_(dv),
        pos_(ChainableStack::instance_->var_stack_.size() - 1) {
    if (A.rows == A.cols && !dv.rows) B_->sink_ = this;  // (square, scalar diagonal)
    smg_ctx* c = amd::ctx();
    const int m = A.rows, n = A.cols, k = m < n ? m : n;
    const double* dvec = dv_.rows ? dv_.val() : nullptr;
    if (m == n) {
      amd::check(smg_add_diag_fwd(c, A_.val(), m, m, d, dvec, B_->val_, m), "add_diag");
    } else if (m && n) {  // copy, then the k x k leading block in place
      amd::check(smg_memcpy_d2d(c, B_->val_, A_.val(), size_t(m) * n * sizeof(double)), "add_diag");
      amd::check(smg_add_diag_fwd(c, B_->val_, m, k, d, dvec, B_->val_, m), "add_diag");
    }
  }
  bool may_write_device_adjoint(const void* node) const override {
    return (A_.vi && node == A_.vi) || (dv_.vi && node == dv_.vi);
  }
  // one deposit per sweep (a second factorisation of B writes its G densely)
  bool take_inverse_adjoint(const inverse_adjoint& d, double*) override {
    if (B_->sink_ != this) return false;
    if (dep_.C && dep_.sweep == ChainableStack::instance_->sweep_) return false;
    dep_ = d;
    return true;
  }
  // B's adjoint read: this sweep's deposit written densely, consumed (exp_)
  // or not yet chained (dep_), as gp_exp_quad_cov_dev_vari::expand_adjoint
  void expand_adjoint() override {
    const size_t sw = ChainableStack::instance_->sweep_;
    if (exp_.C && exp_.sweep == sw) exp_.expand_into(B_->adj_);
    exp_ = inverse_adjoint{};
    if (dep_.C && dep_.sweep == sw) dep_.expand_into(B_->adj_);
    dep_ = inverse_adjoint{};
  }

  void chain() override {
    smg_ctx* c = amd::ctx();
    const int m = A_.rows, n = A_.cols, k = m < n ? m : n;
    if (!m || !n) return;
    auto* st = ChainableStack::instance_;
    if (dep_.C && dep_.sweep == st->sweep_) {
      const inverse_adjoint d = dep_;
      dep_ = inverse_adjoint{};
      if (!others_write_device_adjoint(pos_, B_, d.owner)) {
        // B's whole adjoint is the inverse form G: A' += G (passed on to A's
        // producer when it takes it -- gp_exp_quad_cov reduces it in one pass
        // and writes our d' -- else added densely), d' += sum_i G_ii
        inverse_adjoint pass = d;
        pass.owner = this;
        const bool passed = A_.vi && A_.vi->sink_ && A_.vi->sink_->take_inverse_adjoint(pass, dadj_);
        if (!passed) {
          if (A_.adj()) pass.expand_into(A_.adj());
          if (dadj_)
            amd::check(smg_gp_inverse_adjoint(c, d.C, n, n, d.s, d.k, d.ss, d.adj, nullptr, n, nullptr, 1, 1.0, 1.0,
                                              dadj_, nullptr),
                       "add_diag");
        }
        if (d_vi_) add_pending_adjoint(d_vi_, dadj_);
        exp_ = d;
        return;
      }
      d.expand_into(B_->adj_);  // another node wrote B's adjoint too: the dense sum
    }
    double* dadj = dv_.rows ? dv_.adj() : dadj_;
    if (dadj_) amd::check(smg_memset(c, dadj_, 0, sizeof(double)), "add_diag");
    const int vec = dv_.rows ? 1 : 0;
    if (m == n) {
      amd::check(smg_add_diag_rev(c, B_->adj_, m, m, A_.adj(), m, dadj, vec), "add_diag");
    } else {
      if (A_.adj())
        amd::check(smg_axpy(c, (long long)m * n, 1.0, B_->adj_, 1, A_.adj(), 1), "add_diag");
      amd::check(smg_add_diag_rev(c, B_->adj_, m, k, nullptr, 0, dadj, vec), "add_diag");
    }
    if (d_vi_) add_pending_adjoint(d_vi_, dadj_);
  }
};

/**
 * The factor's adjoint reaches this node in one of two forms:
 *  - dense (L_->adj_): Murray's blocked reverse, like the reference's chain()
 *    (rev/mat/fun/cholesky_decompose.hpp:118-166);
 *  - structured: a multi_normal_cholesky_lpdf consuming the factor deposits
 *    its partials unexpanded (take_mvn_adjoint) instead of writing the dense
 *    adj (tril(s w^T) - diag(1/L_ii)).  When no other node chained after this
 *    one wrote the factor's adjoint (may_write_device_adjoint), the reverse is
 *    the closed form Abar += adj Phi(s s^T - K^{-1}) (smg_cholesky_mvn_rev:
 *    the same 2N^3/3 in a few large GEMMs); otherwise the deposit is expanded
 *    into L_->adj_ first and Murray's reverse runs on the sum.
 */
class cholesky_dev_vari : public device_vari, public structured_adjoint_sink {
 public:
  dev_matrix_vari* A_;
  dev_matrix_vari* L_;
  int n_;
  size_t pos_;  // this node's index in var_stack_
  // the deposited multi_normal_cholesky_lpdf partials
  const vari* dep_owner_ = nullptr;
  const double* dep_ws_ = nullptr;
  double dep_adj_ = 0.0;
  int dep_k_ = 1;  // observations (the array form), [w, s] 2n doubles apart
  size_t dep_sweep_ = 0;
  double* ws_ = nullptr;  // smg_cholesky_mvn_rev's workspace [V = L^{-T}, K^{-1}]
  bool early_ = false;    // the factorisation queued all of K^{-1} into ws_ (progressively, with its panels)
  const double* winv_ = nullptr;  // W = L^{-1} alone, formed with the panels (cholesky_decompose_with_inverse)
  bool v_ready_ = false;  // V queued (smg_cholesky_inv_t_async) by prepare_mvn_adjoint
  bool c_ready_ = false;  // and K^{-1} (after early_)
  // the closed form applied these MVN partials without writing L's dense
  // adjoint (expand_adjoint writes them if L's adjoint is read)
  const double* exp_ws_ = nullptr;
  double exp_adj_ = 0.0;
  int exp_k_ = 1;
  size_t exp_sweep_ = 0;
  // the deposited partials written densely into L's adjoint (what the MVN
  // would have written: one smg_mvn_cholesky_rev per observation)
  void expand(const double* ws, double adj, int k) const {
    for (int o = 0; o < k; ++o)
      amd::check(smg_mvn_cholesky_rev(amd::ctx(), L_->val_, n_, L_->aux_, n_, ws + 2 * size_t(n_) * o, adj, 1, nullptr,
                                      nullptr, L_->adj_, n_),
                 "cholesky_decompose");
  }

  /** Which factorisations took the closed-form reverse last time, by tape
   * position and size: a sampler re-runs the same program every gradient, so
   * the next factorisation at that position forms K^{-1} alongside its panels
   * (smg_cholesky_fwd_checked_mark_inv) instead of after them. */
  static std::vector<std::pair<std::pair<size_t, int>, bool>>& history() {
    static thread_local std::vector<std::pair<std::pair<size_t, int>, bool>> h;
    return h;
  }
  // 1: took the closed form last time, 0: did not, -1: no record
  static int history_of(size_t pos, int n) {
    for (const auto& e : history())
      if (e.first.first == pos && e.first.second == n) return e.second ? 1 : 0;
    return -1;
  }
  static bool predicted(size_t pos, int n) { return history_of(pos, n) == 1; }
  void record(bool closed) const {
    auto& h = history();
    for (auto& e : h)
      if (e.first.first == pos_ && e.first.second == n_) {
        e.second = closed;
        return;
      }
    if (h.size() >= 64) h.erase(h.begin());
    h.push_back({{pos_, n_}, closed});
  }

  static bool closed_form_enabled() {
    // SMG_CHOL_MVN_CLOSED_FORM=0: always the dense adjoint + Murray (A/B, tests)
    static const bool on = [] {
      const char* e = std::getenv("SMG_CHOL_MVN_CLOSED_FORM");
      return !(e && e[0] == '0');
    }();
    return on;
  }

  cholesky_dev_vari(dev_matrix_vari* A, dev_matrix_vari* L)
      : device_vari(0.0), A_(A), L_(L), n_(A->rows_), pos_(ChainableStack::instance_->var_stack_.size() - 1) {
    L->sink_ = this;
  }

  // chain() adds into A's device adjoint only
  bool may_write_device_adjoint(const void* node) const override { return node == A_; }

  // When the factorisation did not already queue K^{-1} (no prediction yet,
  // or a size it cannot form progressively), L^{-T} is formed on the side
  // stream from the MVN's forward on, queued behind the MVN's latency-bound
  // solves so that they are not starved of CUs; unused if the reverse takes
  // the dense path
  void prepare_mvn_adjoint() override {
    if (!closed_form_enabled() || v_ready_) return;
    // (a factor whose adjoint had other writers last time -- the HVP's value
    // factor feeds the tangent nodes too -- would form V for nothing)
    if (history_of(pos_, n_) == 0) return;
    if (!ws_) ws_ = amd::alloc_doubles(smg_cholesky_mvn_rev_ws_doubles(n_));
    int started = 0;
    amd::check(smg_cholesky_inv_t_async(amd::ctx(), L_->val_, n_, L_->aux_, n_, ws_, early_ ? 1 : 0, &started),
               "multi_normal_cholesky_lpdf");
    v_ready_ = started != 0;
    c_ready_ = v_ready_ && early_;
  }

  // W = L^{-1}: the first n^2 doubles of ws_ once the progressive K^{-1}
  // (early_) has queued all of its block rows (chol_mvn.hip)
  const double* inverse_factor() override {
    if (winv_) return smg_cholesky_inverse_wait(amd::ctx()) == SMG_OK ? winv_ : nullptr;
    if (!early_ || !ws_ || n_ % 64 != 0) return nullptr;
    if (smg_cholesky_inverse_wait(amd::ctx()) != SMG_OK) return nullptr;
    return ws_;
  }

  bool take_mvn_adjoint(const vari* owner, const double* ws, double adj, int k) override {
    if (!closed_form_enabled()) return false;
    auto* st = ChainableStack::instance_;
    if (dep_owner_ && dep_sweep_ == st->sweep_ && dep_owner_ != owner) return false;  // one consumer only
    dep_owner_ = owner;
    dep_ws_ = ws;
    dep_adj_ = adj;
    dep_k_ = k;
    dep_sweep_ = st->sweep_;
    return true;
  }

  void expand_adjoint() override {
    auto* st = ChainableStack::instance_;
    if (dep_owner_ && dep_sweep_ == st->sweep_) {  // deposited, and this node was not chained
      dep_owner_ = nullptr;
      expand(dep_ws_, dep_adj_, dep_k_);
    } else if (exp_ws_ && exp_sweep_ == st->sweep_) {  // consumed by the closed form
      const double* ws = exp_ws_;
      exp_ws_ = nullptr;
      expand(ws, exp_adj_, exp_k_);
    }
  }

  void chain() override {
    smg_ctx* c = amd::ctx();
    auto* st = ChainableStack::instance_;
    const size_t nn = size_t(n_) * n_;
    const bool deposit = dep_owner_ && dep_sweep_ == st->sweep_;
    if (deposit) {
      const vari* owner = dep_owner_;
      dep_owner_ = nullptr;
      const bool dense = others_write_device_adjoint(pos_, L_, owner);  // did any other node write L's adjoint?
      record(!dense);
      if (!dense) {
        exp_ws_ = dep_ws_;
        exp_adj_ = dep_adj_;
        exp_k_ = dep_k_;
        exp_sweep_ = st->sweep_;
        // K^{-1} into ws_ + n^2, then its inverse form goes to A's producer
        // when it takes it (add_diag / gp_exp_quad_cov: one fused pass),
        // else the epilogue adds it into A's adjoint
        if (v_ready_) {
          amd::check(smg_cholesky_mvn_rev_v(c, n_, dep_ws_ + n_, dep_k_, 2LL * n_, dep_adj_, nullptr, n_, ws_,
                                            c_ready_ ? 1 : 0),
                     "cholesky_decompose");
        } else {
          if (!ws_) ws_ = amd::alloc_doubles(smg_cholesky_mvn_rev_ws_doubles(n_));
          amd::check(smg_cholesky_mvn_rev(c, L_->val_, n_, L_->aux_, n_, dep_ws_ + n_, dep_k_, 2LL * n_, dep_adj_,
                                          nullptr, n_, ws_),
                     "cholesky_decompose");
        }
        inverse_adjoint d;
        d.owner = this;
        d.C = ws_ + size_t(n_) * n_;
        d.s = dep_ws_ + n_;
        d.n = n_;
        d.k = dep_k_;
        d.ss = 2LL * n_;
        d.adj = dep_adj_;
        d.sweep = st->sweep_;
        if (!(A_->sink_ && A_->sink_->take_inverse_adjoint(d, nullptr))) d.expand_into(A_->adj_);
        return;
      }
      // expand the deposit: the MVN's own lower-only partials, added densely
      expand(dep_ws_, dep_adj_, dep_k_);
    }
    if (!deposit) record(false);
    // Murray's algorithm overwrites its input and reads only its lower triangle
    double* work = amd::alloc_doubles(nn);
    amd::check(smg_copy_tril(c, n_, n_, L_->adj_, n_, work, n_), "cholesky_decompose");
    amd::check(smg_cholesky_rev(c, L_->val_, n_, L_->aux_, work, n_, n_, A_->adj_, n_),
               "cholesky_decompose");
  }
};

inline void check_square(const char* fn, const char* name, int rows, int cols) {
  if (rows != cols) {
    std::ostringstream m;
    m << fn << ": Expecting a square matrix; rows of " << name << " (" << rows << ") and columns of "
      << name << " (" << cols << ") must match in size";
    throw std::invalid_argument(m.str());
  }
}

/** check_symmetric's message for a device matrix the device check flagged
 * (error path: one host copy of A). */
inline void throw_not_symmetric_dev(const char* fn, const char* name, const double* A, int n) {
  std::vector<double> h(size_t(n) * n);
  amd::to_host(h.data(), A, h.size());
  amd::throw_not_symmetric_host(fn, name, h.data(), n);
}


inline dev_var_matrix add_diag_dev(const dev_operand& A, double d, vari* d_vi, const dev_operand& dv) {
  if (dv.rows || dv.cols) {  // check_consistent_size(fn, "number of elements of to_add", to_add, min(rows, cols))
    const size_t k = size_t(A.rows < A.cols ? A.rows : A.cols);
    if (dv.size() != k) {
      std::ostringstream m;
      m << "add_diag: number of elements of to_add has dimension = " << dv.size() << ", expecting dimension = " << k
        << "; a function was called with arguments of different scalar, array, vector, or matrix types, and they "
           "were not consistently sized;  all arguments must be scalars or multidimensional values of the same shape.";
      throw std::invalid_argument(m.str());
    }
  }
  auto* node = new add_diag_dev_vari(A, d, d_vi, dv);
  return dev_var_matrix(node->B_);
}

}  // namespace internal

/** add_diag(mat, to_add) (prim/mat/fun/add_diag.hpp:20-55) on device operands:
 * a scalar or a vector to_add, any var / data combination, rectangular mat. */
inline dev_var_matrix add_diag(const dev_var_matrix& A, const var& d) {
  return internal::add_diag_dev(internal::operand(A), d.val(), d.vi_, {});
}
inline dev_var_matrix add_diag(const dev_var_matrix& A, double d) {
  return internal::add_diag_dev(internal::operand(A), d, nullptr, {});
}
inline dev_var_matrix add_diag(const dev_data<double>& A, const var& d) {
  return internal::add_diag_dev(internal::operand(A), d.val(), d.vi_, {});
}
inline dev_var_matrix add_diag(const dev_var_matrix& A, const dev_var_matrix& d) {
  return internal::add_diag_dev(internal::operand(A), 0.0, nullptr, internal::operand(d));
}
inline dev_var_matrix add_diag(const dev_var_matrix& A, const dev_data<double>& d) {
  return internal::add_diag_dev(internal::operand(A), 0.0, nullptr, internal::operand(d));
}
inline dev_var_matrix add_diag(const dev_data<double>& A, const dev_var_matrix& d) {
  return internal::add_diag_dev(internal::operand(A), 0.0, nullptr, internal::operand(d));
}

namespace internal {
/**
 * cholesky_decompose on a device operand; with host_out (an n x n Eigen
 * matrix of vars, column-major) also the Eigen boundary's output: the
 * factor's host varis -- its lower triangle's, the strict upper on one dummy
 * (cholesky_decompose.hpp:34-48, as internal::materialise) -- are built
 * panel by panel as the factorisation streams each finished panel's columns
 * to the host (smg_cholesky_fwd_checked_mark_stream), instead of after it.
 * Varis built before a failed check are left unreferenced in the arena, as a
 * throwing reference functor leaves its partial allocations.
 */
inline dev_var_matrix cholesky_decompose_impl(const dev_var_matrix& A, var* host_out,
                                              const std::function<bool()>* verify = nullptr, bool want_w = false) {
  const char* fn = "cholesky_decompose";
  internal::check_square(fn, "A", A.rows(), A.cols());
  const int n = A.rows();
  smg_ctx* c = amd::ctx();
  // verify: A is speculative (its host matrix still to be checked); an empty
  // result if the check fails.  It runs once the factorisation is queued when
  // the factor streams to the host, before anything is queued otherwise.
  if (verify && !(host_out && n > 0 && smg_cholesky_stream_panels(n) <= 64)) {
    if (!(*verify)()) return dev_var_matrix();
    verify = nullptr;
  }
  if (n == 0) return dev_var_matrix(new dev_matrix_vari(0, 0, dev_structure::lower));
  auto* L = new dev_matrix_vari(n, n, dev_structure::lower);
  L->aux_ = amd::alloc_doubles(size_t(smg_cholesky_aux_doubles(n)));
  // the node's tape position once pushed (cholesky_dev_vari::pos_)
  const size_t pos = ChainableStack::instance_->var_stack_.size();
  double* inv_ws = nullptr;
  // want_w: W = L^{-1} alone, progressively (the HVP's value factor, whose
  // tangent node reads W); n % 512 == 0 and n >= 1024, else not formed
  want_w = want_w && !host_out && n % 512 == 0 && n >= 1024;
  if (want_w || (internal::cholesky_dev_vari::closed_form_enabled() && internal::cholesky_dev_vari::predicted(pos, n)))
    inv_ws = amd::alloc_doubles(smg_cholesky_mvn_rev_ws_doubles(n));
  // check_symmetric fused with the factorisation's copy of A (one pass); the
  // status is read at the mark after the panels, so the block inverses that
  // follow run while the host builds the next node
  int inv_started = 0;
  const int panels = smg_cholesky_stream_panels(n);
  host_block b{};
  if (host_out && panels <= 64) {
    b.node = L;
    b.rows = b.cols = n;
    b.dirty = false;
    b.layout = layout_lower;
    b.n = tril_count(size_t(n));
    b.first = static_cast<vari*>(ChainableStack::instance_->memalloc_.alloc(b.n * sizeof(vari)));
    b.dummy = new vari(0.0, vari::unstacked_tag{});
    double* packed = amd::alloc_doubles(b.n);
    double* stage = static_cast<double*>(smg_host_scratch(c, b.n * sizeof(double)));
    if (!stage) throw std::bad_alloc();
    amd::phase_mark(20);
    amd::check(smg_cholesky_fwd_checked_mark_stream(c, A.val_ptr(), n, n, L->val_, n, L->aux_, inv_ws, &inv_started,
                                                    packed, stage, 0),
               fn);
    amd::phase_mark(0);
    if (verify && !(*verify)()) {  // (rejected: the queued work drains, its results are dropped)
      amd::check(smg_sync_all(c), fn);
      int st = 0;
      amd::check(smg_status_mark_wait(c, &st), fn);
      return dev_var_matrix();
    }
    amd::phase_mark(21);
    fill_block_pointers(b, host_out);  // addresses only: while the first panel factors
    amd::phase_mark(1);
    for (int p = 0; p < panels; ++p) {
      int j0 = 0, j1 = 0;  // (the library's own panel bounds: what marker p covers)
      amd::check(smg_cholesky_stream_panel_cols(n, p, &j0, &j1), fn);
      const size_t o0 = tril_off(size_t(n), size_t(j0)), o1 = tril_off(size_t(n), size_t(j1));
      amd::check(smg_marker_wait(c, p), fn);
      amd::phase_mark(2 + 2 * p);
      host_parallel_for(o1 - o0, [&](size_t s0, size_t s1) { construct_varis(b.first, stage, o0 + s0, o0 + s1); });
      amd::phase_mark(3 + 2 * p);
    }
  } else if (want_w) {
    amd::check(smg_cholesky_fwd_checked_mark_winv(c, A.val_ptr(), n, n, L->val_, n, L->aux_, inv_ws, &inv_started),
               fn);
  } else if (inv_ws) {
    amd::check(smg_cholesky_fwd_checked_mark_inv(c, A.val_ptr(), n, n, L->val_, n, L->aux_, inv_ws, &inv_started), fn);
  } else {
    amd::check(smg_cholesky_fwd_checked_mark(c, A.val_ptr(), n, n, L->val_, n, L->aux_), fn);
  }
  int st = 0;
  amd::check(smg_status_mark_wait(c, &st), fn);
  amd::phase_mark(30);
  if (st & SMG_ERR_NOT_SYMMETRIC) internal::throw_not_symmetric_dev(fn, "A", A.val_ptr(), n);
  if (st) amd::throw_status(st, fn, "m");
  auto* node = new internal::cholesky_dev_vari(A.vi_, L);
  if (want_w) {  // W alone (inv_started == 3); the closed form, if taken, gets a workspace of its own
    if (inv_started == 3) node->winv_ = inv_ws;
  } else {
    node->ws_ = inv_ws;  // (reused by prepare_mvn_adjoint when the factorisation could not form K^{-1})
  }
  if (inv_started && !want_w) {
    node->early_ = true;
    node->v_ready_ = node->c_ready_ = true;  // all of K^{-1} queued already
  }
  if (b.node) {
    push_block(b);
  } else if (host_out) {  // (more than 64 panels: materialised after the factorisation)
    materialise(L, [&](const host_block& hb) { fill_block_pointers(hb, host_out); });
  }
  return dev_var_matrix(L);
}
}  // namespace internal

inline dev_var_matrix cholesky_decompose(const dev_var_matrix& A) {
  return internal::cholesky_decompose_impl(A, nullptr);
}

namespace internal {
/** cholesky_decompose that also forms W = L^{-1} beside its panels, read
 * through the factor's sink (inverse_factor()) by the Cholesky tangent node
 * and the MVN's W-form forward. */
inline dev_var_matrix cholesky_decompose_with_inverse(const dev_var_matrix& A) {
  return cholesky_decompose_impl(A, nullptr, nullptr, true);
}
}  // namespace internal

}  // namespace math
}  // namespace stan
#endif
