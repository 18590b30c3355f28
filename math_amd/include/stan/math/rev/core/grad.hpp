#ifndef STAN_MATH_REV_CORE_GRAD_HPP
#define STAN_MATH_REV_CORE_GRAD_HPP

// Reverse sweep and tape management.
//   grad                     rev/core/grad.hpp:30-46
//   start_nested             rev/core/start_nested.hpp:13
//   recover_memory(_nested)  rev/core/recover_memory.hpp:18-31,
//                            rev/core/recover_memory_nested.hpp:20-45
//   set_zero_all_adjoints(_nested)  rev/core/set_zero_all_adjoints*.hpp
//   empty_nested / nested_size
// Device extension: the same calls mark / rewind the device arena, zero the
// device adjoint buffers, and land pending device->host adjoint
// contributions (flush_pending) before any host chain() that could read them.

#include <stan/math/amd/device.hpp>
#include <stan/math/rev/core/vari.hpp>

#include <algorithm>
#include <cstdint>
#include <typeinfo>
#include <stdexcept>
#include <vector>

namespace stan {
namespace math {

/** Register a device adjoint buffer with the tape (zeroed now and by
 * set_zero_all_adjoints).  A large buffer is zeroed on the context's zeroing
 * stream, overlapping the rest of the forward pass; only a reverse sweep (or
 * a host read of the adjoint) touches it, and both join that stream first
 * (join_device_adjoints). */
inline void register_device_adjoint(double* p, size_t n) {
  if (n >= (size_t(1) << 17))
    amd::check(smg_memset_async(amd::ctx(), p, n * sizeof(double)), "zero");
  else
    amd::zero(p, n);
  ChainableStack::instance_->dev_adj_stack_.push_back({p, n});
}

/** The main stream waits for every adjoint zeroing still in flight. */
inline void join_device_adjoints() {
  if (amd::has_ctx()) amd::check(smg_join_async(amd::ctx()), "grad");
}

/** Queue target->adj_ += *src (src: device scalar) for the next flush. */
inline void add_pending_adjoint(vari* target, const double* src) {
  ChainableStack::instance_->pending_.push_back({target, src});
}

/** Land every queued device->host adjoint contribution (one sync).  With
 * `status` (the end of the reverse sweep), the device status word is read in
 * the same sync when a launch that can latch it asynchronously was enqueued
 * (a persistent solve / panel whose hand-off timed out: SMG_ERR_SYNC), so
 * such a failure throws from the grad() that ran it. */
inline void flush_pending(bool status = false) {
  auto& pend = ChainableStack::instance_->pending_;
  int armed = 0;
  if (status && amd::has_ctx()) amd::check(smg_status_armed(amd::ctx(), &armed), "grad");
  if (pend.empty() && !armed) return;
  smg_ctx* c = amd::ctx();
  const size_t n = pend.size();
  // one gather kernel into fine-grained pinned memory and one host wait
  // (smg_gather_scalars), not a copy per scalar and a stream sync
  double* stage = static_cast<double*>(smg_pinned_result(c, (n + 1) * sizeof(double)));
  if (!stage) throw std::bad_alloc();
  std::vector<const double*> src(n);
  for (size_t i = 0; i < n; ++i) src[i] = pend[i].src;
  int* st = reinterpret_cast<int*>(stage + n);
  amd::check(smg_gather_scalars(c, src.data(), int(n), stage, armed ? st : nullptr), "flush_pending");
  auto& blocks = ChainableStack::instance_->host_blocks_;
  for (size_t i = 0; i < n; ++i) {
    vari* t = pend[i].target;
    t->adj_ += stage[i];
    for (auto& b : blocks)  // a host block's bridge must then gather (bridge.hpp)
      if (t >= b.first && t < b.first + b.n) b.dirty = true;
  }
  pend.clear();
  if (armed) amd::throw_if_sync(*st, "grad", "the reverse sweep");
}

/** Record which host blocks' varis node v (just chained) may have added into
 * (vari::touches_adjoints_in), stamping them with the sweep: a block's bridge
 * (amd/matrix.hpp dev_to_host_vari) then knows without rescanning the rest of
 * the tape whether any node after it touched its varis.  The blocks, ordered
 * by address, are bisected: O(log B) range queries for a node touching one
 * block, one query for a node touching none. */
inline void log_host_touches(vari* v) {
  auto* st = ChainableStack::instance_;
  auto& blocks = st->host_blocks_;
  if (typeid(*v) == typeid(vari)) return;  // (a leaf: its chain() is empty)
  auto& order = st->block_order_;
  if (st->block_order_sweep_ != st->sweep_) {
    order.clear();
    for (size_t k = 0; k < blocks.size(); ++k)
      if (blocks[k].n) order.push_back(k);
    std::sort(order.begin(), order.end(), [&](size_t a, size_t b) { return blocks[a].first < blocks[b].first; });
    st->block_order_sweep_ = st->sweep_;
  }
  struct bisect {
    static void run(vari* v, std::vector<host_block>& blocks, const std::vector<size_t>& order, size_t a, size_t b,
                    size_t sweep) {
      const vari* lo = blocks[order[a]].first;
      const host_block& last = blocks[order[b - 1]];
      if (!v->touches_adjoints_in(lo, last.first + last.n)) return;
      if (b - a == 1) {
        blocks[order[a]].touched_sweep = sweep;
        return;
      }
      const size_t m = a + (b - a) / 2;
      run(v, blocks, order, a, m, sweep);
      run(v, blocks, order, m, b, sweep);
    }
  };
  if (!order.empty()) bisect::run(v, blocks, order, 0, order.size(), st->sweep_);
}

static inline bool empty_nested() {
  return ChainableStack::instance_->nested_var_stack_sizes_.empty();
}

static inline size_t nested_size() {
  return ChainableStack::instance_->var_stack_.size()
         - ChainableStack::instance_->nested_var_stack_sizes_.back();
}

/**
 * Reverse sweep from vi: adj(vi) = 1, then chain() over var_stack_ in reverse
 * (only the innermost nested window when nested).  Device nodes enqueue their
 * adjoint kernels on the thread's stream; host nodes run inline.
 */
static void grad(vari* vi) {
  using it_t = std::vector<vari*>::reverse_iterator;
  auto* st = ChainableStack::instance_;
  join_device_adjoints();
  ++st->sweep_;
  vi->init_dependent();
  for (auto& b : st->host_blocks_)  // the root itself may be an element of a host block
    if (vi >= b.first && vi < b.first + b.n) b.dirty = true;
  it_t begin = st->var_stack_.rbegin();
  it_t end = empty_nested() ? st->var_stack_.rend() : begin + nested_size();
  for (it_t it = begin; it < end; ++it) {
    // a device->host contribution must land before its target's chain() reads
    // its adj_; nodes that are not a target run without a synchronisation
    // (device nodes keep streaming)
    if (__builtin_expect(!st->pending_.empty(), 0)) {
      // (a plain vari -- a leaf such as var(double)'s -- has an empty chain())
      bool need = (*it)->reads_other_adjoints() && typeid(**it) != typeid(vari);
      for (size_t i = 0; !need && i < st->pending_.size(); ++i) need = st->pending_[i].target == *it;
      if (need) flush_pending();
    }
    (*it)->chain();
    if (!st->host_blocks_.empty()) log_host_touches(*it);
  }
  flush_pending(true);
  if (st->publish_ && st->no_publish_ == 0) st->publish_(empty_nested() ? 0 : st->nested_host_block_sizes_.back());
}

/** While alive, sweeps leave the host blocks' varis unpublished (their
 * device adjoints stay on the device): for callers that read only their
 * independent variables' adjoints and then recover the tape. */
struct no_publish_scope {
  no_publish_scope() { ++ChainableStack::instance_->no_publish_; }
  ~no_publish_scope() { --ChainableStack::instance_->no_publish_; }
  no_publish_scope(const no_publish_scope&) = delete;
  no_publish_scope& operator=(const no_publish_scope&) = delete;
};

static inline void start_nested() {
  auto* st = ChainableStack::instance_;
  st->nested_var_stack_sizes_.push_back(st->var_stack_.size());
  st->nested_var_nochain_stack_sizes_.push_back(st->var_nochain_stack_.size());
  st->nested_var_alloc_stack_starts_.push_back(st->var_alloc_stack_.size());
  st->nested_dev_adj_sizes_.push_back(st->dev_adj_stack_.size());
  st->nested_dev_marks_.push_back(amd::has_ctx() ? smg_arena_mark(amd::ctx()) : SIZE_MAX);
  st->nested_host_block_sizes_.push_back(st->host_blocks_.size());
  st->memalloc_.start_nested();
}

static inline void recover_memory_nested() {
  if (empty_nested())
    throw std::logic_error("empty_nested() must be false before calling recover_memory_nested()");
  auto* st = ChainableStack::instance_;
  st->var_stack_.resize(st->nested_var_stack_sizes_.back());
  while (!st->dev_writers_.empty() && st->dev_writers_.back().pos >= st->var_stack_.size()) st->dev_writers_.pop_back();
  st->nested_var_stack_sizes_.pop_back();
  st->var_nochain_stack_.resize(st->nested_var_nochain_stack_sizes_.back());
  st->nested_var_nochain_stack_sizes_.pop_back();
  for (size_t i = st->nested_var_alloc_stack_starts_.back(); i < st->var_alloc_stack_.size(); ++i)
    delete st->var_alloc_stack_[i];
  st->var_alloc_stack_.resize(st->nested_var_alloc_stack_starts_.back());
  st->nested_var_alloc_stack_starts_.pop_back();
  st->dev_adj_stack_.resize(st->nested_dev_adj_sizes_.back());
  st->nested_dev_adj_sizes_.pop_back();
  const size_t mark = st->nested_dev_marks_.back();
  st->nested_dev_marks_.pop_back();
  st->pending_.clear();
  st->host_blocks_.resize(st->nested_host_block_sizes_.back());
  st->nested_host_block_sizes_.pop_back();
  if (amd::has_ctx()) {
    if (mark == SIZE_MAX)
      smg_arena_recover_all(amd::ctx());
    else
      smg_arena_rewind(amd::ctx(), mark);
  }
  st->memalloc_.recover_nested();
}

static inline void recover_memory() {
  if (!empty_nested())
    throw std::logic_error("empty_nested() must be true before calling recover_memory()");
  auto* st = ChainableStack::instance_;
  st->var_stack_.clear();
  st->dev_writers_.clear();
  st->var_nochain_stack_.clear();
  for (auto* a : st->var_alloc_stack_) delete a;
  st->var_alloc_stack_.clear();
  st->dev_adj_stack_.clear();
  st->pending_.clear();
  st->host_blocks_.clear();
  if (amd::has_ctx()) smg_arena_recover_all(amd::ctx());
  st->memalloc_.recover_all();
}

/** Zero the adjoints of the host blocks from index `from` on (their varis
 * are on no stack; stan/math/amd/matrix.hpp materialise). */
static inline void zero_host_blocks(size_t from) {
  auto& blocks = ChainableStack::instance_->host_blocks_;
  for (size_t k = from; k < blocks.size(); ++k) {
    host_block& b = blocks[k];
    for (size_t i = 0; i < b.n; ++i) b.first[i].adj_ = 0.0;
    if (b.dummy) b.dummy->adj_ = 0.0;
    b.dummy_dev = 0.0;
    b.dirty = false;
  }
}

static inline void set_zero_all_adjoints() {
  auto* st = ChainableStack::instance_;
  ++st->sweep_;  // (a structured adjoint of the last sweep is gone with the dense ones)
  for (auto* v : st->var_stack_) v->set_zero_adjoint();
  for (auto* v : st->var_nochain_stack_) v->set_zero_adjoint();
  for (auto& b : st->dev_adj_stack_) amd::zero(b.ptr, b.n);
  zero_host_blocks(0);
  st->pending_.clear();
}

static inline void set_zero_all_adjoints_nested() {
  if (empty_nested())
    throw std::logic_error(
        "empty_nested() must be false before calling set_zero_all_adjoints_nested()");
  auto* st = ChainableStack::instance_;
  ++st->sweep_;
  const size_t s1 = st->nested_var_stack_sizes_.back();
  for (size_t i = (s1 == 0U) ? 0U : (s1 - 1); i < st->var_stack_.size(); ++i)
    st->var_stack_[i]->set_zero_adjoint();
  const size_t s2 = st->nested_var_nochain_stack_sizes_.back();
  for (size_t i = (s2 == 0U) ? 0U : (s2 - 1); i < st->var_nochain_stack_.size(); ++i)
    st->var_nochain_stack_[i]->set_zero_adjoint();
  for (size_t i = st->nested_dev_adj_sizes_.back(); i < st->dev_adj_stack_.size(); ++i)
    amd::zero(st->dev_adj_stack_[i].ptr, st->dev_adj_stack_[i].n);
  zero_host_blocks(st->nested_host_block_sizes_.back());
  st->pending_.clear();
}

/** Free every arena block but the first (reference: recover_memory + free_all). */
static inline void free_memory() { ChainableStack::instance_->memalloc_.free_all(); }

}  // namespace math
}  // namespace stan
#endif
