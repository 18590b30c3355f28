#ifndef STAN_MATH_AMD_MATRIX_HPP
#define STAN_MATH_AMD_MATRIX_HPP

// Device-resident matrices of vars (struct-of-arrays).
//
// The reference represents an N x N matrix of vars as N^2 host varis
// (AoS, one `vari*` per element) and every matrix functor gathers/scatters
// through those pointers (e.g. rev/mat/fun/cholesky_decompose.hpp:74-92,
// 159-164).  Here a matrix node is ONE arena object holding a device column
// of values and a device column of adjoints; functor nodes (vari subclasses
// on var_stack_) read and write those columns with HIP kernels.  Host varis
// are materialised only at an Eigen boundary (stan/math/eigen/interop.hpp).
//
//   dev_matrix_vari  the node (arena object, never chained itself)
//   dev_var_matrix   the handle user code holds (like var for vari)
//   dev_data         a device copy of constant data (double or int)

#include <stan/math/amd/device.hpp>
#include <stan/math/amd/host_parallel.hpp>
#include <stan/math/rev/core/grad.hpp>
#include <stan/math/rev/core/var.hpp>
#include <stan/math/rev/core/vari.hpp>

#include <algorithm>
#include <cmath>
#include <functional>
#include <new>
#include <sstream>
#include <stdexcept>
#include <vector>

namespace stan {
namespace math {

/** Structural information carried by a matrix node. */
enum class dev_structure : int {
  general = 0,
  lower = 1,     // strict upper triangle is constant zero (cholesky_decompose output)
  symmetric = 2  // values symmetric, and the reference's matrix holds one vari per
                 // (i, j), (j, i) pair (gp_exp_quad_cov output)
};

/** A matrix adjoint in inverse form, G = adj Phi(sum_o s_o s_o^T - k C)
 * (Phi: strict lower + half the diagonal, the reference's lower-entry
 * convention; C = K^{-1} lower, ld n; s_o = s + o ss on the device): the
 * closed-form reverse of cholesky_decompose under multi_normal_cholesky_lpdf
 * (rev/fun/cholesky_decompose.hpp), handed to the producer of the factored
 * matrix unexpanded. */
struct inverse_adjoint {
  const vari* owner = nullptr;  // the depositing node
  const double* C = nullptr;
  const double* s = nullptr;
  int n = 0, k = 1;
  long long ss = 0;
  double adj = 0.0;
  size_t sweep = 0;  // ChainableStack::sweep_ of the deposit
  /** the dense form added into the lower triangle of Aadj (ld n) */
  void expand_into(double* Aadj) const {
    amd::check(smg_cholesky_inverse_adjoint(amd::ctx(), C, n, n, s, k, ss, adj, Aadj, n), "cholesky_decompose");
  }
};

/** True when a node chained after tape position `pos`, other than `except`,
 * may have written the device adjoint of matrix node `node`
 * (vari::may_write_device_adjoint). */
inline bool others_write_device_adjoint(size_t pos, const void* node, const vari* except) {
  // only the nodes that can write device adjoints at all (the tape's
  // dev_writers_, registered at construction), from the first one after pos
  const auto& w = ChainableStack::instance_->dev_writers_;
  auto it = std::upper_bound(w.begin(), w.end(), pos, [](size_t p, const dev_writer& d) { return p < d.pos; });
  for (; it != w.end(); ++it)
    if (it->v != except && it->v->may_write_device_adjoint(node)) return true;
  return false;
}

/** A node that can take a consumer's adjoint contribution in structured
 * (unexpanded) form instead of as a dense device adjoint: cholesky_decompose
 * takes multi_normal_cholesky_lpdf's partials for its factor and applies
 * them in closed form (rev/fun/cholesky_decompose.hpp); add_diag and
 * gp_exp_quad_cov take that closed form's inverse form (inverse_adjoint) for
 * their outputs and reduce it in one pass (rev/fun/gp_exp_quad_cov.hpp). */
class structured_adjoint_sink {
 public:
  /** An inverse-form adjoint for the node's output (valid for the current
   * sweep); dadj (device scalar, may be null): where a depositing add_diag
   * wants its diagonal sum written.  True when taken. */
  virtual bool take_inverse_adjoint(const inverse_adjoint& d, double* dadj) {
    (void)d;
    (void)dadj;
    return false;
  }
  /** owner: the consumer node; ws: its device [w, s] (smg_mvn_cholesky_fwd),
   * k of them 2n doubles apart (the array form's observations); adj: its
   * adjoint.  True when taken (the consumer then writes no dense adjoint for
   * the factor); false: the consumer writes it densely. */
  virtual bool take_mvn_adjoint(const vari* owner, const double* ws, double adj, int k = 1) {
    (void)owner;
    (void)ws;
    (void)adj;
    (void)k;
    return false;
  }
  /** Called by such a consumer's forward pass before its own device work:
   * the node may start, on a side stream, what that reverse will need. */
  virtual void prepare_mvn_adjoint() {}
  /** Before the node's own device adjoint is read (dev_var_matrix::adj()):
   * write the structured contribution of the last sweep into it densely, so
   * that it holds what the reference's varis would (the closed form never
   * formed it). */
  virtual void expand_adjoint() {}
  /** The factor's explicit inverse W = L^{-1} (device, n x n, ld n, lower;
   * stored zeros above the diagonal inside its diagonal 64 x 64 tiles) when
   * the factorisation formed it anyway, with the context's stream already
   * ordered after its completion; null otherwise.  The consumer's forward
   * then takes the reference's products with inv_L instead of two solves. */
  virtual const double* inverse_factor() { return nullptr; }
};

class dev_matrix_vari {
 public:
  const int rows_;
  const int cols_;
  double* val_;  // device, column-major, ld = rows_
  double* adj_;  // device, column-major, registered with the tape
  dev_structure structure_;
  double* aux_;  // node-specific device side data (e.g. Cholesky diagonal-block inverses)
  // set on transpose(A)'s output: multiply(A, transpose(A)) recognises the
  // Gram product (one lower GEMM forward, one GEMM reverse)
  dev_matrix_vari* transpose_of_ = nullptr;
  // the producing node when it accepts structured adjoints (a Cholesky factor)
  structured_adjoint_sink* sink_ = nullptr;

  dev_matrix_vari(int rows, int cols, dev_structure s = dev_structure::general)
      : rows_(rows),
        cols_(cols),
        val_(amd::alloc_doubles(size_t(rows) * cols)),
        adj_(amd::alloc_doubles(size_t(rows) * cols)),
        structure_(s),
        aux_(nullptr) {
    register_device_adjoint(adj_, size_t(rows) * cols);
  }

  size_t size() const { return size_t(rows_) * cols_; }

  static inline void* operator new(size_t nbytes) {
    return ChainableStack::instance_->memalloc_.alloc(nbytes);
  }
  static inline void operator delete(void*) {}
};

class dev_var_matrix {
 public:
  dev_matrix_vari* vi_;

  dev_var_matrix() : vi_(nullptr) {}
  explicit dev_var_matrix(dev_matrix_vari* vi) : vi_(vi) {}

  int rows() const { return vi_->rows_; }
  int cols() const { return vi_->cols_; }
  size_t size() const { return vi_->size(); }
  const double* val_ptr() const { return vi_->val_; }
  double* adj_ptr() const { return vi_->adj_; }

  /** Column-major host copy of the values (synchronising). */
  std::vector<double> val() const {
    std::vector<double> h(size());
    amd::to_host(h.data(), vi_->val_, size());
    return h;
  }
  /** Column-major host copy of the adjoints (synchronising). */
  std::vector<double> adj() const {
    if (vi_->sink_) vi_->sink_->expand_adjoint();
    join_device_adjoints();
    std::vector<double> h(size());
    amd::to_host(h.data(), vi_->adj_, size());
    return h;
  }

#ifdef STAN_MATH_AMD_HAS_EIGEN
  // materialise as N^2 host varis (stan/math/eigen/interop.hpp)
  operator Eigen::Matrix<var, Eigen::Dynamic, Eigen::Dynamic>() const;
  operator Eigen::Matrix<var, Eigen::Dynamic, 1>() const;
#endif
};

/** Device copy of constant data (arena-owned, recovered with the tape). */
template <typename T>
class dev_data {
 public:
  const T* ptr_ = nullptr;
  size_t n_ = 0;
  int rows_ = 0, cols_ = 0;
  dev_data() = default;
  dev_data(const T* p, size_t n, int rows, int cols) : ptr_(p), n_(n), rows_(rows), cols_(cols) {}
  size_t size() const { return n_; }
  int rows() const { return rows_; }
  int cols() const { return cols_; }
  const T* data() const { return ptr_; }
};

inline dev_data<double> to_dev_data(const double* h, size_t n, int rows = -1, int cols = 1) {
  double* d = amd::alloc_doubles(n);
  amd::to_device(d, h, n);
  return dev_data<double>(d, n, rows < 0 ? int(n) : rows, cols);
}
inline dev_data<double> to_dev_data(const std::vector<double>& v) {
  return to_dev_data(v.data(), v.size());
}
inline dev_data<int> to_dev_data(const std::vector<int>& v) {
  int* d = amd::alloc_ints(v.size());
  amd::to_device_int(d, v.data(), v.size());
  return dev_data<int>(d, v.size(), int(v.size()), 1);
}

namespace internal {
/** One operand of a matrix functor: a device var node or constant device data. */
struct dev_operand {
  dev_matrix_vari* vi = nullptr;  // null for data
  const double* data = nullptr;
  int rows = 0, cols = 0;
  const double* val() const { return vi ? vi->val_ : data; }
  double* adj() const { return vi ? vi->adj_ : nullptr; }
  size_t size() const { return size_t(rows) * size_t(cols); }
};
inline dev_operand operand(const dev_var_matrix& m) { return dev_operand{m.vi_, nullptr, m.rows(), m.cols()}; }
inline dev_operand operand(const dev_data<double>& d) { return dev_operand{nullptr, d.data(), d.rows(), d.cols()}; }
}  // namespace internal

/** A fresh device matrix of vars initialised from host values (a leaf:
 * its adjoint is read back by the caller, like x_var in gradient()). */
inline dev_var_matrix to_dev_var_matrix(const double* host_colmajor, int rows, int cols) {
  auto* vi = new dev_matrix_vari(rows, cols);
  amd::to_device(vi->val_, host_colmajor, size_t(rows) * cols);
  return dev_var_matrix(vi);
}

namespace internal {

enum block_layout : int { layout_dense = 0, layout_lower = 1, layout_sym = 2, layout_diag = 3 };

/** packed lower triangle, column-major: column j's rows j..n-1 start at
 * j n - j (j - 1) / 2 (smg_pack_tril) */
inline size_t tril_off(size_t n, size_t j) { return j * n - j * (j - 1) / 2; }
inline size_t tril_count(size_t n) { return n * (n + 1) / 2; }

inline void block_column_ptrs(const std::vector<host_block>& blocks, const host_block& b, size_t j, vari** out);

/** f(i, v) for every row i of column j of a dense, lower or symmetric block
 * (no base block), in order.  The symmetric layout's rows above the diagonal
 * step through the packed columns incrementally: element (i, j), i < j, is
 * packed column i's entry j - i at tril_off(r, i) + j - i, and
 * tril_off(r, i + 1) - tril_off(r, i) = r - i. */
template <typename F>
inline void block_column_own(const host_block& b, size_t j, F&& f) {
  const size_t r = size_t(b.rows);
  switch (b.layout) {
    case layout_lower: {
      for (size_t i = 0; i < j && i < r; ++i) f(i, b.dummy);
      vari* c = b.first + tril_off(r, j) - j;
      for (size_t i = j; i < r; ++i) f(i, c + i);
      break;
    }
    case layout_sym: {
      vari* p = b.first + j;  // (i = 0: tril_off(r, 0) + j)
      for (size_t i = 0; i < j && i < r; ++i) {
        f(i, p);
        p += r - i - 1;
      }
      vari* c = b.first + tril_off(r, j) - j;
      for (size_t i = j; i < r; ++i) f(i, c + i);
      break;
    }
    default: {
      vari* c = b.first + j * r;
      for (size_t i = 0; i < r; ++i) f(i, c + i);
    }
  }
}

/** f(i, v) for every row i of column j of host block b, in order: v is the
 * vari the reference's matrix holds at (i, j) (host_block's layouts).
 * blocks: the tape's host_blocks_ (passed in: the host pool's workers have
 * no tape of their own). */
template <typename F>
inline void block_column(const std::vector<host_block>& blocks, const host_block& b, size_t j, F&& f) {
  if (b.layout != layout_diag) return block_column_own(b, j, f);
  const size_t r = size_t(b.rows);
  vari* own = j < b.n ? b.first + j : nullptr;
  if (b.base >= 0) {
    const host_block& base = blocks[size_t(b.base)];
    if (base.layout != layout_diag) {  // (the common case: add_diag of a materialised node)
      block_column_own(base, j, [&](size_t i, vari* v) { f(i, i == j && own ? own : v); });
      return;
    }
    // (the base's column through a buffer: no recursive instantiation)
    thread_local std::vector<vari*> col;
    col.resize(r);
    block_column_ptrs(blocks, base, j, col.data());
    for (size_t i = 0; i < r; ++i) f(i, i == j && own ? own : col[i]);
  } else {
    vari* const* e = b.base_elems + j * r;
    for (size_t i = 0; i < r; ++i) f(i, i == j && own ? own : e[i]);
  }
}

inline void block_column_ptrs(const std::vector<host_block>& blocks, const host_block& b, size_t j, vari** out) {
  block_column(blocks, b, j, [out](size_t i, vari* v) { out[i] = v; });
}

/** smg_pack_tril's mode for a layout's owned varis (-1: dense, no packing) */
inline int block_pack_mode(int layout) {
  return layout == layout_lower ? 0 : layout == layout_sym ? 1 : layout == layout_diag ? 2 : -1;
}

/** column grain for the host pool: about 2^18 elements per task */
inline size_t col_grain(int rows) { return std::max<size_t>(1, (size_t(1) << 18) / size_t(rows > 0 ? rows : 1)); }

/** Index in host_blocks_ of the block whose elements are exactly d[0..n)
 * (column-major rows x cols) by the block's layout, or -1.  The full pointer
 * check runs on every call (a caller may have replaced single elements); it
 * is one parallel read of n pointers. */
/** The host block d[0..n) may be (its first vari and shape; O(1)), or -1. */
inline long candidate_block_index(const var* d, size_t n, int rows, int cols) {
  if (n == 0) return -1;
  auto& blocks = ChainableStack::instance_->host_blocks_;
  const vari* v0 = d[0].vi_;
  for (size_t k = blocks.size(); k-- > 0;) {
    const host_block& b = blocks[k];
    if (b.first != v0) continue;
    if (b.rows != rows || b.cols != cols || size_t(rows) * size_t(cols) != n) return -1;
    return long(k);
  }
  return -1;
}
/** Whether d (column-major, block k's shape) holds exactly block k's varis:
 * one parallel read of its pointers. */
inline bool block_matches(const var* d, size_t k) {
  auto& blocks = ChainableStack::instance_->host_blocks_;
  const host_block& b = blocks[k];
  const size_t r = size_t(b.rows);
  return host_parallel_all(
      size_t(b.cols),
      [&](size_t j0, size_t j1) {
        bool good = true;
        for (size_t j = j0; good && j < j1; ++j) {
          const var* col = d + j * r;
          block_column(blocks, b, j, [&](size_t i, vari* v) { good &= col[i].vi_ == v; });
        }
        return good;
      },
      col_grain(b.rows));
}
inline long recognise_block_index(const var* d, size_t n, int rows, int cols) {
  const long k = candidate_block_index(d, n, rows, cols);
  return k >= 0 && block_matches(d, size_t(k)) ? k : -1;
}
inline dev_matrix_vari* recognise_block(const var* d, size_t n, int rows, int cols) {
  const long k = recognise_block_index(d, n, rows, cols);
  return k < 0 ? nullptr : static_cast<dev_matrix_vari*>(ChainableStack::instance_->host_blocks_[size_t(k)].node);
}

/** varis first[i] = vari(val[i]) (unstacked) for i in [b, e) */
inline void construct_varis(vari* first, const double* val, size_t b, size_t e) {
  for (size_t i = b; i < e; ++i) ::new (static_cast<void*>(first + i)) vari(val[i], vari::unstacked_tag{});
}

/** Write block b's element varis into d (column-major rows x cols). */
inline void fill_block_pointers(const host_block& b, var* d) {
  const std::vector<host_block>& blocks = ChainableStack::instance_->host_blocks_;
  const size_t r = size_t(b.rows);
  host_parallel_for(
      size_t(b.cols),
      [&](size_t j0, size_t j1) {
        for (size_t j = j0; j < j1; ++j) {
          var* col = d + j * r;
          block_column(blocks, b, j, [&](size_t i, vari* v) { col[i].vi_ = v; });
        }
      },
      col_grain(b.rows));
}

// The bridge of a host block: in the reverse sweep, the host adjoints of the
// varis the block owns are gathered into the device node's adjoint (packed
// layouts into the lower triangle / the diagonal) -- unless no node chained
// after the block touched them (device consumers of the recognised node add
// into its device adjoint directly) and no device->host pending adjoint
// landed in it, in which case they are all still zero.  A shared vari (a
// symmetric block's (i, j) = (j, i), add_diag's off-diagonal elements) is
// gathered once, by the block that owns it.
class dev_to_host_vari : public vari {
 public:
  size_t blk_;  // index in host_blocks_
  size_t pos_;  // this node's index in var_stack_
  size_t ran_ = 0;     // the sweep (ChainableStack::sweep_) of the last chain()
  bool wrote_ = false;  // whether that chain() added into the node's adjoint
  explicit dev_to_host_vari(size_t blk)
      : vari(0.0), blk_(blk), pos_(ChainableStack::instance_->var_stack_.size() - 1) {
    local_adjoint_vari::register_dev_writer(this);  // (it adds gathered host adjoints into the node's)
  }
  bool reads_other_adjoints() const override { return true; }
  bool touches_adjoints_in(const vari*, const vari*) const override { return false; }
  bool may_write_device_adjoint(const void* node) const override {
    auto* st = ChainableStack::instance_;
    return node == st->host_blocks_[blk_].node && (ran_ != st->sweep_ || wrote_);
  }
  void chain() override {
    auto* st = ChainableStack::instance_;
    ran_ = st->sweep_;
    wrote_ = false;
    const host_block b = st->host_blocks_[blk_];
    if (!b.n) return;
    // a node chained before this one in the sweep (after it on the tape)
    // added into the block's host adjoints (grad.hpp log_host_touches), or a
    // device->host pending adjoint landed in one
    const bool touched = b.dirty || b.touched_sweep == st->sweep_;
    if (!touched) return;
    wrote_ = true;
    smg_ctx* c = amd::ctx();
    double* stage = static_cast<double*>(smg_host_scratch(c, b.n * sizeof(double)));
    if (!stage) throw std::bad_alloc();
    host_parallel_for(b.n, [&](size_t s, size_t e) {
      for (size_t i = s; i < e; ++i) stage[i] = b.first[i].adj_;
    });
    double* dst = amd::alloc_doubles(b.n);
    auto* node = static_cast<dev_matrix_vari*>(b.node);
    amd::check(smg_memcpy_h2d(c, dst, stage, b.n * sizeof(double)), "to_host");
    const int mode = block_pack_mode(b.layout);
    if (mode < 0)
      amd::check(smg_axpy(c, (long long)b.n, 1.0, dst, 1, node->adj_, 1), "to_host");
    else
      amd::check(smg_unpack_tril_add(c, mode, mode == 2 ? int(b.n) : b.rows, dst, node->adj_, b.rows), "to_host");
    amd::check(smg_sync(c), "to_host");  // the staging buffer is reused by the next host copy
  }
};

/** After a sweep (grad.hpp): every host block from index `from` on gets its
 * device node's adjoint written into the varis it owns -- what the
 * reference's varis hold after grad(): a symmetric block's shared vari the
 * sum of both elements' adjoints, a Cholesky factor's varis the partials its
 * consumers wrote (a closed-form reverse never formed them: expand_adjoint),
 * and its strict upper triangle's one dummy vari (cholesky_decompose.hpp:34-48)
 * the sum of the adjoints device consumers wrote there.  Every block's pack
 * and copy are queued first and land in ONE synchronisation. */
inline void publish_block_adjoints(size_t from) {
  auto* st = ChainableStack::instance_;
  if (from >= st->host_blocks_.size() || !amd::has_ctx()) return;
  smg_ctx* c = amd::ctx();
  join_device_adjoints();
  const size_t nb = st->host_blocks_.size();
  std::vector<size_t> off(nb + 1, 0);  // each block's doubles in the staging area (+1: a lower block's upper sum)
  for (size_t k = from; k < nb; ++k) {
    const host_block& b = st->host_blocks_[k];
    off[k + 1] = off[k] + (b.n ? b.n + (b.layout == layout_lower ? 1 : 0) : 0);
  }
  if (off[nb] == 0) return;
  double* stage = static_cast<double*>(smg_host_scratch(c, off[nb] * sizeof(double)));
  if (!stage) throw std::bad_alloc();
  for (size_t k = from; k < nb; ++k) {
    const host_block b = st->host_blocks_[k];
    if (!b.n) continue;
    auto* node = static_cast<dev_matrix_vari*>(b.node);
    if (node->sink_) node->sink_->expand_adjoint();
    const double* src = node->adj_;
    const int mode = block_pack_mode(b.layout);
    const size_t cnt = off[k + 1] - off[k];
    if (mode >= 0) {
      double* t = amd::alloc_doubles(cnt);
      amd::check(smg_pack_tril(c, mode, mode == 2 ? int(b.n) : b.rows, node->adj_, b.rows, t), "grad");
      if (b.layout == layout_lower) amd::check(smg_sum_strict_upper(c, b.rows, node->adj_, b.rows, t + b.n), "grad");
      src = t;
    }
    amd::check(smg_memcpy_d2h(c, stage + off[k], src, cnt * sizeof(double)), "grad");
  }
  amd::check(smg_sync(c), "grad");
  for (size_t k = from; k < nb; ++k) {
    host_block& b = st->host_blocks_[k];
    if (!b.n) continue;
    const double* h = stage + off[k];
    host_parallel_for(b.n, [&](size_t s, size_t e) {
      for (size_t i = s; i < e; ++i) b.first[i].adj_ = h[i];
    });
    if (b.layout == layout_lower && b.dummy) {  // (host nodes' contributions are already in it)
      b.dummy->adj_ += h[b.n] - b.dummy_dev;
      b.dummy_dev = h[b.n];
    }
  }
}

/** n varis constructed in place at first from values streamed device->host:
 * `src` (device, n doubles) comes down in chunks (one marker each) and the
 * host constructs chunk k's varis in parallel while chunk k+1 is in flight,
 * after running `overlap` while the first chunk transfers. */
inline void stream_varis(vari* first, const double* src, size_t n, const std::function<void()>& overlap) {
  if (!n) {
    if (overlap) overlap();
    return;
  }
  smg_ctx* c = amd::ctx();
  int armed = 0;
  amd::check(smg_status_armed(c, &armed), "to_host");
  double* stage = static_cast<double*>(smg_host_scratch(c, (n + 1) * sizeof(double)));
  if (!stage) throw std::bad_alloc();
  const int nch = n >= (size_t(1) << 21) ? 8 : 1;
  const size_t chunk = (n + size_t(nch) - 1) / size_t(nch);
  if (armed) amd::check(smg_status_enqueue(c, reinterpret_cast<int*>(stage + n)), "to_host");
  for (int k = 0; k < nch; ++k) {
    const size_t b = size_t(k) * chunk, e = std::min(n, b + chunk);
    amd::check(smg_memcpy_d2h(c, stage + b, src + b, (e - b) * sizeof(double)), "to_host");
    amd::check(smg_marker_record(c, k), "to_host");
  }
  if (overlap) overlap();
  for (int k = 0; k < nch; ++k) {
    const size_t b = size_t(k) * chunk, e = std::min(n, b + chunk);
    amd::check(smg_marker_wait(c, k), "to_host");
    if (k == 0 && armed) amd::throw_if_sync(*reinterpret_cast<int*>(stage + n), "to_host", "a persistent solve");
    host_parallel_for(e - b, [&](size_t s0, size_t s1) { construct_varis(first, stage, b + s0, b + s1); });
  }
}

/** Register block b (its bridge vari on var_stack_) and return its index. */
inline size_t push_block(const host_block& b) {
  auto* st = ChainableStack::instance_;
  st->host_blocks_.push_back(b);
  st->publish_ = &publish_block_adjoints;
  new dev_to_host_vari(st->host_blocks_.size() - 1);
  return st->host_blocks_.size() - 1;
}

/**
 * Materialise device node m as host varis (off every stack; the tape's
 * host_blocks_ owns them) plus one bridge vari on var_stack_, with the
 * reference's vari identity for m's structure: a lower-structured node (a
 * Cholesky factor) owns its lower triangle's varis, the strict upper being
 * one dummy (cholesky_decompose.hpp:34-48); a symmetric one (gp_exp_quad_cov)
 * one vari per (i, j), (j, i) pair (gp_exp_quad_cov.hpp:235); any other node
 * one vari per element.  Only the owned values cross PCIe (packed on the
 * device first).  `overlap` runs while the first chunk of values transfers
 * (work that needs the block's addresses but not its values: the caller's
 * pointer array).  Returns the block's index.
 */
inline size_t materialise(dev_matrix_vari* m, const std::function<void(const host_block&)>& overlap = nullptr) {
  auto* st = ChainableStack::instance_;
  host_block b{};
  b.node = m;
  b.rows = m->rows_;
  b.cols = m->cols_;
  b.dirty = false;
  const bool square = m->rows_ == m->cols_;
  b.layout = square && m->structure_ == dev_structure::lower       ? layout_lower
             : square && m->structure_ == dev_structure::symmetric ? layout_sym
                                                                   : layout_dense;
  b.n = b.layout == layout_dense ? m->size() : tril_count(size_t(m->rows_));
  b.first = static_cast<vari*>(st->memalloc_.alloc((b.n ? b.n : 1) * sizeof(vari)));
  b.dummy = b.layout == layout_lower ? new vari(0.0, vari::unstacked_tag{}) : nullptr;
  const double* src = m->val_;
  if (b.layout != layout_dense && b.n) {
    double* t = amd::alloc_doubles(b.n);
    amd::check(smg_pack_tril(amd::ctx(), 0, b.rows, m->val_, b.rows, t), "to_host");
    src = t;
  }
  stream_varis(b.first, src, b.n, [&] {
    if (overlap) overlap(b);
  });
  return push_block(b);
}

/**
 * add_diag's output at the Eigen boundary (prim/mat/fun/add_diag.hpp:25-27:
 * a copy of mat whose diagonal gets new varis): device node B = mat +
 * diag(d), whose elements off the diagonal are mat's own varis -- host block
 * `base`'s, or base_elems (mat's pointers, column-major) when mat is no
 * block -- and whose min(rows, cols) diagonal varis are new.  Returns the
 * block's index.
 */
inline size_t materialise_diag(dev_matrix_vari* B, long base, vari* const* base_elems) {
  auto* st = ChainableStack::instance_;
  host_block b{};
  b.node = B;
  b.rows = B->rows_;
  b.cols = B->cols_;
  b.dirty = false;
  b.layout = layout_diag;
  b.base = base;
  b.base_elems = base_elems;
  b.n = size_t(std::min(B->rows_, B->cols_));
  b.first = static_cast<vari*>(st->memalloc_.alloc((b.n ? b.n : 1) * sizeof(vari)));
  b.dummy = nullptr;
  if (b.n) {
    double* t = amd::alloc_doubles(b.n);
    amd::check(smg_pack_tril(amd::ctx(), 2, int(b.n), B->val_, b.rows, t), "add_diag");
    stream_varis(b.first, t, b.n, nullptr);
  }
  return push_block(b);
}

// host varis -> device (reverse: device adjoint -> host adjoints)
class host_to_dev_vari : public host_local_vari {
 public:
  dev_matrix_vari* dst_;
  vari** elems_;
  host_to_dev_vari(dev_matrix_vari* dst, vari** elems) : host_local_vari(0.0), dst_(dst), elems_(elems) {}
  bool touches_adjoints_in(const vari* lo, const vari* hi) const override {
    const size_t n = dst_->size();
    return !host_parallel_all(n, [&](size_t s, size_t e) {
      for (size_t i = s; i < e; ++i)
        if (elems_[i] >= lo && elems_[i] < hi) return false;
      return true;
    });
  }
  void chain() override {
    const size_t n = dst_->size();
    if (!n) return;
    smg_ctx* c = amd::ctx();
    int armed = 0;
    amd::check(smg_status_armed(c, &armed), "to_dev");
    double* h = static_cast<double*>(smg_host_scratch(c, (n + 1) * sizeof(double)));
    if (!h) throw std::bad_alloc();
    amd::check(smg_memcpy_d2h(c, h, dst_->adj_, n * sizeof(double)), "to_dev");
    if (armed) amd::check(smg_status_enqueue(c, reinterpret_cast<int*>(h + n)), "to_dev");
    amd::check(smg_sync(c), "to_dev");
    if (armed) amd::throw_if_sync(*reinterpret_cast<int*>(h + n), "to_dev", "a persistent solve");
    // elements may alias one vari (e.g. a broadcast mean): a serial scatter
    for (size_t i = 0; i < n; ++i) elems_[i]->adj_ += h[i];
  }
};

/** Host vars d[0..n) (column-major rows x cols) -> device node: the node a
 * host block mirrors when d is exactly that block, else a gathered copy
 * bridged by host_to_dev_vari.  nan_fn != null: the reference's
 * check_not_nan(nan_fn, nan_name, x) on the values first (throws before the
 * tape is touched; a recognised node is checked on the device). */
inline dev_var_matrix to_dev_vars(const var* d, size_t n, int rows, int cols, const char* nan_fn = nullptr,
                                  const char* nan_name = nullptr);
}  // namespace internal

/** Host vars (column-major; a column vector by default) -> device node
 * (bridged in the reverse sweep). */
inline dev_var_matrix to_dev(const std::vector<var>& v, int rows = -1, int cols = 1) {
  const size_t n = v.size();
  if (rows < 0) rows = int(n);
  if (size_t(rows) * size_t(cols) != n) throw std::invalid_argument("to_dev: rows * cols != size");
  return internal::to_dev_vars(v.data(), n, rows, cols);
}

/** Device node -> host vars, column-major (bridged in the reverse sweep). */
inline std::vector<var> to_var_vector(const dev_var_matrix& m) {
  std::vector<var> out(m.size());
  internal::materialise(m.vi_, [&](const host_block& b) { internal::fill_block_pointers(b, out.data()); });
  return out;
}

namespace internal {
inline void throw_not_nan(const char* fn, const char* name, size_t i) {
  std::ostringstream m;
  m << fn << ": " << name << "[" << i + 1 << "] is nan, but must not be nan!";
  throw std::domain_error(m.str());
}

inline dev_var_matrix to_dev_vars(const var* d, size_t n, int rows, int cols, const char* nan_fn,
                                  const char* nan_name) {
  if (dev_matrix_vari* node = recognise_block(d, n, rows, cols)) {
    if (nan_fn) {  // check_not_nan on the device values (one flag read back)
      smg_ctx* c = amd::ctx();
      double* flag = amd::alloc_doubles(1);
      amd::check(smg_memset(c, flag, 0, sizeof(double)), nan_fn);
      amd::check(smg_check_domain(c, node->val_, (long long)n, 0, flag), nan_fn);
      double f = 0;
      amd::to_host(&f, flag, 1);
      if (f != 0.0)
        for (size_t i = 0; i < n; ++i)
          if (std::isnan(d[i].vi_->val_)) throw_not_nan(nan_fn, nan_name, i);
    }
    return dev_var_matrix(node);
  }
  smg_ctx* c = amd::ctx();
  double* stage = n ? static_cast<double*>(smg_host_scratch(c, n * sizeof(double))) : nullptr;
  if (n && !stage) throw std::bad_alloc();
  vari** elems = ChainableStack::instance_->memalloc_.alloc_array<vari*>(n ? n : 1);
  host_parallel_for(n, [&](size_t s, size_t e) {
    for (size_t i = s; i < e; ++i) {
      elems[i] = d[i].vi_;
      stage[i] = d[i].vi_->val_;
    }
  });
  if (nan_fn)
    for (size_t i = 0; i < n; ++i)
      if (std::isnan(stage[i])) throw_not_nan(nan_fn, nan_name, i);
  auto* node = new dev_matrix_vari(rows, cols);
  if (n) {
    amd::check(smg_memcpy_h2d(c, node->val_, stage, n * sizeof(double)), "to_dev");
    amd::check(smg_sync(c), "to_dev");
  }
  new host_to_dev_vari(node, elems);
  return dev_var_matrix(node);
}
}  // namespace internal

}  // namespace math
}  // namespace stan
#endif
