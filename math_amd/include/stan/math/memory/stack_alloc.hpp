#ifndef STAN_MATH_MEMORY_STACK_ALLOC_HPP
#define STAN_MATH_MEMORY_STACK_ALLOC_HPP

// Host bump arena for vari objects and their operand arrays.
// Same contract as the reference's stan::math::stack_alloc
// (stan/math/memory/stack_alloc.hpp:72-287): 8-byte aligned bump allocation
// from a list of blocks that double in size, nested marks, bulk recovery only,
// no per-object free, in_stack() membership.  Written independently; the
// block list keeps (base, size) pairs and marks are (block, offset) tuples.

#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <new>
#include <vector>

namespace stan {
namespace math {

class stack_alloc {
 public:
  explicit stack_alloc(size_t initial_nbytes = size_t(1) << 16) {
    add_block(initial_nbytes);
    cur_ = 0;
    next_ = blocks_[0].base;
    end_ = next_ + blocks_[0].size;
  }
  stack_alloc(const stack_alloc&) = delete;
  stack_alloc& operator=(const stack_alloc&) = delete;
  ~stack_alloc() {
    for (auto& b : blocks_) std::free(b.base);
  }

  inline void* alloc(size_t len) {
    len = (len + 7) & ~size_t(7);
    char* r = next_;
    next_ += len;
    if (__builtin_expect(next_ > end_, 0)) r = next_block(len);
    return r;
  }

  template <typename T>
  inline T* alloc_array(size_t n) {
    return static_cast<T*>(alloc(n * sizeof(T)));
  }

  inline void recover_all() {
    cur_ = 0;
    next_ = blocks_[0].base;
    end_ = next_ + blocks_[0].size;
  }

  inline void start_nested() { marks_.push_back({cur_, next_, end_}); }

  inline void recover_nested() {
    if (marks_.empty()) {
      recover_all();
      return;
    }
    const mark m = marks_.back();
    marks_.pop_back();
    cur_ = m.block;
    next_ = m.next;
    end_ = m.end;
  }

  inline void free_all() {
    for (size_t i = 1; i < blocks_.size(); ++i) std::free(blocks_[i].base);
    blocks_.resize(1);
    recover_all();
  }

  inline size_t bytes_allocated() const {
    size_t s = 0;
    for (size_t i = 0; i <= cur_; ++i) s += blocks_[i].size;
    return s;
  }

  inline bool in_stack(const void* p) const {
    const char* c = static_cast<const char*>(p);
    for (size_t i = 0; i < cur_; ++i)
      if (c >= blocks_[i].base && c < blocks_[i].base + blocks_[i].size) return true;
    return c >= blocks_[cur_].base && c < next_;
  }

 private:
  struct block {
    char* base;
    size_t size;
  };
  struct mark {
    size_t block;
    char* next;
    char* end;
  };
  std::vector<block> blocks_;
  std::vector<mark> marks_;
  size_t cur_;
  char* next_;
  char* end_;

  void add_block(size_t n) {
    void* p = std::malloc(n);
    if (!p) throw std::bad_alloc();
    blocks_.push_back({static_cast<char*>(p), n});
  }

  char* next_block(size_t len) {
    size_t b = cur_ + 1;
    while (b < blocks_.size() && blocks_[b].size < len) ++b;
    if (b >= blocks_.size()) {
      size_t n = blocks_.back().size * 2;
      if (n < len) n = len;
      add_block(n);
      b = blocks_.size() - 1;
    }
    cur_ = b;
    next_ = blocks_[b].base + len;
    end_ = blocks_[b].base + blocks_[b].size;
    return blocks_[b].base;
  }
};

}  // namespace math
}  // namespace stan
#endif
