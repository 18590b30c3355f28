// The reverse sweep's bookkeeping with host blocks, on the CPU (no device
// call is made): B materialised blocks, each with its bridge on the tape and
// host nodes after it, one of which touches one element of block k0 (that
// block has no bridge: it would gather into a device node).  Prints
//   blocks tape_length sweep_seconds touched_blocks
// and, with argv[1] == "check", exits non-zero unless exactly block k0 is
// stamped touched in the sweep (grad.hpp log_host_touches) -- the bridges'
// check is O(1) per bridge instead of a rescan of the rest of the tape
// (the round-4 form cost O(bridges x tape)).
#include <stan/math.hpp>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>

int main(int argc, char** argv) {
  using namespace stan::math;
  const int B = argc > 2 ? std::atoi(argv[2]) : 1000;
  const int per = 4;  // host nodes after each bridge
  auto* st = ChainableStack::instance_;
  var x = 1.5, acc = 0.0;
  const size_t k0 = size_t(B) / 3;
  std::vector<vari*> firsts;
  for (int k = 0; k < B; ++k) {
    host_block b{};
    b.n = 16;
    b.rows = 4;
    b.cols = 4;
    b.layout = internal::layout_dense;
    b.first = static_cast<vari*>(st->memalloc_.alloc(b.n * sizeof(vari)));
    for (size_t i = 0; i < b.n; ++i) ::new (static_cast<void*>(b.first + i)) vari(0.25 * double(i), vari::unstacked_tag{});
    firsts.push_back(b.first);
    if (size_t(k) == k0)
      st->host_blocks_.push_back(b);  // (no bridge: a touched bridge would gather into the device node)
    else
      internal::push_block(b);
    for (int q = 0; q < per; ++q) acc = acc + x * 1.0001;  // touch no block
    if (size_t(k) == k0) acc = acc + var(b.first + 5) * 2.0;  // touches block k0's element 5
  }
  const size_t tape = st->var_stack_.size();
  auto t0 = std::chrono::steady_clock::now();
  grad(acc.vi_);
  auto t1 = std::chrono::steady_clock::now();
  int touched = 0;
  bool ok = true;
  for (size_t k = 0; k < st->host_blocks_.size(); ++k) {
    const bool t = st->host_blocks_[k].touched_sweep == st->sweep_;
    touched += t;
    if (t != (k == k0)) ok = false;
  }
  const double g_elem = firsts[k0][5].adj_;
  std::printf("%d %zu %.6e %d %.6g %.6g\n", B, tape, std::chrono::duration<double>(t1 - t0).count(), touched,
              x.adj(), g_elem);
  if (argc > 1 && std::string(argv[1]) == "check" && (!ok || g_elem != 2.0)) return 1;
  recover_memory();
  return 0;
}
