#ifndef STAN_MATH_AMD_COMM_HPP
#define STAN_MATH_AMD_COMM_HPP

// The process's place in the multi-GPU job: one process per GPU, one RCCL
// communicator per process (smg_comm_*), plus the host-side view of it the
// header layer needs -- world size, rank, an all-gather of host doubles and a
// sum all-reduce of device doubles.  Both run over RCCL unless a host
// collective is installed with set_host_collective (a test harness's gloo
// process group, or any transport of the caller's); the map_rect executor
// (rev/functor/map_rect.hpp) calls amd::allgather (results) and amd::scatterv
// (its job data, once per call_id), the row-sharded reducers (*_glm_*) only
// amd::allreduce_sum.

#include <stan/math/amd/device.hpp>

#include <algorithm>
#include <stdexcept>
#include <string>
#include <vector>

namespace stan {
namespace math {
namespace amd {

/** recv[r * count + i] = rank r's send[i]; must be called by every rank. */
using allgather_fn = void (*)(const double* send, long long count, double* recv, void* user);
/** buf[i] = sum over ranks of buf[i] (in place, host doubles); every rank calls it. */
using allreduce_fn = void (*)(double* buf, long long count, void* user);
/** recv <- rank r's block of rank 0's send (blocks of counts[0], counts[1],
 * ... doubles back to back; send is read on rank 0 only); every rank calls it. */
using scatterv_fn = void (*)(const double* send, const long long* counts, double* recv, void* user);

struct comm_state {
  int nranks = 1;
  int rank = 0;
  bool rccl = false;
  allgather_fn host_allgather = nullptr;
  allreduce_fn host_allreduce = nullptr;
  scatterv_fn host_scatterv = nullptr;
  void* user = nullptr;
};
inline comm_state& comm_info() {
  static thread_local comm_state s;
  return s;
}

/** Join this process to an RCCL communicator (one per process / GPU).
 * id: 128 bytes from smg_comm_unique_id on rank 0, shared by the launcher. */
inline void comm_init(int nranks, int rank, const char* id) {
  check(smg_comm_init(ctx(), nranks, rank, id), "comm_init");
  comm_state& s = comm_info();
  s.nranks = nranks;
  s.rank = rank;
  s.rccl = true;
}
inline void comm_destroy() {
  if (has_ctx()) check(smg_comm_destroy(ctx()), "comm_destroy");
  comm_info() = comm_state{};
}

/** Use a host collective instead of RCCL for the header layer's exchanges
 * (fn == nullptr restores the single-process default).  ar: the sum
 * all-reduce the row-sharded reducers use (optional; without it they need
 * RCCL). */
inline void set_host_collective(int nranks, int rank, allgather_fn fn, void* user,
                                allreduce_fn ar = nullptr, scatterv_fn sc = nullptr) {
  if (fn && (nranks < 1 || rank < 0 || rank >= nranks))
    throw std::invalid_argument("set_host_collective: rank outside [0, nranks)");
  comm_state& s = comm_info();
  s.host_allgather = fn;
  s.host_allreduce = fn ? ar : nullptr;
  s.host_scatterv = fn ? sc : nullptr;
  s.user = user;
  s.nranks = fn ? nranks : (s.rccl ? s.nranks : 1);
  s.rank = fn ? rank : (s.rccl ? s.rank : 0);
}

inline int world_size() { return comm_info().nranks; }
inline int world_rank() { return comm_info().rank; }
/** The header layer exchanges results across ranks: an RCCL communicator is
 * up (any size, so one GPU exercises the same path) or a host collective
 * joins more than one rank. */
inline bool distributed() {
  const comm_state& s = comm_info();
  return s.host_allgather ? s.nranks > 1 : s.rccl;
}

/** All-gather of host doubles across the job (rank order). */
inline void allgather(const double* send, long long count, double* recv) {
  comm_state& s = comm_info();
  if (s.host_allgather) {
    s.host_allgather(send, count, recv, s.user);
    return;
  }
  if (!s.rccl) {
    if (s.nranks != 1) throw std::logic_error("allgather: no collective for a multi-rank job");
    for (long long i = 0; i < count; ++i) recv[i] = send[i];
    return;
  }
  if (count == 0) return;
  double* d = alloc_doubles(size_t(count) * (s.nranks + 1));
  to_device(d, send, size_t(count));
  check(smg_comm_allgather(ctx(), d, count, d + count), "allgather");
  to_host(recv, d + count, size_t(count) * s.nranks);
}

/** Scatter from rank 0: recv (host, counts[my rank] doubles) <- my block of
 * rank 0's send (host; blocks of counts[0], counts[1], ... back to back).
 * RCCL: point-to-point sends from the root (smg_comm_scatterv); a host
 * collective: its scatterv hook, or -- without one -- an all-gather of the
 * root's whole buffer. */
inline void scatterv(const double* send, const std::vector<long long>& counts, double* recv) {
  comm_state& s = comm_info();
  const int W = s.nranks, me = s.rank;
  if (int(counts.size()) != W) throw std::invalid_argument("scatterv: one count per rank");
  long long total = 0, off = 0;
  for (int r = 0; r < W; ++r) {
    if (r < me) off += counts[size_t(r)];
    total += counts[size_t(r)];
  }
  if (W == 1 || (!s.host_allgather && !s.rccl)) {
    if (W != 1) throw std::logic_error("scatterv: no collective for a multi-rank job");
    for (long long i = 0; i < counts[0]; ++i) recv[i] = send[i];
    return;
  }
  if (s.host_allgather) {
    if (s.host_scatterv) {
      s.host_scatterv(send, counts.data(), recv, s.user);
      return;
    }
    std::vector<double> mine(size_t(total), 0.0), all(size_t(total) * W);
    if (me == 0) std::copy(send, send + total, mine.begin());
    s.host_allgather(mine.data(), total, all.data(), s.user);
    std::copy(all.begin() + off, all.begin() + off + counts[size_t(me)], recv);
    return;
  }
  if (total == 0) return;
  double* d = alloc_doubles(size_t(total) + size_t(counts[size_t(me)]));
  if (me == 0) to_device(d, send, size_t(total));
  check(smg_comm_scatterv(ctx(), d, counts.data(), d + total, 0), "scatterv");
  to_host(recv, d + total, size_t(counts[size_t(me)]));
}

/** Sum all-reduce of `count` device doubles in place, on the tape's stream
 * (RCCL: ncclAllReduce; host collective: staged through host memory).
 * Every rank must call it with the same count.  One process without a
 * communicator: the identity. */
inline void allreduce_sum(double* dev, long long count, const char* fn) {
  comm_state& s = comm_info();
  if (count <= 0) return;
  if (s.host_allgather) {
    if (s.nranks == 1) return;
    if (!s.host_allreduce)
      throw std::logic_error(std::string(fn) + ": host collective has no all-reduce");
    std::vector<double> h(static_cast<size_t>(count));
    to_host(h.data(), dev, size_t(count));
    s.host_allreduce(h.data(), count, s.user);
    to_device(dev, h.data(), size_t(count));
    return;
  }
  if (!s.rccl) {
    if (s.nranks != 1) throw std::logic_error(std::string(fn) + ": no collective for a multi-rank job");
    return;
  }
  check(smg_comm_allreduce_sum(ctx(), dev, count), fn);
}

}  // namespace amd
}  // namespace math
}  // namespace stan
#endif
