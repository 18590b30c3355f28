#ifndef STAN_MATH_AMD_COMM_HPP
#define STAN_MATH_AMD_COMM_HPP

// The process's place in the multi-GPU job: one process per GPU, one RCCL
// communicator per process (smg_comm_*), plus the host-side view of it the
// header layer needs -- world size, rank, an all-gather of host doubles and a
// sum all-reduce of device doubles.  Both run over RCCL unless a host
// collective is installed with set_host_collective (a test harness's gloo
// process group, or any transport of the caller's); the map_rect executor
// (rev/functor/map_rect.hpp) only ever calls amd::allgather, the row-sharded
// reducers (*_glm_*) only amd::allreduce_sum.

#include <stan/math/amd/device.hpp>

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

struct comm_state {
  int nranks = 1;
  int rank = 0;
  bool rccl = false;
  allgather_fn host_allgather = nullptr;
  allreduce_fn host_allreduce = nullptr;
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
                                allreduce_fn ar = nullptr) {
  if (fn && (nranks < 1 || rank < 0 || rank >= nranks))
    throw std::invalid_argument("set_host_collective: rank outside [0, nranks)");
  comm_state& s = comm_info();
  s.host_allgather = fn;
  s.host_allreduce = fn ? ar : nullptr;
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
