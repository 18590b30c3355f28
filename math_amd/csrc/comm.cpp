// RCCL (xGMI) communicator for the row-sharded reducers.
// One communicator per process/device.  The row-sharded reducers' one
// collective is a single fp64 sum all-reduce of [logp, alpha', beta'(M)] per
// gradient; the distributed map_rect executor all-gathers per-job results.
// Replaces map_rect's Boost.MPI reduce/gatherv
// (prim/mat/functor/mpi_parallel_call.hpp:320-392).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>

#include "smg_internal.h"

extern "C" {

int smg_comm_unique_id(char* id) {
  if (!id) return SMG_ERR_ARG;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return SMG_ERR_HIP;
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  std::memcpy(id, &u, sizeof(u));
  return SMG_OK;
}

int smg_comm_init(smg_ctx* ctx, int nranks, int rank, const char* id) {
  if (!ctx || !id || nranks < 1 || rank < 0 || rank >= nranks) return SMG_ERR_ARG;
  if (ctx->comm) return SMG_OK;
  hipSetDevice(ctx->device);
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  ncclComm_t c;
  if (ncclCommInitRank(&c, nranks, u, rank) != ncclSuccess) return SMG_ERR_HIP;
  ctx->comm = (void*)c;
  return SMG_OK;
}

int smg_comm_allreduce_sum(smg_ctx* ctx, double* buf, long long count) {
  if (!ctx || !ctx->comm || (count > 0 && !buf)) return SMG_ERR_ARG;
  if (count == 0) return SMG_OK;
  if (ncclAllReduce(buf, buf, (size_t)count, ncclDouble, ncclSum, (ncclComm_t)ctx->comm,
                    ctx->stream) != ncclSuccess)
    return SMG_ERR_HIP;
  return SMG_OK;
}

int smg_comm_allgather(smg_ctx* ctx, const double* send, long long count, double* recv) {
  if (!ctx || !ctx->comm || count < 0 || (count > 0 && (!send || !recv))) return SMG_ERR_ARG;
  if (count == 0) return SMG_OK;
  if (ncclAllGather(send, recv, (size_t)count, ncclDouble, (ncclComm_t)ctx->comm, ctx->stream) != ncclSuccess)
    return SMG_ERR_HIP;
  return SMG_OK;
}

int smg_comm_destroy(smg_ctx* ctx) {
  if (!ctx || !ctx->comm) return SMG_OK;
  ncclCommDestroy((ncclComm_t)ctx->comm);
  ctx->comm = nullptr;
  return SMG_OK;
}

}  // extern "C"
