// RCCL (xGMI) communicator for the row-sharded reducers.
// One communicator per process/device.  The row-sharded reducers' one
// collective is a single fp64 sum all-reduce of [logp, alpha', beta'(M)] per
// gradient; the distributed map_rect executor all-gathers per-job results and
// scatters each rank's block of the job data once per call_id (scatterv).
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
  smg_prof_scope prof(ctx, SMG_FAM_COMM);
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

int smg_comm_scatterv(smg_ctx* ctx, const double* send, const long long* counts, double* recv, int root) {
  if (!ctx || !ctx->comm || !counts) return SMG_ERR_ARG;
  ncclComm_t c = (ncclComm_t)ctx->comm;
  int n = 0, me = 0;
  if (ncclCommCount(c, &n) != ncclSuccess || ncclCommUserRank(c, &me) != ncclSuccess) return SMG_ERR_HIP;
  if (root < 0 || root >= n) return SMG_ERR_ARG;
  long long total = 0;
  for (int r = 0; r < n; ++r) {
    if (counts[r] < 0) return SMG_ERR_ARG;
    total += counts[r];
  }
  if ((me == root && total > 0 && !send) || (counts[me] > 0 && !recv)) return SMG_ERR_ARG;
  // point-to-point: the root sends rank r its block, each rank receives its own
  if (ncclGroupStart() != ncclSuccess) return SMG_ERR_HIP;
  long long off = 0;
  for (int r = 0; r < n; ++r) {
    if (me == root && r != root && counts[r] > 0 &&
        ncclSend(send + off, (size_t)counts[r], ncclDouble, r, c, ctx->stream) != ncclSuccess) {
      ncclGroupEnd();
      return SMG_ERR_HIP;
    }
    off += counts[r];
  }
  if (me != root && counts[me] > 0 &&
      ncclRecv(recv, (size_t)counts[me], ncclDouble, root, c, ctx->stream) != ncclSuccess) {
    ncclGroupEnd();
    return SMG_ERR_HIP;
  }
  if (ncclGroupEnd() != ncclSuccess) return SMG_ERR_HIP;
  if (me == root && counts[me] > 0) {
    long long o = 0;
    for (int r = 0; r < root; ++r) o += counts[r];
    if (hipMemcpyAsync(recv, send + o, (size_t)counts[me] * sizeof(double), hipMemcpyDeviceToDevice,
                       ctx->stream) != hipSuccess)
      return SMG_ERR_HIP;
  }
  return SMG_OK;
}

int smg_comm_destroy(smg_ctx* ctx) {
  if (!ctx || !ctx->comm) return SMG_OK;
  ncclCommDestroy((ncclComm_t)ctx->comm);
  ctx->comm = nullptr;
  return SMG_OK;
}

}  // extern "C"
