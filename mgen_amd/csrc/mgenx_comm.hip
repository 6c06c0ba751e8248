// mgenx_comm.hip -- the multi-GPU exchange steps of the engine, over RCCL (xGMI).
//
// The hot path shards with no data-path collective: records of a flow live
// on the GPU that owns the flow, stream shards are contiguous byte ranges.  Two small
// exchanges remain, and these are the only collectives in the library:
//   * mgenx_allreduce_flows: the per-flow counter merge after flow-sharded
//     MgenAnalytic::Update (mgenAnalytic.cpp:74-258 on each owner).  Every flow has exactly
//     one owner and the others contribute zero records, so an integer SUM over the 64-byte
//     records reproduces the owner's record bit for bit (FP64 fields included: x + 0 = x on
//     the bit pattern, -0.0 too).  One ncclAllReduce of n_flows x 64 B.
//   * mgenx_allgather_u64: the stream-shard chain stitch (a few u64 per rank).
#include <string.h>

#include <rccl/rccl.h>

#include "mgenx_kernels.hpp"

struct mgenx_comm {
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = 0, device = 0;
};

extern "C" int mgenx_ctx_device(const mgenx_ctx* ctx);

extern "C" {

int mgenx_comm_unique_id(void* id_out) {
  if (!id_out) return MGENX_EINVAL;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return MGENX_EDEVICE;
  memcpy(id_out, &id, sizeof(id));
  return MGENX_OK;
}

int mgenx_comm_init(mgenx_ctx* ctx, int nranks, int rank, const void* id, mgenx_comm** out) {
  if (!ctx || !id || !out || nranks < 1 || rank < 0 || rank >= nranks) return MGENX_EINVAL;
  *out = nullptr;
  const int dev = mgenx_ctx_device(ctx);
  if (hipSetDevice(dev) != hipSuccess) return MGENX_EDEVICE;
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  mgenx_comm* c = new mgenx_comm();
  c->nranks = nranks;
  c->rank = rank;
  c->device = dev;
  if (ncclCommInitRank(&c->comm, nranks, uid, rank) != ncclSuccess) {
    delete c;
    return MGENX_EDEVICE;
  }
  *out = c;
  return MGENX_OK;
}

int mgenx_comm_destroy(mgenx_comm* comm) {
  if (!comm) return MGENX_EINVAL;
  if (comm->comm) ncclCommDestroy(comm->comm);
  delete comm;
  return MGENX_OK;
}

int mgenx_allreduce_flows(mgenx_ctx* ctx, mgenx_comm* comm, mgenx_flow_counters* dev_counters,
                          uint32_t n_flows, void* stream) {
  if (!ctx || !comm || (n_flows && !dev_counters)) return MGENX_EINVAL;
  if (n_flows == 0) return MGENX_OK;
  static_assert(sizeof(mgenx_flow_counters) == 64, "64-byte counter record");
  const size_t count = (size_t)n_flows * (sizeof(mgenx_flow_counters) / 8);
  const ncclResult_t r = ncclAllReduce(dev_counters, dev_counters, count, ncclUint64, ncclSum,
                                       comm->comm, (hipStream_t)stream);
  return r == ncclSuccess ? MGENX_OK : MGENX_EDEVICE;
}

int mgenx_allgather_u64(mgenx_ctx* ctx, mgenx_comm* comm, const uint64_t* dev_in,
                        uint64_t* dev_out, uint32_t count, void* stream) {
  if (!ctx || !comm || (count && (!dev_in || !dev_out))) return MGENX_EINVAL;
  if (count == 0) return MGENX_OK;
  const ncclResult_t r = ncclAllGather(dev_in, dev_out, count, ncclUint64, comm->comm,
                                       (hipStream_t)stream);
  return r == ncclSuccess ? MGENX_OK : MGENX_EDEVICE;
}

}  // extern "C"
