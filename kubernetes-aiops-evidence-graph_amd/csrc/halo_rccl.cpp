// One halo exchange of an edge-cut partitioned plan over an RCCL communicator, for callers of
// libegraph.so that are not torch (SURVEY.md §8b's egr_halo_allgather entry; the torch path is
// egraph/shard.py, which drives the same pack / unpack through torch.distributed): the device
// pack of the boundary rows' non-zero entries into fixed-capacity peer slots, ONE equal-split
// ncclAllToAll of the slots over xGMI, the device unpack -- all enqueued on the caller's
// stream, no host synchronisation.  The exchange itself is the all-to-all, not an all-gather:
// rank r ships rank q only the rows q's rows read.
#include <rccl/rccl.h>

#include <string>

#include "egr_internal.h"

extern "C" int egr_plan_halo_exchange(egr_plan* p, int32_t what, const uint32_t* send_rows,
                                      int64_t n_send, const int64_t* send_seg_dev, int32_t P,
                                      int64_t peer_cap, int64_t* send_slots, int64_t* recv_slots,
                                      const uint32_t* recv_vertex, int64_t n_recv,
                                      const int64_t* recv_base_dev, uint32_t* overflow_dev,
                                      void* rccl_comm, void* stream) {
  if (!p || !rccl_comm || (what != 0 && what != 1) || P < 1 || P > EGR_SX_MAX_PEERS ||
      peer_cap < 1 || !send_slots || !recv_slots || !overflow_dev || !send_seg_dev ||
      (n_recv > 0 && (!recv_vertex || !recv_base_dev)))
    return egr::fail(EGR_EINVAL, "egr_plan_halo_exchange: bad arguments");
  const ncclComm_t comm = static_cast<ncclComm_t>(rccl_comm);
  int nranks = 0;
  ncclResult_t r = ncclCommCount(comm, &nranks);
  if (r != ncclSuccess) return egr::fail(EGR_EDEVICE, std::string("ncclCommCount: ") + ncclGetErrorString(r));
  if (nranks != P)
    return egr::fail(EGR_EINVAL, "egr_plan_halo_exchange: the communicator has " +
                                     std::to_string(nranks) + " ranks, the partition " + std::to_string(P));
  int rc = egr_plan_pack_sparse_cap(p, what, send_rows, n_send, send_seg_dev, P, send_slots, peer_cap,
                                    nullptr, overflow_dev, stream);
  if (rc != EGR_OK) return rc;
  // one slot per peer: a header word (the entry count) + peer_cap entries of 1 (scores) or 2
  // (reach) int64 words
  const size_t slot = 1 + (size_t)peer_cap * (what == 1 ? 2 : 1);
  r = ncclAllToAll(send_slots, recv_slots, slot, ncclInt64, comm, (hipStream_t)stream);
  if (r != ncclSuccess) return egr::fail(EGR_EDEVICE, std::string("ncclAllToAll: ") + ncclGetErrorString(r));
  return egr_plan_unpack_sparse_cap(p, what, recv_vertex, n_recv, recv_slots, peer_cap, overflow_dev,
                                    recv_base_dev, P, stream);
}
