// Factor exchange over RCCL (xGMI on an MI355X node) -- replaces hp:379-387 and carries the
// dense-dW all-reduce variant.  The library owns one ncclComm_t per hdp_comm; the unique id
// is created on rank 0 and shipped by the host (the reference's env:// rendezvous, hp:216).
#include <rccl/rccl.h>

#include <cstring>

#include "hdp_common.h"

struct hdp_comm_s {
  ncclComm_t nccl;
  int nranks, rank;
};

#define HDP_CHECK_NCCL(expr)                                                                  \
  do {                                                                                        \
    ncclResult_t r_ = (expr);                                                                 \
    if (r_ != ncclSuccess) {                                                                  \
      ::hdp::set_error("%s failed: %s (%s:%d)", #expr, ncclGetErrorString(r_), __FILE__, __LINE__); \
      return HDP_ERCCL;                                                                       \
    }                                                                                         \
  } while (0)

extern "C" int hdp_comm_unique_id(unsigned char* id, size_t id_bytes) {
  HDP_CHECK_ARG(id && id_bytes >= sizeof(ncclUniqueId), "hdp_comm_unique_id: need %zu bytes",
                sizeof(ncclUniqueId));
  ncclUniqueId uid;
  HDP_CHECK_NCCL(ncclGetUniqueId(&uid));
  std::memcpy(id, &uid, sizeof(uid));
  return HDP_OK;
}

extern "C" int hdp_comm_init(hdp_comm* comm, const unsigned char* id, size_t id_bytes, int nranks, int rank) {
  HDP_CHECK_ARG(comm && id && id_bytes >= sizeof(ncclUniqueId), "hdp_comm_init: bad id");
  HDP_CHECK_ARG(nranks > 0 && rank >= 0 && rank < nranks, "hdp_comm_init: bad rank %d/%d", rank, nranks);
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  hdp_comm c = new hdp_comm_s;
  c->nranks = nranks;
  c->rank = rank;
  ncclResult_t r = ncclCommInitRank(&c->nccl, nranks, uid, rank);
  if (r != ncclSuccess) {
    hdp::set_error("ncclCommInitRank failed: %s", ncclGetErrorString(r));
    delete c;
    return HDP_ERCCL;
  }
  *comm = c;
  return HDP_OK;
}

extern "C" int hdp_comm_destroy(hdp_comm comm) {
  if (!comm) return HDP_OK;
  ncclResult_t r = ncclCommDestroy(comm->nccl);
  delete comm;
  if (r != ncclSuccess) {
    hdp::set_error("ncclCommDestroy failed: %s", ncclGetErrorString(r));
    return HDP_ERCCL;
  }
  return HDP_OK;
}

extern "C" int hdp_allgather_f32(hdp_comm comm, const float* send, float* recv, int64_t count, void* stream) {
  HDP_CHECK_ARG(comm && send && recv && count >= 0, "hdp_allgather_f32: bad argument");
  if (count == 0) return HDP_OK;
  HDP_CHECK_NCCL(ncclAllGather(send, recv, (size_t)count, ncclFloat32, comm->nccl, hdp::as_stream(stream)));
  return HDP_OK;
}

extern "C" int hdp_allreduce_sum_f32(hdp_comm comm, float* buf, int64_t count, void* stream) {
  HDP_CHECK_ARG(comm && buf && count >= 0, "hdp_allreduce_sum_f32: bad argument");
  if (count == 0) return HDP_OK;
  HDP_CHECK_NCCL(ncclAllReduce(buf, buf, (size_t)count, ncclFloat32, ncclSum, comm->nccl, hdp::as_stream(stream)));
  return HDP_OK;
}

extern "C" int hdp_broadcast_bytes(hdp_comm comm, void* buf, int64_t bytes, int root, void* stream) {
  HDP_CHECK_ARG(comm && buf && bytes >= 0 && root >= 0 && root < comm->nranks, "hdp_broadcast_bytes: bad argument");
  if (bytes == 0) return HDP_OK;
  HDP_CHECK_NCCL(ncclBroadcast(buf, buf, (size_t)bytes, ncclUint8, root, comm->nccl, hdp::as_stream(stream)));
  return HDP_OK;
}

extern "C" int hdp_alltoall_f32(hdp_comm comm, const float* send, float* recv, int64_t count, void* stream) {
  HDP_CHECK_ARG(comm && send && recv && count >= 0, "hdp_alltoall_f32: bad argument");
  if (count == 0) return HDP_OK;
  hipStream_t st = hdp::as_stream(stream);
  HDP_CHECK_NCCL(ncclGroupStart());
  // the group is closed on every path: an error inside it must not leave the communicator in an
  // open group for the next collective (the first error is the one reported)
  ncclResult_t first = ncclSuccess;
  const char* what = nullptr;
  for (int j = 0; j < comm->nranks && first == ncclSuccess; ++j) {
    first = ncclSend(send + (size_t)j * count, (size_t)count, ncclFloat32, j, comm->nccl, st);
    if (first != ncclSuccess) { what = "ncclSend"; break; }
    first = ncclRecv(recv + (size_t)j * count, (size_t)count, ncclFloat32, j, comm->nccl, st);
    if (first != ncclSuccess) what = "ncclRecv";
  }
  ncclResult_t end = ncclGroupEnd();
  if (first == ncclSuccess && end != ncclSuccess) {
    first = end;
    what = "ncclGroupEnd";
  }
  if (first != ncclSuccess) {
    hdp::set_error("hdp_alltoall_f32: %s failed: %s", what, ncclGetErrorString(first));
    return HDP_ERCCL;
  }
  return HDP_OK;
}

extern "C" int hdp_allgather_bytes(hdp_comm comm, const void* send, void* recv, int64_t bytes, void* stream) {
  HDP_CHECK_ARG(comm && send && recv && bytes >= 0, "hdp_allgather_bytes: bad argument");
  if (bytes == 0) return HDP_OK;
  HDP_CHECK_NCCL(ncclAllGather(send, recv, (size_t)bytes, ncclUint8, comm->nccl, hdp::as_stream(stream)));
  return HDP_OK;
}
