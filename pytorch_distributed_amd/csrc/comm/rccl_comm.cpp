// RCCL communicator over xGMI (C ABI, loaded with ctypes by parallel/rccl.py).
//
// Replaces ProcessGroupNCCL / torch.cuda.nccl of the reference stack:
//   * multi-process: ncclGetUniqueId on rank 0 -> exchanged through the torch TCPStore ->
//     ncclCommInitRank (one communicator per process/GPU);
//   * single-process multi-GPU (DataParallel): ncclCommInitAll over the device list, collectives
//     issued for every device inside one ncclGroupStart/End;
//   * every collective takes an explicit hipStream_t (the caller's dedicated comm stream, ordered
//     against the compute stream with HIP events) -- nothing here synchronises the host;
//   * pda_comm_check polls ncclCommGetAsyncError so a dead peer surfaces as an error (and can be
//     aborted) instead of a hang.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <vector>

#include "comm.h"

using pda::Comm;
using pda::to_nccl;

namespace {

ncclRedOp_t to_op(int op) {
  switch (op) {
    case 0: return ncclSum;
    case 1: return ncclAvg;
    case 2: return ncclMax;
    case 3: return ncclMin;
    default: return ncclSum;
  }
}

}  // namespace

extern "C" {

int pda_comm_unique_id(char* out128) {
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return (int)r;
  std::memcpy(out128, id.internal, NCCL_UNIQUE_ID_BYTES);
  return 0;
}

const char* pda_comm_error_string(int r) { return ncclGetErrorString((ncclResult_t)r); }

// multi-process: one rank of nranks on `device`
int pda_comm_init_rank(const char* id128, int nranks, int rank, int device, void** handle) {
  ncclUniqueId id;
  std::memcpy(id.internal, id128, NCCL_UNIQUE_ID_BYTES);
  if (hipSetDevice(device) != hipSuccess) return -1;
  Comm* c = new Comm();
  c->comms.resize(1);
  c->devices.push_back(device);
  ncclResult_t r = ncclCommInitRank(&c->comms[0], nranks, id, rank);
  if (r != ncclSuccess) {
    delete c;
    return (int)r;
  }
  *handle = c;
  return 0;
}

// single-process: one communicator per device
int pda_comm_init_all(const int* devices, int ndev, void** handle) {
  Comm* c = new Comm();
  c->comms.resize(ndev);
  c->devices.assign(devices, devices + ndev);
  ncclResult_t r = ncclCommInitAll(c->comms.data(), ndev, devices);
  if (r != ncclSuccess) {
    delete c;
    return (int)r;
  }
  *handle = c;
  return 0;
}

int pda_comm_destroy(void* h, int abort_) {
  Comm* c = static_cast<Comm*>(h);
  int rc = 0;
  for (auto cm : c->comms) {
    ncclResult_t r = abort_ ? ncclCommAbort(cm) : ncclCommDestroy(cm);
    if (r != ncclSuccess) rc = (int)r;
  }
  delete c;
  return rc;
}

int pda_comm_check(void* h) {
  Comm* c = static_cast<Comm*>(h);
  for (auto cm : c->comms) {
    ncclResult_t ae = ncclSuccess;
    ncclResult_t r = ncclCommGetAsyncError(cm, &ae);
    if (r != ncclSuccess) return (int)r;
    if (ae != ncclSuccess && ae != ncclInProgress) return (int)ae;
  }
  return 0;
}

// ---- multi-process collectives (comms[0]) ------------------------------------------------
int pda_allreduce(void* h, const void* send, void* recv, size_t count, int dt, int op,
                  hipStream_t st) {
  Comm* c = static_cast<Comm*>(h);
  return (int)ncclAllReduce(send, recv, count, to_nccl(dt), to_op(op), c->comms[0], st);
}

int pda_broadcast(void* h, const void* send, void* recv, size_t count, int dt, int root,
                  hipStream_t st) {
  Comm* c = static_cast<Comm*>(h);
  return (int)ncclBroadcast(send, recv, count, to_nccl(dt), root, c->comms[0], st);
}

int pda_reduce(void* h, const void* send, void* recv, size_t count, int dt, int op, int root,
               hipStream_t st) {
  Comm* c = static_cast<Comm*>(h);
  return (int)ncclReduce(send, recv, count, to_nccl(dt), to_op(op), root, c->comms[0], st);
}

int pda_allgather(void* h, const void* send, void* recv, size_t count, int dt, hipStream_t st) {
  Comm* c = static_cast<Comm*>(h);
  return (int)ncclAllGather(send, recv, count, to_nccl(dt), c->comms[0], st);
}

int pda_reduce_scatter(void* h, const void* send, void* recv, size_t count, int dt, int op,
                       hipStream_t st) {
  Comm* c = static_cast<Comm*>(h);
  return (int)ncclReduceScatter(send, recv, count, to_nccl(dt), to_op(op), c->comms[0], st);
}

// ---- in-process (DataParallel) grouped collectives: arrays of per-device pointers/streams --
int pda_group_allreduce(void* h, void* const* bufs, size_t count, int dt, int op,
                        const hipStream_t* streams) {
  Comm* c = static_cast<Comm*>(h);
  ncclResult_t r = ncclGroupStart();
  if (r != ncclSuccess) return (int)r;
  for (size_t i = 0; i < c->comms.size(); ++i) {
    r = ncclAllReduce(bufs[i], bufs[i], count, to_nccl(dt), to_op(op), c->comms[i], streams[i]);
    if (r != ncclSuccess) break;
  }
  ncclResult_t e = ncclGroupEnd();
  return (int)(r != ncclSuccess ? r : e);
}

int pda_group_broadcast(void* h, void* const* bufs, size_t count, int dt, int root,
                        const hipStream_t* streams) {
  Comm* c = static_cast<Comm*>(h);
  ncclResult_t r = ncclGroupStart();
  if (r != ncclSuccess) return (int)r;
  for (size_t i = 0; i < c->comms.size(); ++i) {
    r = ncclBroadcast(bufs[i], bufs[i], count, to_nccl(dt), root, c->comms[i], streams[i]);
    if (r != ncclSuccess) break;
  }
  ncclResult_t e = ncclGroupEnd();
  return (int)(r != ncclSuccess ? r : e);
}

int pda_group_reduce(void* h, void* const* bufs, size_t count, int dt, int op, int root,
                     const hipStream_t* streams) {
  Comm* c = static_cast<Comm*>(h);
  ncclResult_t r = ncclGroupStart();
  if (r != ncclSuccess) return (int)r;
  for (size_t i = 0; i < c->comms.size(); ++i) {
    r = ncclReduce(bufs[i], bufs[i], count, to_nccl(dt), to_op(op), root, c->comms[i], streams[i]);
    if (r != ncclSuccess) break;
  }
  ncclResult_t e = ncclGroupEnd();
  return (int)(r != ncclSuccess ? r : e);
}

}  // extern "C"
