// RCCL communicator over xGMI (C ABI, loaded with ctypes by parallel/rccl.py).
//
// Replaces ProcessGroupNCCL / torch.cuda.nccl of the reference stack:
//   * multi-process: ncclGetUniqueId on rank 0 -> exchanged through the torch TCPStore ->
//     ncclCommInitRank (one communicator per process/GPU);
//   * single-process multi-GPU (DataParallel): ncclCommInitAll over the device list, collectives
//     issued for every device inside one ncclGroupStart/End;
//   * every collective takes an explicit hipStream_t (the caller's dedicated comm stream, ordered
//     against the compute stream with HIP events) -- nothing here synchronises the host;
//   * failure detection: pda_comm_check polls ncclCommGetAsyncError; the watchdog
//     calls pda_comm_abort, which aborts WITHOUT freeing (see comm.h for the lifetime model), so a
//     dead peer surfaces as an error code from the next enqueue instead of a hang or a segfault.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <vector>

#include "comm.h"

using pda::Comm;
using pda::Enqueue;
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

// abort (or destroy) every communicator of c once; caller holds c->mu or gave up waiting for it
int teardown(Comm* c, bool abort_) {
  std::lock_guard<std::mutex> st(c->state_mu);
  if (c->aborted.exchange(true)) return 0;
  int rc = 0;
  for (auto& cm : c->comms) {
    if (!cm) continue;
    ncclResult_t r = abort_ ? ncclCommAbort(cm) : ncclCommDestroy(cm);
    if (r != ncclSuccess) rc = (int)r;
    cm = nullptr;
  }
  return rc;
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

const char* pda_comm_error_string(int r) {
  if (r == pda::kErrAborted) return "communicator aborted";
  if (r == pda::kErrBadArgs) return "invalid arguments";
  if (r < 0) return "HIP runtime error";
  return ncclGetErrorString((ncclResult_t)r);
}

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

// Abort without freeing (watchdog): waits up to timeout_ms for in-flight enqueues, then aborts
// regardless -- an enqueue blocked on a dead peer holds the lock and only the abort releases it.
int pda_comm_abort(void* h, int timeout_ms) {
  Comm* c = static_cast<Comm*>(h);
  bool locked = pda::try_lock_for(c, timeout_ms);
  int rc = teardown(c, true);
  if (locked) c->mu.unlock();
  return rc;
}

// Drop the caller's reference: destroys (or aborts) the RCCL communicators now; the struct
// itself lives on while a reducer still references it (its enqueues then return kErrAborted).
int pda_comm_destroy(void* h, int abort_) {
  Comm* c = static_cast<Comm*>(h);
  int rc;
  {
    std::unique_lock<std::mutex> lk(c->mu);
    rc = teardown(c, abort_ != 0);
  }
  pda::release(c);
  return rc;
}

int pda_comm_is_aborted(void* h) { return static_cast<Comm*>(h)->aborted.load() ? 1 : 0; }

// 0 = healthy; an ncclResult_t async error; kErrAborted once aborted. Does not take the enqueue
// lock (see comm.h), so it still runs while an enqueue is stuck on a dead peer.
int pda_comm_check(void* h) {
  Comm* c = static_cast<Comm*>(h);
  std::lock_guard<std::mutex> st(c->state_mu);
  if (c->aborted.load()) return pda::kErrAborted;
  for (auto cm : c->comms) {
    ncclResult_t ae = ncclSuccess;
    ncclResult_t r = ncclCommGetAsyncError(cm, &ae);
    if (r != ncclSuccess) return (int)r;
    if (ae != ncclSuccess && ae != ncclInProgress) return (int)ae;
  }
  return 0;
}

// number of ranks RCCL itself reports for this communicator (bench: "rccl_world")
int pda_comm_count(void* h, int* out) {
  Comm* c = static_cast<Comm*>(h);
  Enqueue g(c);
  if (!g.ok()) return pda::kErrAborted;
  return (int)ncclCommCount(c->comms[0], out);
}

// ---- multi-process collectives (comms[0]) ------------------------------------------------
int pda_allreduce(void* h, const void* send, void* recv, size_t count, int dt, int op,
                  hipStream_t st) {
  Comm* c = static_cast<Comm*>(h);
  Enqueue g(c);
  if (!g.ok()) return pda::kErrAborted;
  return (int)ncclAllReduce(send, recv, count, to_nccl(dt), to_op(op), c->comms[0], st);
}

int pda_broadcast(void* h, const void* send, void* recv, size_t count, int dt, int root,
                  hipStream_t st) {
  Comm* c = static_cast<Comm*>(h);
  Enqueue g(c);
  if (!g.ok()) return pda::kErrAborted;
  return (int)ncclBroadcast(send, recv, count, to_nccl(dt), root, c->comms[0], st);
}

int pda_reduce(void* h, const void* send, void* recv, size_t count, int dt, int op, int root,
               hipStream_t st) {
  Comm* c = static_cast<Comm*>(h);
  Enqueue g(c);
  if (!g.ok()) return pda::kErrAborted;
  return (int)ncclReduce(send, recv, count, to_nccl(dt), to_op(op), root, c->comms[0], st);
}

int pda_allgather(void* h, const void* send, void* recv, size_t count, int dt, hipStream_t st) {
  Comm* c = static_cast<Comm*>(h);
  Enqueue g(c);
  if (!g.ok()) return pda::kErrAborted;
  return (int)ncclAllGather(send, recv, count, to_nccl(dt), c->comms[0], st);
}

int pda_reduce_scatter(void* h, const void* send, void* recv, size_t count, int dt, int op,
                       hipStream_t st) {
  Comm* c = static_cast<Comm*>(h);
  Enqueue g(c);
  if (!g.ok()) return pda::kErrAborted;
  return (int)ncclReduceScatter(send, recv, count, to_nccl(dt), to_op(op), c->comms[0], st);
}

// ---- in-process (DataParallel) grouped collectives: arrays of per-device pointers/streams --
int pda_group_allreduce(void* h, void* const* bufs, size_t count, int dt, int op,
                        const hipStream_t* streams) {
  Comm* c = static_cast<Comm*>(h);
  Enqueue g(c);
  if (!g.ok()) return pda::kErrAborted;
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
  Enqueue g(c);
  if (!g.ok()) return pda::kErrAborted;
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
  Enqueue g(c);
  if (!g.ok()) return pda::kErrAborted;
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
