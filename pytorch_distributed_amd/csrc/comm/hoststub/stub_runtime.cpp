// Host implementation of the HIP/RCCL stand-ins in this directory (test-only, see rccl/rccl.h).
//
// A "world" is what one ncclUniqueId names. Every rank of it is a host thread; a collective is
// executed synchronously: register pointers -> barrier -> each rank computes its result from every
// rank's send buffer -> barrier -> write -> barrier. ncclCommAbort wakes every rank blocked in a
// barrier with ncclRemoteError and FREES the comm object, exactly the contract of the real
// library -- so a caller that touches an aborted handle afterwards is a use-after-free that
// AddressSanitizer reports. Grouped calls from one thread (the in-process DataParallel pattern)
// are queued and executed together at ncclGroupEnd.
#include "hip/hip_runtime.h"
#include "rccl/rccl.h"

#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

struct pda_stub_event {
  double t = 0.0;
};

namespace {

double now_ms() {
  using namespace std::chrono;
  return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

enum Kind { kAllReduce, kBroadcast, kReduce, kAllGather, kReduceScatter };

struct World {
  explicit World(int n_) : n(n_), send(n_), count(n_), dt(n_), op(n_), root(n_), kind(n_) {}
  int n;
  std::mutex mu;
  std::condition_variable cv;
  bool aborted = false;
  bool async_err = false;
  int arrived = 0;
  long gen = 0;
  std::vector<const void*> send;
  std::vector<size_t> count;
  std::vector<int> dt, op, root, kind;
};

}  // namespace

struct pda_stub_comm {
  std::shared_ptr<World> w;
  int rank = 0;
};

namespace {

std::mutex g_mu;
std::map<std::string, std::shared_ptr<World>> g_worlds;
std::atomic<long> g_ids{0};
std::atomic<long> g_colls{0};

struct Op {
  Kind kind;
  const void* send;
  void* recv;
  size_t count;
  int dt, op, root;
  std::shared_ptr<World> w;
  int rank;
};
thread_local int t_group_depth = 0;
thread_local std::vector<Op> t_group;

size_t esize(int dt) {
  switch (dt) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    default: return 8;
  }
}

template <class T>
void combine_t(const std::vector<const void*>& srcs, size_t src_off, char* out, size_t n, int op) {
  const int nr = (int)srcs.size();
  T* o = reinterpret_cast<T*>(out);
  for (size_t i = 0; i < n; ++i) {
    T acc = reinterpret_cast<const T*>(srcs[0])[src_off + i];
    for (int r = 1; r < nr; ++r) {
      const T v = reinterpret_cast<const T*>(srcs[r])[src_off + i];
      switch (op) {
        case ncclProd: acc = acc * v; break;
        case ncclMax: acc = v > acc ? v : acc; break;
        case ncclMin: acc = v < acc ? v : acc; break;
        default: acc = acc + v; break;
      }
    }
    if (op == ncclAvg) acc = acc / (T)nr;
    o[i] = acc;
  }
}

bool combine(const std::vector<const void*>& srcs, size_t src_off, char* out, size_t n, int dt,
             int op) {
  switch (dt) {
    case ncclFloat32: combine_t<float>(srcs, src_off, out, n, op); return true;
    case ncclFloat64: combine_t<double>(srcs, src_off, out, n, op); return true;
    case ncclInt32: combine_t<int32_t>(srcs, src_off, out, n, op); return true;
    case ncclInt64: combine_t<int64_t>(srcs, src_off, out, n, op); return true;
    case ncclUint8: combine_t<uint8_t>(srcs, src_off, out, n, op); return true;
    default: return false;
  }
}

// result of rank `rank` for the registered collective; returns false if unsupported
bool compute(Kind kind, const std::vector<const void*>& send, size_t count, int dt, int op,
             int root, int rank, int n, std::vector<char>& tmp) {
  const size_t es = esize(dt);
  switch (kind) {
    case kAllReduce:
    case kReduce:
      tmp.resize(count * es);
      return combine(send, 0, tmp.data(), count, dt, op);
    case kBroadcast:
      tmp.resize(count * es);
      std::memcpy(tmp.data(), send[root], count * es);
      return true;
    case kAllGather:
      tmp.resize(count * es * n);
      for (int r = 0; r < n; ++r) std::memcpy(tmp.data() + r * count * es, send[r], count * es);
      return true;
    case kReduceScatter:
      tmp.resize(count * es);
      return combine(send, (size_t)rank * count, tmp.data(), count, dt, op);
  }
  return false;
}

bool writes(Kind kind, int rank, int root) { return kind != kReduce || rank == root; }

// generation barrier; false if the world was aborted before everyone arrived
bool barrier(World& w, std::unique_lock<std::mutex>& lk) {
  if (w.aborted) return false;
  const long g = w.gen;
  if (++w.arrived == w.n) {
    w.arrived = 0;
    ++w.gen;
    w.cv.notify_all();
    return true;
  }
  w.cv.wait(lk, [&] { return w.gen != g || w.aborted; });
  return w.gen != g;
}

ncclResult_t run(Kind kind, const void* send, void* recv, size_t count, int dt, int op, int root,
                 ncclComm_t comm) {
  if (!comm) return ncclInvalidArgument;
  // copy what we need: an abort from another thread frees `comm` while we wait below
  std::shared_ptr<World> w = comm->w;
  const int rank = comm->rank;
  if (t_group_depth > 0) {
    t_group.push_back(Op{kind, send, recv, count, dt, op, root, w, rank});
    return ncclSuccess;
  }
  ++g_colls;
  std::unique_lock<std::mutex> lk(w->mu);
  if (w->aborted) return ncclRemoteError;
  w->send[rank] = send;
  w->count[rank] = count;
  w->dt[rank] = dt;
  w->op[rank] = op;
  w->root[rank] = root;
  w->kind[rank] = kind;
  if (!barrier(*w, lk)) return ncclRemoteError;
  bool ok = true;
  for (int r = 0; r < w->n; ++r)
    ok = ok && w->count[r] == count && w->dt[r] == dt && w->op[r] == op && w->root[r] == root &&
         w->kind[r] == kind;
  std::vector<char> tmp;
  ok = ok && compute(kind, w->send, count, dt, op, root, rank, w->n, tmp);
  if (!barrier(*w, lk)) return ncclRemoteError;   // every rank has read every input
  if (ok && writes(kind, rank, root)) std::memcpy(recv, tmp.data(), tmp.size());
  if (!barrier(*w, lk)) return ncclRemoteError;   // every rank has written before reuse
  return ok ? ncclSuccess : ncclInvalidUsage;
}

}  // namespace

// ------------------------------------------------------------------------------------- HIP
hipError_t hipSetDevice(int) { return hipSuccess; }
hipError_t hipEventCreate(hipEvent_t* e) {
  *e = new pda_stub_event();
  return hipSuccess;
}
hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) { return hipEventCreate(e); }
hipError_t hipEventDestroy(hipEvent_t e) {
  delete e;
  return hipSuccess;
}
hipError_t hipEventRecord(hipEvent_t e, hipStream_t) {
  if (!e) return hipErrorInvalidValue;
  e->t = now_ms();
  return hipSuccess;
}
hipError_t hipStreamWaitEvent(hipStream_t, hipEvent_t e, unsigned) {
  return e ? hipSuccess : hipErrorInvalidValue;
}
hipError_t hipEventElapsedTime(float* ms, hipEvent_t a, hipEvent_t b) {
  if (!a || !b) return hipErrorInvalidValue;
  *ms = (float)(b->t - a->t);
  return hipSuccess;
}

// ------------------------------------------------------------------------------------- RCCL
ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  std::memset(id->internal, 0, sizeof(id->internal));
  std::snprintf(id->internal, sizeof(id->internal), "stub-%d-%ld", (int)getpid(), g_ids.fetch_add(1));
  return ncclSuccess;
}

const char* ncclGetErrorString(ncclResult_t r) {
  switch (r) {
    case ncclSuccess: return "no error";
    case ncclRemoteError: return "remote process exited or there was a network error";
    case ncclInvalidUsage: return "invalid usage";
    case ncclInvalidArgument: return "invalid argument";
    default: return "stub error";
  }
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
  if (nranks <= 0 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
  std::shared_ptr<World> w;
  {
    std::lock_guard<std::mutex> g(g_mu);
    std::string key(id.internal, strnlen(id.internal, NCCL_UNIQUE_ID_BYTES));
    auto it = g_worlds.find(key);
    if (it == g_worlds.end()) it = g_worlds.emplace(key, std::make_shared<World>(nranks)).first;
    w = it->second;
  }
  if (w->n != nranks) return ncclInvalidUsage;
  {
    std::unique_lock<std::mutex> lk(w->mu);   // init blocks until every rank joined (as NCCL)
    if (!barrier(*w, lk)) return ncclRemoteError;
  }
  *comm = new pda_stub_comm{w, rank};
  return ncclSuccess;
}

ncclResult_t ncclCommInitAll(ncclComm_t* comms, int ndev, const int*) {
  auto w = std::make_shared<World>(ndev);
  for (int i = 0; i < ndev; ++i) comms[i] = new pda_stub_comm{w, i};
  return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  delete comm;
  return ncclSuccess;
}

ncclResult_t ncclCommAbort(ncclComm_t comm) {
  if (!comm) return ncclSuccess;
  {
    std::lock_guard<std::mutex> g(comm->w->mu);
    comm->w->aborted = true;
    comm->w->cv.notify_all();
  }
  delete comm;
  return ncclSuccess;
}

ncclResult_t ncclCommGetAsyncError(ncclComm_t comm, ncclResult_t* err) {
  std::lock_guard<std::mutex> g(comm->w->mu);
  *err = (comm->w->aborted || comm->w->async_err) ? ncclRemoteError : ncclSuccess;
  return ncclSuccess;
}

ncclResult_t ncclCommCount(ncclComm_t comm, int* count) {
  *count = comm->w->n;
  return ncclSuccess;
}

ncclResult_t ncclAllReduce(const void* s, void* r, size_t n, ncclDataType_t dt, ncclRedOp_t op,
                           ncclComm_t c, hipStream_t) {
  return run(kAllReduce, s, r, n, dt, op, 0, c);
}
ncclResult_t ncclBroadcast(const void* s, void* r, size_t n, ncclDataType_t dt, int root,
                           ncclComm_t c, hipStream_t) {
  return run(kBroadcast, s, r, n, dt, ncclSum, root, c);
}
ncclResult_t ncclReduce(const void* s, void* r, size_t n, ncclDataType_t dt, ncclRedOp_t op,
                        int root, ncclComm_t c, hipStream_t) {
  return run(kReduce, s, r, n, dt, op, root, c);
}
ncclResult_t ncclAllGather(const void* s, void* r, size_t n, ncclDataType_t dt, ncclComm_t c,
                           hipStream_t) {
  return run(kAllGather, s, r, n, dt, ncclSum, 0, c);
}
ncclResult_t ncclReduceScatter(const void* s, void* r, size_t n, ncclDataType_t dt,
                               ncclRedOp_t op, ncclComm_t c, hipStream_t) {
  return run(kReduceScatter, s, r, n, dt, op, 0, c);
}

ncclResult_t ncclGroupStart() {
  ++t_group_depth;
  return ncclSuccess;
}

// one thread issued every rank's call of each world: execute them together, no barriers
ncclResult_t ncclGroupEnd() {
  if (t_group_depth <= 0) return ncclInvalidUsage;
  if (--t_group_depth > 0) return ncclSuccess;
  std::vector<Op> ops;
  ops.swap(t_group);
  ncclResult_t res = ncclSuccess;
  size_t i = 0;
  while (i < ops.size()) {
    const int n = ops[i].w->n;
    if (i + n > ops.size()) return ncclInvalidUsage;
    std::vector<const void*> send(n, nullptr);
    for (int k = 0; k < n; ++k) {
      const Op& o = ops[i + k];
      if (o.w != ops[i].w || o.kind != ops[i].kind || o.count != ops[i].count) return ncclInvalidUsage;
      send[o.rank] = o.send;
    }
    if (ops[i].w->aborted) return ncclRemoteError;
    ++g_colls;
    std::vector<std::vector<char>> tmp(n);
    for (int k = 0; k < n; ++k) {
      const Op& o = ops[i + k];
      if (!compute(o.kind, send, o.count, o.dt, o.op, o.root, o.rank, n, tmp[k]))
        res = ncclInvalidUsage;
    }
    if (res == ncclSuccess)
      for (int k = 0; k < n; ++k) {
        const Op& o = ops[i + k];
        if (writes(o.kind, o.rank, o.root)) std::memcpy(o.recv, tmp[k].data(), tmp[k].size());
      }
    i += n;
  }
  return res;
}

extern "C" void pda_stub_inject_async_error(ncclComm_t comm) {
  std::lock_guard<std::mutex> g(comm->w->mu);
  comm->w->async_err = true;
}

extern "C" long pda_stub_collectives(void) { return g_colls.load(); }
