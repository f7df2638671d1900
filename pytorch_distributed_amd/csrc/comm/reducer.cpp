// Gradient-bucket reducer (C ABI) -- the native counterpart of torch DDP's C++ Reducer that the
// reference's DDP relied on.
//
// The native ResNet keeps every gradient in ONE flat buffer laid out in gradient-production
// order, so a bucket is just a [begin, end) element range of it (no copy-in/copy-out, the
// parameters' .grad are views). The backward schedule reports how many leading elements are
// final (pda_reducer_ready(upto)); every bucket that became complete is launched right away:
//
//   hipEventRecord(ready[b], producer stream)         -- the stream that wrote the gradients
//   hipStreamWaitEvent(comm stream, ready[b])         -- no host synchronisation anywhere
//   ncclAllReduce(bucket, ncclAvg, comm stream)       -- 1/world inside the collective
//   hipEventRecord(done[b], comm stream)
//
// pda_reducer_finish(consumer stream) launches what is left and makes the consumer (the fused
// SGD's stream) wait on the last bucket's event; buckets run in order on one comm stream, so
// that one event covers all of them. Events are created once (timing disabled) and re-recorded
// every step, so the per-bucket host cost is four HIP/RCCL calls. Bucket boundaries are chosen
// by the Python planner (parallel/reducer.py plan_buckets: small first bucket, 32 MiB middle
// buckets for per-link-bound xGMI rings, a small exposed final bucket).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <vector>

#include "comm.h"

namespace {

struct Reducer {
  pda::Comm* comm = nullptr;
  char* flat = nullptr;
  ncclDataType_t dt = ncclFloat32;
  size_t esize = 4;
  ncclRedOp_t op = ncclAvg;
  hipStream_t comm_stream = nullptr;
  std::vector<long long> beg, end;
  std::vector<hipEvent_t> ready, done;
  int next = 0;   // first bucket not launched this step
  int last = -1;  // last bucket launched this step
  long long launched_total = 0;
};

int launch_upto(Reducer* r, long long upto, hipStream_t producer) {
  const int nb = (int)r->beg.size();
  while (r->next < nb && r->end[r->next] <= upto) {
    const int b = r->next;
    if (hipEventRecord(r->ready[b], producer) != hipSuccess) return -1;
    if (hipStreamWaitEvent(r->comm_stream, r->ready[b], 0) != hipSuccess) return -1;
    char* p = r->flat + (size_t)r->beg[b] * r->esize;
    const size_t n = (size_t)(r->end[b] - r->beg[b]);
    ncclResult_t e = ncclAllReduce(p, p, n, r->dt, r->op, r->comm->comms[0], r->comm_stream);
    if (e != ncclSuccess) return (int)e;
    if (hipEventRecord(r->done[b], r->comm_stream) != hipSuccess) return -1;
    r->last = b;
    r->next = b + 1;
    ++r->launched_total;
  }
  return 0;
}

}  // namespace

extern "C" {

// bounds: nb (begin, end) element pairs, contiguous and increasing; op: 0 sum, 1 avg
int pda_reducer_create(void* comm, void* flat, int dt, int op, const long long* bounds, int nb,
                       hipStream_t comm_stream, void** out) {
  if (!comm || !flat || nb <= 0 || !out) return -1;
  Reducer* r = new Reducer();
  r->comm = static_cast<pda::Comm*>(comm);
  r->flat = static_cast<char*>(flat);
  r->dt = pda::to_nccl(dt);
  r->esize = pda::nccl_elem_bytes(dt);
  r->op = op == 1 ? ncclAvg : ncclSum;
  r->comm_stream = comm_stream;
  for (int b = 0; b < nb; ++b) {
    const long long s = bounds[2 * b], e = bounds[2 * b + 1];
    if (e <= s || (b > 0 && s < r->end.back())) {
      delete r;
      return -2;
    }
    r->beg.push_back(s);
    r->end.push_back(e);
  }
  r->ready.resize(nb);
  r->done.resize(nb);
  for (int b = 0; b < nb; ++b) {
    if (hipEventCreateWithFlags(&r->ready[b], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&r->done[b], hipEventDisableTiming) != hipSuccess)
      return -1;
  }
  *out = r;
  return 0;
}

// launch every not-yet-launched bucket whose end <= upto, ordered after `producer`'s work
int pda_reducer_ready(void* h, long long upto, hipStream_t producer) {
  return launch_upto(static_cast<Reducer*>(h), upto, producer);
}

// launch the remaining buckets, make `consumer` wait for all of them, reset for the next step
int pda_reducer_finish(void* h, hipStream_t producer, hipStream_t consumer) {
  Reducer* r = static_cast<Reducer*>(h);
  int rc = launch_upto(r, r->end.back(), producer);
  if (rc != 0) return rc;
  if (r->last >= 0 && hipStreamWaitEvent(consumer, r->done[r->last], 0) != hipSuccess) return -1;
  r->next = 0;
  r->last = -1;
  return 0;
}

int pda_reducer_reset(void* h) {
  Reducer* r = static_cast<Reducer*>(h);
  r->next = 0;
  r->last = -1;
  return 0;
}

long long pda_reducer_launched(void* h) { return static_cast<Reducer*>(h)->launched_total; }

int pda_reducer_destroy(void* h) {
  Reducer* r = static_cast<Reducer*>(h);
  for (auto e : r->ready) hipEventDestroy(e);
  for (auto e : r->done) hipEventDestroy(e);
  delete r;
  return 0;
}

}  // extern "C"
