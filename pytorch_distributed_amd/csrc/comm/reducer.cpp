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
// by the Python planner (parallel/reducer.py plan_buckets).
//
// Diagnostics (pda_reducer_set_timing): a second set of timing-enabled events brackets every
// bucket all-reduce on the comm stream plus the backward end on the producer stream, so
// pda_reducer_timing reports per-bucket all-reduce time and the EXPOSED communication time
// (backward end -> last bucket done). Off in timed runs.
//
// Lifetime: the reducer holds a reference on the communicator (comm.h) and every launch runs
// under the communicator lock, returning kErrAborted once the watchdog (or close) aborted it.
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
  // timing diagnostics
  bool timing = false;
  bool timed_step = false;  // this step was recorded with timing events
  std::vector<hipEvent_t> t_beg, t_end;
  hipEvent_t t_bwd_end = nullptr;
};

void destroy_events(std::vector<hipEvent_t>& v) {
  for (auto e : v)
    if (e) hipEventDestroy(e);
  v.clear();
}

int launch_upto(Reducer* r, long long upto, hipStream_t producer) {
  const int nb = (int)r->beg.size();
  while (r->next < nb && r->end[r->next] <= upto) {
    const int b = r->next;
    if (hipEventRecord(r->ready[b], producer) != hipSuccess) return -1;
    if (hipStreamWaitEvent(r->comm_stream, r->ready[b], 0) != hipSuccess) return -1;
    if (r->timing && hipEventRecord(r->t_beg[b], r->comm_stream) != hipSuccess) return -1;
    char* p = r->flat + (size_t)r->beg[b] * r->esize;
    const size_t n = (size_t)(r->end[b] - r->beg[b]);
    ncclResult_t e = ncclAllReduce(p, p, n, r->dt, r->op, r->comm->comms[0], r->comm_stream);
    if (e != ncclSuccess) return (int)e;
    if (r->timing && hipEventRecord(r->t_end[b], r->comm_stream) != hipSuccess) return -1;
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
  if (!comm || !flat || nb <= 0 || !out) return pda::kErrBadArgs;
  Reducer* r = new Reducer();
  r->flat = static_cast<char*>(flat);
  r->dt = pda::to_nccl(dt);
  r->esize = pda::nccl_elem_bytes(dt);
  r->op = op == 1 ? ncclAvg : ncclSum;
  r->comm_stream = comm_stream;
  for (int b = 0; b < nb; ++b) {
    const long long s = bounds[2 * b], e = bounds[2 * b + 1];
    if (s < 0 || e <= s || (b > 0 && s < r->end.back())) {
      delete r;
      return pda::kErrBadArgs;
    }
    r->beg.push_back(s);
    r->end.push_back(e);
  }
  r->ready.assign(nb, nullptr);
  r->done.assign(nb, nullptr);
  for (int b = 0; b < nb; ++b) {
    if (hipEventCreateWithFlags(&r->ready[b], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&r->done[b], hipEventDisableTiming) != hipSuccess) {
      destroy_events(r->ready);
      destroy_events(r->done);
      delete r;
      return -1;
    }
  }
  r->comm = static_cast<pda::Comm*>(comm);
  pda::retain(r->comm);
  *out = r;
  return 0;
}

// launch every not-yet-launched bucket whose end <= upto, ordered after `producer`'s work
int pda_reducer_ready(void* h, long long upto, hipStream_t producer) {
  Reducer* r = static_cast<Reducer*>(h);
  pda::Enqueue g(r->comm);
  if (!g.ok()) return pda::kErrAborted;
  return launch_upto(r, upto, producer);
}

// launch the remaining buckets, make `consumer` wait for all of them, reset for the next step
int pda_reducer_finish(void* h, hipStream_t producer, hipStream_t consumer) {
  Reducer* r = static_cast<Reducer*>(h);
  pda::Enqueue g(r->comm);
  if (!g.ok()) return pda::kErrAborted;
  if (r->timing && hipEventRecord(r->t_bwd_end, producer) != hipSuccess) return -1;
  int rc = launch_upto(r, r->end.back(), producer);
  if (rc != 0) return rc;
  if (r->last >= 0 && hipStreamWaitEvent(consumer, r->done[r->last], 0) != hipSuccess) return -1;
  r->timed_step = r->timing && r->next == (int)r->beg.size();
  r->next = 0;
  r->last = -1;
  return 0;
}

int pda_reducer_reset(void* h) {
  Reducer* r = static_cast<Reducer*>(h);
  pda::Enqueue g(r->comm);
  r->next = 0;
  r->last = -1;
  return 0;
}

long long pda_reducer_launched(void* h) { return static_cast<Reducer*>(h)->launched_total; }

int pda_reducer_num_buckets(void* h) { return (int)static_cast<Reducer*>(h)->beg.size(); }

// enable/disable the timing events (takes effect at the next bucket launch; call between steps)
int pda_reducer_set_timing(void* h, int on) {
  Reducer* r = static_cast<Reducer*>(h);
  pda::Enqueue g(r->comm);
  const int nb = (int)r->beg.size();
  if (on && r->t_beg.empty()) {
    r->t_beg.assign(nb, nullptr);
    r->t_end.assign(nb, nullptr);
    for (int b = 0; b < nb; ++b)
      if (hipEventCreate(&r->t_beg[b]) != hipSuccess || hipEventCreate(&r->t_end[b]) != hipSuccess)
        return -1;
    if (hipEventCreate(&r->t_bwd_end) != hipSuccess) return -1;
  }
  r->timing = on != 0;
  r->timed_step = false;
  return 0;
}

// After a timed step has COMPLETED on the device (caller synchronised): out[0] = exposed
// communication ms (backward end -> last bucket done, >= 0), out[1 + b] = all-reduce ms of
// bucket b. Returns kErrBadArgs if no complete timed step was recorded.
int pda_reducer_timing(void* h, float* out) {
  Reducer* r = static_cast<Reducer*>(h);
  if (!r->timed_step) return pda::kErrBadArgs;
  const int nb = (int)r->beg.size();
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, r->t_bwd_end, r->t_end[nb - 1]) != hipSuccess) return -1;
  out[0] = ms > 0.f ? ms : 0.f;
  for (int b = 0; b < nb; ++b) {
    if (hipEventElapsedTime(&ms, r->t_beg[b], r->t_end[b]) != hipSuccess) return -1;
    out[1 + b] = ms;
  }
  return 0;
}

int pda_reducer_destroy(void* h) {
  Reducer* r = static_cast<Reducer*>(h);
  destroy_events(r->ready);
  destroy_events(r->done);
  destroy_events(r->t_beg);
  destroy_events(r->t_end);
  if (r->t_bwd_end) hipEventDestroy(r->t_bwd_end);
  pda::release(r->comm);
  delete r;
  return 0;
}

}  // extern "C"
