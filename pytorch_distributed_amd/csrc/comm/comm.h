// Shared between the RCCL communicator (rccl_comm.cpp) and the gradient-bucket reducer
// (reducer.cpp): the communicator handle handed to Python as an opaque pointer.
//
// Lifetime / failure model:
//   * every enqueue (collective, bucket launch) holds `mu` and first checks `aborted`, so once a
//     communicator is aborted no caller can reach a freed ncclComm_t; the async-error poll does
//     not take `mu` (an enqueue blocked on a dead peer holds it -- that is exactly when the poll
//     must still run) but `state_mu`, which abort/destroy hold while freeing the comms;
//   * the watchdog thread aborts through pda_comm_abort: it takes `mu` (with a timeout -- an
//     enqueue stuck on a dead peer holds it, and ncclCommAbort is what unblocks that enqueue),
//     marks the communicator aborted and calls ncclCommAbort. It never frees the struct;
//   * the struct is reference counted: the Python handle owns one reference, every reducer built
//     on it another, so pda_comm_destroy while a reducer is alive leaves the struct valid (and
//     aborted) until the reducer is destroyed too.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <mutex>
#include <thread>
#include <vector>

namespace pda {

// error codes above ncclNumResults that the C ABI can return besides ncclResult_t / -1 (HIP)
constexpr int kErrAborted = 1001;   // communicator aborted (watchdog or close)
constexpr int kErrBadArgs = 1002;

struct Comm {
  std::vector<ncclComm_t> comms;  // 1 for multi-process, ndev for in-process
  std::vector<int> devices;
  std::mutex mu;                  // held by every enqueue (may block on a dead peer)
  std::mutex state_mu;            // never held across a blocking call: guards comms' lifetime
                                  // between the async-error poll and abort/destroy
  std::atomic<bool> aborted{false};
  std::atomic<int> refs{1};
};

inline void retain(Comm* c) { c->refs.fetch_add(1); }

// try to take c->mu for up to timeout_ms (polling try_lock: sanitizer-friendly, and the wait is
// only ever the watchdog's, off the training thread)
inline bool try_lock_for(Comm* c, int timeout_ms) {
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  for (;;) {
    if (c->mu.try_lock()) return true;
    if (std::chrono::steady_clock::now() >= deadline) return false;
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
}

inline void release(Comm* c) {
  if (c->refs.fetch_sub(1) == 1) delete c;
}

// RAII enqueue guard: holds the communicator lock; `ok()` is false once aborted
class Enqueue {
 public:
  explicit Enqueue(Comm* c) : c_(c), lk_(c->mu) {}
  bool ok() const { return !c_->aborted.load(); }

 private:
  Comm* c_;
  std::unique_lock<std::mutex> lk_;
};

inline ncclDataType_t to_nccl(int dt) {
  switch (dt) {
    case 0: return ncclFloat32;
    case 1: return ncclBfloat16;
    case 2: return ncclFloat16;
    case 3: return ncclInt64;
    case 4: return ncclFloat64;
    case 5: return ncclInt32;
    case 6: return ncclUint8;
    default: return ncclFloat32;
  }
}

inline size_t nccl_elem_bytes(int dt) {
  switch (dt) {
    case 1: case 2: return 2;
    case 3: case 4: return 8;
    case 6: return 1;
    default: return 4;
  }
}

}  // namespace pda
