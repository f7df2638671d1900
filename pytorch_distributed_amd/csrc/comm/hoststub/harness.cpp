// Multi-rank host harness for the C ABI of csrc/comm (communicator + gradient-bucket reducer),
// built against the stub runtime in this directory and run under ASan+UBSan and TSan by
// tests/test_comm_sanitizers_cpu.py (SURVEY §5.2 race detection, §5.3 failure detection).
//
// Every scenario runs world > 1 ranks as threads, calling exactly the functions the Python side
// calls (parallel/rccl.py). Exit code 0 = all scenarios passed; each prints "PASS <name>".
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "comm.h"

extern "C" {
int pda_comm_unique_id(char* out128);
int pda_comm_init_rank(const char* id128, int nranks, int rank, int device, void** handle);
int pda_comm_init_all(const int* devices, int ndev, void** handle);
int pda_comm_abort(void* h, int timeout_ms);
int pda_comm_destroy(void* h, int abort_);
int pda_comm_check(void* h);
int pda_comm_count(void* h, int* out);
int pda_comm_is_aborted(void* h);
int pda_allreduce(void* h, const void* s, void* r, size_t n, int dt, int op, hipStream_t st);
int pda_broadcast(void* h, const void* s, void* r, size_t n, int dt, int root, hipStream_t st);
int pda_allgather(void* h, const void* s, void* r, size_t n, int dt, hipStream_t st);
int pda_reduce_scatter(void* h, const void* s, void* r, size_t n, int dt, int op, hipStream_t st);
int pda_group_allreduce(void* h, void* const* bufs, size_t n, int dt, int op, const hipStream_t* st);
int pda_reducer_create(void* comm, void* flat, int dt, int op, const long long* bounds, int nb,
                       hipStream_t cs, void** out);
int pda_reducer_ready(void* h, long long upto, hipStream_t producer);
int pda_reducer_finish(void* h, hipStream_t producer, hipStream_t consumer);
int pda_reducer_reset(void* h);
long long pda_reducer_launched(void* h);
int pda_reducer_set_timing(void* h, int on);
int pda_reducer_timing(void* h, float* out);
int pda_reducer_destroy(void* h);
}

#define CHECK(cond)                                                                        \
  do {                                                                                     \
    if (!(cond)) {                                                                         \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond);         \
      std::_Exit(1);                                                                       \
    }                                                                                      \
  } while (0)

namespace {

constexpr int kF32 = 0, kI64 = 3, kU8 = 6;
constexpr int kSum = 0, kAvg = 1, kMax = 2, kMin = 3;

template <class F>
void run_ranks(int world, F f) {
  std::vector<std::thread> ts;
  for (int r = 0; r < world; ++r) ts.emplace_back(f, r);
  for (auto& t : ts) t.join();
}

// world W (4, and 8 = the driver's one-node scaling run): buckets launched in rank-specific
// readiness patterns, averaged exactly; timing
void multi_rank_average(const int W) {
  const long long N = 10000;
  const std::vector<long long> bounds = {0, 1000, 1000, 4000, 4000, 4096, 4096, 10000};
  char id[128];
  CHECK(pda_comm_unique_id(id) == 0);
  run_ranks(W, [&](int rank) {
    void* h = nullptr;
    CHECK(pda_comm_init_rank(id, W, rank, 0, &h) == 0);
    int n = 0;
    CHECK(pda_comm_count(h, &n) == 0 && n == W);
    std::vector<float> flat(N);
    void* red = nullptr;
    CHECK(pda_reducer_create(h, flat.data(), kF32, kAvg, bounds.data(), 4, nullptr, &red) == 0);
    std::mt19937 rng(1234 + rank);
    for (int step = 0; step < 6; ++step) {
      if (step == 3) CHECK(pda_reducer_set_timing(red, 1) == 0);
      if (step == 5) CHECK(pda_reducer_set_timing(red, 0) == 0);
      for (long long i = 0; i < N; ++i) flat[i] = (float)(rank * 8 + (i % 97) + step);
      CHECK(pda_reducer_reset(red) == 0);
      long long upto = 0;
      while (upto < N) {   // monotone, rank-specific readiness reports (some not on a boundary)
        upto += 1 + (long long)(rng() % 3000);
        if (upto > N) upto = N;
        CHECK(pda_reducer_ready(red, upto, nullptr) == 0);
      }
      CHECK(pda_reducer_finish(red, nullptr, nullptr) == 0);
      const float avg_rank = 8.f * (float)(W * (W - 1) / 2) / W;
      for (long long i = 0; i < N; ++i) CHECK(flat[i] == avg_rank + (float)(i % 97) + step);
      CHECK(pda_reducer_launched(red) == 4LL * (step + 1));
      if (step == 3) {
        float t[5] = {-1, -1, -1, -1, -1};
        CHECK(pda_reducer_timing(red, t) == 0);
        for (float v : t) CHECK(v >= 0.f);
      }
    }
    CHECK(pda_comm_check(h) == 0);
    CHECK(pda_reducer_destroy(red) == 0);
    CHECK(pda_comm_destroy(h, 0) == 0);
  });
  std::printf("PASS multi_rank_average world %d\n", W);
}

// the Python handle closes the communicator while a reducer still references it
void destroy_comm_before_reducer() {
  const int W = 2;
  char id[128];
  CHECK(pda_comm_unique_id(id) == 0);
  run_ranks(W, [&](int rank) {
    void* h = nullptr;
    CHECK(pda_comm_init_rank(id, W, rank, 0, &h) == 0);
    std::vector<float> flat(256, 1.f);
    const long long b[2] = {0, 256};
    void* red = nullptr;
    CHECK(pda_reducer_create(h, flat.data(), kF32, kSum, b, 1, nullptr, &red) == 0);
    CHECK(pda_reducer_finish(red, nullptr, nullptr) == 0);
    CHECK(flat[7] == 2.f);
    CHECK(pda_comm_destroy(h, 0) == 0);                        // struct kept alive by the reducer
    CHECK(pda_reducer_ready(red, 256, nullptr) == pda::kErrAborted);
    CHECK(pda_reducer_finish(red, nullptr, nullptr) == pda::kErrAborted);
    CHECK(pda_reducer_destroy(red) == 0);                      // last reference frees it
  });
  std::printf("PASS destroy_comm_before_reducer\n");
}

// one rank never joins the step (dead peer): the others block inside a bucket all-reduce while
// holding the communicator lock; their watchdogs see the async error and abort with a timeout;
// the blocked enqueue returns an error, later enqueues return kErrAborted, teardown is clean
void abort_while_enqueuing() {
  const int W = 3;
  char id[128];
  CHECK(pda_comm_unique_id(id) == 0);
  std::atomic<int> blocked_returned{0};
  run_ranks(W, [&](int rank) {
    void* h = nullptr;
    CHECK(pda_comm_init_rank(id, W, rank, 0, &h) == 0);
    if (rank == W - 1) {             // the dead peer: holds its handle, never enqueues
      std::this_thread::sleep_for(std::chrono::milliseconds(400));
      CHECK(pda_comm_destroy(h, 1) == 0);
      return;
    }
    std::vector<float> flat(1024, 1.f);
    const long long b[4] = {0, 512, 512, 1024};
    void* red = nullptr;
    CHECK(pda_reducer_create(h, flat.data(), kF32, kAvg, b, 2, nullptr, &red) == 0);
    // the watchdog of parallel/rccl.py: poll the async error, abort (never free) on error
    std::thread watchdog([&] {
      const auto t0 = std::chrono::steady_clock::now();
      bool injected = false;
      for (;;) {
        if (!injected && rank == 0 &&
            std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(100)) {
          std::lock_guard<std::mutex> st(static_cast<pda::Comm*>(h)->state_mu);
          pda_stub_inject_async_error(static_cast<pda::Comm*>(h)->comms[0]);
          injected = true;
        }
        const int rc = pda_comm_check(h);
        if (rc == pda::kErrAborted) return;
        if (rc != 0) {
          CHECK(pda_comm_abort(h, 50) == 0);
          return;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(5));
      }
    });
    const int rc = pda_reducer_ready(red, 512, nullptr);   // blocks: the dead rank never arrives
    CHECK(rc != 0);
    blocked_returned.fetch_add(1);
    watchdog.join();
    CHECK(pda_comm_is_aborted(h) == 1);
    CHECK(pda_reducer_ready(red, 1024, nullptr) == pda::kErrAborted);
    CHECK(pda_reducer_finish(red, nullptr, nullptr) == pda::kErrAborted);
    CHECK(pda_comm_check(h) == pda::kErrAborted);
    float x = 0.f;
    CHECK(pda_allreduce(h, &x, &x, 1, kF32, kSum, nullptr) == pda::kErrAborted);
    CHECK(pda_comm_destroy(h, 0) == 0);
    CHECK(pda_reducer_destroy(red) == 0);
  });
  CHECK(blocked_returned.load() == W - 1);
  std::printf("PASS abort_while_enqueuing\n");
}

void bad_arguments() {
  char id[128];
  CHECK(pda_comm_unique_id(id) == 0);
  void* h = nullptr;
  CHECK(pda_comm_init_rank(id, 1, 0, 0, &h) == 0);
  std::vector<float> flat(100);
  const long long overlap[4] = {0, 60, 50, 100};
  const long long empty[2] = {10, 10};
  void* red = nullptr;
  CHECK(pda_reducer_create(h, flat.data(), kF32, kAvg, overlap, 2, nullptr, &red) == pda::kErrBadArgs);
  CHECK(pda_reducer_create(h, flat.data(), kF32, kAvg, empty, 1, nullptr, &red) == pda::kErrBadArgs);
  CHECK(pda_reducer_create(h, nullptr, kF32, kAvg, empty, 1, nullptr, &red) == pda::kErrBadArgs);
  const long long ok[2] = {0, 100};
  CHECK(pda_reducer_create(h, flat.data(), kF32, kAvg, ok, 1, nullptr, &red) == 0);
  float t[2];
  CHECK(pda_reducer_timing(red, t) == pda::kErrBadArgs);     // no timed step recorded
  CHECK(pda_reducer_destroy(red) == 0);
  CHECK(pda_comm_destroy(h, 0) == 0);
  std::printf("PASS bad_arguments\n");
}

// other collectives used by DDP construction checks / buffers / validation
void collectives() {
  const int W = 3;
  char id[128];
  CHECK(pda_comm_unique_id(id) == 0);
  run_ranks(W, [&](int rank) {
    void* h = nullptr;
    CHECK(pda_comm_init_rank(id, W, rank, 0, &h) == 0);
    std::vector<unsigned char> bytes(37, (unsigned char)(rank + 1));
    CHECK(pda_broadcast(h, bytes.data(), bytes.data(), bytes.size(), kU8, 1, nullptr) == 0);
    for (auto v : bytes) CHECK(v == 2);
    long long meta[2] = {100 + rank, -rank};
    long long mx[2], mn[2];
    CHECK(pda_allreduce(h, meta, mx, 2, kI64, kMax, nullptr) == 0);
    CHECK(pda_allreduce(h, meta, mn, 2, kI64, kMin, nullptr) == 0);
    CHECK(mx[0] == 100 + W - 1 && mx[1] == 0 && mn[0] == 100 && mn[1] == -(W - 1));
    float mine[2] = {(float)rank, (float)(10 * rank)};
    std::vector<float> all(2 * W);
    CHECK(pda_allgather(h, mine, all.data(), 2, kF32, nullptr) == 0);
    for (int r = 0; r < W; ++r) CHECK(all[2 * r] == (float)r && all[2 * r + 1] == 10.f * r);
    std::vector<float> full(2 * W, 1.f);
    float part[2];
    CHECK(pda_reduce_scatter(h, full.data(), part, 2, kF32, kSum, nullptr) == 0);
    CHECK(part[0] == (float)W && part[1] == (float)W);
    CHECK(pda_comm_destroy(h, 0) == 0);
  });
  std::printf("PASS collectives\n");
}

// in-process DataParallel group: one thread, ncclCommInitAll, grouped all-reduce (D = 4, and 8 =
// resnet_dp.py's node: the segmented replay reduces each gradient slice this way)
void dp_group(const int D) {
  std::vector<int> devs(D);
  for (int d = 0; d < D; ++d) devs[d] = d;
  void* h = nullptr;
  CHECK(pda_comm_init_all(devs.data(), D, &h) == 0);
  std::vector<std::vector<float>> bufs(D, std::vector<float>(333));
  std::vector<void*> ptrs(D);
  std::vector<hipStream_t> sts(D, nullptr);
  for (int d = 0; d < D; ++d) {
    for (int i = 0; i < 333; ++i) bufs[d][i] = (float)(d + i);
    ptrs[d] = bufs[d].data();
  }
  CHECK(pda_group_allreduce(h, ptrs.data(), 333, kF32, kSum, sts.data()) == 0);
  for (int d = 0; d < D; ++d)
    for (int i = 0; i < 333; ++i) CHECK(bufs[d][i] == (float)(D * (D - 1) / 2 + D * i));
  // the segmented DataParallel reduce: consecutive slices of the flat gradient, one grouped call
  // each, in stage order
  const int cuts[4] = {0, 100, 250, 333};
  for (int s = 0; s < 3; ++s) {
    std::vector<void*> sp(D);
    for (int d = 0; d < D; ++d) sp[d] = bufs[d].data() + cuts[s];
    CHECK(pda_group_allreduce(h, sp.data(), cuts[s + 1] - cuts[s], kF32, kSum, sts.data()) == 0);
  }
  for (int d = 0; d < D; ++d)
    for (int i = 0; i < 333; ++i) CHECK(bufs[d][i] == (float)D * (float)(D * (D - 1) / 2 + D * i));
  CHECK(pda_comm_destroy(h, 0) == 0);
  std::printf("PASS dp_group %d devices\n", D);
}

}  // namespace

int main() {
  alarm(120);   // a deadlock fails the test instead of hanging it
  multi_rank_average(4);
  multi_rank_average(8);
  destroy_comm_before_reducer();
  abort_while_enqueuing();
  bad_arguments();
  collectives();
  dp_group(4);
  dp_group(8);
  std::printf("ALL PASS\n");
  return 0;
}
