// Host-side sanitizer check of the request executor (csrc/executor.cpp): slot hand-off between
// request threads and the worker, dynamic batching (row claims, sealing, partial batches),
// multi-row requests (hz_exec_submit_rows) and teardown, under AddressSanitizer+UBSan or
// ThreadSanitizer (tests/test_native_asan_cpu.py builds it both ways with -Xarch_host).
//
// No GPU: hz_prog_replay and the four HIP event calls the executor makes are defined here (the
// executable's definitions take precedence over libamdhip64's). A fake program "runs" at replay
// time -- out row r = f(in row r) over the slot's pinned buffers -- so a launch issued before every
// claimed row was copied, or a result read before its replay, shows up as a wrong row; the fake
// event completes a few microseconds after it is recorded, so the worker really polls.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "hipzap.h"

namespace {

constexpr int kInts = 6;  // ints per row (input and output)

struct FakeProg {
  int32_t* in;
  int32_t* out;
  int rows;
  std::atomic<int> replays{0};
};

struct FakeEvent {
  std::atomic<int64_t> ready_ns{0};
};

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int32_t f(int32_t v, int e) { return v * 3 + 7 + e; }

}  // namespace

extern "C" int hz_prog_replay(HzProgram p, hipStream_t) {
  auto* fp = static_cast<FakeProg*>(p);
  for (int r = 0; r < fp->rows; ++r)
    for (int e = 0; e < kInts; ++e) fp->out[r * kInts + e] = f(fp->in[r * kInts + e], e);
  fp->replays.fetch_add(1, std::memory_order_relaxed);
  return 0;
}

hipError_t hipEventCreateWithFlags(hipEvent_t* ev, unsigned) {
  *ev = reinterpret_cast<hipEvent_t>(new FakeEvent());
  return hipSuccess;
}

hipError_t hipEventRecord(hipEvent_t ev, hipStream_t) {
  reinterpret_cast<FakeEvent*>(ev)->ready_ns.store(now_ns() + 20000, std::memory_order_release);
  return hipSuccess;
}

hipError_t hipEventQuery(hipEvent_t ev) {
  return now_ns() >= reinterpret_cast<FakeEvent*>(ev)->ready_ns.load(std::memory_order_acquire) ? hipSuccess
                                                                                                  : hipErrorNotReady;
}

hipError_t hipEventDestroy(hipEvent_t ev) {
  delete reinterpret_cast<FakeEvent*>(ev);
  return hipSuccess;
}

#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      fprintf(stderr, "CHECK failed line %d: %s\n", __LINE__, #c); \
      return 1;                                                    \
    }                                                              \
  } while (0)

static int run_mode(int rows, int nslots, int clients, int iters) {
  std::vector<FakeProg*> progs;
  std::vector<std::vector<int32_t>> ins(nslots), outs(nslots);
  std::vector<HzProgram> hp;
  std::vector<hipStream_t> streams(nslots, nullptr);
  std::vector<void*> host_in, host_out;
  for (int i = 0; i < nslots; ++i) {
    ins[i].assign(rows * kInts, 0);
    outs[i].assign(rows * kInts, 0);
    auto* p = new FakeProg();
    p->in = ins[i].data();
    p->out = outs[i].data();
    p->rows = rows;
    progs.push_back(p);
    hp.push_back(p);
    host_in.push_back(ins[i].data());
    host_out.push_back(outs[i].data());
  }
  const uint64_t in_bytes = (uint64_t)rows * kInts * 4, out_bytes = in_bytes;
  void* ex = rows == 1 ? hz_exec_create(hp.data(), streams.data(), host_in.data(), &in_bytes, 1, host_out.data(),
                                        out_bytes, nslots)
                       : hz_exec_create_batched(hp.data(), streams.data(), host_in.data(), &in_bytes, 1,
                                                host_out.data(), out_bytes, nslots, rows, 50.0, 1);
  CHECK(ex != nullptr);
  if (rows > 1) {  // argument checks of the multi-row entry point
    int32_t dummy[kInts * 8] = {};
    const void* in1[1] = {dummy};
    CHECK(hz_exec_submit_rows(ex, in1, 0, dummy, nullptr) == -1);
    CHECK(hz_exec_submit_rows(ex, in1, rows + 1, dummy, nullptr) == -1);
  }
  std::atomic<int> bad{0};
  std::atomic<uint64_t> rows_sent{0};
  std::vector<std::thread> th;
  for (int c = 0; c < clients; ++c)
    th.emplace_back([&, c] {
      std::vector<int32_t> in(rows * kInts), out(rows * kInts);
      for (int it = 0; it < iters; ++it) {
        // batched executors: every third request of odd clients carries several rows
        const int m = (rows > 1 && (c & 1) && it % 3 == 0) ? 1 + (c + it) % rows : 1;
        for (int r = 0; r < m; ++r)
          for (int e = 0; e < kInts; ++e) in[r * kInts + e] = c * 1000003 + it * 131 + r * 17 + e;
        std::fill(out.begin(), out.end(), -1);
        const void* ip[1] = {in.data()};
        double lat = 0;
        const int rc = m > 1 ? hz_exec_submit_rows(ex, ip, m, out.data(), &lat) : hz_exec_submit(ex, ip, out.data(), &lat);
        if (rc) {
          bad.fetch_add(1);
          continue;
        }
        rows_sent.fetch_add(m);
        const int nrow = rows == 1 ? 1 : m;
        for (int r = 0; r < nrow; ++r)
          for (int e = 0; e < kInts; ++e)
            if (out[r * kInts + e] != f(in[r * kInts + e], e)) bad.fetch_add(1);
        if (lat < 0) bad.fetch_add(1);
      }
    });
  for (auto& t : th) t.join();
  CHECK(bad.load() == 0);
  uint64_t served = 0, polls = 0, batches = 0;
  hz_exec_stats(ex, &served, &polls);
  hz_exec_batches(ex, &batches);
  CHECK(served == rows_sent.load());
  CHECK(batches >= 1 && batches <= served);
  if (rows == 1) {  // the native closed-loop bench over the same executor
    std::vector<int32_t> in(kInts, 5);
    const void* ip[1] = {in.data()};
    std::vector<double> lat(4 * 50);
    double wall = 0;
    CHECK(hz_exec_bench(ex, 4, 50, ip, lat.data(), &wall) == 0 && wall > 0);
  }
  hz_exec_destroy(ex);
  int replays = 0;
  for (auto* p : progs) {
    replays += p->replays.load();
    delete p;
  }
  CHECK((uint64_t)replays >= batches);
  printf("mode rows=%d slots=%d: %llu rows in %llu replays\n", rows, nslots, (unsigned long long)served,
         (unsigned long long)batches);
  return 0;
}

int main() {
  if (run_mode(1, 3, 8, 300)) return 1;
  if (run_mode(4, 2, 8, 300)) return 1;
  if (run_mode(4, 1, 6, 200)) return 1;  // one slot: every chunk waits for the previous batch
  printf("executor host sanitize: ok\n");
  return 0;
}
