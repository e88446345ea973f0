// Host-side sanitizer check of the batched-decode scheduler (csrc/lmserve.cpp): continuous
// batching, the pipelined pair of programs (host blocks written while the other replay runs,
// alternating per-row output slots), the low-load and one-request program switches and teardown, under
// AddressSanitizer+UBSan or ThreadSanitizer (tests/test_native_asan_cpu.py builds it both ways).
//
// No GPU: hz_prog_replay and the HIP event calls are defined here. A fake "GPU" thread executes the
// queued replays IN ORDER with a small delay, reading the program's host block only when the
// replay runs (as the admit kernel does) and writing each sampled token through the row's output
// pointer from that block: out[i] = token(seed, i). So a block rewritten while its replay is still
// queued, an output slot reused before it was collected, or a result read before its replay ran
// shows up as a wrong token, and every unsynchronised access is a TSan report.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <deque>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#include "hipzap.h"

namespace {

constexpr int kV = 64;  // vocabulary of the fake decoder (logits rows)

struct FakeProg {
  const int* block;
  float* logits;  // [Bp][kV] or null
  int Bp, U;
  bool low;
  bool solo = false;
};

struct FakeEvent {
  bool done = false;
};

// the fake device: a queue of replays and event markers, executed by one thread in order
struct FakeGpu {
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::pair<FakeProg*, FakeEvent*>> q;  // (prog, null) or (null, event)
  bool stop = false;
  std::thread th;
  std::atomic<long> replays{0}, low_replays{0};

  void start() {
    th = std::thread([this] {
      for (;;) {
        std::pair<FakeProg*, FakeEvent*> item;
        {
          std::unique_lock<std::mutex> lk(mu);
          cv.wait(lk, [&] { return stop || !q.empty(); });
          if (q.empty()) return;
          item = q.front();
        }
        if (item.first) {
          std::this_thread::sleep_for(std::chrono::microseconds(30));
          execute(item.first);
        }
        std::lock_guard<std::mutex> g(mu);
        if (item.second) item.second->done = true;
        q.pop_front();
      }
    });
  }
  void halt() {
    {
      std::lock_guard<std::mutex> g(mu);
      stop = true;
    }
    cv.notify_all();
    th.join();
  }
  void execute(FakeProg* p) {
    replays.fetch_add(1);
    if (p->low) low_replays.fetch_add(1);
    const int rs = 8 + 4 * p->U;
    for (int r = 0; r < p->Bp; ++r) {
      const int* b = p->block + 8 + (size_t)r * rs;
      const unsigned long long seed = (unsigned long long)(unsigned)b[1] | ((unsigned long long)(unsigned)b[2] << 32);
      int* outp = reinterpret_cast<int*>((unsigned long long)(unsigned)b[3] | ((unsigned long long)(unsigned)b[4] << 32));
      const HzLmbCtl* c = reinterpret_cast<const HzLmbCtl*>(b + 8);
      for (int u = 0; u < p->U; ++u) {
        if (c[u].tok == -2) continue;
        if (p->low && r >= 16) {  // the low-load program computes rows < 16 only
          fprintf(stderr, "low-load replay with a busy row %d\n", r);
          abort();
        }
        if (p->solo && r != 0) {  // the one-request program computes row 0 only
          fprintf(stderr, "one-request replay with a busy row %d\n", r);
          abort();
        }
        if (c[u].tok == -1 && c[u].out >= 0) outp[c[u].out] = (int)((seed * 2654435761ull + c[u].out * 97ull) % 100003ull);
        if (c[u].rec && p->logits)
          for (int v = 0; v < kV; ++v) p->logits[(size_t)r * kV + v] = (float)((seed + v) % 1009);
      }
    }
  }
};

FakeGpu g_gpu;

unsigned token(unsigned long long seed, int i) { return (unsigned)((seed * 2654435761ull + i * 97ull) % 100003ull); }

}  // namespace

extern "C" int hz_prog_replay(HzProgram p, hipStream_t) {
  std::lock_guard<std::mutex> g(g_gpu.mu);
  g_gpu.q.push_back({static_cast<FakeProg*>(p), nullptr});
  g_gpu.cv.notify_all();
  return 0;
}

hipError_t hipEventCreateWithFlags(hipEvent_t* ev, unsigned) {
  *ev = reinterpret_cast<hipEvent_t>(new FakeEvent());
  return hipSuccess;
}

hipError_t hipEventRecord(hipEvent_t ev, hipStream_t) {
  std::lock_guard<std::mutex> g(g_gpu.mu);
  auto* e = reinterpret_cast<FakeEvent*>(ev);
  e->done = false;
  g_gpu.q.push_back({nullptr, e});
  g_gpu.cv.notify_all();
  return hipSuccess;
}

hipError_t hipEventQuery(hipEvent_t ev) {
  std::lock_guard<std::mutex> g(g_gpu.mu);
  return reinterpret_cast<FakeEvent*>(ev)->done ? hipSuccess : hipErrorNotReady;
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

static int run_mode(int nprog, bool lowload, int clients, int iters, bool solo = false) {
  const int Bp = 32, U = 4, maxn = 64;
  std::vector<std::vector<int>> blocks(2, std::vector<int>(8 + Bp * (8 + 4 * U), 0));
  std::vector<int> out_pool(2 * Bp * maxn, 0);
  std::vector<std::vector<float>> logits(2, std::vector<float>(Bp * kV, 0.f));
  FakeProg progs[2], lo[2], so[2];
  HzProgram hp[2] = {nullptr, nullptr}, hl[2] = {nullptr, nullptr}, hs[2] = {nullptr, nullptr};
  int* bl[2] = {nullptr, nullptr};
  float* lg[2] = {nullptr, nullptr};
  for (int k = 0; k < nprog; ++k) {
    progs[k] = FakeProg{blocks[k].data(), logits[k].data(), Bp, U, false};
    lo[k] = FakeProg{blocks[k].data(), logits[k].data(), Bp, U, true};
    so[k] = FakeProg{blocks[k].data(), logits[k].data(), Bp, U, false, true};
    hp[k] = &progs[k];
    hl[k] = &lo[k];
    hs[k] = &so[k];
    bl[k] = blocks[k].data();
    lg[k] = logits[k].data();
  }
  CHECK(hz_lmb_create(hp, 3, nullptr, bl, Bp, U, 0, maxn, out_pool.data(), lg, kV) == nullptr);  // argument checks
  void* s = hz_lmb_create(hp, nprog, nullptr, bl, Bp, U, 0, maxn, out_pool.data(), lg, kV);
  CHECK(s != nullptr);
  if (lowload) CHECK(hz_lmb_set_lowload(s, hl, 16) == 0);
  if (solo) CHECK(hz_lmb_set_solo(s, hs) == 0);
  std::atomic<int> bad{0};
  std::vector<std::thread> th;
  for (int c = 0; c < clients; ++c)
    th.emplace_back([&, c] {
      std::mt19937 rng(c * 7919 + nprog);
      for (int it = 0; it < iters; ++it) {
        const int P = 1 + (int)(rng() % 5), n = 1 + (int)(rng() % maxn);
        std::vector<int> prompt(P, 3), out(n, -1);
        const unsigned long long seed = ((unsigned long long)c << 32) | (unsigned)it;
        std::vector<float> lgo(kV, -1.f);
        const bool want_logits = (it % 3) == 0;
        double lat = 0;
        const int rc = hz_lmb_submit(s, prompt.data(), P, n, seed, out.data(), want_logits ? lgo.data() : nullptr, &lat);
        if (rc) {
          bad.fetch_add(1);
          continue;
        }
        for (int i = 0; i < n; ++i)
          if ((unsigned)out[i] != token(seed, i)) bad.fetch_add(1);
        if (want_logits)
          for (int v = 0; v < kV; ++v)
            if (lgo[v] != (float)((seed + v) % 1009)) bad.fetch_add(1);
        if (c == 0 && (it & 7) == 0) std::this_thread::sleep_for(std::chrono::microseconds(200));  // load swings
      }
    });
  for (auto& t : th) t.join();
  unsigned long long st[4];
  hz_lmb_stats(s, st);
  const unsigned long long lo_rep = hz_lmb_lo_replays(s), solo_rep = hz_lmb_solo_replays(s);
  hz_lmb_destroy(s);
  CHECK(bad.load() == 0);
  CHECK(st[1] == (unsigned long long)clients * iters);
  CHECK(st[2] <= st[3]);
  if (lowload && clients > 1) CHECK(lo_rep > 0 && lo_rep < st[0]);
  if (!lowload) CHECK(lo_rep == 0);
  if (solo && clients == 1) CHECK(solo_rep == st[0]);  // a lone client always sits in row 0
  if (!solo) CHECK(solo_rep == 0);
  printf("mode nprog=%d lowload=%d solo=%d clients=%d: replays %llu served %llu low %llu solo %llu\n", nprog,
         (int)lowload, (int)solo, clients, st[0], st[1], lo_rep, solo_rep);
  return 0;
}

int main() {
  g_gpu.start();
  int rc = 0;
  for (int nprog : {1, 2})
    for (bool lowload : {false, true})
      if (!rc) rc = run_mode(nprog, lowload, lowload ? 40 : 12, 25);
  for (int nprog : {1, 2}) {  // the one-request program: alone, then under concurrency
    if (!rc) rc = run_mode(nprog, true, 1, 20, true);
    if (!rc) rc = run_mode(nprog, true, 24, 15, true);
  }
  // a lone client mostly runs the low-load program
  g_gpu.halt();
  if (rc) return rc;
  printf("lmserve host sanitize: ok\n");
  return 0;
}
