// Batched-decode scheduler for the AWD-LSTM text endpoint (GET /inference; the kernels are
// csrc/lmbatch.hip). Continuous batching at replay granularity:
//   request thread  hz_lmb_submit: queue the request, sleep on its condition variable
//   worker thread   the only thread touching HIP: before each replay it admits waiting requests
//                   into free rows and writes the replay's control block (per row and sub-step:
//                   forced prompt token / sample / idle, output index, noise step, logits record)
//                   into pinned memory, replays the captured U-step program (its first node, the
//                   admit kernel, copies the block to the device and zeroes admitted rows' state),
//                   waits for the replay's event, then hands finished rows' tokens back.
// A request of P prompt tokens and n words occupies its row for P + n sub-steps (its last token
// is chosen at sub-step P + n - 1); rows are refilled at the next replay boundary, so a request
// waits at most one replay (U steps) to join.
// Low load: with a second program captured for the first row block only (hz_lmb_set_lowload), a
// replay whose busy rows are all below lo_rows runs that one instead: the same per-row arithmetic
// (a row's tokens never depend on the program), half the state traffic and MFMAs at Bp = 32.
// Requests take the lowest free row, so a lone request always qualifies.
#include <hip/hip_runtime.h>

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "hipzap.h"

namespace {

double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Req {
  const int* prompt;
  int P, n;
  unsigned long long seed;
  int* out;
  float* logits_out;
  int t = 0;  // sub-steps run so far
  bool done = false;
  int rc = 0;
  std::condition_variable cv;
};

struct Sched {
  HzProgram prog;
  HzProgram lo = nullptr;  // low-load program (rows < lo_rows only) or null
  int lo_rows = 0;
  hipStream_t st;
  hipEvent_t ev = nullptr;
  int* block;
  int Bp, U, maxp, maxn, V;
  int* out_pool;   // pinned [Bp][maxn]: where the kernels write each row's tokens
  float* logits;   // pinned [Bp][V] or null
  std::mutex mu;
  std::condition_variable cv_work;
  std::deque<Req*> waiting;
  std::vector<Req*> rows;
  int busy = 0;
  bool stop = false;
  std::thread worker;
  long long gstep = 0;
  unsigned long long replays = 0, served = 0, used = 0, offered = 0, lo_replays = 0;

  int row_stride() const { return 8 + 4 * U; }

  void write_block(const std::vector<char>& admitted) {
    block[0] = (int)(gstep & 1);
    for (int r = 0; r < Bp; ++r) {
      int* b = block + 8 + (size_t)r * row_stride();
      Req* q = rows[r];
      b[0] = admitted[r] ? 1 : 0;
      const unsigned long long seed = q ? q->seed : 0ull;
      const unsigned long long op = reinterpret_cast<unsigned long long>(out_pool + (size_t)r * maxn);
      b[1] = (int)(unsigned)seed;
      b[2] = (int)(unsigned)(seed >> 32);
      b[3] = (int)(unsigned)op;
      b[4] = (int)(unsigned)(op >> 32);
      HzLmbCtl* c = reinterpret_cast<HzLmbCtl*>(b + 8);
      for (int u = 0; u < U; ++u) {
        HzLmbCtl e{-2, -1, -1, 0};
        if (q) {
          const int t = q->t + u, total = q->P + q->n;
          if (t < q->P) e.tok = q->prompt[t];
          else if (t < total) e.tok = -1, e.out = t - q->P;
          if (t + 1 >= q->P && t + 1 < total) e.dec_t = t;
          if (q->logits_out && logits && t == q->P - 1) e.rec = 1;
        }
        c[u] = e;
      }
    }
  }

  void run() {
    std::vector<char> admitted(Bp, 0);
    for (;;) {
      bool low = false;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv_work.wait(lk, [&] { return stop || !waiting.empty() || busy > 0; });
        if (stop && busy == 0) {
          for (Req* q : waiting) {
            q->rc = -10;
            q->done = true;
            q->cv.notify_all();
          }
          waiting.clear();
          return;
        }
        for (int r = 0; r < Bp; ++r) {
          admitted[r] = 0;
          if (!rows[r] && !waiting.empty() && !stop) {
            rows[r] = waiting.front();
            waiting.pop_front();
            rows[r]->t = 0;
            admitted[r] = 1;
            ++busy;
          }
        }
        low = lo != nullptr;
        for (int r = lo_rows; low && r < Bp; ++r) low = rows[r] == nullptr;
      }
      write_block(admitted);
      int rc = hz_prog_replay(low ? lo : prog, st);
      lo_replays += low;
      if (!rc) rc = (int)hipEventRecord(ev, st);
      if (!rc) {
        for (;;) {
          const hipError_t q = hipEventQuery(ev);
          if (q == hipSuccess) break;
          if (q != hipErrorNotReady) {
            rc = (int)q;
            break;
          }
          std::this_thread::yield();
        }
      }
      gstep += U;
      ++replays;
      offered += (unsigned long long)Bp * U;
      std::lock_guard<std::mutex> g(mu);
      for (int r = 0; r < Bp; ++r) {
        Req* q = rows[r];
        if (!q) continue;
        const int total = q->P + q->n;
        used += (unsigned long long)std::max(0, std::min(U, total - q->t));
        q->t += U;
        if (q->t < total && !rc) continue;
        if (!rc) {
          std::memcpy(q->out, out_pool + (size_t)r * maxn, sizeof(int) * (size_t)q->n);
          if (q->logits_out) std::memcpy(q->logits_out, logits + (size_t)r * V, sizeof(float) * (size_t)V);
        }
        q->rc = rc;
        q->done = true;
        q->cv.notify_all();
        rows[r] = nullptr;
        --busy;
        ++served;
      }
    }
  }
};

}  // namespace

extern "C" {

void* hz_lmb_create(HzProgram prog, hipStream_t st, int* host_block, int Bp, int U, int maxp, int maxn, int* out_pool,
                    float* logits, int V) {
  if (!prog || !host_block || !out_pool || Bp < 1 || U < 1 || U > HZ_LMB_MAXU || maxn < 1 || V < 1) return nullptr;
  auto* s = new Sched();
  s->prog = prog;
  s->st = st;
  s->block = host_block;
  s->Bp = Bp;
  s->U = U;
  s->maxp = maxp;
  s->maxn = maxn;
  s->V = V;
  s->out_pool = out_pool;
  s->logits = logits;
  s->rows.assign(Bp, nullptr);
  if (hipEventCreateWithFlags(&s->ev, hipEventDisableTiming) != hipSuccess) {
    delete s;
    return nullptr;
  }
  s->worker = std::thread([s] { s->run(); });
  return s;
}

// blocking: prompt[P] token ids, n words -> out[n]; logits_out (optional, [V]): the logits after
// the last prompt token (needs an engine built with a logits buffer); lat_us: submit -> done
int hz_lmb_submit(void* h, const int* prompt, int P, int n, unsigned long long seed, int* out, float* logits_out,
                  double* lat_us) {
  auto* s = static_cast<Sched*>(h);
  if (!s || !prompt || P < 1 || n < 1 || n > s->maxn || !out) return -1;
  const double t0 = now_us();
  Req q;
  q.prompt = prompt;
  q.P = P;
  q.n = n;
  q.seed = seed;
  q.out = out;
  q.logits_out = logits_out;
  std::unique_lock<std::mutex> lk(s->mu);
  if (s->stop) return -10;
  s->waiting.push_back(&q);
  s->cv_work.notify_one();
  q.cv.wait(lk, [&] { return q.done; });
  if (lat_us) *lat_us = now_us() - t0;
  return q.rc;
}

// optional low-load program over the same buffers (kernels with nb_act = rows / 16); call before
// the first submit
int hz_lmb_set_lowload(void* h, HzProgram lo, int rows) {
  auto* s = static_cast<Sched*>(h);
  if (!s || (lo && (rows < 16 || rows % 16 || rows >= s->Bp))) return -1;
  std::lock_guard<std::mutex> g(s->mu);
  s->lo = lo;
  s->lo_rows = lo ? rows : 0;
  return 0;
}

unsigned long long hz_lmb_lo_replays(void* h) {
  auto* s = static_cast<Sched*>(h);
  std::lock_guard<std::mutex> g(s->mu);
  return s->lo_replays;
}

void hz_lmb_stats(void* h, unsigned long long* out4) {
  auto* s = static_cast<Sched*>(h);
  std::lock_guard<std::mutex> g(s->mu);
  out4[0] = s->replays;
  out4[1] = s->served;
  out4[2] = s->used;
  out4[3] = s->offered;
}

// finishes the requests already in rows, fails the ones still waiting, joins the worker
void hz_lmb_destroy(void* h) {
  auto* s = static_cast<Sched*>(h);
  if (!s) return;
  {
    std::lock_guard<std::mutex> g(s->mu);
    s->stop = true;
  }
  s->cv_work.notify_all();
  if (s->worker.joinable()) s->worker.join();
  if (s->ev) (void)hipEventDestroy(s->ev);
  delete s;
}

}  // extern "C"
