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
// waits at most one replay (U steps) to join (two with the pipelined pair of programs).
// Low load: with a second program captured for the first row block only (hz_lmb_set_lowload), a
// replay whose busy rows are all below lo_rows runs that one instead: the same per-row arithmetic
// (a row's tokens never depend on the program), half the state traffic and MFMAs at Bp = 32.
// Requests take the lowest free row, so a lone request always qualifies. One request: with the
// programs of hz_lmb_set_solo (kernels with nb_act = -1), a replay whose only busy row is row 0
// reads and writes that row's state alone (bitwise the same tokens).
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
  int t = 0;                 // sub-steps issued so far
  int row = -1, slot = 0;    // row and output slot (alternating per row admission)
  long long last_seq = -1;   // replay that issued the last sub-step
  long long rec_seq = -1;    // replay that recorded the logits (after the last prompt token)
  int rec_k = 0;             // its program index (logits buffer)
  bool done = false;
  int rc = 0;
  std::condition_variable cv;
};

struct Flight {
  long long seq;
  int k;   // program / block index
  int rc;  // launch status
};

struct Sched {
  HzProgram prog[2] = {nullptr, nullptr};
  HzProgram lo[2] = {nullptr, nullptr};  // low-load programs (rows < lo_rows only) or null
  HzProgram solo[2] = {nullptr, nullptr};  // one-request programs (row 0 only) or null
  int nprog = 1, lo_rows = 0;
  hipStream_t st;
  hipEvent_t ev[2] = {nullptr, nullptr};
  int* block[2] = {nullptr, nullptr};
  int Bp, U, maxp, maxn, V;
  int* out_pool;       // pinned [2 slots][Bp][maxn]: where the kernels write each row's tokens
  float* logits[2];    // pinned [Bp][V] per program, or null
  std::mutex mu;
  std::condition_variable cv_work;
  std::deque<Req*> waiting;
  std::vector<Req*> rows;   // worker thread only
  std::vector<int> slot_of; // next output slot per row (worker thread only)
  int busy = 0;             // rows holding a request with sub-steps still to issue
  bool stop = false;
  std::thread worker;
  unsigned long long replays = 0, served = 0, used = 0, offered = 0, lo_replays = 0, solo_replays = 0;

  int row_stride() const { return 8 + 4 * U; }

  void write_block(int k, long long gstep, const std::vector<char>& admitted) {
    int* blk = block[k];
    blk[0] = (int)(gstep & 1);
    for (int r = 0; r < Bp; ++r) {
      int* b = blk + 8 + (size_t)r * row_stride();
      Req* q = rows[r];
      b[0] = admitted[r] ? 1 : 0;
      const unsigned long long seed = q ? q->seed : 0ull;
      const unsigned long long op =
          reinterpret_cast<unsigned long long>(out_pool + ((size_t)(q ? q->slot : 0) * Bp + r) * maxn);
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
          if (q->logits_out && logits[k] && t == q->P - 1) e.rec = 1;
        }
        c[u] = e;
      }
    }
  }

  hipError_t wait_event(hipEvent_t e) {
    for (;;) {
      const hipError_t q = hipEventQuery(e);
      if (q != hipErrorNotReady) return q;
      std::this_thread::yield();
    }
  }

  // Pipelined with two programs (nprog = 2): replay k + 1 is launched while replay k runs (each
  // program's admit kernel reads its own host block, so the next block is written while the
  // GPU works), and the worker only waits when two replays are in flight. Rows are handed out
  // when their request's last sub-step is ISSUED; outputs go to alternating per-row slots and are
  // copied when the replay that wrote them completes -- before the slot's next user can run,
  // because a launch needs the replay two back completed. nprog = 1: launch, wait, repeat.
  void run() {
    std::vector<char> admitted(Bp, 0);
    std::deque<Flight> inflight;
    std::vector<Req*> pending;  // every sub-step issued, outputs not yet collected
    long long seq = 0, gstep = 0;
    int next_k = 0;
    for (;;) {
      bool launch = false, low = false, one = false;
      {
        std::unique_lock<std::mutex> lk(mu);
        if (inflight.empty() && busy == 0) {
          cv_work.wait(lk, [&] { return stop || !waiting.empty(); });
          if (stop) {
            for (Req* q : waiting) {
              q->rc = -10;
              q->done = true;
              q->cv.notify_all();
            }
            waiting.clear();
            return;
          }
        }
        if ((int)inflight.size() < nprog) {
          for (int r = 0; r < Bp; ++r) {
            admitted[r] = 0;
            if (!rows[r] && !waiting.empty() && !stop) {
              Req* q = waiting.front();
              waiting.pop_front();
              q->t = 0;
              q->row = r;
              q->slot = slot_of[r];
              slot_of[r] ^= 1;
              rows[r] = q;
              admitted[r] = 1;
              ++busy;
            }
          }
          launch = busy > 0;
          low = launch && lo[next_k] != nullptr;
          for (int r = lo_rows; low && r < Bp; ++r) low = rows[r] == nullptr;
          one = launch && solo[next_k] != nullptr && rows[0] != nullptr;
          for (int r = 1; one && r < Bp; ++r) one = rows[r] == nullptr;
        }
      }
      if (launch) {
        const int k = next_k;
        write_block(k, gstep, admitted);
        int rc = hz_prog_replay(one ? solo[k] : low ? lo[k] : prog[k], st);
        if (!rc) rc = (int)hipEventRecord(ev[k], st);
        std::lock_guard<std::mutex> g(mu);
        lo_replays += low && !one;
        solo_replays += one;
        ++replays;
        offered += (unsigned long long)Bp * U;
        for (int r = 0; r < Bp; ++r) {
          Req* q = rows[r];
          if (!q) continue;
          const int total = q->P + q->n;
          used += (unsigned long long)std::max(0, std::min(U, total - q->t));
          if (q->logits_out && logits[k] && q->P - 1 >= q->t && q->P - 1 < q->t + U) q->rec_seq = seq, q->rec_k = k;
          q->t += U;
          if (q->t >= total || rc) {  // every sub-step issued (or the launch failed): free the row
            q->last_seq = seq;
            pending.push_back(q);
            rows[r] = nullptr;
            --busy;
          }
        }
        inflight.push_back({seq, k, rc});
        ++seq;
        gstep += U;
        next_k = nprog == 2 ? k ^ 1 : 0;
        if ((int)inflight.size() < nprog) continue;  // launch the next replay before waiting
      }
      if (inflight.empty()) continue;
      const Flight f = inflight.front();
      inflight.pop_front();
      int rc = f.rc;
      if (!rc) rc = (int)wait_event(ev[f.k]);
      std::lock_guard<std::mutex> g(mu);
      auto collect_logits = [&](Req* q) {
        if (q->rec_seq == f.seq && !rc)
          std::memcpy(q->logits_out, logits[q->rec_k] + (size_t)q->row * V, sizeof(float) * (size_t)V);
      };
      for (Req* q : rows)
        if (q) collect_logits(q);
      for (size_t i = 0; i < pending.size();) {
        Req* q = pending[i];
        collect_logits(q);
        if (q->last_seq != f.seq) {
          ++i;
          continue;
        }
        if (!rc) std::memcpy(q->out, out_pool + ((size_t)q->slot * Bp + q->row) * maxn, sizeof(int) * (size_t)q->n);
        q->rc = rc;
        q->done = true;
        q->cv.notify_all();
        ++served;
        pending[i] = pending.back();
        pending.pop_back();
      }
      if (rc) {  // a failed replay fails every request still in a row as well
        for (int r = 0; r < Bp; ++r) {
          Req* q = rows[r];
          if (!q) continue;
          q->rc = rc;
          q->done = true;
          q->cv.notify_all();
          rows[r] = nullptr;
          --busy;
        }
      }
    }
  }
};

}  // namespace

extern "C" {

// progs[k] (k < nprog, nprog 1 or 2): the captured U-step program whose admit kernel reads
// blocks[k] and whose decoder records logits into logits[k] (or null); out_pool: pinned
// [2][Bp][maxn]
void* hz_lmb_create(const HzProgram* progs, int nprog, hipStream_t st, int* const* blocks, int Bp, int U, int maxp,
                    int maxn, int* out_pool, float* const* logits, int V) {
  if (!progs || !blocks || (nprog != 1 && nprog != 2) || !out_pool || Bp < 1 || U < 1 || U > HZ_LMB_MAXU ||
      maxn < 1 || V < 1)
    return nullptr;
  for (int k = 0; k < nprog; ++k)
    if (!progs[k] || !blocks[k]) return nullptr;
  auto* s = new Sched();
  s->nprog = nprog;
  s->st = st;
  for (int k = 0; k < nprog; ++k) {
    s->prog[k] = progs[k];
    s->block[k] = blocks[k];
    s->logits[k] = logits ? logits[k] : nullptr;
  }
  if (nprog == 1) s->logits[1] = nullptr;
  s->Bp = Bp;
  s->U = U;
  s->maxp = maxp;
  s->maxn = maxn;
  s->V = V;
  s->out_pool = out_pool;
  s->rows.assign(Bp, nullptr);
  s->slot_of.assign(Bp, 0);
  for (int k = 0; k < nprog; ++k)
    if (hipEventCreateWithFlags(&s->ev[k], hipEventDisableTiming) != hipSuccess) {
      for (int j = 0; j < k; ++j) (void)hipEventDestroy(s->ev[j]);
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
  if (logits_out && !s->logits[0]) return -1;
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

// optional low-load programs over the same buffers (kernels with nb_act = rows / 16), one per
// program of hz_lmb_create; call before the first submit
int hz_lmb_set_lowload(void* h, const HzProgram* lo, int rows) {
  auto* s = static_cast<Sched*>(h);
  if (!s || (lo && (rows < 16 || rows % 16 || rows >= s->Bp))) return -1;
  std::lock_guard<std::mutex> g(s->mu);
  for (int k = 0; k < s->nprog; ++k) s->lo[k] = lo ? lo[k] : nullptr;
  s->lo_rows = lo ? rows : 0;
  return 0;
}

// optional one-request programs over the same buffers (kernels with nb_act = -1), one per
// program of hz_lmb_create; call before the first submit
int hz_lmb_set_solo(void* h, const HzProgram* solo) {
  auto* s = static_cast<Sched*>(h);
  if (!s) return -1;
  std::lock_guard<std::mutex> g(s->mu);
  for (int k = 0; k < s->nprog; ++k) s->solo[k] = solo ? solo[k] : nullptr;
  return 0;
}

unsigned long long hz_lmb_solo_replays(void* h) {
  auto* s = static_cast<Sched*>(h);
  std::lock_guard<std::mutex> g(s->mu);
  return s->solo_replays;
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
  for (int k = 0; k < 2; ++k)
    if (s->ev[k]) (void)hipEventDestroy(s->ev[k]);
  delete s;
}

}  // extern "C"
