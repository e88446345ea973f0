// hipzap request executor: the serving scheduler between request threads and the GPU.
//
// Measured problem (profiles/r2_serving): 32 request threads that each hipGraphLaunch +
// hipStreamSynchronize their own context contend inside the HIP runtime (spin-waiting
// synchronisation, submission locks): 5.5k inf/s closed-loop with a 58 ms p99, against 10.4k
// when one thread queues the same replays back to back. The executor keeps that shape:
//   request thread  take a free context slot -> copy its payload into the slot's pinned input
//                   -> queue the slot -> sleep on the slot's condition variable -> copy the
//                   result out of the pinned output -> release the slot
//   worker thread   the ONLY thread that touches HIP on the request path: launches queued
//                   slots (one hipGraphLaunch + one event record each) and polls the in-flight
//                   slots' completion events, waking each request as its replay finishes
// Host copies are spread over the request threads; submissions are serialised on one thread
// (which is how the pipelined device ceiling was measured); request threads never spin.
//
// Dynamic batching (hz_exec_create_batched): the contexts are captured at batch B and every
// request is still ONE image. Request threads claim a row of the single OPEN slot (opening a free
// slot if none is open), copy their payload into that row of its pinned input and wait; the slot
// is sealed when its B rows are claimed, or by the worker as soon as fewer than `min_inflight`
// batches are on the GPU or the slot has been open `max_wait_us`. A sealed slot is launched once
// its last claimed row has been copied; each request copies its own output row out and the
// slot is freed when every claimed row has been read. Unclaimed rows of a partial batch hold stale
// inputs whose outputs nobody reads. At batch 8-16 the conv layers run on the LDS-tiled implicit
// GEMM (gemm.hip CV mode), so one batched replay costs far less than B single-image replays.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "hipzap.h"

namespace {

constexpr int kMaxIn = 4;

double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Slot {
  HzProgram prog = nullptr;
  hipStream_t st = nullptr;
  void* in[kMaxIn] = {};
  void* out = nullptr;
  hipEvent_t ev = nullptr;
  bool done = false;
  std::atomic<bool> done_a{false};  // = done, for the low-load spin of submit_one (set after rc)
  int rc = 0;
  std::condition_variable cv;
  // dynamic batching: rows claimed / payloads copied / outputs read; sealed = no more rows
  int claimed = 0, copied = 0, read = 0;
  bool sealed = false;
  double t_open = 0;
};

struct Exec {
  std::vector<Slot> slots;
  int n_in = 1;
  uint64_t in_bytes[kMaxIn] = {};
  uint64_t out_bytes = 0;
  std::mutex mu;
  std::condition_variable cv_free, cv_work;
  std::vector<int> free_slots;
  std::deque<int> to_launch;
  std::vector<int> inflight;  // worker-owned
  bool stop = false;
  int active = 0;  // request threads inside submit_wait: the worker outlives every one of them
  std::thread worker;
  uint64_t served = 0, polls = 0, batches = 0;
  // dynamic batching (rows > 1)
  int rows = 1, open = -1, min_inflight = 1;
  double max_wait_us = 0;
  uint64_t row_in[kMaxIn] = {};
  uint64_t row_out = 0;
  // low load (HIPZAP_EXEC_SPIN_US, default 300; 0 = off): an idle worker polls for new work and a
  // request thread that is alone (or one of two) polls for its completion for up to this long
  // before sleeping on a condition variable -- two futex wake-ups off a single request's latency.
  // Under load nobody spins: the worker always has replays in flight and requesters sleep.
  double spin_us = 300.0;
  std::atomic<int> work_hint{0};  // bumped whenever work is queued for the worker

  void complete(int s, int rc) {
    std::lock_guard<std::mutex> g(mu);
    slots[s].rc = rc;
    slots[s].done = true;
    slots[s].done_a.store(true, std::memory_order_release);
    slots[s].cv.notify_all();
    served += rows == 1 ? 1 : slots[s].claimed;
    ++batches;
  }

  // mu held: a sealed slot whose claimed rows are all copied goes to the launch queue
  void queue_if_ready(int s) {
    Slot& sl = slots[s];
    if (sl.sealed && sl.copied == sl.claimed) {
      to_launch.push_back(s);
      work_hint.fetch_add(1, std::memory_order_release);
      cv_work.notify_one();
    }
  }

  // mu held
  void seal_open() {
    const int s = open;
    open = -1;
    slots[s].sealed = true;
    queue_if_ready(s);
  }

  void run() {
    std::vector<int> launch;
    double last_busy = now_us();
    for (;;) {
      if (inflight.empty() && spin_us > 0 && now_us() - last_busy < spin_us) {
        // idle but recently busy: poll for new work without the lock instead of sleeping
        const int h0 = work_hint.load(std::memory_order_acquire);
        bool empty;
        {
          std::lock_guard<std::mutex> g(mu);
          empty = to_launch.empty() && open < 0 && !stop;
        }
        while (empty && work_hint.load(std::memory_order_acquire) == h0 && now_us() - last_busy < spin_us)
          std::this_thread::yield();
      }
      {
        std::unique_lock<std::mutex> lk(mu);
        // at shutdown a request may still be copying into a sealed slot (not yet queued): keep
        // serving until every request thread has left, so none waits on a slot nobody launches
        if (to_launch.empty() && inflight.empty())
          cv_work.wait(lk, [&] { return (stop && active == 0) || !to_launch.empty() || open >= 0; });
        if (stop && active == 0 && to_launch.empty() && inflight.empty() && open < 0) return;
        // dynamic batching: close the filling batch when the GPU is short of work or it is old
        if (open >= 0 && ((int)inflight.size() < min_inflight || stop || now_us() - slots[open].t_open >= max_wait_us))
          seal_open();
        launch.assign(to_launch.begin(), to_launch.end());
        to_launch.clear();
      }
      for (int s : launch) {
        int rc = hz_prog_replay(slots[s].prog, slots[s].st);
        if (!rc) rc = (int)hipEventRecord(slots[s].ev, slots[s].st);
        if (rc)
          complete(s, rc);
        else
          inflight.push_back(s);
      }
      bool progressed = !launch.empty();
      if (progressed || !inflight.empty()) last_busy = now_us();
      for (size_t i = 0; i < inflight.size();) {
        const int s = inflight[i];
        const hipError_t q = hipEventQuery(slots[s].ev);
        ++polls;
        if (q == hipErrorNotReady) {
          ++i;
          continue;
        }
        complete(s, q == hipSuccess ? 0 : (int)q);
        inflight[i] = inflight.back();
        inflight.pop_back();
        progressed = true;
      }
      if (!progressed) std::this_thread::yield();
    }
  }

  int submit_batched(const void* const* in, void* out, double* lat_us) {
    const double t0 = now_us();
    int s, r;
    {
      std::unique_lock<std::mutex> lk(mu);
      while (open < 0) {
        if (stop) return -10;
        if (!free_slots.empty()) {
          s = free_slots.back();
          free_slots.pop_back();
          Slot& o = slots[s];
          o.claimed = o.copied = o.read = 0;
          o.sealed = o.done = false;
          o.t_open = now_us();
          open = s;
          work_hint.fetch_add(1, std::memory_order_release);
          cv_work.notify_one();  // the worker decides when to seal
          cv_free.notify_all();  // waiting requests may join this batch
          break;
        }
        cv_free.wait(lk);
      }
      s = open;
      r = slots[s].claimed++;
      if (slots[s].claimed == rows) seal_open();
    }
    Slot& sl = slots[s];
    for (int k = 0; k < n_in; ++k)
      if (in && in[k] && row_in[k]) std::memcpy(static_cast<char*>(sl.in[k]) + r * row_in[k], in[k], row_in[k]);
    int rc;
    {
      std::unique_lock<std::mutex> lk(mu);
      ++sl.copied;
      queue_if_ready(s);
      sl.cv.wait(lk, [&] { return sl.done; });
      rc = sl.rc;
    }
    if (!rc && out && row_out) std::memcpy(out, static_cast<const char*>(sl.out) + r * row_out, row_out);
    {
      std::lock_guard<std::mutex> g(mu);
      if (++sl.read == sl.claimed) {
        free_slots.push_back(s);
        cv_free.notify_all();
      }
    }
    if (lat_us) *lat_us = now_us() - t0;
    return rc;
  }

  // m consecutive rows of one request (m <= rows) from ONE thread: each chunk claims what the open
  // slot has left, copies it, waits for that replay and reads its rows back before the next chunk
  // claims anything, so the thread never holds an unread slot while waiting for a free one
  int submit_rows(const void* const* in, int m, void* out, double* lat_us) {
    const double t0 = now_us();
    int rc = 0;
    for (int done = 0; done < m && !rc;) {
      int s, r, k;
      {
        std::unique_lock<std::mutex> lk(mu);
        while (open < 0) {
          if (stop) return -10;
          if (!free_slots.empty()) {
            s = free_slots.back();
            free_slots.pop_back();
            Slot& o = slots[s];
            o.claimed = o.copied = o.read = 0;
            o.sealed = o.done = false;
            o.t_open = now_us();
            open = s;
            work_hint.fetch_add(1, std::memory_order_release);
            cv_work.notify_one();
            cv_free.notify_all();
            break;
          }
          cv_free.wait(lk);
        }
        s = open;
        r = slots[s].claimed;
        k = std::min(m - done, rows - r);
        slots[s].claimed += k;
        if (slots[s].claimed == rows) seal_open();
      }
      Slot& sl = slots[s];
      for (int q = 0; q < n_in; ++q)
        if (in && in[q] && row_in[q])
          std::memcpy(static_cast<char*>(sl.in[q]) + r * row_in[q], static_cast<const char*>(in[q]) + done * row_in[q],
                      k * row_in[q]);
      {
        std::unique_lock<std::mutex> lk(mu);
        sl.copied += k;
        queue_if_ready(s);
        sl.cv.wait(lk, [&] { return sl.done; });
        rc = sl.rc;
      }
      if (!rc && out && row_out)
        std::memcpy(static_cast<char*>(out) + done * row_out, static_cast<const char*>(sl.out) + r * row_out, k * row_out);
      {
        std::lock_guard<std::mutex> g(mu);
        sl.read += k;
        if (sl.read == sl.claimed) {
          free_slots.push_back(s);
          cv_free.notify_all();
        }
      }
      done += k;
    }
    if (lat_us) *lat_us = now_us() - t0;
    return rc;
  }

  int submit_wait(const void* const* in, void* out, double* lat_us, int m = 1) {
    {
      std::lock_guard<std::mutex> g(mu);
      if (stop) return -10;
      ++active;
    }
    const int rc = rows > 1 ? (m > 1 ? submit_rows(in, m, out, lat_us) : submit_batched(in, out, lat_us))
                            : submit_one(in, out, lat_us);
    {
      std::lock_guard<std::mutex> g(mu);
      if (--active == 0 && stop) cv_work.notify_all();
    }
    return rc;
  }

  int submit_one(const void* const* in, void* out, double* lat_us) {
    const double t0 = now_us();
    int s;
    {
      std::unique_lock<std::mutex> lk(mu);
      cv_free.wait(lk, [&] { return stop || !free_slots.empty(); });
      if (stop) return -10;
      s = free_slots.back();
      free_slots.pop_back();
    }
    Slot& sl = slots[s];
    for (int k = 0; k < n_in; ++k)
      if (in && in[k] && in_bytes[k]) std::memcpy(sl.in[k], in[k], in_bytes[k]);
    int rc;
    bool spin;
    {
      std::unique_lock<std::mutex> lk(mu);
      sl.done = false;
      sl.done_a.store(false, std::memory_order_relaxed);
      to_launch.push_back(s);
      work_hint.fetch_add(1, std::memory_order_release);
      cv_work.notify_one();
      spin = spin_us > 0 && active <= 2;
    }
    if (spin) {  // low load: poll for the completion before sleeping
      const double ts = now_us();
      while (!sl.done_a.load(std::memory_order_acquire) && now_us() - ts < 4.0 * spin_us) std::this_thread::yield();
    }
    {
      std::unique_lock<std::mutex> lk(mu);
      sl.cv.wait(lk, [&] { return sl.done; });
      rc = sl.rc;
    }
    if (!rc && out && out_bytes) std::memcpy(out, sl.out, out_bytes);
    {
      std::lock_guard<std::mutex> g(mu);
      free_slots.push_back(s);
    }
    cv_free.notify_one();
    if (lat_us) *lat_us = now_us() - t0;
    return rc;
  }

  ~Exec() {
    {
      std::lock_guard<std::mutex> g(mu);
      stop = true;
    }
    work_hint.fetch_add(1, std::memory_order_release);
    cv_work.notify_all();
    cv_free.notify_all();
    if (worker.joinable()) worker.join();  // returns once no request thread is inside submit_wait
    for (auto& s : slots)
      if (s.ev) (void)hipEventDestroy(s.ev);
  }
};

}  // namespace

extern "C" {

// progs/streams: n bound, captured contexts; host_in[k * n + i] = context i's pinned input k;
// host_out[i] = its pinned output. The executor does not own any of them.
void* hz_exec_create(HzProgram* progs, hipStream_t* streams, void** host_in, const uint64_t* in_bytes, int n_in,
                     void** host_out, uint64_t out_bytes, int n) {
  if (n <= 0 || n_in < 0 || n_in > kMaxIn) return nullptr;
  auto* e = new Exec();
  e->slots = std::vector<Slot>(n);
  if (const char* sp = getenv("HIPZAP_EXEC_SPIN_US")) e->spin_us = atof(sp);
  e->n_in = n_in;
  for (int k = 0; k < n_in; ++k) e->in_bytes[k] = in_bytes[k];
  e->out_bytes = out_bytes;
  for (int i = 0; i < n; ++i) {
    Slot& s = e->slots[i];
    s.prog = progs[i];
    s.st = streams[i];
    for (int k = 0; k < n_in; ++k) s.in[k] = host_in[k * n + i];
    s.out = host_out[i];
    if (hipEventCreateWithFlags(&s.ev, hipEventDisableTiming) != hipSuccess) {
      delete e;
      return nullptr;
    }
    e->free_slots.push_back(n - 1 - i);  // slot 0 first
  }
  e->worker = std::thread([e] { e->run(); });
  return e;
}

// Dynamic batching over contexts captured at batch `rows`: in_bytes / out_bytes are the whole
// batch's; every request submits ONE row (in_bytes[k] / rows, out_bytes / rows).
void* hz_exec_create_batched(HzProgram* progs, hipStream_t* streams, void** host_in, const uint64_t* in_bytes,
                             int n_in, void** host_out, uint64_t out_bytes, int n, int rows, double max_wait_us,
                             int min_inflight) {
  if (rows < 1 || out_bytes % rows) return nullptr;
  for (int k = 0; k < n_in; ++k)
    if (in_bytes[k] % rows) return nullptr;
  auto* e = static_cast<Exec*>(hz_exec_create(progs, streams, host_in, in_bytes, n_in, host_out, out_bytes, n));
  if (!e) return nullptr;
  {
    std::lock_guard<std::mutex> g(e->mu);
    e->rows = rows;
    e->max_wait_us = max_wait_us;
    e->min_inflight = min_inflight;
    for (int k = 0; k < n_in; ++k) e->row_in[k] = in_bytes[k] / rows;
    e->row_out = out_bytes / rows;
  }
  return e;
}

void hz_exec_batches(void* h, uint64_t* batches) {
  Exec* e = static_cast<Exec*>(h);
  std::lock_guard<std::mutex> g(e->mu);
  *batches = e->batches;
}

int hz_exec_submit(void* h, const void* const* in, void* out, double* lat_us) {
  return static_cast<Exec*>(h)->submit_wait(in, out, lat_us);
}

// dynamic-batching executor only: one request of m (1..rows) consecutive rows, in[k] / out holding
// m rows each; the rows share replays with other requests' rows
int hz_exec_submit_rows(void* h, const void* const* in, int m, void* out, double* lat_us) {
  Exec* e = static_cast<Exec*>(h);
  if (e->rows <= 1 || m < 1 || m > e->rows) return -1;
  return e->submit_wait(in, out, lat_us, m);
}

void hz_exec_stats(void* h, uint64_t* served, uint64_t* polls) {
  Exec* e = static_cast<Exec*>(h);
  std::lock_guard<std::mutex> g(e->mu);
  *served = e->served;
  *polls = e->polls;
}

void hz_exec_destroy(void* h) { delete static_cast<Exec*>(h); }

// `clients` native threads, each serving `iters` requests back to back through the executor
// (payload in[] for every request); per-request latency in lat_us[client * iters + i]
int hz_exec_bench(void* h, int clients, int iters, const void* const* in, double* lat_us, double* wall_us) {
  Exec* e = static_cast<Exec*>(h);
  std::vector<std::thread> th;
  std::vector<int> rcs(clients, 0);
  std::vector<std::vector<uint8_t>> outs(clients, std::vector<uint8_t>(e->out_bytes + 1));
  const double t0 = now_us();
  for (int c = 0; c < clients; ++c)
    th.emplace_back([&, c] {
      for (int it = 0; it < iters && !rcs[c]; ++it)
        rcs[c] = e->submit_wait(in, outs[c].data(), lat_us + (size_t)c * iters + it);
    });
  for (auto& t : th) t.join();
  *wall_us = now_us() - t0;
  int rc = 0;
  for (int r : rcs) rc |= r;
  return rc;
}

}  // extern "C"
