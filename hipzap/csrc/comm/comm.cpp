// hipzap native communicator over RCCL (xGMI), built as libhipzap_comm.so so the 570 MB
// librccl is only mapped by multi-GPU processes (the single-GPU cold path never loads it).
//
// SURVEY.md §2f (C1 broadcast, C2 scatter, C3 gather, C4 health all-reduce) and §5 "failure
// detection": every communicator is NON-BLOCKING (ncclConfig_t.blocking = 0), and every wait
// polls both the collective's completion event and ncclCommGetAsyncError with a deadline. A
// peer that died, a transport error or a timeout therefore ends in ncclCommAbort and an error
// code in bounded time instead of a collective that spins forever on the GPU. Survivors can
// then form a smaller communicator with ncclCommShrink (elastic DP, parallel/cluster.py).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <chrono>
#include <cstring>
#include <string>
#include <thread>

namespace {

thread_local std::string g_err;

enum { HZC_OK = 0, HZC_TIMEOUT = -2, HZC_ABORTED = -3, HZC_BAD = -4 };

struct Comm {
  ncclComm_t comm = nullptr;
  hipStream_t st = nullptr;
  hipEvent_t ev = nullptr;
  int rank = 0, size = 1, device = 0;
  double timeout_s = 60.0;
  bool aborted = false;
};

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int nfail(Comm* c, ncclResult_t r, const char* what) {
  g_err = std::string(what) + ": " + ncclGetErrorString(r);
  if (c && c->comm && !c->aborted) {
    (void)ncclCommAbort(c->comm);
    c->aborted = true;
    c->comm = nullptr;
  }
  return (int)r;
}

// wait until the communicator leaves ncclInProgress (non-blocking init / enqueue)
int wait_ready(Comm* c, const char* what) {
  const double t0 = now_s();
  for (;;) {
    ncclResult_t st = ncclSuccess;
    ncclResult_t r = ncclCommGetAsyncError(c->comm, &st);
    if (r != ncclSuccess) return nfail(c, r, what);
    if (st == ncclSuccess) return HZC_OK;
    if (st != ncclInProgress) return nfail(c, st, what);
    if (now_s() - t0 > c->timeout_s) {
      g_err = std::string(what) + ": timed out";
      (void)ncclCommAbort(c->comm);
      c->aborted = true;
      c->comm = nullptr;
      return HZC_TIMEOUT;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

// after a collective was enqueued on `st`: wait for it, watching for asynchronous errors
int wait_done(Comm* c, hipStream_t st, const char* what) {
  if (hipEventRecord(c->ev, st) != hipSuccess) {
    g_err = std::string(what) + ": event record failed";
    return HZC_BAD;
  }
  const double t0 = now_s();
  int spins = 0;
  for (;;) {
    const hipError_t q = hipEventQuery(c->ev);
    if (q == hipSuccess) return HZC_OK;
    if (q != hipErrorNotReady) {
      g_err = std::string(what) + ": " + hipGetErrorString(q);
      return HZC_BAD;
    }
    ncclResult_t ae = ncclSuccess;
    if (ncclCommGetAsyncError(c->comm, &ae) != ncclSuccess || (ae != ncclSuccess && ae != ncclInProgress))
      return nfail(c, ae, what);
    if (now_s() - t0 > c->timeout_s) {
      g_err = std::string(what) + ": timed out (peer dead or hung?)";
      (void)ncclCommAbort(c->comm);
      c->aborted = true;
      c->comm = nullptr;
      return HZC_TIMEOUT;
    }
    if (++spins > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

Comm* C(void* h) { return static_cast<Comm*>(h); }

int enqueue_result(Comm* c, ncclResult_t r, hipStream_t st, int wait, const char* what) {
  if (r != ncclSuccess && r != ncclInProgress) return nfail(c, r, what);
  if (r == ncclInProgress) {
    int rc = wait_ready(c, what);
    if (rc) return rc;
  }
  return wait ? wait_done(c, st, what) : HZC_OK;
}

int usable(Comm* c) {
  if (!c || !c->comm || c->aborted) {
    g_err = "communicator is aborted";
    return 0;
  }
  return 1;
}

ncclDataType_t dtype(int d) {
  switch (d) {
    case 0: return ncclInt32;
    case 1: return ncclFloat32;
    case 2: return ncclFloat64;
    case 3: return ncclInt64;
    default: return ncclUint8;
  }
}

Comm* make(ncclComm_t comm, int device, double timeout_s) {
  auto* c = new Comm();
  c->comm = comm;
  c->device = device;
  c->timeout_s = timeout_s;
  (void)ncclCommUserRank(comm, &c->rank);
  (void)ncclCommCount(comm, &c->size);
  if (hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev, hipEventDisableTiming) != hipSuccess) {
    g_err = "stream/event creation failed";
    return nullptr;
  }
  return c;
}

}  // namespace

extern "C" {

const char* hz_comm_last_error(void) { return g_err.c_str(); }

int hz_comm_unique_id(unsigned char* out128) {
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return nfail(nullptr, r, "ncclGetUniqueId");
  std::memcpy(out128, id.internal, NCCL_UNIQUE_ID_BYTES);
  return 0;
}

void* hz_comm_init(const unsigned char* id128, int nranks, int rank, int device, double timeout_s) {
  g_err.clear();
  if (hipSetDevice(device) != hipSuccess) {
    g_err = "hipSetDevice failed";
    return nullptr;
  }
  ncclUniqueId id;
  std::memcpy(id.internal, id128, NCCL_UNIQUE_ID_BYTES);
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclComm_t comm = nullptr;
  ncclResult_t r = ncclCommInitRankConfig(&comm, nranks, id, rank, &cfg);
  Comm tmp;
  tmp.comm = comm;
  tmp.timeout_s = timeout_s;
  if (r != ncclSuccess && r != ncclInProgress) {
    nfail(&tmp, r, "ncclCommInitRankConfig");
    return nullptr;
  }
  if (wait_ready(&tmp, "ncclCommInitRankConfig")) return nullptr;
  return make(comm, device, timeout_s);
}

int hz_comm_rank(void* h) { return C(h)->rank; }
int hz_comm_size(void* h) { return C(h)->size; }
void* hz_comm_stream(void* h) { return C(h)->st; }
void hz_comm_set_timeout(void* h, double s) { C(h)->timeout_s = s; }

// 0 healthy, >0 ncclResult_t of an asynchronous error, HZC_ABORTED after an abort
int hz_comm_poll(void* h) {
  Comm* c = C(h);
  if (!c->comm || c->aborted) return HZC_ABORTED;
  ncclResult_t st = ncclSuccess;
  if (ncclCommGetAsyncError(c->comm, &st) != ncclSuccess) return HZC_BAD;
  return st == ncclInProgress ? 0 : (int)st;
}

int hz_comm_abort(void* h) {
  Comm* c = C(h);
  if (c->comm && !c->aborted) {
    (void)ncclCommAbort(c->comm);
    c->aborted = true;
    c->comm = nullptr;
  }
  return 0;
}

// stream 0 -> the communicator's own stream. wait != 0: return after completion (with async
// error polling and the deadline); wait == 0: return once enqueued (caller orders the stream).
int hz_comm_broadcast(void* h, void* buf, uint64_t bytes, int root, void* stream, int wait) {
  Comm* c = C(h);
  if (!usable(c)) return HZC_ABORTED;
  hipStream_t st = stream ? (hipStream_t)stream : c->st;
  return enqueue_result(c, ncclBroadcast(buf, buf, bytes, ncclUint8, root, c->comm, st), st, wait, "broadcast");
}

int hz_comm_scatter(void* h, const void* send, void* recv, uint64_t bytes_per_rank, int root, void* stream, int wait) {
  Comm* c = C(h);
  if (!usable(c)) return HZC_ABORTED;
  hipStream_t st = stream ? (hipStream_t)stream : c->st;
  return enqueue_result(c, ncclScatter(send, recv, bytes_per_rank, ncclUint8, root, c->comm, st), st, wait,
                        "scatter");
}

int hz_comm_gather(void* h, const void* send, void* recv, uint64_t bytes_per_rank, int root, void* stream, int wait) {
  Comm* c = C(h);
  if (!usable(c)) return HZC_ABORTED;
  hipStream_t st = stream ? (hipStream_t)stream : c->st;
  return enqueue_result(c, ncclGather(send, recv, bytes_per_rank, ncclUint8, root, c->comm, st), st, wait,
                        "gather");
}

// dtype: 0 int32, 1 float32, 2 float64, 3 int64; op: 0 sum, 2 max, 3 min (ncclRedOp_t)
int hz_comm_allreduce(void* h, void* buf, uint64_t count, int dt, int op, void* stream, int wait) {
  Comm* c = C(h);
  if (!usable(c)) return HZC_ABORTED;
  hipStream_t st = stream ? (hipStream_t)stream : c->st;
  return enqueue_result(c, ncclAllReduce(buf, buf, count, dtype(dt), (ncclRedOp_t)op, c->comm, st), st, wait,
                        "allreduce");
}

int hz_comm_sync(void* h, void* stream) {
  Comm* c = C(h);
  if (!usable(c)) return HZC_ABORTED;
  return wait_done(c, stream ? (hipStream_t)stream : c->st, "sync");
}

// survivors drop `exclude` ranks (elastic DP); every surviving rank must call it
void* hz_comm_shrink(void* h, const int* exclude, int n_exclude, int abort_parent) {
  Comm* c = C(h);
  g_err.clear();
  if (!c->comm) {
    g_err = "parent communicator already aborted; re-initialise instead";
    return nullptr;
  }
  (void)hipSetDevice(c->device);
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclComm_t nc = nullptr;
  // resolved at run time: a process that loaded an older librccl first (e.g. the one bundled with
  // PyTorch) must still be able to load this library; shrink is then reported as unsupported
  using ShrinkFn = ncclResult_t (*)(ncclComm_t, int*, int, ncclComm_t*, ncclConfig_t*, int);
  auto shrink = reinterpret_cast<ShrinkFn>(dlsym(RTLD_DEFAULT, "ncclCommShrink"));
  if (!shrink) {
    g_err = "ncclCommShrink is not available in the loaded librccl; re-initialise instead";
    return nullptr;
  }
  ncclResult_t r = shrink(c->comm, const_cast<int*>(exclude), n_exclude, &nc, &cfg,
                          abort_parent ? NCCL_SHRINK_ABORT : NCCL_SHRINK_DEFAULT);
  Comm tmp;
  tmp.comm = nc;
  tmp.timeout_s = c->timeout_s;
  if (r != ncclSuccess && r != ncclInProgress) {
    nfail(&tmp, r, "ncclCommShrink");
    return nullptr;
  }
  if (wait_ready(&tmp, "ncclCommShrink")) return nullptr;
  return make(nc, c->device, c->timeout_s);
}

void hz_comm_destroy(void* h) {
  Comm* c = C(h);
  if (c->comm && !c->aborted) {
    // finalize is collective; a dead peer must not hang teardown
    if (ncclCommFinalize(c->comm) == ncclInProgress) {
      Comm tmp = *c;
      tmp.timeout_s = 5.0;
      if (wait_ready(&tmp, "finalize")) c->comm = nullptr;  // aborted inside
    }
    if (c->comm) (void)ncclCommDestroy(c->comm);
  }
  if (c->ev) (void)hipEventDestroy(c->ev);
  if (c->st) (void)hipStreamDestroy(c->st);
  delete c;
}

}  // extern "C"
