// hipzap plan images: a torch-free cold start (VERDICT r1 "next round" #1).
//
// A plan (`<ckpt>.hzplan`, written at deploy time by hipzap/engine/plan.py) is a fully bound
// native Program serialised with relocations instead of pointers:
//   region 0  shared device blob (packed weights + constants; its bytes are in the file)
//   region 1  per-context device block (activation arena + static device I/O), zero-filled
//   region 2  per-context pinned host block (request input / logits, zero-copy I/O)
// Loading is: mmap -> hipMalloc + H2D of the blob (or an RCCL broadcast into it) -> per context
// one hipMalloc + one hipHostMalloc + patch every pointer field -> hz_prog_add_* -> hipGraph
// capture. No Python tensor library, no packing, no planning on the cold path: process start
// -> first logits is HIP init + one DMA of the weights + a graph instantiation.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "hipzap.h"

namespace {

constexpr uint32_t kPlanVersion = 1;
// flags: the file carries no weight bytes (a template: engine/plan.py export_template); the blob
// is filled by the caller, e.g. by packing a .pth checkpoint on the device (csrc/pack.hip)
constexpr uint64_t kFlagWeightless = 1;
constexpr char kMagic[8] = {'H', 'Z', 'P', 'L', 'A', 'N', '0', '1'};
enum : unsigned { kUnitConv = 1, kUnitVision = 2, kUnitGemm = 4, kUnitTransformer = 8, kUnitFp8 = 16, kUnitPack = 32, kUnitBlock = 64 };

// file header: magic + 15 little-endian u64 fields (see plan.py PlanHeader)
struct FileHeader {
  char magic[8];
  uint64_t version, abi, n_ops;
  uint64_t meta_off, meta_len;
  uint64_t ops_off, ops_len;
  uint64_t blob_off, blob_len;
  uint64_t ctx_dev_bytes, ctx_host_bytes;
  uint64_t flags, reserved0, reserved1, reserved2;
};
static_assert(sizeof(FileHeader) == 128, "plan header is 128 bytes");

struct OpHeader {  // followed by plen param bytes (padded to 8) and nrel relocations
  uint32_t type;
  int32_t arg;   // conv cfg or kernel kind
  int32_t slot;
  uint32_t plen;
  uint32_t nrel;
  uint32_t pad;
};
struct Reloc {
  uint32_t off;     // byte offset of the pointer field inside the params
  uint32_t region;  // 0 blob, 1 context device block, 2 context host block
  uint64_t roff;    // offset inside the region
};

struct PlanOp {
  OpHeader h;
  const uint8_t* prm;
  const Reloc* rel;
};

struct PlanCtx {
  void* dev = nullptr;
  void* host = nullptr;
  HzProgram prog = nullptr;
  hipStream_t st = nullptr;
  bool own_stream = true;  // false: borrowed from an earlier context (HIPZAP_CTX_STREAMS)
};

thread_local std::string g_err;

struct Plan;
int capture_ctx_prog(Plan* p, const PlanCtx& c);

int fail(const std::string& msg, int rc = -1) {
  g_err = msg;
  return rc;
}

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// File byte ranges -> device memory through pinned staging buffers: each reader thread has two
// staging buffers and reads chunk j while the DMA of its previous chunk runs; every copy goes on
// `st` (distinct destinations, so their order does not matter). HIPZAP_UPLOAD_THREADS readers
// (default 1, 4-MiB chunks) split the chunks round-robin (2-MiB chunks). Measured (r6 session 18,
// profiles/r6_cold): 4 readers made the plan blob's DMA 4.3 -> 7.8-11.0 ms and the LM checkpoint's
// 340-MB upload no faster (the extra pinned staging buffers cost more than the parallel reads save).
int staged_upload(int fd, int n, const uint64_t* file_off, const uint64_t* nbytes, void* const* dst,
                  hipStream_t st) {
  const char* e = getenv("HIPZAP_UPLOAD_THREADS");
  int T = e ? atoi(e) : 1;
  T = T < 1 ? 1 : T > 8 ? 8 : T;
  const size_t chunk = T == 1 ? size_t(4) << 20 : size_t(2) << 20;
  struct Chunk {
    uint64_t f;
    size_t m;
    uint8_t* d;
  };
  std::vector<Chunk> cs;
  for (int i = 0; i < n; ++i)
    for (uint64_t off = 0; off < nbytes[i]; off += chunk)
      cs.push_back({file_off[i] + off, (size_t)(nbytes[i] - off < chunk ? nbytes[i] - off : chunk),
                    static_cast<uint8_t*>(dst[i]) + off});
  if (cs.empty()) return 0;
  if ((size_t)T > cs.size()) T = (int)cs.size();
  std::vector<int> ok(T, 1);
  auto work = [&](int t) {
    void* stage[2] = {nullptr, nullptr};
    hipEvent_t done[2] = {nullptr, nullptr};
    bool good = hipHostMalloc(&stage[0], chunk, hipHostMallocDefault) == hipSuccess &&
                hipHostMalloc(&stage[1], chunk, hipHostMallocDefault) == hipSuccess &&
                hipEventCreateWithFlags(&done[0], hipEventDisableTiming) == hipSuccess &&
                hipEventCreateWithFlags(&done[1], hipEventDisableTiming) == hipSuccess;
    int k = 0, issued = 0;
    for (size_t j = (size_t)t; good && j < cs.size(); j += (size_t)T, k ^= 1, ++issued) {
      if (issued >= 2) good = hipEventSynchronize(done[k]) == hipSuccess;  // staging buffer k free again
      if (!good) break;
      size_t got = 0;
      while (got < cs[j].m) {
        const ssize_t r = pread(fd, static_cast<uint8_t*>(stage[k]) + got, cs[j].m - got, (off_t)(cs[j].f + got));
        if (r <= 0) break;
        got += (size_t)r;
      }
      good = got == cs[j].m && hipMemcpyAsync(cs[j].d, stage[k], cs[j].m, hipMemcpyHostToDevice, st) == hipSuccess &&
             hipEventRecord(done[k], st) == hipSuccess;
    }
    for (int i = 0; i < 2; ++i) {
      if (done[i]) {
        if (issued > i) good = hipEventSynchronize(done[i]) == hipSuccess && good;  // before its buffer is freed
        (void)hipEventDestroy(done[i]);
      }
      if (stage[i]) (void)hipHostFree(stage[i]);
    }
    ok[t] = good;
  };
  std::vector<std::thread> th;
  for (int t = 1; t < T; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
  for (int v : ok)
    if (!v) return -1;
  return hipStreamSynchronize(st) == hipSuccess ? 0 : -1;
}

struct Plan {
  int device = 0;
  int fd = -1;
  uint8_t* map = nullptr;
  size_t map_len = 0;
  FileHeader h{};
  std::vector<PlanOp> ops;
  void* blob = nullptr;
  std::vector<PlanCtx> ctx;
  std::mutex mu;
  double t[HZ_PLAN_NT] = {};

  hipStream_t spare = nullptr;  // the upload stream, handed to the first context (stream creation is
                                // ~10-25 ms of lazy runtime work in a fresh process)
  hipStream_t cap_st = nullptr;  // private capture stream for contexts on borrowed streams
  // hz_plan_set_stream_priority: contexts after the first get fresh highest-priority streams (HIP
  // keeps a separate set of hardware queues per priority: 2-4 contexts land on distinct queues;
  // engine.py stream_kind, profiles/r6_queues)
  bool prio_high = false;
  std::mutex cap_mu;
  std::thread warm;  // device-code warm-up, joined before hz_plan_open returns
  void join_warm() {
    if (warm.joinable()) warm.join();
  }
  ~Plan() {
    join_warm();
    (void)hipSetDevice(device);
    // borrowed streams first: their owners' free_ctx destroys the stream
    for (auto& c : ctx)
      if (!c.own_stream) free_ctx(c);
    for (auto& c : ctx) free_ctx(c);
    if (spare) (void)hipStreamDestroy(spare);
    if (cap_st) (void)hipStreamDestroy(cap_st);
    if (blob) (void)hipFree(blob);
    if (map) munmap(map, map_len);
    if (fd >= 0) close(fd);
  }

  static void free_ctx(PlanCtx& c) {
    if (c.st) (void)hipStreamSynchronize(c.st);
    if (c.prog) hz_prog_destroy(c.prog);
    if (c.st && c.own_stream) (void)hipStreamDestroy(c.st);
    if (c.dev) (void)hipFree(c.dev);
    if (c.host) (void)hipHostFree(c.host);
    c = PlanCtx{};
  }

  // translation units whose kernels the ops launch (bit set for hz_plan_open's code warm-up)
  unsigned code_units() const {
    unsigned u = 0;
    for (const PlanOp& op : ops) {
      switch (op.h.type) {
        case HZ_PLAN_OP_CONV: u |= op.h.arg >= 16 ? kUnitGemm : kUnitConv; break;
        case HZ_PLAN_OP_CONV2: u |= kUnitConv; break;
        case HZ_PLAN_OP_MAXPOOL:
        case HZ_PLAN_OP_AVGPOOL:
        case HZ_PLAN_OP_PREPROCESS: u |= kUnitVision; break;
        case HZ_PLAN_OP_KERNEL:
          switch (op.h.arg) {
            case HZ_K_LAYERNORM:
            case HZ_K_EMBED:
            case HZ_K_ATTENTION:
            case HZ_K_QKVATT:
            case HZ_K_VIT_TOKENS:
            case HZ_K_SOFTMAX: u |= kUnitTransformer; break;
            case HZ_K_GEMM_FP8:
            case HZ_K_QUANT: u |= kUnitFp8; break;
            case HZ_K_MAXPOOL:
            case HZ_K_POOL_FC: u |= kUnitVision; break;
            case HZ_K_STEM:
            case HZ_K_BNECK:
            case HZ_K_SEAM:
            case HZ_K_KCONV: u |= kUnitBlock; break;
            default: break;
          }
          break;
        default: break;
      }
    }
    return u;
  }

  int parse() {
    if (map_len < sizeof(FileHeader)) return fail("plan: file too small");
    std::memcpy(&h, map, sizeof(h));
    if (std::memcmp(h.magic, kMagic, 8) != 0) return fail("plan: bad magic");
    if (h.version != kPlanVersion) return fail("plan: unsupported version " + std::to_string(h.version));
    if (h.abi != hz_abi_version())
      return fail("plan: written for a different native ABI (" + std::to_string(h.abi) + " != " +
                  std::to_string(hz_abi_version()) + "); re-export it");
    // (subtractive bounds: a forged offset + length must not wrap around)
    if (h.ops_off > map_len || h.ops_len > map_len - h.ops_off ||
        (!(h.flags & kFlagWeightless) && (h.blob_off > map_len || h.blob_len > map_len - h.blob_off)))
      return fail("plan: truncated file");
    const uint8_t* p = map + h.ops_off;
    const uint8_t* end = p + h.ops_len;
    ops.reserve(h.n_ops);
    for (uint64_t i = 0; i < h.n_ops; ++i) {
      if (p + sizeof(OpHeader) > end) return fail("plan: truncated op table");
      PlanOp op;
      std::memcpy(&op.h, p, sizeof(OpHeader));
      p += sizeof(OpHeader);
      const uint64_t rec = (((uint64_t)op.h.plen + 7u) & ~uint64_t(7)) + sizeof(Reloc) * (uint64_t)op.h.nrel;
      if (rec > (uint64_t)(end - p)) return fail("plan: truncated op record");
      op.prm = p;
      op.rel = reinterpret_cast<const Reloc*>(p + (((uint64_t)op.h.plen + 7u) & ~uint64_t(7)));
      p += rec;
      // every op reads a whole parameter struct from its record
      size_t need = 0;
      switch (op.h.type) {
        case HZ_PLAN_OP_CONV: need = sizeof(HzConvParams); break;
        case HZ_PLAN_OP_CONV2: need = 2 * sizeof(HzConvParams); break;
        case HZ_PLAN_OP_MAXPOOL: need = sizeof(HzPoolParams); break;
        case HZ_PLAN_OP_AVGPOOL: need = sizeof(HzAvgpoolArgs); break;
        case HZ_PLAN_OP_PREPROCESS: need = sizeof(HzPreprocessArgs); break;
        case HZ_PLAN_OP_MEMCPY: need = sizeof(HzMemcpyArgs); break;
        case HZ_PLAN_OP_KERNEL: need = hz_kernel_param_size(op.h.arg); break;
        case HZ_PLAN_OP_FORK:
        case HZ_PLAN_OP_JOIN: need = 0; break;
        default: return fail("plan: unknown op type " + std::to_string(op.h.type));
      }
      if ((op.h.type == HZ_PLAN_OP_KERNEL && !need) || op.h.plen < need)
        return fail("plan: op " + std::to_string(i) + " record shorter than its parameters");
      for (uint32_t r = 0; r < op.h.nrel; ++r) {
        const Reloc& rl = op.rel[r];
        const uint64_t lim = rl.region == 0 ? h.blob_len : rl.region == 1 ? h.ctx_dev_bytes : h.ctx_host_bytes;
        if (rl.region > 2 || (uint64_t)rl.off + 8 > op.h.plen || rl.roff > lim)
          return fail("plan: relocation out of range in op " + std::to_string(i));
      }
      ops.push_back(op);
    }
    return 0;
  }

  // blob upload, HIPZAP_PLAN_UPLOAD selects (measured: profiles/r2_coldstart):
  //   register  pin the mmapped file pages in place (hipHostRegister) -> one DMA -> unpin
  //   staged    pread() chunks into pinned staging buffers on HIPZAP_UPLOAD_THREADS readers, the
  //             DMA of each chunk overlapping the next reads (staged_upload)
  //   pageable  hipMemcpyAsync from the mapping (HIP stages pageable memory internally)
  //   kernel    pin the mapping in place, then a copy kernel reads it over PCIe (no DMA engine)
  int upload_blob(hipStream_t st) {
    const char* mode = getenv("HIPZAP_PLAN_UPLOAD");
    const std::string m = mode ? mode : "staged";
    hipError_t e = hipSuccess;
    const char* probe = getenv("HIPZAP_PLAN_PROBE");
    if (probe && probe[0] == '1') {  // diagnostics: cost of the process's first (tiny) DMA alone
      const double t0 = now_ms();
      void* pin = nullptr;
      if (hipHostMalloc(&pin, 4096, hipHostMallocDefault) == hipSuccess) {
        std::memset(pin, 0, 4096);
        (void)hipMemcpyAsync(blob, pin, 4096, hipMemcpyHostToDevice, st);
        (void)hipStreamSynchronize(st);
        (void)hipHostFree(pin);
      }
      t[HZ_PLAN_T_FIRST_COPY] = now_ms() - t0;
    }
    if (m == "kernel" && h.blob_len % 16 == 0) {
      const size_t pg = 4096, off = h.blob_off & ~(pg - 1), len = h.blob_off + h.blob_len - off;
      void* base = map + off;
      if (hipHostRegister(base, len, hipHostRegisterMapped) == hipSuccess) {
        void* dbase = nullptr;
        e = hipHostGetDevicePointer(&dbase, base, 0);
        if (e == hipSuccess)
          e = (hipError_t)hz_diag_launch(1, 1024, 256, static_cast<uint8_t*>(dbase) + (h.blob_off - off), blob,
                                         (long)h.blob_len, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        (void)hipHostUnregister(base);
        if (e == hipSuccess) return 0;
      }
      (void)hipGetLastError();  // fall through to the staged copy
    }
    if (m == "register") {
      const size_t pg = 4096, off = h.blob_off & ~(pg - 1), len = h.blob_off + h.blob_len - off;
      void* base = map + off;
      if (hipHostRegister(base, len, hipHostRegisterDefault) == hipSuccess) {
        void* dptr = nullptr;
        e = hipHostGetDevicePointer(&dptr, base, 0);
        if (e == hipSuccess)
          e = hipMemcpyAsync(blob, map + h.blob_off, h.blob_len, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        (void)hipHostUnregister(base);
        if (e == hipSuccess) return 0;
      }
      (void)hipGetLastError();  // fall through to the staged copy
    }
    if (m != "pageable") {
      const uint64_t off = h.blob_off, len = h.blob_len;
      void* d = blob;
      if (staged_upload(fd, 1, &off, &len, &d, st) == 0) return 0;
      (void)hipGetLastError();
    }
    const uint8_t* src = map + h.blob_off;
    const size_t chunk = size_t(8) << 20;
    for (size_t off = 0; off < h.blob_len; off += chunk) {
      const size_t n = h.blob_len - off < chunk ? h.blob_len - off : chunk;
      e = hipMemcpyAsync(static_cast<uint8_t*>(blob) + off, src + off, n, hipMemcpyHostToDevice, st);
      if (e != hipSuccess) return fail(std::string("plan: blob H2D failed: ") + hipGetErrorString(e), (int)e);
    }
    e = hipStreamSynchronize(st);
    return e == hipSuccess ? 0 : fail("plan: blob H2D sync failed", (int)e);
  }

  int bind(PlanCtx& c) {
    c.prog = hz_prog_create();
    std::vector<uint8_t> buf;
    for (size_t i = 0; i < ops.size(); ++i) {
      const PlanOp& op = ops[i];
      buf.assign(op.prm, op.prm + op.h.plen);
      buf.resize(op.h.plen + 8);  // slack: no op reads past plen
      for (uint32_t r = 0; r < op.h.nrel; ++r) {
        const Reloc& rl = op.rel[r];
        uint8_t* base = static_cast<uint8_t*>(rl.region == 0 ? blob : rl.region == 1 ? c.dev : c.host);
        const uint64_t v = reinterpret_cast<uint64_t>(base + rl.roff);
        std::memcpy(buf.data() + rl.off, &v, 8);
      }
      const void* prm = buf.data();
      int rc = 0;
      switch (op.h.type) {
        case HZ_PLAN_OP_CONV:
          rc = hz_prog_add_conv(c.prog, static_cast<const HzConvParams*>(prm), op.h.arg, op.h.slot);
          break;
        case HZ_PLAN_OP_CONV2: {
          const HzConvParams* a = static_cast<const HzConvParams*>(prm);
          rc = hz_prog_add_conv2(c.prog, a, a + 1, op.h.arg, op.h.slot);
          break;
        }
        case HZ_PLAN_OP_MAXPOOL:
          rc = hz_prog_add_maxpool(c.prog, static_cast<const HzPoolParams*>(prm), op.h.slot);
          break;
        case HZ_PLAN_OP_AVGPOOL: {
          const HzAvgpoolArgs* a = static_cast<const HzAvgpoolArgs*>(prm);
          rc = hz_prog_add_avgpool(c.prog, a->x, a->out, a->N, a->HW, a->C, a->blocked, op.h.slot);
          break;
        }
        case HZ_PLAN_OP_PREPROCESS: {
          const HzPreprocessArgs* a = static_cast<const HzPreprocessArgs*>(prm);
          rc = hz_prog_add_preprocess(c.prog, a->src, a->dst, a->N, a->Cin, a->H, a->W, a->Cpad, a->mode, a->mean,
                                      a->inv_std, op.h.slot);
          break;
        }
        case HZ_PLAN_OP_MEMCPY: {
          const HzMemcpyArgs* a = static_cast<const HzMemcpyArgs*>(prm);
          rc = hz_prog_add_memcpy(c.prog, a->dst, a->src, a->bytes, op.h.slot);
          break;
        }
        case HZ_PLAN_OP_KERNEL: rc = hz_prog_add_kernel(c.prog, op.h.arg, prm, op.h.plen, op.h.slot); break;
        case HZ_PLAN_OP_FORK: rc = hz_prog_add_fork(c.prog, op.h.slot); break;
        case HZ_PLAN_OP_JOIN: rc = hz_prog_add_join(c.prog, op.h.slot); break;
        default: return fail("plan: unknown op type " + std::to_string(op.h.type));
      }
      if (rc) return fail("plan: binding op " + std::to_string(i) + " failed", rc);
    }
    return 0;
  }

  int add_contexts(int n, int capture) {
    for (int k = 0; k < n; ++k) {
      PlanCtx c;
      double t0 = now_ms();
      hipError_t e = hipSuccess;
      // HIPZAP_CTX_STREAMS=k: contexts share k streams round-robin (k ~ the hardware queues)
      // (default 0 = one stream each; see engine.py _new_contexts for the measurements)
      const char* ks = getenv("HIPZAP_CTX_STREAMS");
      const int kshare = ks ? atoi(ks) : 0;
      size_t nctx;
      {
        std::lock_guard<std::mutex> g(mu);
        nctx = ctx.size();
      }
      if (kshare > 0 && nctx >= (size_t)kshare) {
        std::lock_guard<std::mutex> g(mu);
        c.st = ctx[nctx % kshare].st;
        c.own_stream = false;
      } else if (spare) {
        c.st = spare;
        spare = nullptr;
      } else if (prio_high) {
        int lo = 0, hi = 0;
        e = hipDeviceGetStreamPriorityRange(&lo, &hi);
        if (e == hipSuccess) e = hipStreamCreateWithPriority(&c.st, hipStreamNonBlocking, hi);
      } else {
        e = hipStreamCreateWithFlags(&c.st, hipStreamNonBlocking);
      }
      if (e == hipSuccess) e = hipMalloc(&c.dev, h.ctx_dev_bytes ? h.ctx_dev_bytes : 256);
      if (e == hipSuccess && h.ctx_dev_bytes) e = hipMemsetAsync(c.dev, 0, h.ctx_dev_bytes, c.st);
      if (e == hipSuccess) e = hipHostMalloc(&c.host, h.ctx_host_bytes ? h.ctx_host_bytes : 256, hipHostMallocDefault);
      if (e != hipSuccess) {
        free_ctx(c);
        return fail(std::string("plan: context allocation failed: ") + hipGetErrorString(e), (int)e);
      }
      std::memset(c.host, 0, h.ctx_host_bytes);
      double t1 = now_ms();
      int rc = bind(c);
      double t2 = now_ms();
      if (!rc && capture) rc = capture_ctx_prog(this, c);
      if (!rc && hipStreamSynchronize(c.st) != hipSuccess) rc = fail("plan: context sync failed");
      double t3 = now_ms();
      if (rc) {
        if (g_err.empty()) g_err = "plan: capture failed rc=" + std::to_string(rc);
        free_ctx(c);
        return rc;
      }
      t[HZ_PLAN_T_CTX_ALLOC] += t1 - t0;
      t[HZ_PLAN_T_BIND] += t2 - t1;
      t[HZ_PLAN_T_CAPTURE] += t3 - t2;
      std::lock_guard<std::mutex> g(mu);
      ctx.push_back(c);
    }
    return 0;
  }
};

Plan* P(void* h) { return static_cast<Plan*>(h); }

// Capture a context's program. A borrowed (shared) stream may carry other contexts' replays
// issued by other threads meanwhile, which a capture on it would swallow: capture those on a
// private stream instead (a graph replays on any stream).
int capture_ctx_prog(Plan* p, const PlanCtx& c) {
  if (c.own_stream) {
    int rc = hz_prog_capture(c.prog, c.st);
    return rc ? rc : (int)hipStreamSynchronize(c.st);
  }
  std::lock_guard<std::mutex> g(p->cap_mu);  // one private capture stream per plan
  if (!p->cap_st && hipStreamCreateWithFlags(&p->cap_st, hipStreamNonBlocking) != hipSuccess) {
    p->cap_st = nullptr;
    return fail("plan: stream creation failed");
  }
  int rc = hz_prog_capture(c.prog, p->cap_st);
  return rc ? rc : (int)hipStreamSynchronize(p->cap_st);
}

}  // namespace

extern "C" {

uint64_t hz_abi_version(void) {
  // FNV-1a over the plan format version and every struct a plan serialises: a library whose
  // parameter layouts changed refuses old plans instead of launching garbage
  const uint64_t parts[] = {kPlanVersion,
                            sizeof(HzConvParams),
                            sizeof(HzPoolParams),
                            sizeof(HzPoolFcParams),
                            sizeof(HzLayerNormParams),
                            sizeof(HzEmbedParams),
                            sizeof(HzAttentionParams),
                            sizeof(HzVitTokensParams),
                            sizeof(HzSoftmaxParams),
                            sizeof(HzQuantParams),
                            sizeof(HzGemmFp8Params),
                            sizeof(HzLstmParams),
                            sizeof(HzDecoderParams),
                            sizeof(HzSamplerParams),
                            sizeof(HzAvgpoolArgs),
                            sizeof(HzPreprocessArgs),
                            sizeof(HzMemcpyArgs),
                            sizeof(HzStemParams),
                            sizeof(HzBneckParams),
                            sizeof(HzSeamParams),
                            sizeof(HzKconvParams),
                            sizeof(HzQkvAttParams),
                            HZ_ABI_EPOCH};
  uint64_t x = 1469598103934665603ull;
  for (uint64_t v : parts) {
    x ^= v;
    x *= 1099511628211ull;
  }
  return x & 0x7fffffffffffffffull;
}

const char* hz_plan_last_error(void) { return g_err.c_str(); }

// file byte ranges -> device pointers (staged_upload: the plan blob upload's scheme); synchronous
int hz_upload_file(const char* path, int n, const uint64_t* file_off, const uint64_t* nbytes, void* const* dst,
                   void* stream) {
  g_err.clear();
  const int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return fail(std::string("upload: cannot open ") + path);
  const int rc = staged_upload(fd, n, file_off, nbytes, dst, static_cast<hipStream_t>(stream));
  close(fd);
  return rc == 0 ? 0 : fail("upload: read or copy failed");
}

void* hz_plan_open(const char* path, int device, int read_blob, double* timings) {
  g_err.clear();
  double t0 = now_ms();
  auto* p = new Plan();
  p->device = device;
  p->fd = open(path, O_RDONLY | O_CLOEXEC);
  if (p->fd < 0) {
    fail(std::string("plan: cannot open ") + path);
    delete p;
    return nullptr;
  }
  struct stat st {};
  fstat(p->fd, &st);
  p->map_len = (size_t)st.st_size;
  void* m = mmap(nullptr, p->map_len, PROT_READ, MAP_PRIVATE, p->fd, 0);
  if (m == MAP_FAILED) {
    fail("plan: mmap failed");
    delete p;
    return nullptr;
  }
  p->map = static_cast<uint8_t*>(m);
  if (p->parse()) {
    delete p;
    return nullptr;
  }
  if ((p->h.flags & kFlagWeightless) && read_blob) {
    fail("plan: weightless template (its blob comes from a checkpoint: open with read_blob = 0)");
    delete p;
    return nullptr;
  }
  // the weights are read once, sequentially
  if (!(p->h.flags & kFlagWeightless))
    madvise(p->map + (p->h.blob_off & ~size_t(4095)), p->h.blob_len, MADV_SEQUENTIAL | MADV_WILLNEED);
  double t1 = now_ms();
  p->t[HZ_PLAN_T_PARSE] = t1 - t0;
  // first HIP call of a fresh process: runtime + device initialisation
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipFree(nullptr);
  double t2 = now_ms();
  p->t[HZ_PLAN_T_HIP_INIT] = t2 - t1;
  // have the runtime load the device code of every translation unit the plan's ops launch (and
  // the packer's, for a weightless template) on a helper thread while this one uploads the
  // weights, instead of at the first request's first launches (HIPZAP_PLAN_CODE_WARM=0: off).
  // Joined before returning: left running into the caller's context setup (stream creation,
  // hipMemsetAsync), it crashed the runtime in a process that already held RCCL communicators
  // (tests/test_cluster_gpu.py, profiles/r3_warm3/README.md).
  // Order (HIPZAP_PLAN_WARM_ORDER): "init" (default) starts the thread right after HIP init;
  // "stream" waits until the upload stream exists, so the process's first hipStreamCreate (HIP's
  // lazy queue setup) never runs beside the code-object loads (the driver's round-4 box showed the
  // first stream finishing only when the warm thread did). Measured negative:
  // 10 interleaved trials each (profiles/r5_cold) gave p50 228.1 ms "init" vs 238.8 ms "stream"
  // -- the stream took ~20.7 ms either way and "stream" added a 6.7 ms wait for the warm thread.
  const char* cw = getenv("HIPZAP_PLAN_CODE_WARM");
  const char* wo = getenv("HIPZAP_PLAN_WARM_ORDER");
  const bool warm_on = !(cw && cw[0] == '0');
  const bool warm_early = !(wo && std::strcmp(wo, "stream") == 0);
  auto start_warm = [&]() {
    const unsigned units = p->code_units() | ((p->h.flags & kFlagWeightless) ? kUnitPack : 0u);
    double* t_warm = &p->t[HZ_PLAN_T_WARM_THREAD];  // written by the thread, read after the join
    p->warm = std::thread([device, units, t_warm] {
      const double w0 = now_ms();
      if (hipSetDevice(device) != hipSuccess) return;
      if (units & kUnitConv) (void)hz_conv_code_warm();
      if (units & kUnitVision) (void)hz_vision_code_warm();
      if (units & kUnitGemm) (void)hz_gemm_code_warm();
      if (units & kUnitTransformer) (void)hz_transformer_code_warm();
      if (units & kUnitFp8) (void)hz_fp8_code_warm();
      if (units & kUnitPack) (void)hz_pack_code_warm();
      if (units & kUnitBlock) (void)hz_block_code_warm();
      *t_warm = now_ms() - w0;
    });
  };
  if (e == hipSuccess && warm_on && warm_early) start_warm();
  if (e == hipSuccess) e = hipMalloc(&p->blob, p->h.blob_len ? p->h.blob_len : 256);
  p->t[HZ_PLAN_T_BLOB_ALLOC] = now_ms() - t2;
  if (e != hipSuccess) {
    fail(std::string("plan: device init/alloc failed: ") + hipGetErrorString(e));
    delete p;
    return nullptr;
  }
  {  // the upload stream: kept, it becomes the first context's stream (a weightless template's
     // caller fills the blob on it, hz_plan_upload_stream, instead of creating a stream of its own)
    hipStream_t s = nullptr;
    const double ts = now_ms();
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
      fail("plan: stream creation failed");
      delete p;
      return nullptr;
    }
    p->spare = s;
    const double tu = now_ms();
    p->t[HZ_PLAN_T_STREAM] = tu - ts;
    if (warm_on && !warm_early) start_warm();  // beside the blob's read + DMA, after the first stream
    if (read_blob && p->upload_blob(s)) {
      delete p;
      return nullptr;
    }
    p->t[HZ_PLAN_T_UPLOAD_DMA] = now_ms() - tu;
  }
  const double tw = now_ms();
  p->join_warm();
  p->t[HZ_PLAN_T_WARM_WAIT] = now_ms() - tw;
  p->t[HZ_PLAN_T_UPLOAD] = now_ms() - t2 - p->t[HZ_PLAN_T_BLOB_ALLOC];
  if (timings) std::memcpy(timings, p->t, sizeof(p->t));
  return p;
}

int hz_plan_add_contexts(void* h, int n, int capture) {
  g_err.clear();
  if (hipSetDevice(P(h)->device) != hipSuccess) return fail("plan: hipSetDevice failed");
  return P(h)->add_contexts(n, capture);
}

void hz_plan_set_stream_priority(void* h, int high) { P(h)->prio_high = high != 0; }

int hz_plan_num_contexts(void* h) {
  std::lock_guard<std::mutex> g(P(h)->mu);
  return (int)P(h)->ctx.size();
}

void hz_plan_timings(void* h, double* out) { std::memcpy(out, P(h)->t, sizeof(P(h)->t)); }

void* hz_plan_blob(void* h, uint64_t* bytes) {
  if (bytes) *bytes = P(h)->h.blob_len;
  return P(h)->blob;
}

// the stream hz_plan_open created for the blob upload until the first context takes it over
// (NULL afterwards): fill a weightless template's blob on it before adding contexts
void* hz_plan_upload_stream(void* h) {
  std::lock_guard<std::mutex> g(P(h)->mu);
  return (void*)P(h)->spare;
}

void* hz_plan_host(void* h, int ctx) {
  std::lock_guard<std::mutex> g(P(h)->mu);
  return ctx < (int)P(h)->ctx.size() ? P(h)->ctx[ctx].host : nullptr;
}

void* hz_plan_device(void* h, int ctx) {
  std::lock_guard<std::mutex> g(P(h)->mu);
  return ctx < (int)P(h)->ctx.size() ? P(h)->ctx[ctx].dev : nullptr;
}

void* hz_plan_stream(void* h, int ctx) {
  std::lock_guard<std::mutex> g(P(h)->mu);
  return ctx < (int)P(h)->ctx.size() ? (void*)P(h)->ctx[ctx].st : nullptr;
}

static PlanCtx get_ctx(Plan* p, int i) {
  std::lock_guard<std::mutex> g(p->mu);
  return i >= 0 && i < (int)p->ctx.size() ? p->ctx[i] : PlanCtx{};
}

int hz_plan_replay(void* h, int ctx) {
  PlanCtx c = get_ctx(P(h), ctx);
  if (!c.prog) return fail("plan: no such context");
  return hz_prog_replay(c.prog, c.st);
}

int hz_plan_sync(void* h, int ctx) {
  PlanCtx c = get_ctx(P(h), ctx);
  if (!c.st) return fail("plan: no such context");
  return (int)hipStreamSynchronize(c.st);
}

// one request on context `ctx`: copy the payload into the pinned input, replay, wait, copy the
// result out (called from Python with the GIL released, one thread per in-flight request)
int hz_plan_infer(void* h, int ctx, const void* in, uint64_t in_off, uint64_t in_bytes, void* out, uint64_t out_off,
                  uint64_t out_bytes) {
  Plan* p = P(h);
  PlanCtx c = get_ctx(p, ctx);
  if (!c.prog) return fail("plan: no such context");
  if (in_off + in_bytes > p->h.ctx_host_bytes || out_off + out_bytes > p->h.ctx_host_bytes)
    return fail("plan: I/O outside the host block");
  uint8_t* host = static_cast<uint8_t*>(c.host);
  if (in && in_bytes) std::memcpy(host + in_off, in, in_bytes);
  int rc = hz_prog_replay(c.prog, c.st);
  if (rc) return fail("plan: replay failed", rc);
  hipError_t e = hipStreamSynchronize(c.st);
  if (e != hipSuccess) return fail(std::string("plan: sync failed: ") + hipGetErrorString(e), (int)e);
  if (out && out_bytes) std::memcpy(out, host + out_off, out_bytes);
  return 0;
}

double hz_plan_bench(void* h, int iters) {
  Plan* p = P(h);
  std::vector<HzProgram> progs;
  std::vector<hipStream_t> sts;
  {
    std::lock_guard<std::mutex> g(p->mu);
    for (auto& c : p->ctx) {
      progs.push_back(c.prog);
      sts.push_back(c.st);
    }
  }
  return hz_prog_bench(progs.data(), sts.data(), (int)progs.size(), iters);
}

HzProgram hz_plan_prog(void* h, int ctx) { return get_ctx(P(h), ctx).prog; }

// capture a context that was added with capture = 0 (lazy capture: its first requests ran the
// program eagerly); no request may be in flight on it
int hz_plan_capture_ctx(void* h, int ctx) {
  Plan* p = P(h);
  PlanCtx c = get_ctx(p, ctx);
  if (!c.prog) return fail("plan: no such context");
  if (hipSetDevice(p->device) != hipSuccess) return fail("plan: hipSetDevice failed");
  const double t0 = now_ms();
  int rc = capture_ctx_prog(p, c);
  p->t[HZ_PLAN_T_CAPTURE] += now_ms() - t0;
  return rc;
}

void hz_plan_close(void* h) { delete P(h); }

}  // extern "C"
