// hipzap native runtime: static op programs with hipGraph capture/replay.
//
// A model is lowered once (at cold start) into a Program: an ordered list of fully bound
// kernel launches (all pointers fixed into a static activation arena, weights packed), plus
// fork/join markers that put independent branches (e.g. a ResNet downsample conv) on side
// streams. The warm path is the Program captured as ONE hipGraph and replayed per request,
// so per-request host cost is a single hipGraphLaunch (north star "warm-path
// invocation captured as a hipGraph"). Nothing here allocates or synchronises inside the
// launch sequence, so capture is always legal (cdna_hip_programming.md §6 Guideline 9).
#include <hip/hip_runtime.h>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <thread>
#include <vector>

#include "common.h"
#include "hipzap.h"

namespace {

struct Op {
  int slot;  // 0 = main stream, k>0 = side stream k
  enum Kind { LAUNCH, FORK, JOIN } kind;
  std::function<int(hipStream_t)> fn;
};

struct Program {
  std::vector<Op> ops;
  std::vector<hipStream_t> side;     // side[k-1]
  std::vector<hipEvent_t> fork_ev;   // one per fork/join op (indexed by op)
  hipGraph_t graph = nullptr;
  // atomic: a program captured lazily (hz_prog_capture from one thread) may be replayed op by op
  // (hz_prog_replay from another) until the instantiated graph is published
  std::atomic<hipGraphExec_t> exec{nullptr};
  int max_slot = 0;

  ~Program() {
    if (hipGraphExec_t x = exec.load()) (void)hipGraphExecDestroy(x);
    if (graph) (void)hipGraphDestroy(graph);
    for (auto s : side) (void)hipStreamDestroy(s);
    for (auto e : fork_ev)
      if (e) (void)hipEventDestroy(e);
  }

  int ensure_streams() {
    while ((int)side.size() < max_slot) {
      hipStream_t s;
      if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return -1;
      side.push_back(s);
    }
    // one event per fork/join op (kernel ops need none: a program without branches touches no
    // HIP object on the host side, which is what the host-sanitizer test relies on)
    while (fork_ev.size() < ops.size()) {
      hipEvent_t e = nullptr;
      if (ops[fork_ev.size()].kind != Op::LAUNCH &&
          hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
        return -1;
      fork_ev.push_back(e);
    }
    return 0;
  }

  int run(hipStream_t main) {
    if (ensure_streams()) return -1;
    for (size_t i = 0; i < ops.size(); ++i) {
      Op& op = ops[i];
      hipStream_t s = op.slot == 0 ? main : side[op.slot - 1];
      int rc = 0;
      switch (op.kind) {
        case Op::LAUNCH: rc = op.fn(s); break;
        case Op::FORK:  // side waits for main
          rc = (int)hipEventRecord(fork_ev[i], main);
          if (!rc) rc = (int)hipStreamWaitEvent(side[op.slot - 1], fork_ev[i], 0);
          break;
        case Op::JOIN:  // main waits for side
          rc = (int)hipEventRecord(fork_ev[i], side[op.slot - 1]);
          if (!rc) rc = (int)hipStreamWaitEvent(main, fork_ev[i], 0);
          break;
      }
      if (rc) {
        fprintf(stderr, "hipzap: program op %zu failed rc=%d\n", i, rc);
        return rc;
      }
    }
    return 0;
  }
};

}  // namespace

size_t hz_excl_pad(const void* fn, size_t dyn) {
  static const size_t target = [] {
    const char* e = getenv("HIPZAP_EXCL_LDS");
    return e ? (size_t)strtoul(e, nullptr, 10) : (size_t)0;
  }();
  if (!target || target > 160 * 1024) return dyn;
  hipFuncAttributes a;
  if (hipFuncGetAttributes(&a, fn) != hipSuccess) return dyn;
  const size_t tot = a.sharedSizeBytes + dyn;
  return tot >= target ? dyn : dyn + (target - tot);
}

extern "C" {

HzProgram hz_prog_create(void) { return new Program(); }
void hz_prog_destroy(HzProgram p) { delete static_cast<Program*>(p); }
int hz_prog_num_ops(HzProgram p) { return (int)static_cast<Program*>(p)->ops.size(); }

static int add_op(Program* P, int slot, Op::Kind kind, std::function<int(hipStream_t)> fn) {
  if (P->exec) return -3;  // frozen after capture
  if (slot < 0 || slot > 8) return -4;
  if (slot > P->max_slot) P->max_slot = slot;
  P->ops.push_back(Op{slot, kind, std::move(fn)});
  return 0;
}

int hz_prog_add_conv(HzProgram h, const HzConvParams* cp, int cfg, int slot) {
  HzConvParams c = *cp;
  return add_op(static_cast<Program*>(h), slot, Op::LAUNCH,
                [c, cfg](hipStream_t s) { return hz_conv_launch(&c, cfg, s); });
}
int hz_prog_add_conv2(HzProgram h, const HzConvParams* a, const HzConvParams* b, int cfg, int slot) {
  HzConvParams c0 = *a, c1 = *b;
  return add_op(static_cast<Program*>(h), slot, Op::LAUNCH,
                [c0, c1, cfg](hipStream_t s) { return hz_conv2_launch(&c0, &c1, cfg, s); });
}
int hz_prog_add_maxpool(HzProgram h, const HzPoolParams* pp, int slot) {
  HzPoolParams c = *pp;
  return add_op(static_cast<Program*>(h), slot, Op::LAUNCH, [c](hipStream_t s) { return hz_maxpool_launch(&c, s); });
}
int hz_prog_add_avgpool(HzProgram h, const unsigned short* x, unsigned short* out, int N, int HW, int C, int blocked,
                        int slot) {
  return add_op(static_cast<Program*>(h), slot, Op::LAUNCH,
                [=](hipStream_t s) { return hz_avgpool_launch(x, out, N, HW, C, blocked, s); });
}
int hz_prog_add_preprocess(HzProgram h, const void* src, unsigned short* dst, int N, int Cin, int H, int W, int Cpad,
                           int mode, const float* mean, const float* inv_std, int slot) {
  return add_op(static_cast<Program*>(h), slot, Op::LAUNCH, [=](hipStream_t s) {
    return hz_preprocess_launch(src, dst, N, Cin, H, W, Cpad, mode, mean, inv_std, s);
  });
}
int hz_prog_add_memcpy(HzProgram h, void* dst, const void* src, size_t bytes, int slot) {
  return add_op(static_cast<Program*>(h), slot, Op::LAUNCH,
                [=](hipStream_t s) { return (int)hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, s); });
}
int hz_prog_add_lstm(HzProgram h, const HzLstmParams* lp, int slot) {
  HzLstmParams c = *lp;
  return add_op(static_cast<Program*>(h), slot, Op::LAUNCH, [c](hipStream_t s) { return hz_lstm_cell_launch(&c, s); });
}
int hz_prog_add_decoder(HzProgram h, const HzDecoderParams* dp, int slot) {
  HzDecoderParams c = *dp;
  return add_op(static_cast<Program*>(h), slot, Op::LAUNCH, [c](hipStream_t s) { return hz_decoder_launch(&c, s); });
}
int hz_prog_add_sampler(HzProgram h, const HzSamplerParams* sp, int slot) {
  HzSamplerParams c = *sp;
  return add_op(static_cast<Program*>(h), slot, Op::LAUNCH, [c](hipStream_t s) { return hz_sampler_launch(&c, s); });
}
int hz_prog_add_step_bump(HzProgram h, int* step, int n, int slot) {
  return add_op(static_cast<Program*>(h), slot, Op::LAUNCH, [=](hipStream_t s) { return hz_step_bump_launch(step, n, s); });
}
int hz_prog_add_fork(HzProgram h, int slot) {
  if (slot < 1) return -4;
  return add_op(static_cast<Program*>(h), slot, Op::FORK, nullptr);
}
int hz_prog_add_join(HzProgram h, int slot) {
  if (slot < 1) return -4;
  return add_op(static_cast<Program*>(h), slot, Op::JOIN, nullptr);
}

int hz_prog_run(HzProgram h, hipStream_t st) { return static_cast<Program*>(h)->run(st); }

int hz_prog_capture(HzProgram h, hipStream_t st) {
  Program* P = static_cast<Program*>(h);
  if (P->exec) return 0;
  if (P->ensure_streams()) return -1;
  hipError_t e = hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
  if (e != hipSuccess) return (int)e;
  int rc = P->run(st);
  hipGraph_t g = nullptr;
  e = hipStreamEndCapture(st, &g);
  if (rc) {
    if (g) (void)hipGraphDestroy(g);
    return rc;
  }
  if (e != hipSuccess) return (int)e;
  P->graph = g;
  hipGraphExec_t x = nullptr;
  e = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
  if (e != hipSuccess) return (int)e;
  // upload once so the first replay does not pay for it; then publish
  (void)hipGraphUpload(x, st);
  P->exec.store(x);
  return 0;
}

int hz_prog_prepare(HzProgram h) {  // the side streams / events a run needs, made before any run
  return static_cast<Program*>(h)->ensure_streams();
}

int hz_prog_is_captured(HzProgram h) { return static_cast<Program*>(h)->exec.load() != nullptr; }

int hz_prog_replay(HzProgram h, hipStream_t st) {
  Program* P = static_cast<Program*>(h);
  hipGraphExec_t x = P->exec.load();
  if (!x) return P->run(st);
  return (int)hipGraphLaunch(x, st);
}

double hz_prog_bench(HzProgram* progs, hipStream_t* streams, int n, int iters) {
  auto t0 = std::chrono::steady_clock::now();
  for (int it = 0; it < iters; ++it)
    for (int i = 0; i < n; ++i)
      if (hz_prog_replay(progs[i], streams[i])) return -1.0;
  for (int i = 0; i < n; ++i)
    if (hipStreamSynchronize(streams[i]) != hipSuccess) return -2.0;
  auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<double, std::micro>(t1 - t0).count();
}

int hz_prog_add_diag(HzProgram h, int kind, int blocks, int threads, void* a, void* b, long bytes, int slot) {
  return add_op(static_cast<Program*>(h), slot, Op::LAUNCH,
                [=](hipStream_t s) { return hz_diag_launch(kind, blocks, threads, a, b, bytes, s); });
}

// out[0] = host submission time (us), out[1] = submission + drain (us).
// threads != 0: one host thread per stream submits its own replays concurrently.
int hz_prog_bench2(HzProgram* progs, hipStream_t* streams, int n, int iters, int threads, double* out) {
  auto t0 = std::chrono::steady_clock::now();
  int rc = 0;
  if (!threads) {
    for (int it = 0; it < iters && !rc; ++it)
      for (int i = 0; i < n && !rc; ++i) rc = hz_prog_replay(progs[i], streams[i]);
  } else {
    std::vector<std::thread> th;
    std::vector<int> rcs(n, 0);
    for (int i = 0; i < n; ++i)
      th.emplace_back([&, i] {
        for (int it = 0; it < iters && !rcs[i]; ++it) rcs[i] = hz_prog_replay(progs[i], streams[i]);
      });
    for (auto& t : th) t.join();
    for (int r : rcs) rc |= r;
  }
  auto t1 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i)
    if (hipStreamSynchronize(streams[i]) != hipSuccess) rc = -2;
  auto t2 = std::chrono::steady_clock::now();
  out[0] = std::chrono::duration<double, std::micro>(t1 - t0).count();
  out[1] = std::chrono::duration<double, std::micro>(t2 - t0).count();
  return rc;
}

// Closed-loop serving benchmark: one host thread per context, each serving `iters` requests
// back to back the way a request thread does: copy the payload into the pinned input, replay,
// wait for THIS request's completion, copy the result out. Per-request latency (submission ->
// result in host memory) goes to lat_us[ctx * iters + i]; wall_us = total wall time. Unlike
// hz_prog_bench (replays queued back to back, no host work), every request here pays its own
// host copies and synchronisation, so throughput and p99 are what concurrent clients see.
int hz_serve_bench(HzProgram* progs, hipStream_t* streams, void** in_dst, void** in_src, uint64_t in_bytes,
                   void** out_src, void** out_dst, uint64_t out_bytes, int n, int iters, double* lat_us,
                   double* wall_us) {
  std::vector<std::thread> th;
  std::vector<int> rcs(n, 0);
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i)
    th.emplace_back([&, i] {
      for (int it = 0; it < iters && !rcs[i]; ++it) {
        auto a = std::chrono::steady_clock::now();
        if (in_bytes) memcpy(in_dst[i], in_src[i], in_bytes);
        int rc = hz_prog_replay(progs[i], streams[i]);
        if (!rc) rc = (int)hipStreamSynchronize(streams[i]);
        if (!rc && out_bytes) memcpy(out_dst[i], out_src[i], out_bytes);
        rcs[i] = rc;
        lat_us[(size_t)i * iters + it] =
            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
      }
    });
  for (auto& t : th) t.join();
  *wall_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  int rc = 0;
  for (int r : rcs) rc |= r;
  return rc;
}

}  // extern "C"

// 1 when this library was built with the measured-negative experiment kernels (HZ_EXPERIMENTS)
extern "C" int hz_experiments(void) { return HZ_EXPERIMENTS; }

extern "C" int hz_prog_replay_n(HzProgram h, hipStream_t st, int n) {
  for (int i = 0; i < n; ++i) {
    const int rc = hz_prog_replay(h, st);
    if (rc) return rc;
  }
  return 0;
}

extern "C" int hz_launch_kernel(int kind, const void* prm, hipStream_t st) {
  switch (kind) {
    case HZ_K_LAYERNORM: return hz_layernorm_launch(static_cast<const HzLayerNormParams*>(prm), st);
    case HZ_K_EMBED: return hz_embed_ln_launch(static_cast<const HzEmbedParams*>(prm), st);
    case HZ_K_ATTENTION: return hz_attention_launch(static_cast<const HzAttentionParams*>(prm), st);
    case HZ_K_VIT_TOKENS: return hz_vit_tokens_launch(static_cast<const HzVitTokensParams*>(prm), st);
    case HZ_K_LSTM: return hz_lstm_cell_launch(static_cast<const HzLstmParams*>(prm), st);
    case HZ_K_DECODER: return hz_decoder_launch(static_cast<const HzDecoderParams*>(prm), st);
    case HZ_K_SAMPLER: return hz_sampler_launch(static_cast<const HzSamplerParams*>(prm), st);
    case HZ_K_MAXPOOL: return hz_maxpool_launch(static_cast<const HzPoolParams*>(prm), st);
    case HZ_K_QUANT: return hz_quant_launch(static_cast<const HzQuantParams*>(prm), st);
    case HZ_K_GEMM_FP8: return hz_gemm_fp8_launch(static_cast<const HzGemmFp8Params*>(prm), st);
    case HZ_K_SOFTMAX: return hz_softmax_launch(static_cast<const HzSoftmaxParams*>(prm), st);
    case HZ_K_POOL_FC: return hz_pool_fc_launch(static_cast<const HzPoolFcParams*>(prm), st);
    case HZ_K_LMB_LAYER: return hz_lmb_layer_launch(static_cast<const HzLmbLayerParams*>(prm), st);
    case HZ_K_LMB_DEC: return hz_lmb_dec_launch(static_cast<const HzLmbDecParams*>(prm), st);
    case HZ_K_LMB_ADMIT: return hz_lmb_admit_launch(static_cast<const HzLmbAdmitParams*>(prm), st);
    case HZ_K_QKVATT: return hz_qkvatt_launch(static_cast<const HzQkvAttParams*>(prm), st);
    case HZ_K_STEM: return hz_stem_launch(static_cast<const HzStemParams*>(prm), st);
    case HZ_K_BNECK: return hz_bneck_launch(static_cast<const HzBneckParams*>(prm), st);
    case HZ_K_SEAM: return hz_seam_launch(static_cast<const HzSeamParams*>(prm), st);
    case HZ_K_KCONV: return hz_kconv_launch(static_cast<const HzKconvParams*>(prm), st);
    default: return -100;
  }
}

// bytes of the parameter struct hz_launch_kernel reads for `kind` (0: unknown kind)
extern "C" size_t hz_kernel_param_size(int kind) {
  switch (kind) {
    case HZ_K_LAYERNORM: return sizeof(HzLayerNormParams);
    case HZ_K_EMBED: return sizeof(HzEmbedParams);
    case HZ_K_ATTENTION: return sizeof(HzAttentionParams);
    case HZ_K_VIT_TOKENS: return sizeof(HzVitTokensParams);
    case HZ_K_LSTM: return sizeof(HzLstmParams);
    case HZ_K_DECODER: return sizeof(HzDecoderParams);
    case HZ_K_SAMPLER: return sizeof(HzSamplerParams);
    case HZ_K_MAXPOOL: return sizeof(HzPoolParams);
    case HZ_K_QUANT: return sizeof(HzQuantParams);
    case HZ_K_GEMM_FP8: return sizeof(HzGemmFp8Params);
    case HZ_K_SOFTMAX: return sizeof(HzSoftmaxParams);
    case HZ_K_POOL_FC: return sizeof(HzPoolFcParams);
    case HZ_K_LMB_LAYER: return sizeof(HzLmbLayerParams);
    case HZ_K_LMB_DEC: return sizeof(HzLmbDecParams);
    case HZ_K_LMB_ADMIT: return sizeof(HzLmbAdmitParams);
    case HZ_K_QKVATT: return sizeof(HzQkvAttParams);
    case HZ_K_STEM: return sizeof(HzStemParams);
    case HZ_K_BNECK: return sizeof(HzBneckParams);
    case HZ_K_SEAM: return sizeof(HzSeamParams);
    case HZ_K_KCONV: return sizeof(HzKconvParams);
    default: return 0;
  }
}

extern "C" int hz_prog_add_kernel(HzProgram h, int kind, const void* params, size_t size, int slot) {
  // the launcher reads a whole parameter struct: refuse unknown kinds and short records (a plan
  // image's op record, for instance) instead of reading past them when the op is replayed
  const size_t need = hz_kernel_param_size(kind);
  if (!need || size < need) return -101;
  auto buf = std::make_shared<std::vector<char>>(static_cast<const char*>(params), static_cast<const char*>(params) + size);
  return add_op(static_cast<Program*>(h), slot, Op::LAUNCH,
                [buf, kind](hipStream_t s) { return hz_launch_kernel(kind, buf->data(), s); });
}
