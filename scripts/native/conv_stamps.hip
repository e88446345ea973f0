// Where does a bs=1 ResNet-50 conv kernel spend its ~3 us? Per-wave s_memtime stamps at the phase
// boundaries of conv_tile (start, prologue loads issued, K loop done, cross-wave reduction done,
// epilogue issued) for one launch of each representative shape, next to the per-launch time of
// 64 back-to-back launches captured in a hipGraph. Built and run by scripts/conv_stamps.sh.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

__device__ unsigned long long* g_stamps;
#define HZ_STAMP_DECL unsigned long long hz_st[5] = {0, 0, 0, 0, 0};
#define HZ_STAMP(i) hz_st[i] = __builtin_amdgcn_s_memtime()
#define HZ_STAMP_FLUSH                                                                          \
  do {                                                                                          \
    if ((threadIdx.x & 63) == 0 && g_stamps) {                                                  \
      unsigned long long* d = g_stamps + ((size_t)blockIdx.x * 16 + (threadIdx.x >> 6)) * 5;    \
      for (int i = 0; i < 5; ++i) d[i] = hz_st[i];                                              \
    }                                                                                           \
  } while (0)
#include "../../hipzap/csrc/conv.hip"

extern "C" int hz_gemm_lds_launch(const HzConvParams*, int, hipStream_t) { return -1; }

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      std::printf("{\"error\": \"%s line %d\"}\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                           \
    }                                                                     \
  } while (0)

struct Shape {
  const char* name;
  int H, W, C, Cout, R, stride, cfg, kw;
};

int run(const Shape& sh) {
  const int pad = sh.R / 2, P = (sh.H + 2 * pad - sh.R) / sh.stride + 1, Q = P;
  const int K = sh.R * sh.R * sh.C, ksteps = K / 32;
  const int cout_pad = (sh.Cout + 63) / 64 * 64;
  void *x, *w, *bias, *out;
  CK(hipMalloc(&x, (size_t)sh.H * sh.W * sh.C * 2));
  CK(hipMalloc(&w, (size_t)cout_pad / 16 * ksteps * 512 * 2));
  CK(hipMalloc(&bias, (size_t)sh.Cout * 4));
  CK(hipMalloc(&out, (size_t)P * Q * sh.Cout * 2));
  CK(hipMemset(x, 0, (size_t)sh.H * sh.W * sh.C * 2));
  CK(hipMemset(w, 0, (size_t)cout_pad / 16 * ksteps * 512 * 2));
  CK(hipMemset(bias, 0, (size_t)sh.Cout * 4));
  HzConvParams p{};
  p.x = (const unsigned short*)x;
  p.w = (const unsigned short*)w;
  p.bias = (const float*)bias;
  p.out = out;
  p.N = 1, p.H = sh.H, p.W = sh.W, p.C = sh.C, p.Cout = sh.Cout, p.R = sh.R, p.S = sh.R;
  p.stride = sh.stride, p.pad = pad, p.P = P, p.Q = Q, p.M = P * Q, p.K = K, p.ksteps = ksteps;
  p.act = 1, p.kw = sh.kw;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  // per-launch time inside a graph of 64 dependent launches (includes the kernel boundary)
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < 64; ++i)
    if (hz_conv_launch(&p, sh.cfg, st)) {
      std::printf("{\"error\": \"launch rejected\"}\n");
      return 1;
    }
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, st));
  CK(hipEventRecord(e0, st));
  for (int i = 0; i < 10; ++i) CK(hipGraphLaunch(ge, st));
  CK(hipEventRecord(e1, st));
  CK(hipStreamSynchronize(st));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us_per_launch = ms * 1e3 / (10 * 64);
  // one stamped launch
  const int tiles_n = (sh.Cout + 16 * (1 << (sh.cfg / 3)) - 1) / (16 * (1 << (sh.cfg / 3)));
  const int fp = 1 << (sh.cfg % 3);
  const int nwg = tiles_n * ((p.M + 16 * fp - 1) / (16 * fp));
  unsigned long long* d_st;
  CK(hipMalloc(&d_st, (size_t)nwg * 16 * 5 * 8));
  CK(hipMemset(d_st, 0, (size_t)nwg * 16 * 5 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &d_st, sizeof(d_st)));
  for (int rep = 0; rep < 2; ++rep) {  // the second launch runs with warm caches, like the graph
    if (hz_conv_launch(&p, sh.cfg, st)) return 1;
    CK(hipStreamSynchronize(st));
  }
  std::vector<unsigned long long> h((size_t)nwg * 16 * 5);
  CK(hipMemcpy(h.data(), d_st, h.size() * 8, hipMemcpyDeviceToHost));
  unsigned long long first = ~0ull, last = 0;
  double ph[4] = {0, 0, 0, 0};
  int nw = 0;
  for (int b = 0; b < nwg; ++b)
    for (int wv = 0; wv < sh.kw; ++wv) {
      const unsigned long long* s = &h[((size_t)b * 16 + wv) * 5];
      if (!s[0] || !s[4]) continue;
      first = std::min(first, s[0]);
      last = std::max(last, s[4]);
      for (int i = 0; i < 4; ++i) ph[i] += (double)(s[i + 1] - s[i]);
      ++nw;
    }
  const unsigned long long zero = 0;
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &zero, sizeof(zero)));
  std::printf("{\"shape\": \"%s\", \"cfg\": %d, \"kw\": %d, \"workgroups\": %d, \"waves\": %d, "
              "\"us_per_launch_in_graph\": %.2f, \"span_first_wave_start_to_last_wave_end_cycles\": %llu, "
              "\"mean_wave_cycles\": {\"prologue_issue\": %.0f, \"k_loop\": %.0f, \"reduce\": %.0f, \"epilogue_issue\": %.0f}}\n",
              sh.name, sh.cfg, sh.kw, nwg, nw, us_per_launch, last - first, ph[0] / nw, ph[1] / nw, ph[2] / nw,
              ph[3] / nw);
  CK(hipFree(d_st));
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipFree(x));
  CK(hipFree(w));
  CK(hipFree(bias));
  CK(hipFree(out));
  CK(hipStreamDestroy(st));
  return 0;
}

int main() {
  const Shape shapes[] = {
      {"layer3 1x1 196x256x1024", 14, 14, 1024, 256, 1, 1, 3, 16},
      {"layer3 3x3 196x256x2304", 14, 14, 256, 256, 3, 1, 3, 16},
      {"layer1 1x1 3136x64x256", 56, 56, 256, 64, 1, 1, 6, 4},
      {"layer4 3x3 49x512x4608", 7, 7, 512, 512, 3, 1, 3, 16},
      {"layer2 1x1 784x512x128", 28, 28, 128, 512, 1, 1, 3, 2},
  };
  for (const Shape& s : shapes)
    if (run(s)) return 1;
  return 0;
}
