// Where do the fused ResNet kernels (csrc/block.hip) spend their time? s_memrealtime stamps (100 MHz)
// of wave 0 of every workgroup at the phase boundaries, for one launch of the stem kernel and of
// the two layer1 bottleneck kernels at bs=1 (random operands), next to the per-launch time of 64
// back-to-back launches captured in a hipGraph. Stem phases: 0 start, 1 patch in LDS, 2 MFMAs
// done, 3 stem outputs in LDS, 4 pooled stores issued. Bottleneck phases: 0 start, 1 input patch
// in LDS, 2 conv1 done, 3 conv2 MFMAs done, 4 conv2 epilogue done, 5 conv3 MFMAs done, 6 stores.
// Layer2 bottleneck (weight-streaming): 0 start, 1 patch in LDS, 2 conv1 done, 3 conv2 done,
// 4 conv3 MFMAs done, 5 stores issued.
// Build + run: scripts/sessions/gpu_r4_stamps.sh (hipcc --offload-arch=gfx950 -I hipzap/csrc).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

__device__ unsigned long long g_bstamps[5][512][8];
__device__ unsigned long long g_bclock[5][512][2];  // s_memtime (shader clock) at the first / last stamp
#define HZ_BSTAMP 1
#define HZ_BSTAMP_DECL unsigned long long hz_bst[8] = {0, 0, 0, 0, 0, 0, 0, 0}, hz_clk0 = __builtin_amdgcn_s_memtime();
#define HZ_BSTAMP(i) hz_bst[i] = __builtin_amdgcn_s_memrealtime()
#define HZ_BSTAMP_FLUSH(kind)                                                            \
  do {                                                                                   \
    const unsigned long long clk1_ = __builtin_amdgcn_s_memtime();                      \
    if (threadIdx.x == 0 && blockIdx.x < 512) {                                          \
      for (int i_ = 0; i_ < 8; ++i_) g_bstamps[kind][blockIdx.x][i_] = hz_bst[i_];       \
      g_bclock[kind][blockIdx.x][0] = hz_clk0;                                           \
      g_bclock[kind][blockIdx.x][1] = clk1_;                                             \
    }                                                                                    \
  } while (0)
#include "../../hipzap/csrc/block.hip"

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::printf("{\"error\": \"%s line %d\"}\n", hipGetErrorString(e_), __LINE__);   \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

static void* dev_random(size_t bytes, unsigned seed, bool bf16) {
  std::vector<unsigned short> h((bytes + 1) / 2);
  srand(seed);
  for (auto& v : h) {
    // bf16 in [-0.06, 0.06] (weights / activations of a plausible scale); raw bits otherwise
    const float f = ((rand() % 2001) - 1000) * 6e-5f;
    unsigned u;
    memcpy(&u, &f, 4);
    v = bf16 ? (unsigned short)(u >> 16) : (unsigned short)rand();
  }
  void* d = nullptr;
  (void)hipMalloc(&d, h.size() * 2);
  (void)hipMemcpy(d, h.data(), h.size() * 2, hipMemcpyHostToDevice);
  return d;
}

static int report(const char* name, int kind, int nwg, int nph, double launch_us) {
  unsigned long long h[512][8], ck[512][2];
  CK(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_bstamps), sizeof(h), (size_t)kind * sizeof(h), hipMemcpyDeviceToHost));
  CK(hipMemcpyFromSymbol(ck, HIP_SYMBOL(g_bclock), sizeof(ck), (size_t)kind * sizeof(ck), hipMemcpyDeviceToHost));
  std::vector<double> mhz;
  for (int b = 0; b < nwg; ++b)
    if (h[b][nph - 1] > h[b][0]) mhz.push_back((double)(ck[b][1] - ck[b][0]) / (double)(h[b][nph - 1] - h[b][0]) * 100.0);
  std::sort(mhz.begin(), mhz.end());
  std::printf("{\"kernel\": \"%s\", \"workgroups\": %d, \"graph_launch_us\": %.2f, \"phase_us_median\": [", name, nwg,
              launch_us);
  for (int ph = 1; ph < nph; ++ph) {
    std::vector<double> d;
    for (int b = 0; b < nwg; ++b) d.push_back((double)(h[b][ph] - h[b][ph - 1]) * 0.01);  // 100 MHz ticks -> us
    std::sort(d.begin(), d.end());
    std::printf("%s%.2f", ph > 1 ? ", " : "", d[d.size() / 2]);
  }
  unsigned long long t0 = ~0ull, t1 = 0;
  for (int b = 0; b < nwg; ++b) {
    t0 = std::min(t0, h[b][0]);
    t1 = std::max(t1, h[b][nph - 1]);
  }
  std::vector<double> st;
  for (int b = 0; b < nwg; ++b) st.push_back((double)(h[b][0] - t0) * 0.01);
  std::sort(st.begin(), st.end());
  std::printf("], \"first_to_last_us\": %.2f, \"start_skew_us_p50_max\": [%.2f, %.2f], \"shader_mhz_p50\": %.0f}\n",
              (double)(t1 - t0) * 0.01, st[st.size() / 2], st.back(), mhz.empty() ? 0.0 : mhz[mhz.size() / 2]);
  return 0;
}

template <class F>
static double graph_us(F launch, hipStream_t st, int n) {
  hipGraph_t g;
  hipGraphExec_t ge;
  (void)hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
  for (int i = 0; i < n; ++i) launch();
  (void)hipStreamEndCapture(st, &g);
  (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  for (int w = 0; w < 30; ++w) (void)hipGraphLaunch(ge, st);  // ~clock ramp before the timed replays
  (void)hipStreamSynchronize(st);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a, st);
  for (int r = 0; r < 5; ++r) (void)hipGraphLaunch(ge, st);
  (void)hipEventRecord(b, st);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipGraphExecDestroy(ge);
  (void)hipGraphDestroy(g);
  return ms * 1e3 / (5.0 * n);
}

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  // ---- stem: 224x224x3 uint8 image (device memory) -> [1][2][56][56][32]
  HzStemParams sp{};
  sp.src = dev_random(224 * 224 * 3, 1, false);
  sp.w = (const unsigned short*)dev_random(4 * 13 * 512 * 2, 2, true);
  sp.bias = (const float*)dev_random(64 * 4, 3, false);
  CK(hipMemset((void*)sp.bias, 0, 256));
  CK(hipMalloc((void**)&sp.out, 2 * 56 * 56 * 32 * 2));
  sp.N = 1, sp.H = 224, sp.W = 224, sp.mode = 1, sp.SH = 112, sp.SW = 112, sp.PH = 56, sp.PW = 56, sp.norm = 1;
  for (int c = 0; c < 3; ++c) sp.mean[c] = 0.45f, sp.inv_std[c] = 4.4f;
  CK((hipError_t)hz_stem_launch(&sp, st));
  CK(hipStreamSynchronize(st));
  const double t_stem = graph_us([&] { hz_stem_launch(&sp, st); }, st, 64);
  report("stem", 0, 98, 5, t_stem);
  // ---- layer1 bottlenecks at 56x56
  for (int th : {8, 4})
  for (int cin : {64, 256}) {
    HzBneckParams bp{};
    bp.x = (const unsigned short*)dev_random((size_t)cin * 56 * 56 * 2, 4, true);
    bp.w1 = (const unsigned short*)dev_random((size_t)64 * cin * 2, 5, true);
    bp.b1 = (const float*)dev_random(1024, 6, false);
    bp.w2 = (const unsigned short*)dev_random((size_t)64 * 576 * 2, 7, true);
    bp.b2 = (const float*)dev_random(1024, 8, false);
    bp.w3 = (const unsigned short*)dev_random((size_t)256 * 64 * 2, 9, true);
    bp.b3 = (const float*)dev_random(1024, 10, false);
    for (const float* b : {bp.b1, bp.b2, bp.b3}) CK(hipMemset((void*)b, 0, 1024));
    if (cin == 64) {
      bp.wd = (const unsigned short*)dev_random((size_t)256 * 64 * 2, 11, true);
      bp.bd = (const float*)dev_random(1024, 12, false);
      CK(hipMemset((void*)bp.bd, 0, 1024));
    }
    CK(hipMalloc((void**)&bp.out, (size_t)256 * 56 * 56 * 2));
    bp.N = 1, bp.H = 56, bp.W = 56, bp.Cin = cin, bp.Cmid = 64, bp.Cout = 256, bp.tile_h = th;
    CK((hipError_t)hz_bneck_launch(&bp, st));
    CK(hipStreamSynchronize(st));
    const double t = graph_us([&] { hz_bneck_launch(&bp, st); }, st, 64);
    char name[64];
    snprintf(name, sizeof name, "bneck_cin%d%s_th%d", cin, cin == 64 ? "_ds" : "", th);
    report(name, cin == 64 ? 1 : 2, 56 / th * 7, 7, t);
  }
  // ---- layer2 identity bottleneck at 28x28 (Cin = Cout = 512, Cmid 128)
  {
    HzBneckParams bp{};
    bp.x = (const unsigned short*)dev_random((size_t)512 * 28 * 28 * 2, 14, true);
    bp.w1 = (const unsigned short*)dev_random((size_t)128 * 512 * 2, 15, true);
    bp.b1 = (const float*)dev_random(2048, 16, false);
    bp.w2 = (const unsigned short*)dev_random((size_t)128 * 1152 * 2, 17, true);
    bp.b2 = (const float*)dev_random(2048, 18, false);
    bp.w3 = (const unsigned short*)dev_random((size_t)512 * 128 * 2, 19, true);
    bp.b3 = (const float*)dev_random(2048, 20, false);
    for (const float* b : {bp.b1, bp.b2, bp.b3}) CK(hipMemset((void*)b, 0, 2048));
    CK(hipMalloc((void**)&bp.out, (size_t)512 * 28 * 28 * 2));
    bp.N = 1, bp.H = 28, bp.W = 28, bp.Cin = 512, bp.Cmid = 128, bp.Cout = 512;
    CK((hipError_t)hz_bneck_launch(&bp, st));
    CK(hipStreamSynchronize(st));
    const double t = graph_us([&] { hz_bneck_launch(&bp, st); }, st, 64);
    report("bneck2_cin512", 3, 49, 6, t);
  }
  // ---- first layer2 block: 56x56x256 -> 28x28x512 (stride-2 3x3 and downsample)
  {
    HzBneckParams bp{};
    bp.x = (const unsigned short*)dev_random((size_t)256 * 56 * 56 * 2, 24, true);
    bp.w1 = (const unsigned short*)dev_random((size_t)128 * 256 * 2, 25, true);
    bp.b1 = (const float*)dev_random(2048, 26, false);
    bp.w2 = (const unsigned short*)dev_random((size_t)128 * 1152 * 2, 27, true);
    bp.b2 = (const float*)dev_random(2048, 28, false);
    bp.w3 = (const unsigned short*)dev_random((size_t)512 * 128 * 2, 29, true);
    bp.b3 = (const float*)dev_random(2048, 30, false);
    bp.wd = (const unsigned short*)dev_random((size_t)512 * 256 * 2, 31, true);
    bp.bd = (const float*)dev_random(2048, 32, false);
    for (const float* b : {bp.b1, bp.b2, bp.b3, bp.bd}) CK(hipMemset((void*)b, 0, 2048));
    CK(hipMalloc((void**)&bp.out, (size_t)512 * 28 * 28 * 2));
    bp.N = 1, bp.H = 28, bp.W = 28, bp.Cin = 256, bp.Cmid = 128, bp.Cout = 512;
    CK((hipError_t)hz_bneck_launch(&bp, st));
    CK(hipStreamSynchronize(st));
    const double t = graph_us([&] { hz_bneck_launch(&bp, st); }, st, 64);
    report("bneck2d_cin256_ds", 4, 49, 6, t);
  }
  return 0;
}
