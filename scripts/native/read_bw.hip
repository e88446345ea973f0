// HBM read-bandwidth ceiling probe: sum-reduce B bytes with 16-B loads, N loads in flight per
// lane, one-shot (each wave reads N * 1 KB once) vs grid-stride; buffers alternate between two
// 160 MB regions (> 256 MB Infinity Cache together) so every launch streams from HBM.
//   hipcc --offload-arch=gfx950 -O3 read_bw.hip -o read_bw && ./read_bw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int N>
__global__ __launch_bounds__(256) void oneshot(const u32x4* __restrict__ p, long n16, float* out) {
  const long base = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * N * 64 + (threadIdx.x & 63);
  u32x4 v[N];
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = base + i * 64 < n16 ? p[base + i * 64] : u32x4{0, 0, 0, 0};
  unsigned s = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) s += v[i][0] ^ v[i][1] ^ v[i][2] ^ v[i][3];
  if (s == 0x12345678u) out[blockIdx.x] = (float)s;
}

template <int N>
__global__ __launch_bounds__(256) void stride(const u32x4* __restrict__ p, long n16, float* out) {
  unsigned s = 0;
  const long step = (long)gridDim.x * 256 * N;
  for (long b = (long)blockIdx.x * 256 * N + threadIdx.x; b < n16; b += step) {
    u32x4 v[N];
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = b + i * 256 < n16 ? p[b + i * 256] : u32x4{0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < N; ++i) s += v[i][0] ^ v[i][1] ^ v[i][2] ^ v[i][3];
  }
  if (s == 0x12345678u) out[blockIdx.x] = (float)s;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
  const long bytes = 150l << 20, n16 = bytes / 16;
  char* buf;
  float* out;
  CK(hipMalloc(&buf, 2 * bytes + 4096));
  CK(hipMalloc(&out, 1 << 20));
  CK(hipMemset(buf, 1, 2 * bytes));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const char* name, auto launch) -> int {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int r = 0; r < 20; ++r) launch((const u32x4*)(buf + (r & 1) * bytes));
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(a, st));
    for (int i = 0; i < 5; ++i) CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / 100;
    printf("{\"kernel\": \"%s\", \"us\": %.2f, \"TB_s\": %.3f}\n", name, us, bytes / us / 1e6);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    return 0;
  };
#define ONESHOT(N) \
  run("oneshot_" #N, [&](const u32x4* p) { hipLaunchKernelGGL((oneshot<N>), dim3((n16 + N * 256 - 1) / (N * 256)), dim3(256), 0, st, p, n16, out); })
#define STRIDE(N, G) \
  run("stride_" #N "_g" #G, [&](const u32x4* p) { hipLaunchKernelGGL((stride<N>), dim3(G), dim3(256), 0, st, p, n16, out); })
  if (ONESHOT(4) || ONESHOT(8) || ONESHOT(16)) return 1;
  if (STRIDE(4, 1024) || STRIDE(8, 1024) || STRIDE(4, 2048) || STRIDE(8, 2048) || STRIDE(16, 1024) || STRIDE(8, 4096)) return 1;
  return 0;
}
