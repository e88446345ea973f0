// Per-CU operand-staging rate of a GEMM-like stage loop (profiles/r5_mx: cfg 24's two 8-wave
// workgroups per CU move ~36 GB/s per CU, every one-workgroup-per-CU MX tile built ~11-15): each
// wave issues L 1-KiB loads (64 lanes x 16 B) of a "stage", waits for them (vmcnt 0: one stage in
// flight, as the NS = 2 kernels), then a workgroup barrier, for S stages; through VGPRs or through
// global_load_lds into an LDS ring. The source is a 32 MB window (L2 / Infinity Cache resident, as
// the GEMM operands) read at a different offset per workgroup and stage. Prints GB/s per CU for
// workgroups per CU x waves per workgroup x loads per wave per stage x path.
//   hipcc --offload-arch=gfx950 -O3 cu_stage_bw.hip -o cu_stage_bw && ./cu_stage_bw
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void glds16(const void* g, void* lds) {
  __builtin_amdgcn_global_load_lds(g, (lds_void*)lds, 16, 0, 0);
}

template <int L, bool DMA>
__global__ void stage_kernel(const u32x4* __restrict__ src, long win16, int stages, unsigned* out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];  // DMA: [waves][L] KiB
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  unsigned acc = 0;
  for (int s = 0; s < stages; ++s) {
    // this wave's L KiB of stage s: a pseudo-random 1-KiB-aligned spot of the window
    const long base = (((long)blockIdx.x * 7919 + (long)s * 104729 + wave * 131) * L * 64) % (win16 - L * 64);
    const long b = base & ~63l;
    if constexpr (DMA) {
#pragma unroll
      for (int i = 0; i < L; ++i) glds16(src + b + i * 64 + lane, lds + ((wave * L + i) << 10));
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      u32x4 v[L];
#pragma unroll
      for (int i = 0; i < L; ++i) v[i] = src[b + i * 64 + lane];
#pragma unroll
      for (int i = 0; i < L; ++i) acc ^= v[i][0] ^ v[i][3];
    }
    __syncthreads();
  }
  if (DMA) acc ^= reinterpret_cast<const unsigned*>(lds)[threadIdx.x];
  if (acc == 0x9e3779b9u) out[blockIdx.x] = acc;  // keep the loads
  (void)nw;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int L, bool DMA>
int run(const u32x4* src, long win16, unsigned* out, int cus, int wgpc, int waves) {
  const int stages = 64, grid = cus * wgpc, block = 64 * waves;
  const size_t lds = DMA ? (size_t)waves * L * 1024 : 0;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL((stage_kernel<L, DMA>), dim3(grid), dim3(block), lds, 0, src, win16, stages, out);
  CK(hipEventRecord(a));
  const int reps = 5;
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((stage_kernel<L, DMA>), dim3(grid), dim3(block), lds, 0, src, win16, stages, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const double bytes = (double)reps * grid * waves * L * 1024.0 * stages;
  const double us = ms * 1e3 / reps;
  printf("{\"wg_per_cu\": %d, \"waves\": %d, \"kib_per_wave_stage\": %d, \"path\": \"%s\", \"kib_in_flight_per_cu\": %d, "
         "\"us\": %.2f, \"gb_s_per_cu\": %.1f, \"tb_s_chip\": %.2f}\n",
         wgpc, waves, L, DMA ? "lds_dma" : "vgpr", wgpc * waves * L, us, bytes / reps / (us * 1e-6) / cus / 1e9,
         bytes / reps / (us * 1e-6) / 1e12);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return 0;
}

int main() {
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const long win = 32l << 20, win16 = win / 16;
  u32x4* src;
  unsigned* out;
  CK(hipMalloc(&src, win));
  CK(hipMalloc(&out, 1 << 20));
  CK(hipMemset(src, 1, win));
  for (int wgpc : {1, 2})
    for (int waves : {4, 8}) {
      if (run<4, false>(src, win16, out, cus, wgpc, waves)) return 1;
      if (run<8, false>(src, win16, out, cus, wgpc, waves)) return 1;
      if (run<4, true>(src, win16, out, cus, wgpc, waves)) return 1;
      if (run<8, true>(src, win16, out, cus, wgpc, waves)) return 1;
    }
  CK(hipDeviceSynchronize());
  CK(hipFree(src));
  CK(hipFree(out));
  return 0;
}
