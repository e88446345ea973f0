// Diagnostic kernels for measuring the launch/boundary floor of the runtime on MI355X:
// a no-op kernel and a 16-B-per-lane copy, both addable to a Program so their cost can be
// measured inside hipGraphs exactly like model kernels (scripts/diag_runtime.py).
#include <functional>

#include "common.h"
#include "hipzap.h"

namespace {
__global__ void noop_kernel(int* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 0x7fffffff) p[0] = 1;
}
__global__ __launch_bounds__(256) void copy_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst, long n16) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (long)gridDim.x * blockDim.x) dst[i] = src[i];
}

// Operand-layout probe for v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3, unit E8M0 scales):
// ab = [A: 16 rows x 128 k][B^T: 16 cols x 128 k] bytes; lane l loads byte j of its operand
// from k = kmap(layout, l, j); C is written through the standard 16x16 C/D map. The host test
// (tests/test_fp8_gpu.py) checks which (A map, B map) combinations give A @ B exactly.
__device__ __forceinline__ int probe_k(int layout, int l, int j) {
  if (layout == 0) return 32 * (l >> 4) + j;                   // 32 consecutive k per lane
  return 8 * (l >> 4) + 32 * (j >> 3) + (j & 7);               // 4 blocks of the 16x16x32 map
}
__global__ void probe_mfma_f8_kernel(const unsigned char* ab, float* c, int layout) {
  const int l = threadIdx.x;
  typedef int i32x8 __attribute__((ext_vector_type(8)));
  i32x8 a, b;
  unsigned char* pa = reinterpret_cast<unsigned char*>(&a);
  unsigned char* pb = reinterpret_cast<unsigned char*>(&b);
  for (int j = 0; j < 32; ++j) {  // layout bit 0: A's lane->k map, bit 1: B's
    pa[j] = ab[(l & 15) * 128 + probe_k(layout & 1, l, j)];
    pb[j] = ab[2048 + (l & 15) * 128 + probe_k((layout >> 1) & 1, l, j)];
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
  for (int i = 0; i < 4; ++i) c[(4 * (l >> 4) + i) * 16 + (l & 15)] = acc[i];
}

// Block-scale probe: ab = [A 16x128][B^T 16x128] e4m3 bytes (layout 0 map) + [64 x int scale_a]
// + [64 x int scale_b] (E8M0 in the low byte, opsel 0); writes D through the C/D map.
__global__ void probe_mfma_scale_kernel(const unsigned char* ab, float* c) {
  const int l = threadIdx.x;
  typedef int i32x8 __attribute__((ext_vector_type(8)));
  i32x8 a, b;
  unsigned char* pa = reinterpret_cast<unsigned char*>(&a);
  unsigned char* pb = reinterpret_cast<unsigned char*>(&b);
  for (int j = 0; j < 32; ++j) {
    pa[j] = ab[(l & 15) * 128 + probe_k(0, l, j)];
    pb[j] = ab[2048 + (l & 15) * 128 + probe_k(0, l, j)];
  }
  const int* sc = reinterpret_cast<const int*>(ab + 4096);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, sc[l], 0, sc[64 + l]);
  for (int i = 0; i < 4; ++i) c[(4 * (l >> 4) + i) * 16 + (l & 15)] = acc[i];
}

// Raw-register block-scale probe: ab = [A regs: 64 lanes x 32 B][B regs: 64 x 32 B]
// [scale_a: 64 x int][scale_b: 64 x int]; each lane's operand registers are loaded verbatim,
// so the host decides which register byte carries which value (maps a register byte to the
// scale lane that governs it: the K order the block scales assume).
__global__ void probe_mfma_scale_raw_kernel(const unsigned char* ab, float* c) {
  const int l = threadIdx.x;
  typedef int i32x8 __attribute__((ext_vector_type(8)));
  i32x8 a, b;
  unsigned char* pa = reinterpret_cast<unsigned char*>(&a);
  unsigned char* pb = reinterpret_cast<unsigned char*>(&b);
  for (int j = 0; j < 32; ++j) {
    pa[j] = ab[l * 32 + j];
    pb[j] = ab[2048 + l * 32 + j];
  }
  const int* sc = reinterpret_cast<const int*>(ab + 4096);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, sc[l], 0, sc[64 + l]);
  for (int i = 0; i < 4; ++i) c[(4 * (l >> 4) + i) * 16 + (l & 15)] = acc[i];
}
}  // namespace

extern "C" int hz_diag_launch(int kind, int blocks, int threads, void* a, void* b, long bytes, hipStream_t st) {
  if (kind == 4) {  // raw-register block-scale probe
    hipLaunchKernelGGL(probe_mfma_scale_raw_kernel, dim3(1), dim3(64), 0, st, (const unsigned char*)a, (float*)b);
    return (int)hipGetLastError();
  }
  if (kind == 3) {  // MFMA block-scale probe
    hipLaunchKernelGGL(probe_mfma_scale_kernel, dim3(1), dim3(64), 0, st, (const unsigned char*)a, (float*)b);
    return (int)hipGetLastError();
  }
  if (kind == 2) {  // MFMA f8f6f4 layout probe: blocks = layout id
    hipLaunchKernelGGL(probe_mfma_f8_kernel, dim3(1), dim3(64), 0, st, (const unsigned char*)a, (float*)b, blocks);
    return (int)hipGetLastError();
  }
  if (kind == 0) hipLaunchKernelGGL(noop_kernel, dim3(blocks), dim3(threads), 0, st, (int*)a);
  else hipLaunchKernelGGL(copy_kernel, dim3(blocks), dim3(threads), 0, st, (const u32x4*)a, (u32x4*)b, bytes / 16);
  return (int)hipGetLastError();
}
