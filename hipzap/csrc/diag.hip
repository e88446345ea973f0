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
}  // namespace

extern "C" int hz_diag_launch(int kind, int blocks, int threads, void* a, void* b, long bytes, hipStream_t st) {
  if (kind == 0) hipLaunchKernelGGL(noop_kernel, dim3(blocks), dim3(threads), 0, st, (int*)a);
  else hipLaunchKernelGGL(copy_kernel, dim3(blocks), dim3(threads), 0, st, (const u32x4*)a, (u32x4*)b, bytes / 16);
  return (int)hipGetLastError();
}
