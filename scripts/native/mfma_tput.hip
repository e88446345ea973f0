#include <hip/hip_runtime.h>
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
template <int MODE>
__global__ __launch_bounds__(256) void mfma_tput(float* out, int iters) {
  const int l = threadIdx.x;
  i32x8 a = {l, l + 1, l + 2, l + 3, l, l, l, l}, b = a;
  f32x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  f32x16 d0 = {}, d1 = {}, d2 = {}, d3 = {};
  f32x4 e0 = c0, e1 = c0, e2 = c0, e3 = c0;
  for (int i = 0; i < iters; ++i) {
    if constexpr (MODE == 0) {
      c0 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c0, 0, 0, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
      c1 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c1, 0, 0, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
      c2 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c2, 0, 0, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
      c3 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c3, 0, 0, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
    } else if constexpr (MODE == 1) {
      d0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, d0, 0, 0, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
      d1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, d1, 0, 0, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
      d2 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, d2, 0, 0, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
      d3 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, d3, 0, 0, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
    } else if constexpr (MODE == 2) {
      const long x = ((long)a[0] << 32) | a[1];
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(x, x, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(x, x, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(x, x, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(x, x, c3, 0, 0, 0);
    } else if constexpr (MODE == 5) {  // 16x16x32 bf16 with 8 independent accumulators
      bf16x8 x = __builtin_bit_cast(bf16x8, __builtin_shufflevector(a, a, 0, 1, 2, 3));
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, x, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, x, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, x, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, x, c3, 0, 0, 0);
        e0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, x, e0, 0, 0, 0);
        e1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, x, e1, 0, 0, 0);
        e2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, x, e2, 0, 0, 0);
        e3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, x, e3, 0, 0, 0);
      }
    } else if constexpr (MODE == 4) {
      bf16x8 x = __builtin_bit_cast(bf16x8, __builtin_shufflevector(a, a, 0, 1, 2, 3));
      d0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, x, d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, x, d1, 0, 0, 0);
      d2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, x, d2, 0, 0, 0);
      d3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, x, d3, 0, 0, 0);
    } else {
      bf16x8 x = __builtin_bit_cast(bf16x8, __builtin_shufflevector(a, a, 0, 1, 2, 3));
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, x, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, x, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, x, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, x, c3, 0, 0, 0);
    }
  }
  float s = c0[0] + c1[1] + c2[2] + c3[3] + d0[0] + d1[1] + d2[2] + d3[3] + e0[0] + e1[1] + e2[2] + e3[3];
  out[blockIdx.x * 256 + l] = s;
}

// MFMA issue-rate probe: every wave runs `iters` x 4 independent MFMAs; grid = 4 x 256 CUs.
// FLOP per instruction: scaled 16x16x128 = 65536, scaled 32x32x64 = 131072, fp8 16x16x32 = 16384,
// bf16 16x16x32 = 16384.
#include <cstdio>
int main() {
  float* out = nullptr;
  const int blocks = 1024, iters = 4096;
  if (hipMalloc(&out, blocks * 256 * sizeof(float)) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[6] = {"scale_16x16x128_f8", "scale_32x32x64_f8", "16x16x32_fp8", "16x16x32_bf16", "32x32x16_bf16",
                          "16x16x32_bf16_8acc"};
  const double flop[6] = {65536, 131072, 16384, 16384, 32768, 16384 * 4};  // mode 5: 16 MFMAs per iteration
  for (int rep = 0; rep < 2; ++rep)
    for (int m = 0; m < 6; ++m) {
      void (*k)(float*, int) = m == 0 ? mfma_tput<0> : m == 1 ? mfma_tput<1> : m == 2 ? mfma_tput<2> : m == 3 ? mfma_tput<3>
                             : m == 4 ? mfma_tput<4> : mfma_tput<5>;
      hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 16);
      hipEventRecord(e0, 0);
      hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, iters);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double total = (double)blocks * 4 * iters * 4 * flop[m];
      if (rep) std::printf("{\"mfma\": \"%s\", \"ms\": %.3f, \"tflops\": %.1f}\n", names[m], ms, total / ms / 1e9);
    }
  hipFree(out);
  return 0;
}
