// hipzap common device helpers — gfx950 (CDNA4) only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Exclusive-CU launches (A/B switch HIPZAP_EXCL_LDS=<bytes>, csrc/runtime.cpp hz_excl_pad): every
// HZ_LAUNCH asks for at least that much LDS (static + dynamic), so two workgroups -- of this kernel
// or of a concurrent request's -- never share a CU when it exceeds half of the 160 KiB. Off (0) by
// default: the dynamic LDS argument is passed through unchanged.
size_t hz_excl_pad(const void* fn, size_t dyn_lds);
#define HZ_LAUNCH(K, GRID, BLOCK, LDS, ST, ...) \
  hipLaunchKernelGGL(K, GRID, BLOCK, hz_excl_pad(reinterpret_cast<const void*>(&(K)), (LDS)), ST, __VA_ARGS__)

typedef unsigned short bf16_t;                                   // storage type
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));       // MFMA A/B fragment (4 VGPR)
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));         // 16x16 MFMA accumulator
typedef float f32x16 __attribute__((ext_vector_type(16)));       // 32x32 MFMA accumulator
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

#define HZ_WAVE 64

// HZ_EXPERIMENTS=1 (python -m hipzap.build --experiments -> libhipzap_exp.so, selected with
// HIPZAP_LIB): kernel variants that were built, measured and LOST against the defaults, kept for
// re-measurement but not shipped in the product library: the persistent conv
// chain (conv.hip, profiles/r3_chain), the 32x32x16 LDS-GEMM tiles cfg 64-77 (gemm.hip,
// profiles/r3_m32), the folded-LayerNorm GEMM epilogue (gemm.hip, profiles/r1_ab/bert_lnfold.txt)
// and the 256-row MX pipelines cfg 43-47 (fp8.hip, profiles/r3_mxk).
#ifndef HZ_EXPERIMENTS
#define HZ_EXPERIMENTS 0
#endif

// ---- DEBUG kernel variant (SURVEY.md §5 "bounds-check asserts in a DEBUG kernel variant") ----
// `python -m hipzap.build --debug` compiles every source with -DHZ_DEBUG into
// hipzap/_lib/libhipzap_debug.so; HIPZAP_DEBUG=1 makes hipzap._native load that library.
// HZ_DCHECK(cond) guards a global access or a launch contract: in the release build it is the
// constant `true` (compiled away); in the debug build a false condition records (line, block,
// thread) of the FIRST failure of the translation unit in a device word, counts all failures,
// and evaluates to false so the caller SKIPS the access — a failed check never faults the GPU
// (a kernel fault can reset every GPU of the host). The host reads and clears the records with
// hz_debug_poll_<unit>() after a sync (hipzap/utils/kcheck.py). Each .hip file that uses
// HZ_DCHECK instantiates its own record with HZ_DEBUG_UNIT(<unit>) at file scope.
#ifdef HZ_DEBUG
#define HZ_DEBUG_UNIT(UNIT)                                                             \
  static __device__ unsigned hz_dbg_rec[4];                                             \
  static __device__ __noinline__ bool hz_dbg_fail(int line) {                          \
    if (atomicCAS(&hz_dbg_rec[0], 0u, (unsigned)line) == 0u) {                          \
      atomicExch(&hz_dbg_rec[1], blockIdx.x + (blockIdx.y << 20));                      \
      atomicExch(&hz_dbg_rec[2], threadIdx.x);                                          \
    }                                                                                   \
    atomicAdd(&hz_dbg_rec[3], 1u);                                                      \
    return false;                                                                       \
  }                                                                                     \
  extern "C" int hz_debug_poll_##UNIT(unsigned* out) {                                  \
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(hz_dbg_rec), sizeof(hz_dbg_rec)) != hipSuccess) \
      return -1;                                                                        \
    const unsigned z[4] = {0, 0, 0, 0};                                                 \
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(hz_dbg_rec), z, sizeof(z));                \
  }
#define HZ_DCHECK(cond) (__builtin_expect(!!(cond), 1) ? true : hz_dbg_fail(__LINE__))
#else
#define HZ_DEBUG_UNIT(UNIT)
#define HZ_DCHECK(cond) true
#endif

#define HZ_CHECK(x)                                                              \
  do {                                                                           \
    hipError_t e__ = (x);                                                        \
    if (e__ != hipSuccess) {                                                     \
      fprintf(stderr, "hipzap: %s failed: %s (%s:%d)\n", #x,                     \
              hipGetErrorString(e__), __FILE__, __LINE__);                       \
      return (int)e__;                                                           \
    }                                                                            \
  } while (0)

// Deterministic cross-workgroup sums (the ResNet seam / K-split accumulators, csrc/block.hip): every
// term added into such an accumulator -- the preset bias and each workgroup's partial -- is first
// rounded to a multiple of 2^-10. While |sum| < 2^24 * 2^-10 = 16384 every partial sum of such terms
// is exactly representable in fp32, so the memory-side float atomics give the same bits in any
// arrival order (replays, stream counts, XCD placement). 16384 leaves 2x headroom over the largest
// accumulator of the random-init benchmark model (7,520 in layer4; trained ResNets stay in the tens);
// the rounding (<= 4.9e-4 per term) sits below the bf16 the consumer converts the sum to for the
// activations that matter (|x| >~ 0.1).
#ifdef HZ_NO_FIXQ  // (A/B build only: HIPZAP_CFLAGS=-DHZ_NO_FIXQ python -m hipzap.build --experiments)
__device__ __forceinline__ float hz_fixq(float x) { return x; }
#else
__device__ __forceinline__ float hz_fixq(float x) { return __builtin_rintf(x * 1024.f) * (1.f / 1024.f); }
#endif
__device__ __forceinline__ f32x4 hz_fixq4(f32x4 v) {
  return f32x4{hz_fixq(v[0]), hz_fixq(v[1]), hz_fixq(v[2]), hz_fixq(v[3])};
}

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((unsigned)v) << 16);
}
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32 (RNE, NaN-preserving)
  return __builtin_bit_cast(bf16_t, b);
}
// 8 bf16 packed in a uint4 <-> floats
__device__ __forceinline__ void unpack8(const u32x4 v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v[i] << 16);
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ unsigned pack2(float a, float b) {
  return (unsigned)f2bf(a) | ((unsigned)f2bf(b) << 16);
}
__device__ __forceinline__ u32x4 pack8(const float* f) {
  u32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = pack2(f[2 * i], f[2 * i + 1]);
  return r;
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Bijective XCD-aware remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective"):
// blocks b and b+8 share an XCD under round-robin dispatch; give each XCD a contiguous
// chunk of the logical id space. Pure speed choice, never a correctness assumption.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  if (nwg < 16) return bid;
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7, idx = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// a / b for 0 <= a < 2^24, 1 <= b < 2^24 with a / b < 2^20 (index math: tiles, pixels, K
// positions): a float-reciprocal estimate (within 1 of the quotient there) fixed up exactly --
// about 8 VALU instead of the ~20-instruction integer division sequence, which dominated the
// prologue of the bs=1 conv kernels (scripts/native/conv_stamps.hip). HZ_INT_DIV: plain division.
__device__ __forceinline__ int fdiv(int a, int b) {
#ifdef HZ_INT_DIV
  return a / b;
#else
  int q = (int)((float)a * __builtin_amdgcn_rcpf((float)b));
  const int r = a - q * b;
  q -= r < 0;
  q += r >= b;
  return q;
#endif
}

// Grouped tile raster: consecutive logical tiles (= one XCD's share after xcd_remap) walk
// group_m tile rows before the next column tile, so the XCD's L2 holds a group_m-row block of the
// row operand and a few column tiles of the other instead of whole row panels x ALL columns.
// group_m = 1 is the plain row-major raster.
__device__ __forceinline__ void grouped_tile(int lid, int tiles_m, int tiles_n, int group_m, int& tile_m, int& tile_n) {
  const int per_group = group_m * tiles_n, gid = lid / per_group, first_m = gid * group_m;
  const int gsz = min(tiles_m - first_m, group_m);
  tile_m = first_m + (lid - gid * per_group) % gsz;
  tile_n = (lid - gid * per_group) / gsz;
}

__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
}

// 4 floats -> 4 OCP e4m3fn bytes (gfx950 v_cvt_pk_fp8_f32; callers clamp to +-448 first)
__device__ __forceinline__ unsigned pack4_fp8(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return (unsigned)w;
}

// OCP MX E8M0 block scale for e4m3 data: the exponent e of the smallest power of two with
// amax / 2^e <= 448 (frexp: amax/448 = m * 2^e, m in [0.5, 1) => 2^e > amax/448); byte = e + 127.
__device__ __forceinline__ int mx_exp(float amax) {
  if (!(amax > 0.f)) return -127;
  int e;
  frexpf(amax * (1.f / 448.f), &e);
  return e < -127 ? -127 : (e > 127 ? 127 : e);
}

// ---- Philox4x32-10 Gumbel noise of the AWD-LSTM samplers (csrc/lstm.hip, csrc/lmbatch.hip):
// the key of vocabulary row j at step t of a request seeded `seed` is logit + gumbel(seed, t, j),
// the same function in both engines so a request samples the same tokens in either. One Philox
// block (counter (j >> 2, t, 0x5eed, 0), key = seed) yields the noise of the 4 rows 4(j>>2)..+3.
__device__ __forceinline__ u32x4 philox4(unsigned c0, unsigned c1, unsigned c2, unsigned c3, unsigned k0,
                                         unsigned k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const unsigned long long p0 = (unsigned long long)0xD2511F53u * c0;
    const unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c2;
    const unsigned h0 = (unsigned)(p0 >> 32), l0 = (unsigned)p0;
    const unsigned h1 = (unsigned)(p1 >> 32), l1 = (unsigned)p1;
    const unsigned n0 = h1 ^ c1 ^ k0, n2 = h0 ^ c3 ^ k1;
    c0 = n0;
    c1 = l1;
    c2 = n2;
    c3 = l0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return u32x4{c0, c1, c2, c3};
}

__device__ __forceinline__ float gumbel_of(unsigned r) {
  const float u = ((r >> 8) + 0.5f) * (1.0f / 16777216.0f);  // (0, 1)
  return -__logf(-__logf(u));
}

// noise of rows j0 .. j0+3 (j0 % 4 == 0): one Philox block
__device__ __forceinline__ f32x4 gumbel4(unsigned long long seed, int t, int j0) {
  const u32x4 r = philox4((unsigned)j0 >> 2, (unsigned)t, 0x5eedu, 0u, (unsigned)seed, (unsigned)(seed >> 32));
  return f32x4{gumbel_of(r[0]), gumbel_of(r[1]), gumbel_of(r[2]), gumbel_of(r[3])};
}

__device__ __forceinline__ float gumbel(unsigned long long seed, int t, int j) {
  const u32x4 r = philox4((unsigned)j >> 2, (unsigned)t, 0x5eedu, 0u, (unsigned)seed, (unsigned)(seed >> 32));
  const int q = j & 3;
  return gumbel_of(q == 0 ? r[0] : q == 1 ? r[1] : q == 2 ? r[2] : r[3]);
}
