// Vision helper kernels: NHWC max-pool, global average pool, image pre-processing.
//  All are HBM/latency bound: 16-B vector loads (8 bf16
// channels per lane), one output vector per lane, grid sized to the output.
#include "common.h"
#include "hipzap.h"

HZ_DEBUG_UNIT(vision)

namespace {

// K x K window. With K known at compile time (the ResNet 3x3/2 stem pool) every tap is loaded
// before the first max: out-of-range taps are clamped to the nearest border pixel, which lies in
// the same window (a window overlapping the image contains its clamped taps), so the max is
// unchanged and no load is predicated — one memory round trip instead of a dependent chain of
// K*K (the runtime-K loop below compiled to one wait per tap).
template <int K>
__global__ __launch_bounds__(256) void maxpool_kernel(const HzPoolParams p) {
  const int C8 = p.C >> 3;
  const long total = (long)p.N * p.P * p.Q * C8;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c8 = i % C8;
  long t = i / C8;
  const int q = t % p.Q;
  t /= p.Q;
  const int pp = t % p.P;
  const int n = t / p.P;
  float m[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) m[e] = -INFINITY;
  const int h0 = pp * p.stride - p.pad, w0 = q * p.stride - p.pad;
  if (!HZ_DCHECK(h0 < p.H && w0 < p.W && h0 + p.k > 0 && w0 + p.k > 0)) return;  // window overlaps the image
  if constexpr (K > 0) {
    u32x4 v[K * K];
#pragma unroll
    for (int r = 0; r < K; ++r) {
      const int ih = min(max(h0 + r, 0), p.H - 1);
#pragma unroll
      for (int s = 0; s < K; ++s) {
        const int iw = min(max(w0 + s, 0), p.W - 1);
        v[r * K + s] = *reinterpret_cast<const u32x4*>(p.x + (((long)n * p.H + ih) * p.W + iw) * p.C + c8 * 8);
      }
    }
#pragma unroll
    for (int j = 0; j < K * K; ++j) {
      float f[8];
      unpack8(v[j], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], f[e]);
    }
  } else {
    for (int r = 0; r < p.k; ++r) {
      const int ih = h0 + r;
      if ((unsigned)ih >= (unsigned)p.H) continue;
      for (int s = 0; s < p.k; ++s) {
        const int iw = w0 + s;
        if ((unsigned)iw >= (unsigned)p.W) continue;
        const u32x4 v = *reinterpret_cast<const u32x4*>(p.x + (((long)n * p.H + ih) * p.W + iw) * p.C + c8 * 8);
        float f[8];
        unpack8(v, f);
#pragma unroll
        for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], f[e]);
      }
    }
  }
  *reinterpret_cast<u32x4*>(p.out + i * 8) = pack8(m);
}

// [N, HW, C] -> [N, C]. One block per (image, 64 channels): 8 channel groups x 32 pixel
// lanes, so every lane issues only ceil(HW/32) independent 16-B loads (a serial HW loop per
// lane was a 49-deep dependent load chain: 15.7 us on MI355X), then an LDS reduction.
__global__ __launch_bounds__(256) void avgpool_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ out,
                                                      int N, int HW, int C, int blocked) {
  __shared__ float red[32][65];
  const int t = threadIdx.x, cg = t & 7, pl = t >> 3;
  const int cblk = C >> 6;
  const int n = blockIdx.x / cblk, c0 = (blockIdx.x - n * cblk) * 64;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int c = c0 + cg * 8;
  // blocked: [N][C/32][HW][32]; else NHWC [N][HW][C]
  const bf16_t* base = blocked ? x + (((long)n * (C >> 5) + (c >> 5)) * HW) * 32 + (c & 31) : x + (long)n * HW * C + c;
  const long pstride = blocked ? 32 : C;
  for (int j = pl; j < HW; j += 32) {
    float f[8];
    unpack8(*reinterpret_cast<const u32x4*>(base + (long)j * pstride), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] += f[e];
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[pl][cg * 8 + e] = s[e];
  __syncthreads();
  if (t < 64) {
    float a = 0.f;
#pragma unroll 8
    for (int q = 0; q < 32; ++q) a += red[q][t];
    out[(long)n * C + c0 + t] = f2bf(a / HW);
  }
}

// Fused global-average-pool + FC (one launch instead of avgpool + FC GEMM + a kernel boundary).
// Block = one 16-row weight group x one image (blockIdx.y); its 4 waves split the channels
// (K) four ways, so each wave pools ONLY its own C/4 channels (fp32, into its LDS slice) and
// then dots them with its K-quarter of the group's weights; the 4 partial sums meet in LDS.
// Pooling: lane l reads 16 B (8 channels) of channel block (l>>2) of the wave's slice at every
// pixel. Weights are fragment-major (one contiguous 1 KiB per 32-deep k-step); the 4 lanes
// sharing an output row (l, l^16, l^32, l^48) reduce by shuffles.
// Latency: the wave's first WB weight fragments are issued before the pooling (independent of
// it). NB = ceil(HW/8) > 0 additionally issues ALL pixel loads before the first use (one round
// trip instead of one per 8 pixels) but needs 384 VGPRs at HW = 49: one workgroup per CU, which
// measured -1.5 % at 8 concurrent request streams (profiles/r1_ab/vision_latency.txt), so the
// runtime loop (NB = 0) is the default (HZ_POOLFC_STATIC).
#ifndef HZ_POOLFC_PB
#define HZ_POOLFC_PB 16  // pixel loads in flight per lane in the runtime loop: 4 round trips at HW = 49 (8: 7)
#endif
template <int NB>
__global__ __launch_bounds__(256) void pool_fc_kernel(const HzPoolFcParams p) {
  extern __shared__ __attribute__((aligned(16))) float pooled[];  // [C] + [4][16] partials
  constexpr int WB = 16;  // weight fragments in flight per wave
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int b = blockIdx.y, g = blockIdx.x;
  const int ncb = p.C >> 5;
  const int cpw = (ncb + 3) >> 2;  // channel blocks per wave
  const int cb_lo = wave * cpw, cb_hi = min(ncb, cb_lo + cpw);
  const float inv = 1.f / p.HW;
  const int ks = p.C >> 5;
  const bf16_t* wg = p.w + ((long)g * ks * 64 + lane) * 8;
  if (!HZ_DCHECK(p.ldo >= p.N && p.C % 32 == 0)) return;
  // first batch of weight fragments: independent of the pooling, so in flight with it
  u32x4 wv[WB];
#pragma unroll
  for (int j = 0; j < WB; ++j) wv[j] = *reinterpret_cast<const u32x4*>(wg + (long)min(cb_lo + j, cb_hi - 1) * 512);
  if (p.pooled) {  // x = the fp32 channel means already (a tail seam, block.hip): copy the wave's slice
    const float* xp = reinterpret_cast<const float*>(p.x) + (long)b * p.C;
    for (int c = cb_lo * 32 + lane * 4; c < cb_hi * 32; c += 256)
      *reinterpret_cast<f32x4*>(pooled + c) = *reinterpret_cast<const f32x4*>(xp + c);
  }
  for (int cb0 = cb_lo; cb0 < (p.pooled ? cb_lo : cb_hi); cb0 += 16) {
    const int cb = cb0 + (lane >> 2), sub = lane & 3;
    if (cb < cb_hi) {
      const bf16_t* src = p.x + (((long)b * ncb + cb) * p.HW) * 32 + sub * 8;
      float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if constexpr (NB > 0) {
        u32x4 v[NB * 8];
#pragma unroll
        for (int j = 0; j < NB * 8; ++j) v[j] = *reinterpret_cast<const u32x4*>(src + min(j, p.HW - 1) * 32);
#pragma unroll
        for (int j = 0; j < NB * 8; ++j) {
          float f[8];
          unpack8(v[j], f);
          const float wj = j < p.HW ? 1.f : 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) s[e] += wj * f[e];
        }
      } else {
        for (int hw0 = 0; hw0 < p.HW; hw0 += HZ_POOLFC_PB) {  // PB independent loads in flight per lane
          u32x4 v[HZ_POOLFC_PB];
#pragma unroll
          for (int j = 0; j < HZ_POOLFC_PB; ++j)
            v[j] = *reinterpret_cast<const u32x4*>(src + min(hw0 + j, p.HW - 1) * 32);
#pragma unroll
          for (int j = 0; j < HZ_POOLFC_PB; ++j) {
            float f[8];
            unpack8(v[j], f);
            const float wj = hw0 + j < p.HW ? 1.f : 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) s[e] += wj * f[e];
          }
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) pooled[cb * 32 + sub * 8 + e] = s[e] * inv;
    }
  }
  // the wave reads back only its own slice: a wave-level LDS fence is enough
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const float* pl = pooled + (lane >> 4) * 8;
  float acc = 0.f;
  for (int k0 = cb_lo; k0 < cb_hi; k0 += WB) {
    if (k0 != cb_lo) {  // later batches (C/4 > WB*32 channels per wave)
#pragma unroll
      for (int j = 0; j < WB; ++j) wv[j] = *reinterpret_cast<const u32x4*>(wg + (long)min(k0 + j, cb_hi - 1) * 512);
    }
#pragma unroll
    for (int j = 0; j < WB; ++j) {
      const int k = min(k0 + j, cb_hi - 1);
      float f[8];
      unpack8(wv[j], f);
      const f32x4 p0 = *reinterpret_cast<const f32x4*>(pl + k * 32);
      const f32x4 p1 = *reinterpret_cast<const f32x4*>(pl + k * 32 + 4);
      const float d = f[0] * p0[0] + f[1] * p0[1] + f[2] * p0[2] + f[3] * p0[3] + f[4] * p1[0] + f[5] * p1[1] +
                      f[6] * p1[2] + f[7] * p1[3];
      acc += k0 + j < cb_hi ? d : 0.f;
    }
  }
  acc += __shfl_xor(acc, 16, 64);
  acc += __shfl_xor(acc, 32, 64);
  float* part = pooled + p.C;  // [4 waves][16 rows]
  if (lane < 16) part[wave * 16 + lane] = acc;
  __syncthreads();
  const int n = g * 16 + t;
  if (t < 16 && n < p.N)
    p.out[(long)b * p.ldo + n] = part[t] + part[16 + t] + part[32 + t] + part[48 + t] + (p.bias ? p.bias[n] : 0.f);
}

// mode 0: src fp32 NCHW (already normalised unless mean/inv_std given)
// mode 1: src uint8 NHWC (raw image bytes, normalised with mean/inv_std in 0..1 scale)
__global__ __launch_bounds__(256) void preprocess_kernel(const void* __restrict__ src, bf16_t* __restrict__ dst,
                                                         int N, int Cin, int H, int W, int Cpad, int mode,
                                                         const float* __restrict__ mean,
                                                         const float* __restrict__ inv_std) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;  // pixel index
  const long HWl = (long)H * W;
  if (i >= N * HWl) return;
  const long n = i / HWl, hw = i - n * HWl;
  // every channel's load (and the normalisation constants) issued before the first use: a
  // runtime channel loop waited once per channel — over PCIe when the request is read zero-copy
  float v[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    float f = 0.f;
    if (c < Cin) {
      if (mode == 0) f = reinterpret_cast<const float*>(src)[(n * Cin + c) * HWl + hw];
      else f = (float)reinterpret_cast<const unsigned char*>(src)[i * Cin + c] * (1.0f / 255.0f);
    }
    v[c] = f;
  }
  if (mean) {
#pragma unroll
    for (int c = 0; c < 8; ++c)
      if (c < Cin) v[c] = (v[c] - mean[c]) * inv_std[c];
  }
  bf16_t* o = dst + i * Cpad;
  *reinterpret_cast<u32x4*>(o) = pack8(v);
  for (int c = 8; c < Cpad; c += 8) *reinterpret_cast<u32x4*>(o + c) = u32x4{0, 0, 0, 0};
}

// uint8 HWC, 3 channels (the request payload of the vision models), read zero-copy from pinned host
// memory: the generic kernel's per-thread byte loads at stride 3 make every wave instruction touch the
// same three 64 B lines again (uncached over PCIe). Here a workgroup owns 1024 pixels = 3072 bytes:
// three fully coalesced dword loads per thread (768 distinct dwords, each read once), restaged through
// LDS so thread t then owns bytes [12t, 12t+12) = 4 whole pixels. Needs npix % 4 == 0 and a 4-byte
// aligned source (checked by the launcher; the generic kernel covers the rest).
__global__ __launch_bounds__(256) void preprocess_u8c3_kernel(const unsigned* __restrict__ src,
                                                              bf16_t* __restrict__ dst, long npix, int Cpad,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ inv_std) {
  __shared__ __attribute__((aligned(16))) unsigned buf[768];
  const int t = threadIdx.x;
  const long ndw = npix / 4 * 3;
  const long d0 = (long)blockIdx.x * 768;
  // the block's 3 KiB of request bytes as 16-B loads by threads 0..191 (zero-copy: the request is
  // read across PCIe, so fewer, wider requests: 1 KiB per wave instruction instead of 256 B)
  u32x4 r = u32x4{0u, 0u, 0u, 0u};
  if (t < 192) {
    const long d = d0 + 4 * t;
    if (d + 4 <= ndw) {
      r = *reinterpret_cast<const u32x4*>(src + d);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) r[k] = d + k < ndw ? src[d + k] : 0u;
    }
  }
  float mu[3] = {0.f, 0.f, 0.f}, is[3] = {1.f, 1.f, 1.f};
  if (mean) {
#pragma unroll
    for (int c = 0; c < 3; ++c) mu[c] = mean[c], is[c] = inv_std[c];
  }
  if (t < 192) *reinterpret_cast<u32x4*>(buf + 4 * t) = r;
  __syncthreads();
  const long px = (long)blockIdx.x * 1024 + 4 * t;
  if (px >= npix) return;
  const unsigned w[3] = {buf[3 * t], buf[3 * t + 1], buf[3 * t + 2]};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int b = 3 * q + c;  // byte within the thread's 12
      const float f = (float)((w[b >> 2] >> (8 * (b & 3))) & 0xffu) * (1.0f / 255.0f);
      v[c] = mean ? (f - mu[c]) * is[c] : f;
    }
    bf16_t* o = dst + (px + q) * Cpad;
    *reinterpret_cast<u32x4*>(o) = pack8(v);
    for (int c = 8; c < Cpad; c += 8) *reinterpret_cast<u32x4*>(o + c) = u32x4{0, 0, 0, 0};
  }
}

// mode 2 (ViT patch embedding as a plain GEMM): src fp32 NCHW -> bf16 patch rows
// [N * (H/P) * (W/P)][Cin * P * P], column (c, ky, kx) = the flattened [D][Cin][P][P] conv weight's
// K order, so the patch projection is a row-major GEMM with K = Cin * P * P (768 at P = 16, Cin = 3)
// instead of an implicit-GEMM conv over 8-channel padded pixels (K 2048). A thread owns one
// (patch, c, ky) run of P pixels: P / 4 16-B loads, P / 8 16-B stores.
template <int P>
__global__ __launch_bounds__(256) void patchify_kernel(const float* __restrict__ src, bf16_t* __restrict__ dst,
                                                       int N, int Cin, int H, int W,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ inv_std) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;  // (patch row, c, ky)
  const int px = W / P, py = H / P;
  const long runs = (long)N * py * px * Cin * P;
  if (i >= runs) return;
  const int ky = (int)(i % P);
  const long t = i / P;
  const int c = (int)(t % Cin);
  const long row = t / Cin;  // n * py * px + pyi * px + pxi
  const int pxi = (int)(row % px);
  const long t2 = row / px;
  const int pyi = (int)(t2 % py);
  const long n = t2 / py;
  const float* s = src + ((n * Cin + c) * H + (long)pyi * P + ky) * W + (long)pxi * P;
  float v[P];
#pragma unroll
  for (int q = 0; q < P / 4; ++q) {
    const f32x4 f = *reinterpret_cast<const f32x4*>(s + 4 * q);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[4 * q + e] = f[e];
  }
  if (mean) {
    const float mu = mean[c], is = inv_std[c];
#pragma unroll
    for (int e = 0; e < P; ++e) v[e] = (v[e] - mu) * is;
  }
  bf16_t* o = dst + row * ((long)Cin * P * P) + (c * P + ky) * P;
#pragma unroll
  for (int q = 0; q < P / 8; ++q) *reinterpret_cast<u32x4*>(o + 8 * q) = pack8(v + 8 * q);
}

__global__ void cast_f32_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, long n) {
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i + 3 < n) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(x + i);
    *reinterpret_cast<u32x2*>(y + i) = u32x2{pack2(v[0], v[1]), pack2(v[2], v[3])};
  } else {
    for (long j = i; j < n; ++j) y[j] = f2bf(x[j]);
  }
}
__global__ void cast_bf16_f32_kernel(const bf16_t* __restrict__ x, float* __restrict__ y, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = bf2f(x[i]);
}

}  // namespace

extern "C" int hz_maxpool_launch(const HzPoolParams* pp, hipStream_t st) {
  const HzPoolParams& p = *pp;
  if (p.C % 8) return -1;
  const long total = (long)p.N * p.P * p.Q * (p.C / 8);
  // clamped taps are only inside the window when the padding is smaller than the window
  if (p.k == 3 && p.pad < 3) HZ_LAUNCH(maxpool_kernel<3>, dim3((total + 255) / 256), dim3(256), 0, st, p);
  else HZ_LAUNCH(maxpool_kernel<0>, dim3((total + 255) / 256), dim3(256), 0, st, p);
  return (int)hipGetLastError();
}

extern "C" int hz_avgpool_launch(const unsigned short* x, unsigned short* out, int N, int HW, int C, int blocked,
                                 hipStream_t st) {
  if (C % 64) return -1;
  HZ_LAUNCH(avgpool_kernel, dim3(N * (C / 64)), dim3(256), 0, st, x, out, N, HW, C, blocked);
  return (int)hipGetLastError();
}

extern "C" int hz_pool_fc_launch(const HzPoolFcParams* pp, hipStream_t st) {
  const HzPoolFcParams& p = *pp;
  if (p.C % 32 || p.C > 16384 || p.HW < 1 || p.N < 1) return -1;
  const int groups = (p.N + 15) / 16;
  const size_t lds = (size_t)(p.C + 64) * sizeof(float);
  const dim3 grid(groups, p.B);
#ifndef HZ_POOLFC_STATIC
#define HZ_POOLFC_STATIC 0  // 1: measured -1.5 % at 8 streams (384 VGPRs, one workgroup per CU)
#endif
  switch (HZ_POOLFC_STATIC ? (p.HW + 7) / 8 : 0) {  // compile-time pixel batches: every pooling load in flight
    case 1: HZ_LAUNCH(pool_fc_kernel<1>, grid, dim3(256), lds, st, p); break;
    case 2: HZ_LAUNCH(pool_fc_kernel<2>, grid, dim3(256), lds, st, p); break;
    case 4: HZ_LAUNCH(pool_fc_kernel<4>, grid, dim3(256), lds, st, p); break;
    case 7: HZ_LAUNCH(pool_fc_kernel<7>, grid, dim3(256), lds, st, p); break;  // 7x7 (ResNet @224)
    default: HZ_LAUNCH(pool_fc_kernel<0>, grid, dim3(256), lds, st, p); break;
  }
  return (int)hipGetLastError();
}

#ifndef HZ_PREPROC_GENERIC
#define HZ_PREPROC_GENERIC 0  // 1: uint8 3-channel payloads through the generic per-pixel kernel (A/B)
#endif
extern "C" int hz_preprocess_launch(const void* src, unsigned short* dst, int N, int Cin, int H, int W, int Cpad,
                                    int mode, const float* mean, const float* inv_std, hipStream_t st) {
  if (mode == 2) {  // patch rows; Cpad carries the patch size
    if (Cpad != 16 || H % 16 || W % 16 || Cin < 1 || Cin > 8 || ((uintptr_t)src & 15) || ((uintptr_t)dst & 15))
      return -1;
    const long runs = (long)N * (H / 16) * (W / 16) * Cin * 16;
    HZ_LAUNCH(patchify_kernel<16>, dim3((runs + 255) / 256), dim3(256), 0, st,
                       static_cast<const float*>(src), reinterpret_cast<bf16_t*>(dst), N, Cin, H, W, mean, inv_std);
    return (int)hipGetLastError();
  }
  if (Cpad % 8 || Cin > 8) return -1;
  const long total = (long)N * H * W;
  if (mode == 1 && Cin == 3 && total % 4 == 0 && ((uintptr_t)src & 15) == 0 && !HZ_PREPROC_GENERIC) {
    HZ_LAUNCH(preprocess_u8c3_kernel, dim3((total + 1023) / 1024), dim3(256), 0, st,
                       static_cast<const unsigned*>(src), dst, total, Cpad, mean, inv_std);
    return (int)hipGetLastError();
  }
  HZ_LAUNCH(preprocess_kernel, dim3((total + 255) / 256), dim3(256), 0, st, src, dst, N, Cin, H, W, Cpad,
                     mode, mean, inv_std);
  return (int)hipGetLastError();
}

extern "C" int hz_cast_f32_bf16(const float* x, unsigned short* y, long n, hipStream_t st) {
  const long threads = (n + 3) / 4;
  HZ_LAUNCH(cast_f32_bf16_kernel, dim3((threads + 255) / 256), dim3(256), 0, st, x, y, n);
  return (int)hipGetLastError();
}
extern "C" int hz_cast_bf16_f32(const unsigned short* x, float* y, long n, hipStream_t st) {
  HZ_LAUNCH(cast_bf16_f32_kernel, dim3((n + 255) / 256), dim3(256), 0, st, x, y, n);
  return (int)hipGetLastError();
}

// Load this translation unit's device code now (hipFuncGetAttributes makes the runtime load the
// code object of the fatbin that holds the kernel, without a launch or a stream): the plan loader
// calls it on a helper thread while the weight blob uploads, so the first request does not pay
// the load (csrc/plan.cpp hz_plan_open).
__global__ void hz_vision_code_warm_kernel() {}
extern "C" int hz_vision_code_warm(void) {
  hipFuncAttributes a;
  return (int)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&hz_vision_code_warm_kernel));
}
