// LDS-tiled bf16 GEMM for large-M transformer projections (BERT bs=16: M = 2048 tokens).
//
//   out[m][n] = act( sum_k X[m][k] * W[n][k] + bias[n] (+ res[m][n]) ),  X row-major [M][ldx]
//
// The K-across-waves kernel (conv.hip) is right for bs=1 (every operand byte used once), but
// at M >= ~512 each weight fragment is re-read by every M tile and each activation fragment
// by every N tile straight from L2: per-CU load bandwidth, not MFMA, was the limit (BERT-base
// bs=16 at ~205 TFLOP/s). Here a 256-thread workgroup (2x2 waves) owns a BM x BN tile and
// stages BOTH operands through LDS once per 64-deep K step:
//   * operands are staged in MFMA fragment order — weights are already packed
//     fragment-major [N/16][K/32][64][8] (1 KiB per fragment, contiguous), activation fragments
//     are gathered per lane (16 rows x 64 B) — with global_load_lds (16 B per lane; the LDS image
//     is lane-linear, cdna_hip_programming.md §5 "Async global->LDS copy"), so every
//     ds_read_b128 of a fragment is lane-linear and bank-conflict free (no swizzle needed);
//   * each fragment read from LDS feeds 2-4 MFMAs (waves sharing a row or column of the tile);
//   * double-buffered stages: the glds of stage t+1 is issued before the MFMAs of stage t
//     ("Minimum 2-phase" recipe, §5.5 T3+T4), one vmcnt(0) + barrier per stage;
//   * same swapped orientation and fused epilogue as conv.hip (4 consecutive output features
//     per lane: 16-B bias, 8-B residual, 8-B store), XCD-aware tile order.
// Requirements (checked by the launcher): K % 64 == 0, ldx % 8 == 0, weight rows padded to 128.
#include "common.h"
#include "hipzap.h"

namespace {

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void glds16(const void* g, char* lds) {
  __builtin_amdgcn_global_load_lds(g, (lds_void*)lds, 16, 0, 0);
}

template <int BM, int BN>
__global__ __launch_bounds__(256) void gemm_lds_kernel(const HzConvParams p) {
  constexpr int FCW = BN / 32, FPW = BM / 32;  // fragments per wave (2x2 waves)
  constexpr int NWF = BN / 16, NAF = BM / 16;  // fragments per 32-deep k-step in the tile
  constexpr int KF = NWF + NAF;
  constexpr int STAGE_FR = 2 * KF;             // BK = 64 = two k-steps per stage
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE_FR * 1024];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave & 1, wm = wave >> 1;
  const int tiles_n = (p.Cout + BN - 1) / BN;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile_n = lid % tiles_n, tile_m = lid / tiles_n;
  const int n0 = tile_n * BN, m0 = tile_m * BM;
  const int nst = p.ksteps >> 1;

  // per-lane source row of each activation fragment this wave stages (clamped: rows >= M are
  // computed on duplicated data and never stored)
  auto stage = [&](int buf, int st) {
    char* base = smem + buf * STAGE_FR * 1024;
#pragma unroll
    for (int f = wave; f < STAGE_FR; f += 4) {
      const int ks = f / KF, q = f - ks * KF;
      const int kstep = st * 2 + ks;
      const void* src;
      if (q < NWF) {
        src = p.w + (((long)((n0 >> 4) + q) * p.ksteps + kstep) * 64 + lane) * 8;
      } else {
        const int row = min(m0 + (q - NWF) * 16 + (lane & 15), p.M - 1);
        src = p.x + (long)row * p.ldx + kstep * 32 + (lane >> 4) * 8;
      }
      glds16(src, base + f * 1024);
    }
  };

  f32x4 acc[FCW][FPW];
#pragma unroll
  for (int i = 0; i < FCW; ++i)
#pragma unroll
    for (int j = 0; j < FPW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    const int cur = st & 1;
    if (st + 1 < nst) stage(cur ^ 1, st + 1);
    const char* base = smem + cur * STAGE_FR * 1024 + lane * 16;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 a[FCW], b[FPW];
#pragma unroll
      for (int i = 0; i < FCW; ++i) a[i] = *reinterpret_cast<const bf16x8*>(base + (ks * KF + wn * FCW + i) * 1024);
#pragma unroll
      for (int j = 0; j < FPW; ++j)
        b[j] = *reinterpret_cast<const bf16x8*>(base + (ks * KF + NWF + wm * FPW + j) * 1024);
#pragma unroll
      for (int i = 0; i < FCW; ++i)
#pragma unroll
        for (int j = 0; j < FPW; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- fused epilogue (row-major out) ----
  const int lrow = lane & 15;
#pragma unroll
  for (int j = 0; j < FPW; ++j) {
    const int m = m0 + wm * (BM / 2) + j * 16 + lrow;
    if (m >= p.M) continue;
#pragma unroll
    for (int i = 0; i < FCW; ++i) {
      const int n = n0 + wn * (BN / 2) + i * 16 + (lane >> 4) * 4;
      if (n >= p.Cout) continue;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (p.bias) {
        const f32x4 bb = *reinterpret_cast<const f32x4*>(p.bias + n);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += bb[e];
      }
      const long o = (long)m * p.ldo + n;
      if (p.res) {
        const u32x2 rr = *reinterpret_cast<const u32x2*>(p.res + o);
        v[0] += __uint_as_float(rr[0] << 16);
        v[1] += __uint_as_float(rr[0] & 0xffff0000u);
        v[2] += __uint_as_float(rr[1] << 16);
        v[3] += __uint_as_float(rr[1] & 0xffff0000u);
      }
      if (p.act == HZ_ACT_RELU) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
      } else if (p.act == HZ_ACT_GELU) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = gelu_erf(v[e]);
      } else if (p.act == HZ_ACT_TANH) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = tanhf(v[e]);
      }
      if (p.out_f32) *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p.out) + o) = f32x4{v[0], v[1], v[2], v[3]};
      else *reinterpret_cast<u32x2*>(reinterpret_cast<bf16_t*>(p.out) + o) = u32x2{pack2(v[0], v[1]), pack2(v[2], v[3])};
    }
  }
}

template <int BM, int BN>
int launch_lds(const HzConvParams& p, hipStream_t st) {
  const int tiles = ((p.Cout + BN - 1) / BN) * ((p.M + BM - 1) / BM);
  hipLaunchKernelGGL((gemm_lds_kernel<BM, BN>), dim3(tiles), dim3(256), 0, st, p);
  return (int)hipGetLastError();
}

}  // namespace

// cfg 16: 128x128, 17: 64x128 (BM x BN), 18: 128x64, 19: 64x64; row-major activations only.
extern "C" int hz_gemm_lds_launch(const HzConvParams* pp, int cfg, hipStream_t st) {
  const HzConvParams& p = *pp;
  if (!p.x_rowmajor || !p.out_rowmajor || p.K % 64 || p.ksteps * 32 != p.K || p.ldx % 8 || p.Cout % 4) return -1;
  switch (cfg) {
    case 16: return launch_lds<128, 128>(p, st);
    case 17: return launch_lds<64, 128>(p, st);
    case 18: return launch_lds<128, 64>(p, st);
    case 19: return launch_lds<64, 64>(p, st);
    default: return -2;
  }
}
