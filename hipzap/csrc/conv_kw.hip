// Implicit-GEMM convolution, "K across waves" variant (v2) — the bs=1 workhorse.
//
// Same math, layouts and fused epilogue as conv.hip, but the reduction dimension is split
// across the KW waves of ONE workgroup instead of across workgroups:
//   * every wave owns the whole (FC*16 channels x FP*16 pixels) output tile for 1/KW of K,
//   * partial accumulators meet in LDS (KW x FC*FP x 64 lanes x 16 B, lane-linear so every
//     ds_write_b128/ds_read_b128 is conflict-free), summed in wave order (deterministic),
//   * no global split-K slabs, no tickets, no agent-scope release/acquire.
// The first MI355X profile showed the cross-workgroup last-arriver reduction of conv.hip
// costing 5-25 us per layer at bs=1 (release+acquire ~1.7 us each plus serial reads of up
// to 512 KB of slabs by one workgroup); K-across-waves removes that entirely while small
// output tiles (16x16..64x64) still give hundreds of workgroups.
// Each wave streams straight to VGPRs with a DEPTH-deep register ring (DEPTH grows as the
// per-step fragment count shrinks), because at bs=1 every operand is read once per wave.
#include "common.h"
#include "hipzap.h"

namespace {

template <int FC, int FP>
struct Depth {
  static constexpr int value = (FC + FP <= 2) ? 6 : (FC + FP <= 3) ? 4 : (FC + FP <= 4) ? 3 : 2;
};

// keep the register ring out of scratch: 1024 threads cap a wave at 128 VGPRs
constexpr int kw_max_threads(int nf) { return nf >= 16 ? 256 : nf >= 8 ? 512 : 1024; }

template <int FC, int FP, bool FAST, bool IS1X1>
__global__ __launch_bounds__(kw_max_threads(FC * FP)) void conv_kw_kernel(const HzConvParams p) {
  constexpr int DEPTH = Depth<FC, FP>::value;
  constexpr int NF = FC * FP;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int KW = blockDim.x >> 6;
  const int lrow = lane & 15, lk = (lane >> 4) * 8;

  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile_n = lid % p.tiles_n;
  const int tile_m = lid / p.tiles_n;
  const int n0 = tile_n * FC * 16;
  const int m0 = tile_m * FP * 16;

  const int K = p.K, C = p.C;
  const int steps = (K + 31) >> 5;
  const int spw = (steps + KW - 1) / KW;
  const int s_begin = wave * spw;
  const int nsteps = max(0, min(steps, s_begin + spw) - s_begin);
  const int k_begin = s_begin * 32;

  int pbase[FP], pih[FP], piw[FP];
  bool pval[FP];
#pragma unroll
  for (int f = 0; f < FP; ++f) {
    const int m = m0 + f * 16 + lrow;
    pval[f] = m < p.M;
    const int mm = pval[f] ? m : 0;
    if constexpr (IS1X1) {
      pbase[f] = mm * C;
      pih[f] = piw[f] = 0;
    } else {
      const int PQ = p.P * p.Q;
      const int ni = mm / PQ;
      const int rem = mm - ni * PQ;
      const int oh = rem / p.Q;
      const int ow = rem - oh * p.Q;
      pih[f] = oh * p.stride - p.pad;
      piw[f] = ow * p.stride - p.pad;
      pbase[f] = ni * p.H * p.W;
    }
  }
  const bf16_t* __restrict__ X = p.x;
  const bf16_t* __restrict__ Wt = p.w;
  const long ldw = p.ldw;

  bf16x8 fa[DEPTH + 1][FC], fb[DEPTH + 1][FP];
  f32x4 acc[FC][FP];
#pragma unroll
  for (int i = 0; i < FC; ++i)
#pragma unroll
    for (int j = 0; j < FP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto load_step = [&](int t, bf16x8(&a)[FC], bf16x8(&b)[FP]) {
    const int k = k_begin + t * 32;
    const int kk = k + lk;
#pragma unroll
    for (int i = 0; i < FC; ++i)
      a[i] = *reinterpret_cast<const bf16x8*>(Wt + (long)(n0 + i * 16 + lrow) * ldw + kk);
    if constexpr (IS1X1) {
#pragma unroll
      for (int j = 0; j < FP; ++j) {
        if (pval[j]) b[j] = *reinterpret_cast<const bf16x8*>(X + (long)pbase[j] + kk);
        else b[j] = bf16x8{};
      }
    } else {
      int r, s, c;
      bool kval = true;
      if constexpr (FAST) {
        const int rs = k / C;
        c = k - rs * C + lk;
        r = rs / p.S;
        s = rs - r * p.S;
      } else {
        kval = kk < K;
        const int rs = kk / C;
        c = kk - rs * C;
        r = rs / p.S;
        s = rs - r * p.S;
      }
#pragma unroll
      for (int j = 0; j < FP; ++j) {
        const int ih = pih[j] + r, iw = piw[j] + s;
        const bool v = kval && pval[j] && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
        if (v) b[j] = *reinterpret_cast<const bf16x8*>(X + ((long)(pbase[j] + ih * p.W + iw)) * C + c);
        else b[j] = bf16x8{};
      }
    }
  };

#pragma unroll
  for (int u = 0; u < DEPTH; ++u)
    if (u < nsteps) load_step(u, fa[u], fb[u]);
  for (int t = 0; t < nsteps; t += DEPTH + 1) {
#pragma unroll
    for (int u = 0; u <= DEPTH; ++u) {
      const int tt = t + u;
      if (tt + DEPTH < nsteps) load_step(tt + DEPTH, fa[(u + DEPTH) % (DEPTH + 1)], fb[(u + DEPTH) % (DEPTH + 1)]);
      if (tt < nsteps) {
#pragma unroll
        for (int i = 0; i < FC; ++i)
#pragma unroll
          for (int j = 0; j < FP; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[u][i], fb[u][j], acc[i][j], 0, 0, 0);
      }
    }
  }

  auto epilogue = [&](int i, int j, f32x4 a) {
    const int m = m0 + j * 16 + lrow;
    const int n = n0 + i * 16 + (lane >> 4) * 4;
    if (m >= p.M || n >= p.Cout) return;
    float v[4] = {a[0], a[1], a[2], a[3]};
    if (p.bias) {
      const f32x4 bb = *reinterpret_cast<const f32x4*>(p.bias + n);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] += bb[e];
    }
    if (p.res) {
      const u32x2 rr = *reinterpret_cast<const u32x2*>(p.res + (long)m * p.ldr + n);
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
    const long o = (long)m * p.ldo + n;
    if (p.out_f32) *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p.out) + o) = f32x4{v[0], v[1], v[2], v[3]};
    else *reinterpret_cast<u32x2*>(reinterpret_cast<bf16_t*>(p.out) + o) = u32x2{pack2(v[0], v[1]), pack2(v[2], v[3])};
  };

  if (KW == 1) {
#pragma unroll
    for (int i = 0; i < FC; ++i)
#pragma unroll
      for (int j = 0; j < FP; ++j) epilogue(i, j, acc[i][j]);
    return;
  }
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  f32x4* red = reinterpret_cast<f32x4*>(smem_raw);  // [KW][NF][64]
#pragma unroll
  for (int i = 0; i < FC; ++i)
#pragma unroll
    for (int j = 0; j < FP; ++j) red[(wave * NF + i * FP + j) * 64 + lane] = acc[i][j];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < FC; ++i)
#pragma unroll
    for (int j = 0; j < FP; ++j) {
      const int ij = i * FP + j;
      if ((ij % KW) != wave) continue;
      f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int w = 0; w < KW; ++w) s += red[(w * NF + ij) * 64 + lane];
      epilogue(i, j, s);
    }
}

template <int FC, int FP>
int launch_kw(const HzConvParams& p, hipStream_t st) {
  HzConvParams q = p;
  const int kw = p.kw < 1 ? 1 : p.kw;
  if (kw > 16 || kw * FC * FP > 64 || 64 * kw > kw_max_threads(FC * FP)) return -5;
  q.tiles_n = (p.Cout + FC * 16 - 1) / (FC * 16);
  const int tiles_m = (p.M + FP * 16 - 1) / (FP * 16);
  const bool is1x1 = p.R == 1 && p.S == 1 && p.stride == 1 && p.pad == 0;
  const bool fast = (p.C % 32) == 0;
  dim3 grid(q.tiles_n * tiles_m), block(64 * kw);
  const size_t lds = kw > 1 ? (size_t)kw * FC * FP * 64 * 16 : 0;
  if (is1x1 && fast) hipLaunchKernelGGL((conv_kw_kernel<FC, FP, true, true>), grid, block, lds, st, q);
  else if (fast) hipLaunchKernelGGL((conv_kw_kernel<FC, FP, true, false>), grid, block, lds, st, q);
  else hipLaunchKernelGGL((conv_kw_kernel<FC, FP, false, false>), grid, block, lds, st, q);
  return (int)hipGetLastError();
}

}  // namespace

// cfg = 100 + fci*3 + fpi with FC = 1<<fci, FP = 1<<fpi (1,2,4); waves per WG = p->kw.
// Mirrored by hipzap/ops/conv.py (kw_config).
int hz_conv_kw_launch(const HzConvParams* pp, int cfg, hipStream_t st) {
  const HzConvParams& p = *pp;
  switch (cfg - 100) {
    case 0: return launch_kw<1, 1>(p, st);
    case 1: return launch_kw<1, 2>(p, st);
    case 2: return launch_kw<1, 4>(p, st);
    case 3: return launch_kw<2, 1>(p, st);
    case 4: return launch_kw<2, 2>(p, st);
    case 5: return launch_kw<2, 4>(p, st);
    case 6: return launch_kw<4, 1>(p, st);
    case 7: return launch_kw<4, 2>(p, st);
    case 8: return launch_kw<4, 4>(p, st);
    default: return -2;
  }
}
