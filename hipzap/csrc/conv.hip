// Implicit-GEMM convolution (and plain GEMM/Linear as the 1x1 case) on CDNA4 MFMA.
//
//   out[m][n] = act( sum_k W[n][k] * im2col(X)[m][k] + bias[n] (+ res[m][n]) )
//
// * Activations are NHWC bf16, so an 8-element K chunk of one im2col row is 16 contiguous
//   bytes of one input pixel: every MFMA fragment is one 16-B global load straight into
//   VGPRs (no LDS round trip — the latency-bound bs=1 regime of cdna_hip_programming.md §5,
//   'GEMV / M <= 16' row; operands are L2/MALL resident, ResNet-50 bf16 is 51 MB).
// * "Swapped" orientation: the MFMA A operand is the weight (rows = output channels), B is
//   the activation (cols = output pixels). With mfma_f32_16x16x32_bf16's C/D map
//   (col = lane&15, row = 4*(lane>>4)+i) each lane then owns 4 CONSECUTIVE output channels
//   of one pixel, so the fused epilogue (folded-BN bias, residual add, ReLU) does one 16-B
//   bias load, one 8-B residual load and one 8-B store per accumulator.
// * bs=1 late stages have tiny M (49 px) and huge K (4608): split-K across workgroups with
//   an in-launch last-arriver reduction (agent-scope release/acquire ticket protocol of
//   cdna_hip_programming.md §5 'Projection GEMM at M = 256' item 2), so a split conv is
//   still ONE launch and the partial slabs never leave L2 for long.
// * Register-ring software pipeline: fragments of step t+DEPTH are in flight while step t
//   computes (hipcc emits counted vmcnt waits for plain loads).
//
// Reference parity: this replaces the conv/BN/ReLU stack the north star asks for
// (SURVEY.md §2e N1, N3-FC, N4); the reference itself only runs aten::addmm/lstm on CPU
// (SURVEY.md §2d).
#include "common.h"
#include "hipzap.h"

namespace {

constexpr int THREADS = 256;
constexpr int DEPTH = 2;  // loads in flight ahead of the MFMA step

template <int WC, int WP, int FC, int FP, bool FAST, bool IS1X1>
__global__ __launch_bounds__(THREADS) void conv_igemm_kernel(const HzConvParams p) {
  static_assert(WC * WP == 4, "4 waves");
  constexpr int BNC = WC * FC * 16;  // output channels per block
  constexpr int BMP = WP * FP * 16;  // output pixels per block
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave % WC, wp = wave / WC;
  const int lrow = lane & 15, lk = (lane >> 4) * 8;

  const int nwg = gridDim.x;
  const int lid = xcd_remap(blockIdx.x, nwg);
  const int tile = lid / p.splitk;
  const int slice = lid - tile * p.splitk;
  const int tile_n = tile % p.tiles_n;
  const int tile_m = tile / p.tiles_n;
  const int n0 = tile_n * BNC + wc * FC * 16;
  const int m0 = tile_m * BMP + wp * FP * 16;

  const int K = p.K, C = p.C;
  const int k_begin = slice * p.kslice;
  const int k_end = min(K, k_begin + p.kslice);
  const int nsteps = (k_end - k_begin + 31) >> 5;

  // ---- per-pixel precompute (B operand rows = output pixels) ----
  int pbase[FP], pih[FP], piw[FP];
  bool pval[FP];
#pragma unroll
  for (int f = 0; f < FP; ++f) {
    const int m = m0 + f * 16 + lrow;
    pval[f] = m < p.M;
    const int mm = pval[f] ? m : 0;
    if constexpr (IS1X1) {
      pbase[f] = mm * C;
      pih[f] = 0;
      piw[f] = 0;
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
    const int k = k_begin + t * 32;  // wave-uniform
    const int kk = k + lk;           // this lane's 8-chunk
#pragma unroll
    for (int i = 0; i < FC; ++i) {
      const bf16_t* src = Wt + (long)(n0 + i * 16 + lrow) * ldw + kk;
      a[i] = *reinterpret_cast<const bf16x8*>(src);
    }
    if constexpr (IS1X1) {
#pragma unroll
      for (int j = 0; j < FP; ++j) {
        if (pval[j]) b[j] = *reinterpret_cast<const bf16x8*>(X + (long)pbase[j] + kk);
        else b[j] = bf16x8{};
      }
    } else {
      int r, s, c;
      bool kval = true;
      if constexpr (FAST) {  // C % 32 == 0: (r,s) uniform over the 32-wide step
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

  // prologue
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

  // ---- split-K: in-launch last-arriver reduction ----
  if (p.splitk > 1) {
    __shared__ int s_last;
    f32x4* slab = reinterpret_cast<f32x4*>(p.ws) + (long)(tile * p.splitk) * (FC * FP * THREADS);
    f32x4* mine = slab + (long)slice * (FC * FP * THREADS);
#pragma unroll
    for (int i = 0; i < FC; ++i)
#pragma unroll
      for (int j = 0; j < FP; ++j) mine[(i * FP + j) * THREADS + tid] = acc[i][j];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int old = __hip_atomic_fetch_add(p.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = (old == p.splitk - 1);
    }
    __syncthreads();
    if (!s_last) return;
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    // deterministic: sum the slices in slice order whoever arrives last
    f32x4 tot[FC][FP];
#pragma unroll
    for (int i = 0; i < FC; ++i)
#pragma unroll
      for (int j = 0; j < FP; ++j) tot[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int sl = 0; sl < p.splitk; ++sl) {
      const f32x4* other = slab + (long)sl * (FC * FP * THREADS);
#pragma unroll
      for (int i = 0; i < FC; ++i)
#pragma unroll
        for (int j = 0; j < FP; ++j) tot[i][j] += (sl == slice) ? acc[i][j] : other[(i * FP + j) * THREADS + tid];
    }
#pragma unroll
    for (int i = 0; i < FC; ++i)
#pragma unroll
      for (int j = 0; j < FP; ++j) acc[i][j] = tot[i][j];
    if (tid == 0) __hip_atomic_store(p.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }

  // ---- fused epilogue: bias (folded BN) + residual + ReLU, 4 consecutive channels/lane ----
#pragma unroll
  for (int j = 0; j < FP; ++j) {
    const int m = m0 + j * 16 + lrow;
    if (m >= p.M) continue;
#pragma unroll
    for (int i = 0; i < FC; ++i) {
      const int n = n0 + i * 16 + (lane >> 4) * 4;
      if (n >= p.Cout) continue;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (p.bias) {
        const f32x4 bb = *reinterpret_cast<const f32x4*>(p.bias + n);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += bb[e];
      }
      const long o = (long)m * p.ldo + n;
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
      if (p.out_f32) {
        *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p.out) + o) = f32x4{v[0], v[1], v[2], v[3]};
      } else {
        *reinterpret_cast<u32x2*>(reinterpret_cast<bf16_t*>(p.out) + o) = u32x2{pack2(v[0], v[1]), pack2(v[2], v[3])};
      }
    }
  }
}

template <int WC, int WP, int FC, int FP>
int launch_cfg(const HzConvParams& p, hipStream_t st) {
  constexpr int BNC = WC * FC * 16, BMP = WP * FP * 16;
  HzConvParams q = p;
  q.tiles_n = (p.Cout + BNC - 1) / BNC;
  const int tiles_m = (p.M + BMP - 1) / BMP;
  const int nblk = q.tiles_n * tiles_m * q.splitk;
  const bool is1x1 = p.R == 1 && p.S == 1 && p.stride == 1 && p.pad == 0;
  const bool fast = (p.C % 32) == 0;
  dim3 grid(nblk), block(THREADS);
  if (is1x1 && fast)
    hipLaunchKernelGGL((conv_igemm_kernel<WC, WP, FC, FP, true, true>), grid, block, 0, st, q);
  else if (fast)
    hipLaunchKernelGGL((conv_igemm_kernel<WC, WP, FC, FP, true, false>), grid, block, 0, st, q);
  else
    hipLaunchKernelGGL((conv_igemm_kernel<WC, WP, FC, FP, false, false>), grid, block, 0, st, q);
  return (int)hipGetLastError();
}

}  // namespace

// Config table: (WC, WP, FC, FP). Block tile = (WC*FC*16 channels) x (WP*FP*16 pixels).
// Index order is part of the ABI with hipzap/ops/conv.py (CONV_CONFIGS).
extern "C" int hz_conv_launch(const HzConvParams* pp, int cfg, hipStream_t st) {
  const HzConvParams& p = *pp;
  if (p.Cout % 4 != 0 || p.C % 8 != 0 || p.ldw % 32 != 0 || p.splitk < 1) return -1;
  if (cfg >= 100) return hz_conv_kw_launch(pp, cfg, st);
  switch (cfg) {
    case 0: return launch_cfg<2, 2, 2, 2>(p, st);  //  64ch x  64px
    case 1: return launch_cfg<4, 1, 1, 1>(p, st);  //  64ch x  16px
    case 2: return launch_cfg<4, 1, 2, 1>(p, st);  // 128ch x  16px
    case 3: return launch_cfg<1, 4, 1, 1>(p, st);  //  16ch x  64px
    case 4: return launch_cfg<2, 2, 1, 1>(p, st);  //  32ch x  32px
    case 5: return launch_cfg<2, 2, 4, 4>(p, st);  // 128ch x 128px
    case 6: return launch_cfg<2, 2, 2, 4>(p, st);  //  64ch x 128px
    case 7: return launch_cfg<2, 2, 4, 2>(p, st);  // 128ch x  64px
    case 8: return launch_cfg<4, 1, 1, 2>(p, st);  //  64ch x  32px
    case 9: return launch_cfg<1, 4, 2, 1>(p, st);  //  32ch x  64px
    case 10: return launch_cfg<4, 1, 2, 2>(p, st); // 128ch x  32px
    case 11: return launch_cfg<1, 4, 1, 2>(p, st); //  16ch x 128px
    default: return -2;
  }
}
