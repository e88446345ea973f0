// LDS-tiled bf16 GEMM for large-M transformer projections (BERT bs=16: M = 2048 tokens).
//
//   out[m][n] = act( sum_k X[m][k] * W[n][k] + bias[n] (+ res[m][n]) ),  X row-major [M][ldx]
//
// The K-across-waves kernel (conv.hip) is right for bs=1 (every operand byte used once), but
// at M >= ~512 each weight fragment is re-read by every M tile and each activation fragment
// by every N tile: the per-CU load path, not the MFMA, was the limit. Here a 256-thread
// workgroup (2x2 waves, each a (BM/2) x (BN/2) sub-tile of 16x16x32 MFMAs) owns a BM x BN
// tile and stages BOTH operands through LDS once per 64-deep K step:
//   * weights are packed fragment-major [N/16][K/32][64][8] (1 KiB per fragment, contiguous):
//     one global_load_lds (16 B/lane) per fragment, lane-linear LDS image;
//   * activations are staged in FULL 128-B lines (8 rows x 64 k per wave-instruction), not as
//     16-row x 64-B fragments (cdna_hip_programming.md §5 "Projection GEMM": fragment-shaped x
//     loads cost 18-45 %). The LDS image [BM][128 B] is XOR-swizzled per 16-B chunk,
//     chunk' = chunk ^ ((row >> 1) & 7), so the 16 rows of a ds_read_b128 lane group land in
//     16 distinct 16-B bank slots (conflict-free); glds writes lane-linearly, so the swizzle is
//     applied to the per-lane GLOBAL source address;
//   * 2, 3 or 4 LDS stages (up to NS-1 K steps in flight; the N=768 projections are latency-bound
//     with 12 K steps per tile): counted `s_waitcnt vmcnt(k*G)` + raw s_barrier (never
//     __syncthreads(), whose fence would drain the in-flight DMA — §5 "Pipelining across barriers");
//   * same swapped orientation and fused epilogue as conv.hip (4 consecutive output features
//     per lane: 16-B bias, 8-B residual, 8-B store), XCD-aware tile order.
// Requirements (checked by the launcher): K % 64 == 0, ldx % 8 == 0, weight rows padded to 128.
//
// CV (implicit-GEMM convolution at large M, e.g. ResNet-50 at batch >= 4): the same tile, the same
// LDS image, only the activation SOURCE changes. Rows are output pixels of a channel-blocked
// [N][C/32][H][W][32] input (C % 64 == 0, so a 64-deep K step is two 32-channel blocks of ONE
// filter tap (r, s)); each lane's 16-B chunk is fetched with buffer_load ... lds through a buffer
// descriptor over the whole input, and a tap that falls into the zero padding gets an offset past
// the descriptor's range, which the hardware range check turns into zeros in LDS (no zero buffer,
// no predicated DMA). The running (r, s, channel block) of the next staged K step is scalar and
// advances incrementally; the epilogue stores channel-blocked output (+ residual in that layout).
#include <cstdlib>

#include "common.h"
#include "hipzap.h"

HZ_DEBUG_UNIT(gemm)

namespace {

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void glds16(const void* g, char* lds) {
  __builtin_amdgcn_global_load_lds(g, (lds_void*)lds, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// mean / rstd of this lane's FPW rows (m = mbase + 16 j) from a producer's (sum, sumsq) slabs
// (HzLnFold). The 4 lane groups sharing a row split the slabs (group g: slabs g, g+4, ...), every
// load is unconditional (clamped slab / row, zero weight) so all of them are in flight at once —
// one memory latency per tile instead of a serial chain — then an xor-shuffle combines the groups.
// Wave-uniform call (shuffles). nslab <= 4 * HZ_LNF_MAXT (checked by the host).
#define HZ_LNF_MAXT 6
template <int FPW>
__device__ __forceinline__ void rows_stats(const float* __restrict__ st, int nslab, int ld, int mbase, int M,
                                           float inv_d, float eps, float (&mu)[FPW], float (&rs)[FPW]) {
  const int g = (threadIdx.x & 63) >> 4;
  float a[FPW], b[FPW];
#pragma unroll
  for (int j = 0; j < FPW; ++j) a[j] = b[j] = 0.f;
#pragma unroll
  for (int t = 0; t < HZ_LNF_MAXT; ++t) {
    const int s = g + 4 * t;
    const float w = s < nslab ? 1.f : 0.f;
    const long sb = (long)min(s, nslab - 1) * ld;
#pragma unroll
    for (int j = 0; j < FPW; ++j) {
      const float2 v = *reinterpret_cast<const float2*>(st + 2 * (sb + min(mbase + 16 * j, M - 1)));
      a[j] += w * v.x;
      b[j] += w * v.y;
    }
  }
#pragma unroll
  for (int j = 0; j < FPW; ++j) {
    a[j] += __shfl_xor(a[j], 16);
    b[j] += __shfl_xor(b[j], 16);
    a[j] += __shfl_xor(a[j], 32);
    b[j] += __shfl_xor(b[j], 32);
    mu[j] = a[j] * inv_d;
    rs[j] = rsqrtf(fmaxf(b[j] * inv_d - mu[j] * mu[j], 0.f) + eps);
  }
}

// LNF: folded-LayerNorm variant (p.lnf != NULL); a separate instantiation so the plain GEMM keeps
// its register budget (the fold's statistics cost ~60 VGPRs, which halves occupancy)
// WM x WN waves (4 or 8): wave (wm, wn) owns rows wm*BM/WM.. and features wn*BN/WN..
// (a variant reading the same LDS image as 32x32x16 operands, cfg 64-77, was a measured negative,
// profiles/r3_m32, deleted in round 5)
template <int BM, int BN, int NS, bool LNF, int WM, int WN, bool CV = false>
__global__ __launch_bounds__(64 * WM * WN) void gemm_lds_kernel(const HzConvParams p, int group_m) {
  constexpr int NW = WM * WN;
  constexpr int FCW = BN / WN / 16, FPW = BM / WM / 16;  // 16x16 fragments per wave
  constexpr int NWG = BN / 16;                 // weight fragments per 32-deep k-step
  constexpr int XBYTES = BM * 128;             // activation bytes per stage (BK = 64 bf16 = 128 B)
  constexpr int SBYTES = XBYTES + BN * 128;    // + 2 k-steps x NWG fragments x 1 KiB
  constexpr int XPW = BM / 8 / NW, WPW = 2 * NWG / NW;  // glds pieces per wave per stage (x, w)
  static_assert(XPW * 8 * NW == BM && WPW * NW == 2 * NWG && FCW >= 1 && FPW >= 1, "tile / wave split");
  constexpr int G = XPW + WPW;
  __shared__ __attribute__((aligned(16))) char smem[NS * SBYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave % WN, wm = wave / WN;
  const int tiles_n = (p.Cout + BN - 1) / BN, tiles_m = (p.M + BM - 1) / BM;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  // grouped raster (common.h): an XCD's L2 holds a group_m-row block of X and a few W column
  // tiles instead of two X row-panels x ALL of W (5.1 MB > 4 MB L2 at BERT FFN1)
  int tile_m, tile_n;
  grouped_tile(lid, tiles_m, tiles_n, group_m, tile_m, tile_n);
  const int n0 = tile_n * BN, m0 = tile_m * BM;
  const int nst = p.ksteps >> 1;

  // staging sources: x piece q = wave + 4i covers tile rows 8q .. 8q+7, lane -> row 8q + (lane>>3),
  // swizzled chunk (lane&7) ^ (((q&1)<<2) + (lane>>4)); rows >= M are clamped (never stored)
  const bf16_t* xsrc[XPW];
  // CV: per piece, the element offset of the lane's chunk at tap (0, 0) of channel block 0 and the
  // input-window origin (ih0, iw0) of its output pixel
  int xb[XPW], xih[XPW], xiw[XPW];
  const int PQ = p.P * p.Q, HW = p.H * p.W;
#pragma unroll
  for (int i = 0; i < XPW; ++i) {
    const int q = wave + NW * i;
    const int row = min(m0 + q * 8 + (lane >> 3), p.M - 1);
    const int chunk = (lane & 7) ^ (((q & 1) << 2) + (lane >> 4));
    if constexpr (CV) {
      const int ni = fdiv(row, PQ), hw = row - ni * PQ;
      const int oh = fdiv(hw, p.Q), ow = hw - oh * p.Q;
      xih[i] = oh * p.stride - p.pad;
      xiw[i] = ow * p.stride - p.pad;
      xb[i] = ((ni * (p.C >> 5) + (chunk >> 2)) * HW + xih[i] * p.W + xiw[i]) * 32 + (chunk & 3) * 8;
      xsrc[i] = p.x;
    } else {
      xsrc[i] = p.x + (long)row * p.ldx + chunk * 8;
    }
  }
  // CV: descriptor over the whole input (launcher: < 2^31 bytes); scalar running tap position
  const __amdgpu_buffer_rsrc_t xrsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.x, (short)0, CV ? p.N * p.C * HW * 2 : 0, 0x00020000);
  int cv_cb = 0, cv_r = 0, cv_s = 0;
  const bf16_t* wsrc = p.w + ((long)(n0 >> 4) * p.ksteps * 64 + lane) * 8;
  // debug contracts: the tile's weight rows exist in the 128-row padded packing, and the last
  // staged activation line lies inside [M][ldx] (the DMA cannot be skipped, so a violation
  // re-points the sources at the tensor bases instead)
  if (!HZ_DCHECK(n0 + BN <= ((p.Cout + 127) / 128) * 128)) wsrc = p.w + lane * 8;
  if constexpr (!CV) {
#pragma unroll
    for (int i = 0; i < XPW; ++i)
      if (!HZ_DCHECK(xsrc[i] - p.x + (long)(nst - 1) * 64 + 8 <= (long)p.M * p.ldx)) xsrc[i] = p.x;
  }
  auto stage = [&](int buf, int st) {
    char* base = smem + buf * SBYTES;
    if constexpr (CV) {  // stage() runs for st = 0, 1, 2, ... in order: the tap position is running
      const int u = ((cv_cb * p.H + cv_r) * p.W + cv_s) * 32;
#pragma unroll
      for (int i = 0; i < XPW; ++i) {
        const bool v = (unsigned)(xih[i] + cv_r) < (unsigned)p.H && (unsigned)(xiw[i] + cv_s) < (unsigned)p.W;
        const unsigned voff = v ? (unsigned)(xb[i] + u) * 2u : 0x80000000u;  // past the range -> zeros
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xrsrc, (lds_void*)(base + (wave + NW * i) * 1024), 16, voff, 0, 0, 0);
      }
      cv_cb += 2;  // C % 64 == 0: a 64-deep step never straddles a tap
      if (cv_cb == (p.C >> 5)) {
        cv_cb = 0;
        if (++cv_s == p.S) {
          cv_s = 0;
          ++cv_r;
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < XPW; ++i) glds16(xsrc[i] + st * 64, base + (wave + NW * i) * 1024);
    }
#pragma unroll
    for (int i = 0; i < WPW; ++i) {
      const int f = wave + NW * i;  // f = ks * NWG + g
      const int ks = f / NWG, g = f - ks * NWG;
      glds16(wsrc + ((long)g * p.ksteps + st * 2 + ks) * 512, base + XBYTES + f * 1024);
    }
  };

  // reader offsets: B fragment j of k-step ks = rows wm*BM/2 + 16j + (lane&15), chunk 4ks + (lane>>4)
  const int lr = lane & 15, sw = (lane >> 1) & 7;
  const int boff0 = (wm * (BM / WM) + lr) * 128 + (((lane >> 4)) ^ sw) * 16;
  const int boff1 = (wm * (BM / WM) + lr) * 128 + ((4 + (lane >> 4)) ^ sw) * 16;
  const int aoff = XBYTES + (wn * FCW) * 1024 + lane * 16;

  f32x4 acc[FCW][FPW];
#pragma unroll
  for (int i = 0; i < FCW; ++i)
#pragma unroll
    for (int j = 0; j < FPW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s0 = 0; s0 < NS - 1; ++s0)
    if (s0 < nst) stage(s0, s0);
  // folded LayerNorm: row statistics of the producer are complete at kernel start; their loads
  // go out behind the first stages' DMA, so the wait overlaps the first K step's
  const HzLnFold* __restrict__ lf = LNF ? p.lnf : nullptr;
  const bool f_in = LNF && lf->stats_in, f_res = LNF && lf->res_stats, f_out = LNF && lf->stats_out;
  const int lrow = lane & 15;
  float mu_in[FPW], rs_in[FPW], mu_r[FPW], rs_r[FPW];
  if (f_in)
    rows_stats<FPW>(lf->stats_in, lf->nslab_in, lf->ld_stats, m0 + wm * (BM / WM) + lrow, p.M, lf->inv_d, lf->eps_in,
                    mu_in, rs_in);
  if (f_res)
    rows_stats<FPW>(lf->res_stats, lf->nslab_res, lf->ld_stats, m0 + wm * (BM / WM) + lrow, p.M, lf->inv_d,
                    lf->eps_res, mu_r, rs_r);
  int cur = 0;
  for (int st = 0; st < nst; ++st) {
    // stages issued ahead of st: min(NS-2, nst-1-st) may stay in flight
    const int ahead = min(NS - 2, nst - 1 - st);
    if (NS > 3 && ahead >= 2) wait_vm<(NS > 3 ? 2 * G : 0)>();
    else if (NS > 2 && ahead >= 1) wait_vm<(NS > 2 ? G : 0)>();
    else wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (st + NS - 1 < nst) stage(cur == 0 ? NS - 1 : cur - 1, st + NS - 1);
    const char* base = smem + cur * SBYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 a[FCW], b[FPW];
#pragma unroll
      for (int i = 0; i < FCW; ++i) a[i] = *reinterpret_cast<const bf16x8*>(base + aoff + (ks * NWG + i) * 1024);
#pragma unroll
      for (int j = 0; j < FPW; ++j)
        b[j] = *reinterpret_cast<const bf16x8*>(base + (ks ? boff1 : boff0) + j * 16 * 128);
#pragma unroll
      for (int i = 0; i < FCW; ++i)
#pragma unroll
        for (int j = 0; j < FPW; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    cur = cur == NS - 1 ? 0 : cur + 1;
  }

  // ---- fused epilogue (row-major out) ----
  // Optional folded LayerNorm (HzLnFold, hipzap.h): input-side correction rstd*(acc - mean*c1),
  // normalised residual, and per-row (sum, sumsq) partials of the stored bf16 output.
#pragma unroll
  for (int j = 0; j < FPW; ++j) {
    const int m = m0 + wm * (BM / WM) + j * 16 + lrow;
    const bool mval = m < p.M;
    float s1 = 0.f, s2 = 0.f;
    int ni_m = 0, hw_m = 0;  // CV: channel-blocked [N][Cout/32][P*Q][32] output
    if constexpr (CV) {
      ni_m = fdiv(mval ? m : 0, PQ);
      hw_m = m - ni_m * PQ;
    }
#pragma unroll
    for (int i = 0; i < FCW; ++i) {
      const int n = n0 + wn * (BN / WN) + i * 16 + (lane >> 4) * 4;
      const long o = CV ? (((long)ni_m * (p.Cout >> 5) + (n >> 5)) * PQ + hw_m) * 32 + (n & 31) : (long)m * p.ldo + n;
      const long olim = CV ? (long)p.N * p.Cout * PQ : (long)(p.M - 1) * p.ldo + p.Cout;
      if (!mval || n >= p.Cout || !HZ_DCHECK(o + 4 <= olim)) continue;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (f_in) {
        const f32x4 c = *reinterpret_cast<const f32x4*>(lf->c1 + n);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = rs_in[j] * (v[e] - mu_in[j] * c[e]);
      }
      if (p.bias) {
        const f32x4 bb = *reinterpret_cast<const f32x4*>(p.bias + n);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += bb[e];
      }
      if (p.res) {
        const u32x2 rr = *reinterpret_cast<const u32x2*>(p.res + o);
        float r[4] = {__uint_as_float(rr[0] << 16), __uint_as_float(rr[0] & 0xffff0000u),
                      __uint_as_float(rr[1] << 16), __uint_as_float(rr[1] & 0xffff0000u)};
        if (f_res) {
          const f32x4 gg = *reinterpret_cast<const f32x4*>(lf->res_gamma + n);
          const f32x4 bt = *reinterpret_cast<const f32x4*>(lf->res_beta + n);
#pragma unroll
          for (int e = 0; e < 4; ++e) r[e] = (r[e] - mu_r[j]) * rs_r[j] * gg[e] + bt[e];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += r[e];
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
        const u32x2 q = u32x2{pack2(v[0], v[1]), pack2(v[2], v[3])};
        *reinterpret_cast<u32x2*>(reinterpret_cast<bf16_t*>(p.out) + o) = q;
        if (f_out) {  // statistics of exactly what the consumers will read (bf16-rounded)
          const float a0 = __uint_as_float(q[0] << 16), a1 = __uint_as_float(q[0] & 0xffff0000u);
          const float a2 = __uint_as_float(q[1] << 16), a3 = __uint_as_float(q[1] & 0xffff0000u);
          s1 += (a0 + a1) + (a2 + a3);
          s2 += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
        }
      }
    }
    if (f_out) {  // wave-uniform: every lane reaches the shuffles. Lanes l, l^16, l^32, l^48 share row m.
      s1 += __shfl_xor(s1, 16);
      s2 += __shfl_xor(s2, 16);
      s1 += __shfl_xor(s1, 32);
      s2 += __shfl_xor(s2, 32);
      const long so = 2 * ((long)(tile_n * WN + wn) * lf->ld_stats + m);
      if (lane < 16 && mval && HZ_DCHECK(m < lf->ld_stats))
        *reinterpret_cast<float2*>(lf->stats_out + so) = make_float2(s1, s2);
    }
  }
}

template <int BM, int BN, int NS, int WM = 2, int WN = 2, bool CVOK = false>
int launch_lds(const HzConvParams& p, hipStream_t st) {
  // the last feature tile must stay inside the 128-row padded weight packing (BN = 96 / 192 / 288
  // tiles fit only some widths: every BERT / ViT projection, not arbitrary N)
  if (((p.Cout + BN - 1) / BN) * BN > ((p.Cout + 127) / 128) * 128) return -4;
  const int tiles = ((p.Cout + BN - 1) / BN) * ((p.M + BM - 1) / BM);
  const dim3 block(64 * WM * WN);
  static const int group_env = getenv("HIPZAP_GEMM_GROUP") ? atoi(getenv("HIPZAP_GEMM_GROUP")) : 8;
  const int group_m = group_env < 1 ? 1 : group_env;
  if (!p.x_rowmajor) {  // implicit-GEMM conv (CV): every feature tile lies inside Cout (rows padded to 64)
    // (instantiated only for the CV-capable tiles: every kernel variant is code the serving
    // process loads at its first launch, i.e. part of the cold start)
    if constexpr (CVOK) {
      if (p.out_rowmajor || p.lnf || p.C % 64 || p.Cout % BN || p.Cout % 32 || p.K != p.R * p.S * p.C ||
          (long)p.N * p.C * p.H * p.W * 2 >= (1L << 31))
        return -1;
      hipLaunchKernelGGL((gemm_lds_kernel<BM, BN, NS, false, WM, WN, true>), dim3(tiles), block, 0, st, p, group_m);
      return (int)hipGetLastError();
    } else {
      return -1;
    }
  }
  if (p.lnf) {  // the folded-LayerNorm statistics slabs assume 2 feature halves per tile
    if constexpr (WN != 2 || !HZ_EXPERIMENTS) {
      return -3;  // (the LN-fold epilogue is an experiment: not in the product library)
    } else {
      hipLaunchKernelGGL((gemm_lds_kernel<BM, BN, NS, true, WM, 2>), dim3(tiles), block, 0, st, p, group_m);
    }
  } else {
    hipLaunchKernelGGL((gemm_lds_kernel<BM, BN, NS, false, WM, WN, false>), dim3(tiles), block, 0, st, p, group_m);
  }
  return (int)hipGetLastError();
}

}  // namespace

// cfg 16: 128x128, 17: 64x128 (BM x BN), 18: 128x64, 19: 64x64 with 3 LDS stages; cfg 20-23: the same
// tiles with 2 stages (less LDS: more workgroups per CU); cfg 24-27: 4 stages (deeper prefetch for
// short-K / latency-bound shapes); cfg 28-33: 8-wave workgroups (128x128 3/2 stages, 256x128,
// 128x64, 64x128, 256x64); cfg 34-40: one-tile-per-CU shapes for M = 2048 (64x96, 128x192,
// 64x288, 256x96). Row-major activations only.
extern "C" int hz_gemm_lds_launch(const HzConvParams* pp, int cfg, hipStream_t st) {
  const HzConvParams& p = *pp;
  if (!p.x_rowmajor) {  // implicit-GEMM conv on channel-blocked activations: the 4- and 8-wave tiles
    if (p.K % 64 || p.ksteps * 32 != p.K || p.Cout % 4) return -1;
    switch (cfg) {
      case 16: return launch_lds<128, 128, 3, 2, 2, true>(p, st);
      case 20: return launch_lds<128, 128, 2, 2, 2, true>(p, st);
      case 17: return launch_lds<64, 128, 3, 2, 2, true>(p, st);
      case 21: return launch_lds<64, 128, 2, 2, 2, true>(p, st);
      case 18: return launch_lds<128, 64, 3, 2, 2, true>(p, st);
      case 22: return launch_lds<128, 64, 2, 2, 2, true>(p, st);
      case 19: return launch_lds<64, 64, 3, 2, 2, true>(p, st);
      case 23: return launch_lds<64, 64, 2, 2, 2, true>(p, st);
      case 28: return launch_lds<128, 128, 3, 2, 4, true>(p, st);
      case 29: return launch_lds<128, 128, 2, 2, 4, true>(p, st);
      case 30: return launch_lds<256, 128, 2, 4, 2, true>(p, st);
      case 31: return launch_lds<128, 64, 3, 4, 2, true>(p, st);
      case 32: return launch_lds<64, 128, 3, 2, 4, true>(p, st);
      case 33: return launch_lds<256, 64, 2, 4, 2, true>(p, st);
      default: return -2;
    }
  }
  if (!p.out_rowmajor || p.K % 64 || p.ksteps * 32 != p.K || p.ldx % 8 || p.Cout % 4) return -1;
  switch (cfg) {
    case 16: return launch_lds<128, 128, 3>(p, st);
    case 20: return launch_lds<128, 128, 2>(p, st);
    case 17: return launch_lds<64, 128, 3>(p, st);
    case 21: return launch_lds<64, 128, 2>(p, st);
    case 18: return launch_lds<128, 64, 3>(p, st);
    case 22: return launch_lds<128, 64, 2>(p, st);
    case 19: return launch_lds<64, 64, 3>(p, st);
    case 23: return launch_lds<64, 64, 2>(p, st);
    case 24: return launch_lds<128, 128, 4>(p, st);
    case 25: return launch_lds<64, 128, 4>(p, st);
    case 26: return launch_lds<128, 64, 4>(p, st);
    case 27: return launch_lds<64, 64, 4>(p, st);
    // 8 waves per workgroup (two per SIMD at one workgroup per CU)
    case 28: return launch_lds<128, 128, 3, 2, 4>(p, st);
    case 29: return launch_lds<128, 128, 2, 2, 4>(p, st);
    case 30: return launch_lds<256, 128, 2, 4, 2>(p, st);
    case 31: return launch_lds<128, 64, 3, 4, 2>(p, st);
    case 32: return launch_lds<64, 128, 3, 2, 4>(p, st);
    case 33: return launch_lds<256, 64, 2, 4, 2>(p, st);
    // tiles sized so that an M = 2048 projection makes exactly 256 tiles (one per CU): N = 768 ->
    // 64 x 96, N = 3072 -> 128 x 192, N = 2304 -> 64 x 288, N = 3072 -> 256 x 96
    case 34: return launch_lds<64, 96, 3, 2, 2>(p, st);
    case 35: return launch_lds<128, 192, 3, 2, 4>(p, st);
    case 36: return launch_lds<128, 192, 2, 2, 4>(p, st);
    case 37: return launch_lds<64, 288, 2, 2, 2>(p, st);
    case 38: return launch_lds<64, 288, 3, 2, 2>(p, st);
    case 39: return launch_lds<256, 96, 2, 2, 2>(p, st);
    case 40: return launch_lds<64, 96, 4, 2, 2>(p, st);
    default: return -2;
  }
}

// Load this translation unit's device code without a launch (see hz_conv_code_warm in conv.hip).
__global__ void hz_gemm_code_warm_kernel() {}
extern "C" int hz_gemm_code_warm(void) {
  hipFuncAttributes a;
  return (int)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&hz_gemm_code_warm_kernel));
}
