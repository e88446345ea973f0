// FP8 (OCP e4m3fn) inference GEMM path for gfx950 (north-star config 5
// "ViT-B/16 fp8 weights ... CDNA4 fp8 MFMA GEMM").
//   * quant_rows: per-row dynamic activation quantisation, x_fp8 = cvt(x / s_m) with
//     s_m = amax_m / 448 (one wave per row, 16-B loads), scale kept in fp32;
//   * gemm_fp8:   y[m][n] = s_m * s_n * sum_k x8[m][k] w8[n][k] (+ bias, act, residual) on
//     v_mfma_f32_16x16x32_fp8_fp8. Same K-across-waves / fragment-major design as the bf16
//     conv kernel (csrc/conv.hip), but every fragment is 8 B per lane (half the bytes of bf16):
//     at bs<=64 these GEMMs are operand-streaming bound, so bytes — not the MFMA rate — are
//     what fp8 buys. Weights: per-output-channel scales s_n, packed [N/16][K/32][64][8] bytes.
// gfx950 converts with v_cvt_pk_fp8_f32, which on CDNA4 is the OCP e4m3fn encoding (NOT the
// MI300 FNUZ variant) — checked against torch.float8_e4m3fn in tests/test_fp8_gpu.py.
#include <cstdlib>
#include <type_traits>

#include <utility>

#include "common.h"
#include "hipzap.h"

namespace {

constexpr float FP8_MAX = 448.f;
constexpr int QCH = 8;  // 16-B chunks per lane: rows up to 64*8*8 = 4096 elements


__global__ __launch_bounds__(256) void quant_rows_kernel(const HzQuantParams p) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= p.rows) return;
  const bf16_t* x = p.x + (long)row * p.ldx;
  const int nch = p.D >> 3;
  float v[QCH][8];
  float amax = 0.f;
#pragma unroll
  for (int c = 0; c < QCH; ++c) {
    const int ch = c * 64 + lane;
    if (ch < nch) {
      unpack8(*reinterpret_cast<const u32x4*>(x + ch * 8), v[c]);
#pragma unroll
      for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(v[c][e]));
    }
  }
  amax = warp_max(amax);
  const float scale = fmaxf(amax, 1e-12f) / FP8_MAX;
  const float inv = 1.f / scale;
  unsigned char* o = p.out + (long)row * p.ldo;
#pragma unroll
  for (int c = 0; c < QCH; ++c) {
    const int ch = c * 64 + lane;
    if (ch < nch) {
      float q[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) q[e] = fminf(fmaxf(v[c][e] * inv, -FP8_MAX), FP8_MAX);
      *reinterpret_cast<u32x2*>(o + ch * 8) = u32x2{pack4_fp8(q[0], q[1], q[2], q[3]), pack4_fp8(q[4], q[5], q[6], q[7])};
    }
  }
  if (lane == 0) p.scale[row] = scale;
}

__device__ __attribute__((aligned(256))) unsigned int g_zero8[512] = {0};  // spread zero slots (see conv.hip)

template <int FC, int FP>
struct Depth8 {
  static constexpr int value = (FC + FP <= 2) ? 8 : (FC + FP <= 3) ? 6 : (FC + FP <= 4) ? 4 : 3;
};
constexpr int fp8_max_threads(int nf) { return nf >= 16 ? 256 : nf >= 8 ? 512 : 1024; }

template <int FC, int FP>
__global__ __launch_bounds__(fp8_max_threads(FC * FP)) void gemm_fp8_kernel(const HzGemmFp8Params p) {
  constexpr int DEPTH = Depth8<FC, FP>::value;
  constexpr int NF = FC * FP;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int KW = blockDim.x >> 6;
  const int lrow = lane & 15, lk = (lane >> 4) * 8;
  const int tiles_n = (p.N + FC * 16 - 1) / (FC * 16);
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile_n = lid % tiles_n, tile_m = lid / tiles_n;
  const int n0 = tile_n * FC * 16, m0 = tile_m * FP * 16;
  const int steps = p.ksteps;
  const int spw = (steps + KW - 1) / KW;
  const int s_begin = wave * spw;
  const int nsteps = max(0, min(steps, s_begin + spw) - s_begin);
  const unsigned char* __restrict__ Wf = p.w + ((long)(n0 >> 4) * steps) * 512 + lane * 8;
  bool pval[FP];
#pragma unroll
  for (int j = 0; j < FP; ++j) pval[j] = (m0 + j * 16 + lrow) < p.M;

  long fa[DEPTH + 1][FC], fb[DEPTH + 1][FP];
  f32x4 acc[FC][FP];
#pragma unroll
  for (int i = 0; i < FC; ++i)
#pragma unroll
    for (int j = 0; j < FP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // branch-free loads (zero bytes for invalid lanes / steps): see conv.hip load_step
  const unsigned char* __restrict__ Z = reinterpret_cast<const unsigned char*>(g_zero8) + ((lane + (lid & 3) * 64) & 255) * 8;
  auto load_step = [&](int t, long(&a)[FC], long(&b)[FP]) {
    const bool sv = t < nsteps;
    const int s_idx = s_begin + t;
    const int kk = s_idx * 32 + lk;
#pragma unroll
    for (int i = 0; i < FC; ++i)
      a[i] = *reinterpret_cast<const long*>(sv ? Wf + ((long)i * steps + s_idx) * 512 : Z);
#pragma unroll
    for (int j = 0; j < FP; ++j) {
      const bool v = sv && pval[j] && kk < p.K;
      b[j] = *reinterpret_cast<const long*>(v ? p.x + (long)(m0 + j * 16 + lrow) * p.ldx + kk : Z);
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
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(fa[u][i], fb[u][j], acc[i][j], 0, 0, 0);
      }
    }
  }

  auto epilogue = [&](int i, int j, f32x4 a) {
    const int m = m0 + j * 16 + lrow;
    const int n = n0 + i * 16 + (lane >> 4) * 4;
    if (m >= p.M || n >= p.N) return;
    const float sx = p.sx[m];
    const f32x4 sw = *reinterpret_cast<const f32x4*>(p.sw + n);
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = a[e] * sx * sw[e];
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
  };
  if (KW == 1) {
#pragma unroll
    for (int i = 0; i < FC; ++i)
#pragma unroll
      for (int j = 0; j < FP; ++j) epilogue(i, j, acc[i][j]);
    return;
  }
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  f32x4* red = reinterpret_cast<f32x4*>(smem_raw);
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
int launch8(const HzGemmFp8Params& p, hipStream_t st) {
  const int kw = p.kw < 1 ? 1 : p.kw;
  if (kw > 16 || kw * FC * FP > 64 || 64 * kw > fp8_max_threads(FC * FP)) return -5;
  const int tiles = ((p.N + FC * 16 - 1) / (FC * 16)) * ((p.M + FP * 16 - 1) / (FP * 16));
  const size_t lds = kw > 1 ? (size_t)kw * FC * FP * 64 * 16 : 0;
  hipLaunchKernelGGL((gemm_fp8_kernel<FC, FP>), dim3(tiles), dim3(64 * kw), lds, st, p);
  return (int)hipGetLastError();
}

}  // namespace

extern "C" int hz_quant_launch(const HzQuantParams* pp, hipStream_t st) {
  const HzQuantParams& p = *pp;
  if (p.D % 8 || p.D > 64 * 8 * QCH || p.ldo % 8) return -1;
  hipLaunchKernelGGL(quant_rows_kernel, dim3((p.rows + 3) / 4), dim3(256), 0, st, p);
  return (int)hipGetLastError();
}

// --------------------------------------------------------------------------- MX fp8 LDS GEMM
// Large-M fp8 GEMM on v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3): twice the bf16 MFMA
// rate (MI355X_MICROARCH.md, MFMA table). The block scales are all 1.0 (E8M0 0x7f); the real
// per-row activation and per-channel weight scales stay fp32 and are applied in the epilogue,
// so the numerics equal the 16x16x32 fp8 kernel above. Operand map: lane l holds row l&15 and,
// in register half h, k = 64h + 16*(l>>4) + j, j < 16 — the hardware K order, which only the
// block scales can observe (tests/test_fp8_gpu.py::test_mfma_block_scale_kblock_map; MX input
// scales of lane l apply to row l&15, 32-k block l>>4).
//   * weights MX-packed [N/16][K/128][half][64 lanes][16 B]: a 2-KiB fragment is two lane-linear
//     1-KiB glds pieces, and each half is read back with a conflict-free ds_read_b128;
//   * activations (row-major fp8, 128-B rows per 128-deep k-step) staged in full 128-B lines,
//     16-B chunks XOR-swizzled with MX_SWZ (chunk' = c ^ f((row>>1)&7), f found by exhaustive
//     search to make the 16 rows of every ds_read_b128 lane group hit 16 distinct bank slots
//     for this kernel's chunk pattern (l>>4)+4*half — conflict-free, as for the earlier pattern);
//   * 3 LDS stages, counted vmcnt + raw s_barrier, as csrc/gemm.hip.
namespace {

constexpr unsigned MX_SWZ = 0x32765410u;  // nibble i = f(i)
__device__ __forceinline__ int mx_swz(int i) { return (MX_SWZ >> (4 * i)) & 7; }

typedef __attribute__((address_space(3))) void lds_void8;
typedef int i32x8 __attribute__((ext_vector_type(8)));

// (a __device__ wrapper: called directly in the template kernel body, the builtin made hipcc drop
// the kernel's host stub without a diagnostic — undefined symbol at dlopen)
__device__ __forceinline__ void glds16_8(const void* g, char* lds) {
  __builtin_amdgcn_global_load_lds(g, (lds_void8*)lds, 16, 0, 0);
}

__device__ __forceinline__ void glds4_8(const void* g, char* lds) {
  __builtin_amdgcn_global_load_lds(g, (lds_void8*)lds, 4, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm8() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Fused epilogue of the MX GEMMs: per-row (sx) x per-channel (sw) scales, bias, residual,
// activation; bf16 / fp32 output, or MX8 (e4m3 + one E8M0 scale per (row, 32 columns)). The
// wave owns FPW token fragments from row mw and FCW feature fragments from column nw; lane l
// holds token mw + 16j + (l&15), features nw + 16i + 4(l>>4) .. +3. Wave-uniform (shuffles).
template <int FCW, int FPW>
__device__ __forceinline__ void mx_epilogue(const HzGemmFp8Params& p, const f32x4 (&acc)[FCW][FPW], int mw, int nw,
                                            int lane) {
  const int lrow = lane & 15;
  if (p.out8) {  // MX8 output: per (row, 32-column block) E8M0 scale; no early exits (shuffles)
#pragma unroll
    for (int j = 0; j < FPW; ++j) {
      const int m = mw + j * 16 + lrow;
      const bool mv = m < p.M;
      const float sx = p.sx ? p.sx[min(m, p.M - 1)] : 1.f;
#pragma unroll
      for (int i = 0; i < FCW; i += 2) {
        float v[2][4];
        float amax = 0.f;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int n = min(nw + (i + h) * 16 + (lane >> 4) * 4, p.N - 4);
          const f32x4 sw = *reinterpret_cast<const f32x4*>(p.sw + n);
          const f32x4 bb = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float x = acc[i + h][j][e] * sx * sw[e] + bb[e];
            if (p.act == HZ_ACT_RELU) x = fmaxf(x, 0.f);
            else if (p.act == HZ_ACT_GELU) x = gelu_erf(x);
            else if (p.act == HZ_ACT_TANH) x = tanhf(x);
            v[h][e] = x;
            amax = fmaxf(amax, fabsf(x));
          }
        }
        amax = fmaxf(amax, __shfl_xor(amax, 16, 64));
        amax = fmaxf(amax, __shfl_xor(amax, 32, 64));
        const int ex = mx_exp(amax);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int n = nw + (i + h) * 16 + (lane >> 4) * 4;
          float q[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) q[e] = fminf(fmaxf(ldexpf(v[h][e], -ex), -448.f), 448.f);
          if (mv && n < p.N)
            *reinterpret_cast<unsigned*>(p.out8 + (long)m * p.ldo + n) = pack4_fp8(q[0], q[1], q[2], q[3]);
        }
        const int nb = nw + i * 16;
        if (mv && (lane >> 4) == 0 && nb < p.N) p.os8[(long)m * (p.ldo >> 5) + (nb >> 5)] = (unsigned char)(ex + 127);
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < FPW; ++j) {
    const int m = mw + j * 16 + lrow;
    if (m >= p.M) continue;
    const float sx = p.sx ? p.sx[m] : 1.f;
#pragma unroll
    for (int i = 0; i < FCW; ++i) {
      const int n = nw + i * 16 + (lane >> 4) * 4;
      if (n >= p.N) continue;
      const f32x4 sw = *reinterpret_cast<const f32x4*>(p.sw + n);
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] * sx * sw[e];
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

// XS: the activations carry MX block scales (p.xs, one E8M0 byte per 32 k): each wave also
// stages one 4-byte-per-lane piece (64 rows x the 4 block scales of this 128-deep k-step) and
// the scale goes to the MFMA's B-scale operand: lane l supplies token l&15's scale of 32-k block
// l>>4 (the hardware K order above: block b lives in the register halves of lane groups
// 2(b&1)..2(b&1)+1, not in lane group b).
// WM x WN waves (4 or 8; 8 = two waves per SIMD at one workgroup per CU, whose ds_reads and
// MFMAs interleave): wave (wm, wn) owns rows wm*BM/WM.. and features wn*BN/WN..
template <int BM, int BN, int NS, bool XS, int WM = 2, int WN = 2>
__global__ __launch_bounds__(64 * WM * WN) void gemm_mx_kernel(const HzGemmFp8Params p, int group_m) {
  constexpr int NW = WM * WN;
  constexpr int FCW = BN / WN / 16, FPW = BM / WM / 16;
  constexpr int NWG = BN / 16;                // weight fragments (2 KiB) per stage
  constexpr int XBYTES = BM * 128;
  constexpr int WBYTES = NWG * 2048;
  constexpr int SBYTES = XBYTES + WBYTES + (XS ? NW * 256 : 0);
  constexpr int XPW = BM / 8 / NW, WPW = NWG * 2 / NW;  // glds pieces per wave per stage
  static_assert(XPW * 8 * NW == BM && WPW * NW == NWG * 2 && FCW % 2 == 0 && FPW >= 1 && BM / 64 <= NW,
                "tile / wave split");
  constexpr int G = XPW + WPW + (XS ? 1 : 0);
  __shared__ __attribute__((aligned(16))) char smem[NS * SBYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave % WN, wm = wave / WN;
  const int tiles_n = (p.N + BN - 1) / BN, tiles_m = (p.M + BM - 1) / BM;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  int tile_m, tile_n;
  grouped_tile(lid, tiles_m, tiles_n, group_m, tile_m, tile_n);
  const int n0 = tile_n * BN, m0 = tile_m * BM;
  const int kb = p.K >> 7;  // 128-deep k-steps = stages

  const unsigned char* xsrc[XPW];
#pragma unroll
  for (int i = 0; i < XPW; ++i) {
    const int q = wave + NW * i;
    const int row = min(m0 + q * 8 + (lane >> 3), p.M - 1);
    const int chunk = (lane & 7) ^ mx_swz(((q & 1) << 2) + (lane >> 4));
    xsrc[i] = p.x + (long)row * p.ldx + chunk * 16;
  }
  const unsigned char* wsrc = p.wmx + (long)(n0 >> 4) * kb * 2048 + lane * 16;
  // scale piece of this wave: rows (wave % (BM/64))*64 + lane (waves beyond BM/64 duplicate)
  const unsigned char* ssrc = XS ? p.xs + (long)min(m0 + (wave % (BM / 64)) * 64 + lane, p.M - 1) * (p.K >> 5) : nullptr;
  auto stage = [&](int buf, int st) {
    char* base = smem + buf * SBYTES;
    if constexpr (XS) glds4_8(ssrc + st * 4, base + XBYTES + WBYTES + wave * 256);
#pragma unroll
    for (int i = 0; i < XPW; ++i)
      glds16_8(xsrc[i] + st * 128, base + (wave + NW * i) * 1024);
#pragma unroll
    for (int i = 0; i < WPW; ++i) {
      const int piece = wave + NW * i;  // = g * 2 + half
      const int g = piece >> 1, h = piece & 1;
      glds16_8(wsrc + ((long)g * kb + st) * 2048 + h * 1024, base + XBYTES + piece * 1024);
    }
  };

  const int lr = lane & 15, swz = mx_swz((lane >> 1) & 7);
  const int brow = (wm * (BM / WM) + lr) * 128;
  // hardware K order of the f8f6f4 MFMA (what the E8M0 block scales index): lane group g holds
  // k = 16g..16g+15 in its low 16 B and 64+16g.. in its high 16 B
  const int boff0 = brow + ((lane >> 4) ^ swz) * 16;
  const int boff1 = brow + ((4 + (lane >> 4)) ^ swz) * 16;
  const int aoff = XBYTES + (wn * FCW) * 2048 + lane * 16;

  f32x4 acc[FCW][FPW];
#pragma unroll
  for (int i = 0; i < FCW; ++i)
#pragma unroll
    for (int j = 0; j < FPW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s0 = 0; s0 < NS - 1; ++s0)
    if (s0 < kb) stage(s0, s0);
  int cur = 0;
  for (int st = 0; st < kb; ++st) {
    // stages issued ahead of st: min(NS-2, kb-1-st) may stay in flight (NS = 4: two, the K = 768
    // projections have only 6 stages, so the prologue's loads are most of a tile's latency)
    const int ahead = min(NS - 2, kb - 1 - st);
    if (NS > 3 && ahead >= 2) wait_vm8<(NS > 3 ? 2 * G : 0)>();
    else if (NS > 2 && ahead >= 1) wait_vm8<(NS > 2 ? G : 0)>();
    else wait_vm8<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (st + NS - 1 < kb) stage(cur == 0 ? NS - 1 : cur - 1, st + NS - 1);
    const char* base = smem + cur * SBYTES;
    i32x8 a[FCW], b[FPW];
#pragma unroll
    for (int i = 0; i < FCW; ++i) {
      const u32x4 lo = *reinterpret_cast<const u32x4*>(base + aoff + i * 2048);
      const u32x4 hi = *reinterpret_cast<const u32x4*>(base + aoff + i * 2048 + 1024);
      a[i] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
    }
#pragma unroll
    for (int j = 0; j < FPW; ++j) {
      const u32x4 lo = *reinterpret_cast<const u32x4*>(base + boff0 + j * 16 * 128);
      const u32x4 hi = *reinterpret_cast<const u32x4*>(base + boff1 + j * 16 * 128);
      b[j] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
    }
    int sb[FPW];
#pragma unroll
    for (int j = 0; j < FPW; ++j) {
      if constexpr (XS) {
        const int r = wm * (BM / WM) + j * 16 + (lane & 15);
        sb[j] = *reinterpret_cast<const unsigned char*>(base + XBYTES + WBYTES + (r >> 6) * 256 + (r & 63) * 4 +
                                                        (lane >> 4));
      } else {
        sb[j] = 0x7f7f7f7f;
      }
    }
#pragma unroll
    for (int i = 0; i < FCW; ++i)
#pragma unroll
      for (int j = 0; j < FPW; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[i], b[j], acc[i][j], 0, 0, 0, 0x7f7f7f7f, 0,
                                                                      sb[j]);
    cur = cur == NS - 1 ? 0 : cur + 1;
  }

  mx_epilogue<FCW, FPW>(p, acc, m0 + wm * (BM / WM), n0 + wn * (BN / WN), lane);
}

// Role-split MX GEMM (round 6; cfg 40 / 41): the 128 x 128 tile of cfg 24,
// but its 8 MFMA waves never issue a global load and never meet at a workgroup barrier. Two loader
// waves stage the k-steps into an NS-deep LDS ring with global_load_lds (wave 8: the activation
// pieces and the block-scale pieces, wave 9: the weight pieces), keeping up to AH = NS - 2 stages
// in flight, and publish each stage with an LDS counter once its loads have landed (vmcnt); an
// MFMA wave waits for that count, reads its fragments exactly as cfg 24 does, and returns the slot
// with a second counter once its ds_reads are in registers. Both counters only grow (the round
// r = st / NS of a slot is part of the expected value), so no wave ever resets shared state.
// Every wait is bounded (RS_SPIN polls): a broken handshake ends the kernel with wrong results
// instead of a hang. Same MFMAs in the same order per accumulator as cfg 24: bitwise cfg 24.
constexpr int RS_SPIN = 1 << 22;

__device__ __forceinline__ int lds_load_relaxed(int* a) {
  return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ void lds_add(int* a) {
  __hip_atomic_fetch_add(a, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// wait until *a >= v (one lane polls; the value is wave-uniform through readfirstlane)
__device__ __forceinline__ void lds_wait_ge(int* a, int v) {
  for (int i = 0; i < RS_SPIN; ++i) {
    if (__builtin_amdgcn_readfirstlane(lds_load_relaxed(a)) >= v) break;
    __builtin_amdgcn_s_sleep(1);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

template <int NS, bool XS>
__global__ __launch_bounds__(64 * 10) void gemm_mx_rs_kernel(const HzGemmFp8Params p, int group_m) {
  constexpr int BM = 128, BN = 128, WM = 2, WN = 4, MW = WM * WN;
  constexpr int FCW = BN / WN / 16, FPW = BM / WM / 16;
  constexpr int NWG = BN / 16;
  constexpr int XBYTES = BM * 128, WBYTES = NWG * 2048, SCB = XS ? (BM / 64) * 256 : 0;
  constexpr int SBYTES = XBYTES + WBYTES + SCB;
  constexpr int XP = BM / 8, WP = NWG * 2, SP = XS ? BM / 64 : 0;
  constexpr int AH = NS - 2;  // stages a loader keeps in flight behind the one it publishes
  static_assert(NS >= 2 && AH * (XP + SP) < 64 && AH * WP < 64, "vmcnt range");
  __shared__ __attribute__((aligned(16))) char smem[NS * SBYTES];
  __shared__ int loaded[NS], consumed[NS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (tid < NS) {
    loaded[tid] = 0;
    consumed[tid] = 0;
  }
  __syncthreads();  // the only workgroup barrier: the counters exist
  const int tiles_n = (p.N + BN - 1) / BN, tiles_m = (p.M + BM - 1) / BM;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  int tile_m, tile_n;
  grouped_tile(lid, tiles_m, tiles_n, group_m, tile_m, tile_n);
  const int n0 = tile_n * BN, m0 = tile_m * BM;
  const int kb = p.K >> 7;

  if (wave >= MW) {  // ------------------------------------------------------------ loader waves
    const bool xw = wave == MW;  // wave 8: activations (+ scales); wave 9: weights
    const unsigned char* xsrc[XP];
#pragma unroll
    for (int q = 0; q < XP; ++q) {
      const int row = min(m0 + q * 8 + (lane >> 3), p.M - 1);
      const int chunk = (lane & 7) ^ mx_swz(((q & 1) << 2) + (lane >> 4));
      xsrc[q] = p.x + (long)row * p.ldx + chunk * 16;
    }
    const unsigned char* wsrc = p.wmx + (long)(n0 >> 4) * kb * 2048 + lane * 16;
    const unsigned char* ssrc[SP > 0 ? SP : 1];
#pragma unroll
    for (int q = 0; q < SP; ++q) ssrc[q] = p.xs + (long)min(m0 + q * 64 + lane, p.M - 1) * (p.K >> 5);
    for (int st = 0; st < kb + AH; ++st) {
      if (st < kb) {
        const int buf = st % NS;
        lds_wait_ge(&consumed[buf], MW * (st / NS));  // every MFMA wave is done with round st/NS - 1
        char* base = smem + buf * SBYTES;
        if (xw) {
#pragma unroll
          for (int q = 0; q < SP; ++q) glds4_8(ssrc[q] + st * 4, base + XBYTES + WBYTES + q * 256);
#pragma unroll
          for (int q = 0; q < XP; ++q) glds16_8(xsrc[q] + st * 128, base + q * 1024);
        } else {
#pragma unroll
          for (int q = 0; q < WP; ++q)
            glds16_8(wsrc + ((long)(q >> 1) * kb + st) * 2048 + (q & 1) * 1024, base + XBYTES + q * 1024);
        }
      }
      const int done = st - AH;  // the stage whose loads must have landed now
      if (done >= 0) {
        // loads retire in issue order: with the later stages' pieces still allowed in flight
        const int later = min(AH, kb - 1 - done);
        if (xw) {
          if (later >= 2) wait_vm8<2 * (XP + SP) < 64 ? 2 * (XP + SP) : 0>();
          else if (later == 1) wait_vm8<XP + SP>();
          else wait_vm8<0>();
        } else {
          if (later >= 2) wait_vm8<2 * WP < 64 ? 2 * WP : 0>();
          else if (later == 1) wait_vm8<WP>();
          else wait_vm8<0>();
        }
        if (lane == 0) lds_add(&loaded[done % NS]);
      }
    }
    return;
  }

  // ------------------------------------------------------------------------------ MFMA waves
  const int wn = wave % WN, wm = wave / WN;
  const int lr = lane & 15, swz = mx_swz((lane >> 1) & 7);
  const int brow = (wm * (BM / WM) + lr) * 128;
  const int boff0 = brow + ((lane >> 4) ^ swz) * 16;
  const int boff1 = brow + ((4 + (lane >> 4)) ^ swz) * 16;
  const int aoff = XBYTES + (wn * FCW) * 2048 + lane * 16;
  f32x4 acc[FCW][FPW];
#pragma unroll
  for (int i = 0; i < FCW; ++i)
#pragma unroll
    for (int j = 0; j < FPW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int st = 0; st < kb; ++st) {
    const int buf = st % NS;
    lds_wait_ge(&loaded[buf], 2 * (st / NS + 1));  // both loader waves published stage st
    const char* base = smem + buf * SBYTES;
    i32x8 a[FCW], b[FPW];
#pragma unroll
    for (int i = 0; i < FCW; ++i) {
      const u32x4 lo = *reinterpret_cast<const u32x4*>(base + aoff + i * 2048);
      const u32x4 hi = *reinterpret_cast<const u32x4*>(base + aoff + i * 2048 + 1024);
      a[i] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
    }
#pragma unroll
    for (int j = 0; j < FPW; ++j) {
      const u32x4 lo = *reinterpret_cast<const u32x4*>(base + boff0 + j * 16 * 128);
      const u32x4 hi = *reinterpret_cast<const u32x4*>(base + boff1 + j * 16 * 128);
      b[j] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
    }
    int sb[FPW];
#pragma unroll
    for (int j = 0; j < FPW; ++j) {
      if constexpr (XS) {
        const int r = wm * (BM / WM) + j * 16 + (lane & 15);
        sb[j] = *reinterpret_cast<const unsigned char*>(base + XBYTES + WBYTES + (r >> 6) * 256 + (r & 63) * 4 +
                                                        (lane >> 4));
      } else {
        sb[j] = 0x7f7f7f7f;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the fragments are in registers: return the slot
    if (lane == 0) lds_add(&consumed[buf]);
#pragma unroll
    for (int i = 0; i < FCW; ++i)
#pragma unroll
      for (int j = 0; j < FPW; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[i], b[j], acc[i][j], 0, 0, 0, 0x7f7f7f7f, 0,
                                                                      sb[j]);
  }
  mx_epilogue<FCW, FPW>(p, acc, m0 + wm * (BM / WM), n0 + wn * (BN / WN), lane);
}

template <int NS>
int launch_mx_rs(const HzGemmFp8Params& p, hipStream_t st) {
  if (p.N % 128) return -4;
  const int tiles = (p.N / 128) * ((p.M + 127) / 128);
  static const int group_env = getenv("HIPZAP_GEMM_GROUP") ? atoi(getenv("HIPZAP_GEMM_GROUP")) : 8;
  const int group_m = group_env < 1 ? 1 : group_env;
  if (p.xs) hipLaunchKernelGGL((gemm_mx_rs_kernel<NS, true>), dim3(tiles), dim3(640), 0, st, p, group_m);
  else hipLaunchKernelGGL((gemm_mx_rs_kernel<NS, false>), dim3(tiles), dim3(640), 0, st, p, group_m);
  return (int)hipGetLastError();
}

// Measured-negative MX schedules removed in round 5, their numbers committed: the
// ping-pong 128x128 tile with two wave groups a phase apart (cfg 34-36, 1.4x slower than cfg 24,
// profiles/r4_mx), the 256-row tiles with a branch-free main loop (cfg 43-45) and the ring-pipelined
// 256-row kernel with K unrolled (cfg 46-47), 1.15-1.6x slower (profiles/r3_mx256, r3_mxk). Source:
// git history before the round-5 cleanup.

template <int BM, int BN, int NS, int WM = 2, int WN = 2>
int launch_mx(const HzGemmFp8Params& p, hipStream_t st) {
  // the 8-wave tiles read BN weight rows per tile: N must fill them (the 4-wave tiles predate this)
  if (WM * WN > 4 && p.N % BN) return -4;
  const int tiles = ((p.N + BN - 1) / BN) * ((p.M + BM - 1) / BM);
  static const int group_env = getenv("HIPZAP_GEMM_GROUP") ? atoi(getenv("HIPZAP_GEMM_GROUP")) : 8;
  const int group_m = group_env < 1 ? 1 : group_env;
  const dim3 block(64 * WM * WN);
  if (p.xs) hipLaunchKernelGGL((gemm_mx_kernel<BM, BN, NS, true, WM, WN>), dim3(tiles), block, 0, st, p, group_m);
  else hipLaunchKernelGGL((gemm_mx_kernel<BM, BN, NS, false, WM, WN>), dim3(tiles), block, 0, st, p, group_m);
  return (int)hipGetLastError();
}

}  // namespace

extern "C" int hz_gemm_fp8_launch(const HzGemmFp8Params* pp, hipStream_t st) {
  const HzGemmFp8Params& p = *pp;
  if (p.cfg >= 16) {
    if (!p.wmx || p.K % 128 || p.ldx % 16 || p.N % 4) return -1;
    if (!p.sx && !p.xs) return -1;
    if (p.out8 && (!p.os8 || p.ldo % 32 || p.N % 32)) return -1;
    switch (p.cfg) {
      case 16: return launch_mx<128, 128, 3>(p, st);
      case 20: return launch_mx<128, 128, 2>(p, st);
      case 17: return launch_mx<64, 128, 3>(p, st);
      case 21: return launch_mx<64, 128, 2>(p, st);
      case 18: return launch_mx<128, 64, 3>(p, st);
      case 22: return launch_mx<128, 64, 2>(p, st);
      case 19: return launch_mx<64, 64, 3>(p, st);
      case 23: return launch_mx<64, 64, 2>(p, st);
      // 8-wave workgroups (two waves per SIMD): 128x128, 256x128, 128x256 at 2 / 3 LDS stages
      case 24: return launch_mx<128, 128, 2, 2, 4>(p, st);
      case 25: return launch_mx<256, 128, 2, 4, 2>(p, st);
      case 26: return launch_mx<128, 256, 2, 2, 4>(p, st);
      case 27: return launch_mx<128, 128, 3, 2, 4>(p, st);
      case 28: return launch_mx<256, 128, 3, 4, 2>(p, st);
      case 29: return launch_mx<128, 256, 3, 2, 4>(p, st);
      // 4 LDS stages (two K steps in flight): 8-wave 128x128, 4-wave 64x128 / 128x64
      case 30: return launch_mx<128, 128, 4, 2, 4>(p, st);
      case 31: return launch_mx<64, 128, 4>(p, st);
      case 32: return launch_mx<128, 64, 4>(p, st);
      // 8-wave 256x256 tile of the plain kernel (all fragments read before the MFMAs)
      case 33: return launch_mx<256, 256, 2, 2, 4>(p, st);
      // role-split 128x128 (8 MFMA waves + 2 loader waves, LDS FULL / FREE counters): 4 / 3 stages
      case 40: return launch_mx_rs<4>(p, st);
      case 41: return launch_mx_rs<3>(p, st);
      case 42: return launch_mx_rs<2>(p, st);  // 66 KB of LDS: two workgroups (20 waves) per CU
      default: return -2;
    }
  }
  if (p.N % 4 || p.ldx % 8 || p.ksteps * 32 < p.K || !p.sx || p.xs || p.out8) return -1;  // ring: per-row scales only
  switch (p.cfg) {
    case 0: return launch8<1, 1>(p, st);
    case 1: return launch8<1, 2>(p, st);
    case 2: return launch8<1, 4>(p, st);
    case 3: return launch8<2, 1>(p, st);
    case 4: return launch8<2, 2>(p, st);
    case 5: return launch8<2, 4>(p, st);
    case 6: return launch8<4, 1>(p, st);
    case 7: return launch8<4, 2>(p, st);
    case 8: return launch8<4, 4>(p, st);
    default: return -2;
  }
}

// Load this translation unit's device code without a launch (see hz_conv_code_warm in conv.hip).
__global__ void hz_fp8_code_warm_kernel() {}
extern "C" int hz_fp8_code_warm(void) {
  hipFuncAttributes a;
  return (int)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&hz_fp8_code_warm_kernel));
}
