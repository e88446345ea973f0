// Transformer kernels for BERT-base / ViT-B/16 serving:
//   * layernorm  — one wave per row, 16-B loads, two-pass mean/var in registers, optional
//                  fused residual add, bf16 out (and optionally a strided output row, e.g.
//                  the CLS-only final LN of ViT);
//   * embed_ln   — BERT word + position + token-type gather-sum + LayerNorm in one pass;
//   * attention  — fused softmax(Q K^T * scale + mask) V per (batch, head, 64-query block),
//                  K and V^T staged in LDS, S kept in MFMA accumulators, row softmax via
//                  16-lane shuffles, P written once to LDS as bf16 and re-read as the A
//                  operand of P.V. L <= 256, head dim 64 (BERT L=128, ViT L=197).
//   * patch_tokens — ViT: CLS token + position embedding add around the patch-embed GEMM.
#include <cstdlib>

#include "common.h"
#include "hipzap.h"

HZ_DEBUG_UNIT(transformer)

namespace {

// --------------------------------------------------------------------------- LayerNorm
// rows x D (D % 8 == 0, D <= 64*8*NC): each lane holds up to NC 16-B chunks of its row (NC sized
// to D at launch: at D = 768 two, so the kernel holds ~100 instead of 174 VGPRs). A wave owns
// RPW consecutive rows: gamma / beta are loaded once per wave (not once per row: 6 KB a row at
// D = 768), and row i+1's loads are issued before row i's reductions, so a wave pays one memory
// latency for its RPW rows (RPW = 1: a wave per row, the round-1..4 kernel). Same per-row math in
// the same order: bitwise the same outputs for every RPW.
template <int NC, int RPW>
__global__ __launch_bounds__(256) void layernorm_kernel(const HzLayerNormParams p) {
  const int lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
  if (row0 >= p.rows) return;
  if (!HZ_DCHECK(p.D <= NC * 64 * 8 && p.ldx >= p.D && (!p.res || p.ldr >= p.D))) return;
  const int nch = p.D >> 3;
  u32x4 xr[NC], rr4[NC];
  auto load_row = [&](int row, u32x4 (&xo)[NC], u32x4 (&ro)[NC]) {
    const bf16_t* x = p.x + (long)row * p.ldx;
    const bf16_t* r = p.res ? p.res + (long)row * p.ldr : nullptr;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int ch = c * 64 + lane;
      if (ch < nch) {
        xo[c] = *reinterpret_cast<const u32x4*>(x + ch * 8);
        if (r) ro[c] = *reinterpret_cast<const u32x4*>(r + ch * 8);
      }
    }
  };
  // every load of the first row first -- x, residual, then gamma, beta -- so the wave pays ONE
  // memory latency before the reductions
  load_row(row0, xr, rr4);
  f32x4 g4[NC][2], b4[NC][2];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int ch = c * 64 + lane;
    if (ch < nch) {
      g4[c][0] = *reinterpret_cast<const f32x4*>(p.gamma + ch * 8);
      g4[c][1] = *reinterpret_cast<const f32x4*>(p.gamma + ch * 8 + 4);
      b4[c][0] = *reinterpret_cast<const f32x4*>(p.beta + ch * 8);
      b4[c][1] = *reinterpret_cast<const f32x4*>(p.beta + ch * 8 + 4);
    }
  }
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    const int row = row0 + i;
    if (row >= p.rows) break;  // wave-uniform
    u32x4 xn[NC], rn[NC];
    if (RPW > 1 && i + 1 < RPW && row + 1 < p.rows) load_row(row + 1, xn, rn);  // in flight over this row
    float v[NC][8];
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int ch = c * 64 + lane;
      if (ch < nch) {
        unpack8(xr[c], v[c]);
        if (p.res) {
          float rr[8];
          unpack8(rr4[c], rr);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[c][e] += rr[e];
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) s += v[c][e];
      }
    }
    const float mean = warp_sum(s) / p.D;
    float q = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int ch = c * 64 + lane;
      if (ch < nch) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = v[c][e] - mean;
          q += d * d;
        }
      }
    }
    const float rstd = rsqrtf(warp_sum(q) / p.D + p.eps);
    float amax = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int ch = c * 64 + lane;
      if (ch < nch) {
        const f32x4 g0 = g4[c][0], g1 = g4[c][1], b0 = b4[c][0], b1 = b4[c][1];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[c][e] = (v[c][e] - mean) * rstd * g0[e] + b0[e];
          v[c][e + 4] = (v[c][e + 4] - mean) * rstd * g1[e] + b1[e];
        }
        if (p.out) *reinterpret_cast<u32x4*>(p.out + (long)row * p.ldo + ch * 8) = pack8(v[c]);
#pragma unroll
        for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(v[c][e]));
      }
    }
    if (p.out8) {
      // fused fp8 quantisation (same rule as fp8.hip quant_rows: s = amax / 448, e4m3fn)
      amax = warp_max(amax);
      const float scale = fmaxf(amax, 1e-12f) / 448.f, inv = 1.f / scale;
      unsigned char* o8 = p.out8 + (long)row * p.D;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int ch = c * 64 + lane;
        if (ch < nch) {
          float q8[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) q8[e] = fminf(fmaxf(v[c][e] * inv, -448.f), 448.f);
          *reinterpret_cast<u32x2*>(o8 + ch * 8) =
              u32x2{pack4_fp8(q8[0], q8[1], q8[2], q8[3]), pack4_fp8(q8[4], q8[5], q8[6], q8[7])};
        }
      }
      if (lane == 0) p.scale8[row] = scale;
    }
    if constexpr (RPW > 1) {
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        xr[c] = xn[c];
        rr4[c] = rn[c];
      }
    }
  }
}

// --------------------------------------------------------------------------- BERT embeddings
__global__ __launch_bounds__(256) void embed_ln_kernel(const HzEmbedParams p) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= p.rows) return;
  const int tok = min(max(p.ids[row], 0), p.vocab - 1);
  const int pos = row % p.L;
  const int tt = p.types ? min(max(p.types[row], 0), p.ntypes - 1) : 0;
  const bf16_t* w = p.word + (long)tok * p.D;
  const bf16_t* ps = p.pos + (long)pos * p.D;
  const bf16_t* ty = p.type + (long)tt * p.D;
  const int nch = p.D >> 3;
  float v[4][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int ch = c * 64 + lane;
    if (ch < nch) {
      float a[8], b[8], d[8];
      unpack8(*reinterpret_cast<const u32x4*>(w + ch * 8), a);
      unpack8(*reinterpret_cast<const u32x4*>(ps + ch * 8), b);
      unpack8(*reinterpret_cast<const u32x4*>(ty + ch * 8), d);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[c][e] = a[e] + b[e] + d[e];
        s += v[c][e];
      }
    }
  }
  const float mean = warp_sum(s) / p.D;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int ch = c * 64 + lane;
    if (ch < nch) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = v[c][e] - mean;
        q += d * d;
      }
    }
  }
  const float rstd = rsqrtf(warp_sum(q) / p.D + p.eps);
  bf16_t* o = p.out + (long)row * p.D;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int ch = c * 64 + lane;
    if (ch < nch) {
      float y[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) y[e] = (v[c][e] - mean) * rstd * p.gamma[ch * 8 + e] + p.beta[ch * 8 + e];
      *reinterpret_cast<u32x4*>(o + ch * 8) = pack8(y);
    }
  }
}

// --------------------------------------------------------------------------- attention
// softmax(Q K^T * scale + mask) V per (batch, head, block of 16*NW queries); one wave owns 16
// queries and all keys (L <= 256). Keys live on the MFMA lane (cdna_hip_programming.md §3 'An
// accumulator tile as the next MFMA's operand'):
//   S^T = K Q^T   (A = K rows from LDS, B = Q^T from global): lane (q = l&15, g = l>>4) holds
//                 the scores of query q for keys kt*16 + 4g + i, i < 4;
//   softmax       row max / sum over the lane's values + 2 shuffles (xor 16, 32);
//   O^T = V^T P^T the P accumulators ARE the B operand (converted to bf16 in registers, k order
//                 permuted: element j of group g = key 32c + 4g + j (j < 4), 32c + 16 + 4g + j-4);
//                 A = V^T in the same k order, read from the row-major V image with two
//                 ds_read_b64_tr_b16 per fragment (T10) — no transposed staging, no P image.
//   O^T accumulators give each lane 4 consecutive head dims of one query: 8-byte stores.
// K and V are staged once per workgroup with 16-B loads/stores; padding keys (L <= key < Lp)
// re-read row L-1 (finite) and are masked to -inf, so their probabilities are exactly 0.
#ifndef HZ_ATT_NW8_MINL
#define HZ_ATT_NW8_MINL 64
#endif
constexpr int ATT_D = 64;
constexpr int ATT_LMAX = 256;
// Row strides (bf16) of the K and V images, both 160 B: for the K fragment reads
// (ds_read_b128, lane l -> row l&15, 16-B chunk l>>4) every one of the instruction's four 16-lane
// groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, ... (MI355X_MICROARCH.md §LDS) then covers the 64
// banks exactly once; the former 144-B stride was 2-way in every group (SQ_LDS_BANK_CONFLICT
// ratio 0.22, profiles/r2_pmc_fp8). For the V transposed reads (ds_read_b64_tr_b16, 32-lane
// halves) the 8 rows of a half land on 8 distinct 32-B bank slots.
constexpr int ATT_KST = ATT_D + 16;
constexpr int ATT_VST = ATT_D + 16;

typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

__device__ __forceinline__ unsigned pack_bf16x2(float a, float b) {
  return (unsigned)f2bf(a) | ((unsigned)f2bf(b) << 16);
}

template <int NW>
__global__ __launch_bounds__(64 * NW) void attention_kernel(const HzAttentionParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int Lp = (p.L + 31) & ~31;  // keys padded to the 32-wide MFMA K step
  bf16_t* Ks = reinterpret_cast<bf16_t*>(smem);  // [Lp][ATT_KST]
  bf16_t* Vs = Ks + Lp * ATT_KST;                // [Lp][ATT_VST] row-major
  float* Ms = reinterpret_cast<float*>(Vs + Lp * ATT_VST);  // [Lp] additive mask (-inf for padding keys)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bh = blockIdx.x;
  const int b = bh / p.heads, h = bh - b * p.heads;
  const long row0 = (long)b * p.L;
  const bf16_t* Q = p.qkv + row0 * p.ldqkv + h * ATT_D;
  const bf16_t* K = Q + p.k_off;
  const bf16_t* V = Q + p.v_off;
  // debug contracts (uniform per block, before any barrier): the head's Q/K/V columns and its
  // output columns lie inside their rows, and the sequence fits the LDS staging
  if (!HZ_DCHECK(b < p.B && p.L <= ATT_LMAX && h * ATT_D + max(0, max(p.k_off, p.v_off)) + ATT_D <= p.ldqkv &&
                 h * ATT_D + ATT_D <= p.ldo))
    return;
  // ---- every global load first: this wave's Q^T fragments (B operand: k = head dim, col =
  // query; rows past L clamp to L-1 and are never stored), then K, V and the mask ----
  const int q0 = blockIdx.y * 16 * NW + wave * 16;
  const int lq = lane & 15, g = lane >> 4;
  bf16x8 qb[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
    qb[ks] = *reinterpret_cast<const bf16x8*>(Q + (long)min(q0 + lq, p.L - 1) * p.ldqkv + ks * 32 + g * 8);
  constexpr int SIT = ATT_LMAX * 8 / (64 * NW);
  u32x4 kv[SIT], vv[SIT];
#pragma unroll
  for (int it = 0; it < SIT; ++it) {
    const int i = tid + it * 64 * NW;
    if (i >= Lp * 8) break;  // uniform per iteration count (Lp*8 is a multiple of 64*NW/..): guarded per lane
    const int key = min(i >> 3, p.L - 1), c = (i & 7) * 8;
    kv[it] = *reinterpret_cast<const u32x4*>(K + (long)key * p.ldqkv + c);
    vv[it] = *reinterpret_cast<const u32x4*>(V + (long)key * p.ldqkv + c);
  }
  for (int k = tid; k < Lp; k += 64 * NW)
    Ms[k] = k < p.L ? (p.mask ? p.mask[(long)b * p.L + k] : 0.f) : -INFINITY;
#pragma unroll
  for (int it = 0; it < SIT; ++it) {
    const int i = tid + it * 64 * NW;
    if (i >= Lp * 8) break;
    const int key = i >> 3, c = (i & 7) * 8;
    *reinterpret_cast<u32x4*>(Ks + key * ATT_KST + c) = kv[it];
    *reinterpret_cast<u32x4*>(Vs + key * ATT_VST + c) = vv[it];
  }
  __syncthreads();
  if (q0 >= p.L) return;  // no barrier follows (the transposed reads below need full EXEC: whole waves only)
  // ---- S^T = K Q^T: s[kt][i] = score(query q0+lq, key kt*16 + 4g + i) ----
  const int nkt = Lp / 16;
  f32x4 s[ATT_LMAX / 16];
#pragma unroll
  for (int kt = 0; kt < ATT_LMAX / 16; ++kt) {
    s[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (kt < nkt) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 ka = *reinterpret_cast<const bf16x8*>(Ks + (kt * 16 + lq) * ATT_KST + ks * 32 + g * 8);
        s[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, qb[ks], s[kt], 0, 0, 0);
      }
    }
  }
  // ---- scale + mask + softmax over the keys of query lq (4 lanes x the lane's values) ----
  float mx = -INFINITY;
#pragma unroll
  for (int kt = 0; kt < ATT_LMAX / 16; ++kt) {
    if (kt < nkt) {
      const f32x4 madd = *reinterpret_cast<const f32x4*>(Ms + kt * 16 + 4 * g);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        s[kt][i] = s[kt][i] * p.scale + madd[i];
        mx = fmaxf(mx, s[kt][i]);
      }
    }
  }
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int kt = 0; kt < ATT_LMAX / 16; ++kt) {
    if (kt < nkt) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float e = __expf(s[kt][i] - mx);
        s[kt][i] = e;
        sum += e;
      }
    }
  }
  sum += __shfl_xor(sum, 16, 64);
  sum += __shfl_xor(sum, 32, 64);
  const float inv = 1.f / sum;
  // ---- O^T = V^T P^T over 32-key steps ----
  f32x4 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  // transposed-read address of this lane: block row (lane&15)>>2 of the group's 4 rows, columns
  // 4*(lane&3) .. +3 of the 16-dim tile (T10: lane 4r+c supplies row r, columns 4c..4c+3)
  const int tr_row = (lane & 15) >> 2, tr_col = (lane & 3) * 4;
#pragma unroll
  for (int c = 0; c < ATT_LMAX / 32; ++c) {
    if (c < Lp / 32) {
      const f32x4 pa = s[2 * c], pb = s[2 * c + 1];
      const u32x4 pw = u32x4{pack_bf16x2(pa[0] * inv, pa[1] * inv), pack_bf16x2(pa[2] * inv, pa[3] * inv),
                             pack_bf16x2(pb[0] * inv, pb[1] * inv), pack_bf16x2(pb[2] * inv, pb[3] * inv)};
      const bf16x8 pfrag = *reinterpret_cast<const bf16x8*>(&pw);
      const int r_lo = 32 * c + 4 * g + tr_row, r_hi = r_lo + 16;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(Vs + r_lo * ATT_VST + dt * 16 + tr_col));
        const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(Vs + r_hi * ATT_VST + dt * 16 + tr_col));
        const short vv8[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        const bf16x8 va = *reinterpret_cast<const bf16x8*>(vv8);
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pfrag, o[dt], 0, 0, 0);
      }
    }
  }
  // lane holds O[q0 + lq][dt*16 + 4g + i]
  const int q = q0 + lq;
  if (p.out8) {  // MX8 output: head dims [0,32) = dt 0,1 and [32,64) = dt 2,3 are two E8M0 blocks
#pragma unroll
    for (int hb = 0; hb < 2; ++hb) {
      float amax = 0.f;
#pragma unroll
      for (int d = 0; d < 2; ++d)
#pragma unroll
        for (int i = 0; i < 4; ++i) amax = fmaxf(amax, fabsf(o[2 * hb + d][i]));
      amax = fmaxf(amax, __shfl_xor(amax, 16, 64));
      amax = fmaxf(amax, __shfl_xor(amax, 32, 64));
      const int ex = mx_exp(amax);
      if (q < p.L) {
        unsigned char* o8 = p.out8 + (row0 + q) * p.ldo + h * ATT_D + hb * 32;
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          float x[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) x[i] = fminf(fmaxf(ldexpf(o[2 * hb + d][i], -ex), -448.f), 448.f);
          *reinterpret_cast<unsigned*>(o8 + d * 16 + 4 * g) = pack4_fp8(x[0], x[1], x[2], x[3]);
        }
        if (g == 0) p.os8[(row0 + q) * (p.ldo >> 5) + h * 2 + hb] = (unsigned char)(ex + 127);
      }
    }
    return;
  }
  if (q < p.L) {
    bf16_t* out = p.out + (row0 + q) * p.ldo + h * ATT_D + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
      *reinterpret_cast<u32x2*>(out + dt * 16) = u32x2{pack_bf16x2(o[dt][0], o[dt][1]), pack_bf16x2(o[dt][2], o[dt][3])};
  }
}

// --------------------------------------------------------------------------- QKV + attention
// A BERT-class self-attention block in ONE launch (HzQkvAttParams; VERDICT r4 "next round" 4). A
// workgroup per (sequence b, head h) computes its head's Q, K and V for the sequence's L <= 128
// tokens as one 128 x 192 LDS-tiled GEMM tile over K = D (the tile and pipeline of gemm.hip's
// gemm_lds_kernel<128, 192, NS, .., 2, 4>: 2 x 4 waves, 64-deep stages, swizzled 128-B activation
// lines, fragment-major weights through global_load_lds) -- the packed QKV weight rows of head h
// are the three 64-row spans h*64, D + h*64 and 2D + h*64, picked per weight fragment, so the
// standalone GEMM's packing serves unchanged. The epilogue adds the bias and writes Q, K, V as bf16
// images into the LDS the stages used; the attention (attention_kernel's math: S^T = K Q^T,
// softmax over the lane's keys + 2 shuffles, O^T = V^T P^T with transposed V reads) then runs from
// there. The QKV activations never go to memory, and the attention's launch and its kernel
// boundary are gone: 6 kernels per encoder layer instead of 7.
__device__ __forceinline__ void qa_glds16(const void* g, char* lds) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}
template <int N>
__device__ __forceinline__ void qa_wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
constexpr int QA_BM = 128, QA_NWG = 12, QA_XBYTES = QA_BM * 128, QA_SBYTES = QA_XBYTES + QA_NWG * 2 * 1024;
constexpr int QA_IMG = QA_BM * ATT_KST;  // bf16 elements of one Q / K / V image (row stride ATT_KST)
static_assert(3 * QA_IMG * 2 + QA_BM * 4 <= 2 * QA_SBYTES, "the attention images alias the GEMM stages");

template <int NS>
__global__ __launch_bounds__(512) void qkvatt_kernel(const HzQkvAttParams p) {
  constexpr int G = 2 + 3;  // global_load_lds per wave per stage: 2 activation pieces, 3 weight fragments
  __shared__ __attribute__((aligned(16))) char smem[NS * QA_SBYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave & 3, wm = wave >> 2;
  // consecutive workgroups (one XCD) are the heads of one sequence: its 128 x D activations hit L2
  const int bh = xcd_remap(blockIdx.x, gridDim.x);
  const int b = bh / p.heads, h = bh - b * p.heads;
  const int L = p.L, nst = p.ksteps >> 1;
  const long row0 = (long)b * L;
  // activation piece q = wave + 8i: tile rows 8q .. 8q+7, lane -> row 8q + (lane >> 3), 16-B chunk
  // (lane & 7) of the row XOR-swizzled as gemm_lds_kernel's image; rows past L repeat token L-1
  const bf16_t* xsrc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = wave + 8 * i;
    const int row = min(q * 8 + (lane >> 3), L - 1);
    const int chunk = (lane & 7) ^ (((q & 1) << 2) + (lane >> 4));
    xsrc[i] = p.x + (row0 + row) * p.ldx + chunk * 8;
  }
  // weight piece f = wave + 8i (f = ks * 12 + g): tile fragment g = packed fragment (g/4) * D/16 + 4h + g%4
  const bf16_t* wsrc[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int f = wave + 8 * i, ks = f / QA_NWG, g = f - ks * QA_NWG;
    const int frag = (g >> 2) * (p.D >> 4) + 4 * h + (g & 3);
    wsrc[i] = p.w + (((long)frag * p.ksteps + ks) * 64 + lane) * 8;
  }
  auto stage = [&](int buf, int st) {
    char* base = smem + buf * QA_SBYTES;
#pragma unroll
    for (int i = 0; i < 2; ++i) qa_glds16(xsrc[i] + st * 64, base + (wave + 8 * i) * 1024);
#pragma unroll
    for (int i = 0; i < 3; ++i) qa_glds16(wsrc[i] + st * 2 * 512, base + QA_XBYTES + (wave + 8 * i) * 1024);
  };
  // the epilogue's operands go out first (independent of the GEMM): bias of this lane's features,
  // the additive key mask (threads < 128)
  f32x4 bias[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int fl = wn * 48 + 16 * i + 4 * (lane >> 4);
    bias[i] = *reinterpret_cast<const f32x4*>(p.bias + (fl >> 6) * p.D + h * ATT_D + (fl & 63));
  }
  const int Lp = (L + 31) & ~31;
  float mk = 0.f;
  if (tid < Lp) mk = tid < L ? (p.mask ? p.mask[row0 + tid] : 0.f) : -INFINITY;
  // ---- the 128 x 192 x D GEMM (gemm_lds_kernel's schedule) ----
  const int lr = lane & 15, sw = (lane >> 1) & 7;
  const int boff0 = (wm * 64 + lr) * 128 + ((lane >> 4) ^ sw) * 16;
  const int boff1 = (wm * 64 + lr) * 128 + ((4 + (lane >> 4)) ^ sw) * 16;
  const int aoff = QA_XBYTES + (wn * 3) * 1024 + lane * 16;
  f32x4 acc[3][4];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s0 = 0; s0 < NS - 1; ++s0)
    if (s0 < nst) stage(s0, s0);
  int cur = 0;
  for (int st = 0; st < nst; ++st) {
    const int ahead = min(NS - 2, nst - 1 - st);
    if (NS > 2 && ahead >= 1) qa_wait_vm<(NS > 2 ? G : 0)>();
    else qa_wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (st + NS - 1 < nst) stage(cur == 0 ? NS - 1 : cur - 1, st + NS - 1);
    const char* base = smem + cur * QA_SBYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 a[3], bb[4];
#pragma unroll
      for (int i = 0; i < 3; ++i) a[i] = *reinterpret_cast<const bf16x8*>(base + aoff + (ks * QA_NWG + i) * 1024);
#pragma unroll
      for (int j = 0; j < 4; ++j) bb[j] = *reinterpret_cast<const bf16x8*>(base + (ks ? boff1 : boff0) + j * 16 * 128);
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], bb[j], acc[i][j], 0, 0, 0);
    }
    cur = cur == NS - 1 ? 0 : cur + 1;
  }
  // ---- Q, K, V (+ bias, bf16) into LDS images over the stages: lane holds features
  // wn*48 + 16i + 4(lane>>4) + e of token wm*64 + 16j + (lane&15) ----
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // every wave is done reading the stages
  bf16_t* img = reinterpret_cast<bf16_t*>(smem);  // [3][QA_BM][ATT_KST]: Q, K, V
  float* Ms = reinterpret_cast<float*>(smem + 3 * QA_IMG * 2);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int fl = wn * 48 + 16 * i + 4 * (lane >> 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int tok = wm * 64 + 16 * j + lr;
      const f32x4 v = acc[i][j] + bias[i];
      *reinterpret_cast<u32x2*>(img + (fl >> 6) * QA_IMG + tok * ATT_KST + (fl & 63)) =
          u32x2{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
    }
  }
  if (tid < Lp) Ms[tid] = mk;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  const bf16_t* Qs = img;
  const bf16_t* Ks = img + QA_IMG;
  const bf16_t* Vs = img + 2 * QA_IMG;
  // ---- attention for queries q0 .. q0+15 of this wave (attention_kernel's math) ----
  const int q0 = wave * 16;
  if (q0 >= L) return;  // whole waves only (the transposed reads need full EXEC); no barrier follows
  const int lq = lane & 15, g = lane >> 4;
  bf16x8 qb[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) qb[ks] = *reinterpret_cast<const bf16x8*>(Qs + (q0 + lq) * ATT_KST + ks * 32 + g * 8);
  const int nkt = Lp / 16;
  f32x4 s[QA_BM / 16];
#pragma unroll
  for (int kt = 0; kt < QA_BM / 16; ++kt) {
    s[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (kt < nkt) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 ka = *reinterpret_cast<const bf16x8*>(Ks + (kt * 16 + lq) * ATT_KST + ks * 32 + g * 8);
        s[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, qb[ks], s[kt], 0, 0, 0);
      }
    }
  }
  float mx = -INFINITY;
#pragma unroll
  for (int kt = 0; kt < QA_BM / 16; ++kt) {
    if (kt < nkt) {
      const f32x4 madd = *reinterpret_cast<const f32x4*>(Ms + kt * 16 + 4 * g);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        s[kt][i] = s[kt][i] * p.scale + madd[i];
        mx = fmaxf(mx, s[kt][i]);
      }
    }
  }
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int kt = 0; kt < QA_BM / 16; ++kt) {
    if (kt < nkt) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float e = __expf(s[kt][i] - mx);
        s[kt][i] = e;
        sum += e;
      }
    }
  }
  sum += __shfl_xor(sum, 16, 64);
  sum += __shfl_xor(sum, 32, 64);
  const float inv = 1.f / sum;
  f32x4 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int tr_row = (lane & 15) >> 2, tr_col = (lane & 3) * 4;
#pragma unroll
  for (int c = 0; c < QA_BM / 32; ++c) {
    if (c < Lp / 32) {
      const f32x4 pa = s[2 * c], pb = s[2 * c + 1];
      const u32x4 pw = u32x4{pack_bf16x2(pa[0] * inv, pa[1] * inv), pack_bf16x2(pa[2] * inv, pa[3] * inv),
                             pack_bf16x2(pb[0] * inv, pb[1] * inv), pack_bf16x2(pb[2] * inv, pb[3] * inv)};
      const bf16x8 pfrag = *reinterpret_cast<const bf16x8*>(&pw);
      const int r_lo = 32 * c + 4 * g + tr_row, r_hi = r_lo + 16;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(Vs + r_lo * ATT_VST + dt * 16 + tr_col));
        const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(Vs + r_hi * ATT_VST + dt * 16 + tr_col));
        const short vv8[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        const bf16x8 va = *reinterpret_cast<const bf16x8*>(vv8);
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pfrag, o[dt], 0, 0, 0);
      }
    }
  }
  const int q = q0 + lq;
  if (q < L) {
    bf16_t* out = p.out + (row0 + q) * p.ldo + h * ATT_D + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
      *reinterpret_cast<u32x2*>(out + dt * 16) = u32x2{pack_bf16x2(o[dt][0], o[dt][1]), pack_bf16x2(o[dt][2], o[dt][3])};
  }
}

// --------------------------------------------------------------------------- ViT tokens
// out[b][0] = cls + pos[0]; out[b][1+i] = patches[b*np + i] + pos[1+i]   (bf16, D % 8 == 0)
__global__ __launch_bounds__(256) void vit_tokens_kernel(const HzVitTokensParams p) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;  // 8-element chunk index
  const int nch = p.D >> 3;
  const int T = p.np + 1;
  if (i >= (long)p.B * T * nch) return;
  const int ch = i % nch;
  const long rt = i / nch;
  const int t = rt % T;
  const int b = rt / T;
  float a[8], q[8];
  if (t == 0) unpack8(*reinterpret_cast<const u32x4*>(p.cls + ch * 8), a);
  else unpack8(*reinterpret_cast<const u32x4*>(p.patches + ((long)b * p.np + t - 1) * p.D + ch * 8), a);
  unpack8(*reinterpret_cast<const u32x4*>(p.pos + (long)t * p.D + ch * 8), q);
#pragma unroll
  for (int e = 0; e < 8; ++e) a[e] += q[e];
  *reinterpret_cast<u32x4*>(p.out + rt * p.D + ch * 8) = pack8(a);
}

}  // namespace

// --------------------------------------------------------------------------- row softmax
// One wave per row; the row is read twice (max/sum pass, normalise pass) — rows are classifier
// logits or attention-score rows of <= a few thousand elements, L2-resident after the first pass.
__global__ __launch_bounds__(256) void softmax_kernel(const HzSoftmaxParams p) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= p.rows) return;
  auto val = [&](int i) {
    float v = p.x_bf16 ? bf2f(reinterpret_cast<const bf16_t*>(p.x)[(long)row * p.ldx + i])
                       : reinterpret_cast<const float*>(p.x)[(long)row * p.ldx + i];
    v *= p.scale;
    return p.mask ? v + p.mask[i] : v;
  };
  float m = -INFINITY;
  for (int i = lane; i < p.D; i += 64) m = fmaxf(m, val(i));
  m = warp_max(m);
  float s = 0.f;
  for (int i = lane; i < p.D; i += 64) s += __expf(val(i) - m);
  const float inv = 1.f / warp_sum(s);
  float* o = p.out + (long)row * p.ldo;
  for (int i = lane; i < p.D; i += 64) o[i] = __expf(val(i) - m) * inv;
}

extern "C" int hz_softmax_launch(const HzSoftmaxParams* pp, hipStream_t st) {
  const HzSoftmaxParams& p = *pp;
  if (p.D < 1 || p.rows < 1) return -1;
  hipLaunchKernelGGL(softmax_kernel, dim3((p.rows + 3) / 4), dim3(256), 0, st, p);
  return (int)hipGetLastError();
}

extern "C" int hz_layernorm_launch(const HzLayerNormParams* pp, hipStream_t st) {
  const HzLayerNormParams& p = *pp;
  if (p.D % 8 || p.D > 2048) return -1;
  // (a half-wave-per-row variant, 3 chunks per lane at D = 768 and 8 rows per workgroup, measured
  // equal end to end on BERT / ViT: profiles/r2_transformers/layernorm_halfwave_ab)
  // rows per wave: HIPZAP_LN_RPW = 1 (default), 2 or 4. Measured (profiles/r5_tx/ln_ab.jsonl):
  // BERT bs16 16.70k / 16.45k / 15.34k seq/s, ViT fp8 bs64 16.1k / 16.0k / 15.5k img/s -- with the
  // kernel sized to D, one row per wave already keeps 7 waves per SIMD resident
  static const int rpw_env = getenv("HIPZAP_LN_RPW") ? atoi(getenv("HIPZAP_LN_RPW")) : 1;
  const int rpw = rpw_env == 2 || rpw_env == 4 ? rpw_env : 1;
  const dim3 grid((p.rows + 4 * rpw - 1) / (4 * rpw));
  const int nc = (p.D / 8 + 63) / 64;
#define HZ_LN(NC)                                                                           \
  if (rpw == 4) hipLaunchKernelGGL((layernorm_kernel<NC, 4>), grid, dim3(256), 0, st, p);   \
  else if (rpw == 2) hipLaunchKernelGGL((layernorm_kernel<NC, 2>), grid, dim3(256), 0, st, p); \
  else hipLaunchKernelGGL((layernorm_kernel<NC, 1>), grid, dim3(256), 0, st, p);
  switch (nc) {
    case 1: HZ_LN(1) break;
    case 2: HZ_LN(2) break;
    case 3: HZ_LN(3) break;
    default: HZ_LN(4) break;
  }
#undef HZ_LN
  return (int)hipGetLastError();
}

extern "C" int hz_embed_ln_launch(const HzEmbedParams* pp, hipStream_t st) {
  const HzEmbedParams& p = *pp;
  if (p.D % 8 || p.D > 2048) return -1;
  if (p.vocab < 1 || (p.types && p.ntypes < 1)) return -1;  // the id clamps need non-empty tables
  hipLaunchKernelGGL(embed_ln_kernel, dim3((p.rows + 3) / 4), dim3(256), 0, st, p);
  return (int)hipGetLastError();
}

extern "C" int hz_attention_launch(const HzAttentionParams* pp, hipStream_t st) {
  const HzAttentionParams& p = *pp;
  if (p.head_dim != ATT_D || p.L > ATT_LMAX || p.L < 1) return -1;
  if (p.out8 && (!p.os8 || p.ldo % 32)) return -1;
  if (p.ldqkv % 8 || p.k_off % 8 || p.v_off % 8 || p.ldo % 4) return -1;  // 16-B staging, 8-B stores
  const int Lp = (p.L + 31) & ~31;
  const size_t lds = (size_t)Lp * (ATT_KST + ATT_VST) * sizeof(bf16_t) + (size_t)Lp * sizeof(float);
  // 8 waves (128 queries) per workgroup for long sequences: K/V staged half as often
  static const int nw8_minl = getenv("HIPZAP_ATT_NW8_MINL") ? atoi(getenv("HIPZAP_ATT_NW8_MINL")) : HZ_ATT_NW8_MINL;
  // HIPZAP_ATT_NW16=1: 16 waves (256 queries) for L > 128, one workgroup per (batch, head) staging
  // K/V once instead of once per 128-query block. Same-box A/B on ViT (L = 197): bs64 fp8 +0.4 %,
  // bs8 -2 % (profiles/r2_att16) -> off by default
  static const bool nw16 = getenv("HIPZAP_ATT_NW16") && atoi(getenv("HIPZAP_ATT_NW16")) != 0;
  if (nw16 && p.L > 128) hipLaunchKernelGGL(attention_kernel<16>, dim3(p.B * p.heads, 1), dim3(1024), lds, st, p);
  else if (p.L > nw8_minl) hipLaunchKernelGGL(attention_kernel<8>, dim3(p.B * p.heads, (p.L + 127) / 128), dim3(512), lds, st, p);
  else hipLaunchKernelGGL(attention_kernel<4>, dim3(p.B * p.heads, (p.L + 63) / 64), dim3(256), lds, st, p);
  return (int)hipGetLastError();
}

extern "C" int hz_qkvatt_launch(const HzQkvAttParams* pp, hipStream_t st) {
  const HzQkvAttParams& p = *pp;
  if (!p.x || !p.w || !p.bias || !p.out || p.B < 1 || p.heads < 1) return -1;
  if (p.L < 1 || p.L > QA_BM || p.D != p.heads * ATT_D || p.ksteps * 32 != p.D || p.ksteps % 2) return -1;
  if (p.ldx % 8 || p.ldx < p.D || p.ldo % 4 || p.ldo < p.D) return -1;
  // stages: HIPZAP_QKVATT_NS = 2 (default: 80 KiB of LDS, two workgroups per CU) or 3
  static const int ns = getenv("HIPZAP_QKVATT_NS") && atoi(getenv("HIPZAP_QKVATT_NS")) == 3 ? 3 : 2;
  if (ns == 3) hipLaunchKernelGGL(qkvatt_kernel<3>, dim3(p.B * p.heads), dim3(512), 0, st, p);
  else hipLaunchKernelGGL(qkvatt_kernel<2>, dim3(p.B * p.heads), dim3(512), 0, st, p);
  return (int)hipGetLastError();
}

extern "C" int hz_vit_tokens_launch(const HzVitTokensParams* pp, hipStream_t st) {
  const HzVitTokensParams& p = *pp;
  if (p.D % 8) return -1;
  const long total = (long)p.B * (p.np + 1) * (p.D / 8);
  hipLaunchKernelGGL(vit_tokens_kernel, dim3((total + 255) / 256), dim3(256), 0, st, p);
  return (int)hipGetLastError();
}

// Load this translation unit's device code without a launch (see hz_conv_code_warm in conv.hip).
__global__ void hz_transformer_code_warm_kernel() {}
extern "C" int hz_transformer_code_warm(void) {
  hipFuncAttributes a;
  return (int)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&hz_transformer_code_warm_kernel));
}
