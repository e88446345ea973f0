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
#include "common.h"
#include "hipzap.h"

namespace {

// --------------------------------------------------------------------------- LayerNorm
// rows x D (D % 8 == 0, D <= 64*8*4): each lane holds up to 4 16-B chunks of its row.
__global__ __launch_bounds__(256) void layernorm_kernel(const HzLayerNormParams p) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= p.rows) return;
  const bf16_t* x = p.x + (long)row * p.ldx;
  const bf16_t* r = p.res ? p.res + (long)row * p.ldr : nullptr;
  const int nch = p.D >> 3;
  float v[4][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int ch = c * 64 + lane;
    if (ch < nch) {
      unpack8(*reinterpret_cast<const u32x4*>(x + ch * 8), v[c]);
      if (r) {
        float rr[8];
        unpack8(*reinterpret_cast<const u32x4*>(r + ch * 8), rr);
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
  float amax = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int ch = c * 64 + lane;
    if (ch < nch) {
      const f32x4 g0 = *reinterpret_cast<const f32x4*>(p.gamma + ch * 8);
      const f32x4 g1 = *reinterpret_cast<const f32x4*>(p.gamma + ch * 8 + 4);
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(p.beta + ch * 8);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(p.beta + ch * 8 + 4);
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
  if (!p.out8) return;
  // fused fp8 quantisation (same rule as fp8.hip quant_rows: s = amax / 448, e4m3fn)
  amax = warp_max(amax);
  const float scale = fmaxf(amax, 1e-12f) / 448.f, inv = 1.f / scale;
  unsigned char* o8 = p.out8 + (long)row * p.D;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int ch = c * 64 + lane;
    if (ch < nch) {
      float q[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) q[e] = fminf(fmaxf(v[c][e] * inv, -448.f), 448.f);
      *reinterpret_cast<u32x2*>(o8 + ch * 8) = u32x2{pack4_fp8(q[0], q[1], q[2], q[3]), pack4_fp8(q[4], q[5], q[6], q[7])};
    }
  }
  if (lane == 0) p.scale8[row] = scale;
}

// --------------------------------------------------------------------------- BERT embeddings
__global__ __launch_bounds__(256) void embed_ln_kernel(const HzEmbedParams p) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= p.rows) return;
  const int tok = p.ids[row];
  const int pos = row % p.L;
  const int tt = p.types ? p.types[row] : 0;
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
constexpr int ATT_D = 64;
constexpr int ATT_LMAX = 256;

constexpr int ATT_KST = ATT_D + 8;  // padded K row stride: the 16 rows of a fragment read hit distinct banks

__global__ __launch_bounds__(256) void attention_kernel(const HzAttentionParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int Lp = (p.L + 31) & ~31;  // keys padded to the 32-wide MFMA K step
  const int VST = Lp + 8;           // padded V^T / P row strides (bank-conflict-free fragment reads)
  bf16_t* Ks = reinterpret_cast<bf16_t*>(smem);          // [Lp][ATT_KST]
  bf16_t* Vt = Ks + Lp * ATT_KST;                       // [64][VST]
  bf16_t* Ps = Vt + ATT_D * VST;                        // [4 waves][16][VST]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bh = blockIdx.x;
  const int b = bh / p.heads, h = bh - b * p.heads;
  const long row0 = (long)b * p.L;
  const bf16_t* Q = p.qkv + row0 * p.ldqkv + h * ATT_D;
  const bf16_t* K = Q + p.k_off;
  const bf16_t* V = Q + p.v_off;
  // ---- stage K (row-major) and V^T in LDS: every load issued first — one round trip, not one
  // per iteration. Padding keys (L <= key < Lp) re-read row L-1: their scores are masked to -inf
  // and their probabilities are exactly 0, so any finite row is correct (no branch, no zero
  // buffer hotspot) ----
  constexpr int SIT = ATT_LMAX * 8 / 256;
  u32x4 kv[SIT], vv[SIT];
#pragma unroll
  for (int it = 0; it < SIT; ++it) {
    if (it * 32 >= Lp) break;  // block-uniform
    const int i = tid + it * 256;
    const int key = min(i >> 3, p.L - 1), c = (i & 7) * 8;
    kv[it] = *reinterpret_cast<const u32x4*>(K + (long)key * p.ldqkv + c);
    vv[it] = *reinterpret_cast<const u32x4*>(V + (long)key * p.ldqkv + c);
  }
#pragma unroll
  for (int it = 0; it < SIT; ++it) {
    if (it * 32 >= Lp) break;
    const int i = tid + it * 256;
    const int key = i >> 3, c = (i & 7) * 8;
    {
      *reinterpret_cast<u32x4*>(Ks + key * ATT_KST + c) = kv[it];
      const bf16_t* ve = reinterpret_cast<const bf16_t*>(&vv[it]);
#pragma unroll
      for (int e = 0; e < 8; ++e) Vt[(c + e) * VST + key] = ve[e];
    }
  }
  __syncthreads();
  const int q0 = blockIdx.y * 64 + wave * 16;
  if (q0 >= p.L) return;  // no barrier follows
  const int lrow = lane & 15, lk = (lane >> 4) * 8;
  // ---- Q fragments (A operand: rows = queries, k = head dim) ----
  bf16x8 qa[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const int q = q0 + lrow;
    qa[ks] = *reinterpret_cast<const bf16x8*>(Q + (long)min(q, p.L - 1) * p.ldqkv + ks * 32 + lk);  // rows >= L discarded
  }
  // ---- S = Q K^T: lane holds S[q0 + 4*(lane>>4) + i][kt*16 + lrow] ----
  const int nkt = Lp / 16;
  f32x4 s[ATT_LMAX / 16];
#pragma unroll
  for (int kt = 0; kt < ATT_LMAX / 16; ++kt) {
    s[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (kt < nkt) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 kb = *reinterpret_cast<const bf16x8*>(Ks + (kt * 16 + lrow) * ATT_KST + ks * 32 + lk);
        s[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa[ks], kb, s[kt], 0, 0, 0);
      }
    }
  }
  // ---- scale + mask + row softmax (row values live in the 16 lanes of one lane>>4 group) ----
  float mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
  for (int kt = 0; kt < ATT_LMAX / 16; ++kt) {
    if (kt < nkt) {
      const int key = kt * 16 + lrow;
      const float madd = key < p.L ? (p.mask ? p.mask[(long)b * p.L + key] : 0.f) : -INFINITY;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        s[kt][i] = s[kt][i] * p.scale + madd;
        mx[i] = fmaxf(mx[i], s[kt][i]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) mx[i] = fmaxf(mx[i], __shfl_xor(mx[i], o, 64));
  float sum[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kt = 0; kt < ATT_LMAX / 16; ++kt) {
    if (kt < nkt) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float e = __expf(s[kt][i] - mx[i]);
        s[kt][i] = e;
        sum[i] += e;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) sum[i] += __shfl_xor(sum[i], o, 64);
  bf16_t* P = Ps + wave * 16 * VST;
#pragma unroll
  for (int kt = 0; kt < ATT_LMAX / 16; ++kt) {
    if (kt < nkt) {
#pragma unroll
      for (int i = 0; i < 4; ++i) P[(4 * (lane >> 4) + i) * VST + kt * 16 + lrow] = f2bf(s[kt][i] / sum[i]);
    }
  }
  // P is private to this wave: make the writes visible to the wave's own cross-lane reads
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
  // ---- O = P V: A = P (rows q, k = keys), B = V (k = keys, cols = d) via V^T rows ----
  f32x4 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int ks = 0; ks < Lp / 32; ++ks) {
    const bf16x8 pa = *reinterpret_cast<const bf16x8*>(P + lrow * VST + ks * 32 + lk);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const bf16x8 vb = *reinterpret_cast<const bf16x8*>(Vt + (dt * 16 + lrow) * VST + ks * 32 + lk);
      o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, vb, o[dt], 0, 0, 0);
    }
  }
  // lane holds O[q0 + 4*(lane>>4) + i][dt*16 + lrow]
  if (p.out8) {  // MX8 output: head columns [0,32) = dt 0,1 and [32,64) = dt 2,3 are two E8M0 blocks
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = q0 + 4 * (lane >> 4) + i;
#pragma unroll
      for (int hb = 0; hb < 2; ++hb) {
        float amax = fmaxf(fabsf(o[2 * hb][i]), fabsf(o[2 * hb + 1][i]));
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) amax = fmaxf(amax, __shfl_xor(amax, off, 64));
        const int ex = mx_exp(amax);
        if (q < p.L) {
          unsigned char* o8 = p.out8 + (row0 + q) * p.ldo + h * ATT_D + hb * 32;
#pragma unroll
          for (int d = 0; d < 2; ++d) {
            const float x = fminf(fmaxf(ldexpf(o[2 * hb + d][i], -ex), -448.f), 448.f);
            o8[d * 16 + lrow] = (unsigned char)(__builtin_amdgcn_cvt_pk_fp8_f32(x, 0.f, 0, false) & 0xff);
          }
          if (lrow == 0) p.os8[(row0 + q) * (p.ldo >> 5) + h * 2 + hb] = (unsigned char)(ex + 127);
        }
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = q0 + 4 * (lane >> 4) + i;
    if (q >= p.L) continue;
    bf16_t* out = p.out + (row0 + q) * p.ldo + h * ATT_D;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) out[dt * 16 + lrow] = f2bf(o[dt][i]);
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
  hipLaunchKernelGGL(layernorm_kernel, dim3((p.rows + 3) / 4), dim3(256), 0, st, p);
  return (int)hipGetLastError();
}

extern "C" int hz_embed_ln_launch(const HzEmbedParams* pp, hipStream_t st) {
  const HzEmbedParams& p = *pp;
  if (p.D % 8 || p.D > 2048) return -1;
  hipLaunchKernelGGL(embed_ln_kernel, dim3((p.rows + 3) / 4), dim3(256), 0, st, p);
  return (int)hipGetLastError();
}

extern "C" int hz_attention_launch(const HzAttentionParams* pp, hipStream_t st) {
  const HzAttentionParams& p = *pp;
  if (p.head_dim != ATT_D || p.L > ATT_LMAX || p.L < 1) return -1;
  if (p.out8 && (!p.os8 || p.ldo % 32)) return -1;
  const int Lp = (p.L + 31) & ~31;
  const size_t lds = (size_t)(Lp * ATT_KST + ATT_D * (Lp + 8) + 4 * 16 * (Lp + 8)) * sizeof(bf16_t);
  hipLaunchKernelGGL(attention_kernel, dim3(p.B * p.heads, (p.L + 63) / 64), dim3(256), lds, st, p);
  return (int)hipGetLastError();
}

extern "C" int hz_vit_tokens_launch(const HzVitTokensParams* pp, hipStream_t st) {
  const HzVitTokensParams& p = *pp;
  if (p.D % 8) return -1;
  const long total = (long)p.B * (p.np + 1) * (p.D / 8);
  hipLaunchKernelGGL(vit_tokens_kernel, dim3((total + 255) / 256), dim3(256), 0, st, p);
  return (int)hipGetLastError();
}
