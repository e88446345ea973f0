// AWD-LSTM decode on device (the reference's model, /root/reference/main.py:40-103 hot loop;
// SURVEY.md §2d K1-K7 / §2e N12-N13). One decode step = 3 fused LSTM-cell kernels + a
// decoder GEMV + an on-device sampler; all state lives on the GPU so a whole request
// (prompt feed + 200 sampled tokens) is a chain of hipGraph replays with ONE host sync.
//
// * lstm_cell: gates = [W_ih | W_hh] . [x ; h] + (b_ih + b_hh) as ONE GEMV over a packed,
//   gate-interleaved matrix (row 4j+q = gate q of hidden unit j), so the wave that computes
//   unit j's four gate rows applies the cell update itself (no second pass, no global sync).
//   Layer 0 gathers its input straight from the (tied) embedding table by the device-side
//   token id (K1 fused into the layer-0 load). h/c are fp32, ping-ponged by step parity.
// * decoder: logits = E . h + b over the tied embedding (bf16, K padded to 1024), grid-stride
//   over row quads, 16-B weight loads, fp32 accumulate — an HBM/MALL-streaming GEMV.
// * sampler: Gumbel-top-10 with a counter-based Philox4x32-10 stream (seed, step, index):
//   the 10 largest perturbed logits in descending order ARE 10 draws without replacement
//   with P ∝ exp(logit) (Plackett-Luce), i.e. torch.multinomial(exp(logits), 10) of
//   main.py:61 in distribution, without exp() overflow. The main.py:63-68 selection rule
//   (first draw not 0 and not excluded, else the first draw) runs on device too.
#include "common.h"
#include "hipzap.h"

namespace {

constexpr int CHUNK = 8;  // bf16 per 16-B lane load

// --------------------------------------------------------------------------- LSTM cell
// NCH = ldk / 512 is a template parameter so every weight load of a wave (4 gate rows x NCH
// 16-B chunks) is issued before the first use — with a runtime chunk loop hipcc waited
// vmcnt(0) per chunk (one L2/HBM round trip each). The input staging likewise issues all of a
// thread's loads first (address selects instead of branches around loads).
template <int NCH>
__global__ __launch_bounds__(256) void lstm_cell_kernel(const HzLstmParams p) {
  extern __shared__ __attribute__((aligned(16))) float vin[];  // [ldk] = [x ; h_prev ; 0-pad]
  constexpr int PER = NCH * 512 / 256;  // staged elements per thread
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int t = *p.step;
  const int par = t & 1;
  const float* h_prev = p.h_state + par * p.H;
  const int tok = p.emb ? p.tok_seq[t] : 0;
  const bf16_t* erow = p.emb ? p.emb + (long)tok * p.lde : nullptr;
  const float* xprev = p.x_state + (par ^ 1) * p.In;  // previous layer's output of THIS step
  // weights do not depend on the input vector: issue them first so their latency overlaps
  // the staging loads (inactive tail waves read row H-1 and write nothing)
  const int j = blockIdx.x * 4 + wave;  // hidden unit of this wave
  const bf16_t* w = p.w + (long)(4 * min(j, p.H - 1)) * p.ldk + lane * 8;
  u32x4 wv[4][NCH];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int c = 0; c < NCH; ++c) wv[q][c] = *reinterpret_cast<const u32x4*>(w + (long)q * p.ldk + c * 512);
  // ---- stage the input vector in LDS (fp32): all loads first, then the selects ----
  float fv[PER];
  unsigned short ev[PER];
#pragma unroll
  for (int r = 0; r < PER; ++r) {
    const int i = tid + r * 256;
    const bool in_x = i < p.In, in_h = !in_x && i < p.In + p.H;
    const float* fsrc = in_h ? h_prev + (i - p.In) : (in_x && !erow ? xprev + i : h_prev);
    fv[r] = *fsrc;
    ev[r] = erow ? erow[in_x ? i : 0] : 0;
  }
#pragma unroll
  for (int r = 0; r < PER; ++r) {
    const int i = tid + r * 256;
    const bool in_x = i < p.In, in_h = !in_x && i < p.In + p.H;
    vin[i] = in_h ? fv[r] : in_x ? (erow ? bf2f(ev[r]) : fv[r]) : 0.f;
  }
  __syncthreads();
  if (j >= p.H) return;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int k = c * 512 + lane * 8;
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(vin + k);
    const f32x4 v1 = *reinterpret_cast<const f32x4*>(vin + k + 4);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float f[8];
      unpack8(wv[q][c], f);
      acc[q] += f[0] * v0[0] + f[1] * v0[1] + f[2] * v0[2] + f[3] * v0[3] + f[4] * v1[0] + f[5] * v1[1] +
                f[6] * v1[2] + f[7] * v1[3];
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = warp_sum(acc[q]);
  if (lane == 0) {
    const float gi = acc[0] + p.bias[4 * j + 0];
    const float gf = acc[1] + p.bias[4 * j + 1];
    const float gg = acc[2] + p.bias[4 * j + 2];
    const float go = acc[3] + p.bias[4 * j + 3];
    const float si = 1.f / (1.f + __expf(-gi));
    const float sf = 1.f / (1.f + __expf(-gf));
    const float so = 1.f / (1.f + __expf(-go));
    const float c_new = sf * p.c_state[par * p.H + j] + si * tanhf(gg);
    const float h_new = so * tanhf(c_new);
    p.c_state[(par ^ 1) * p.H + j] = c_new;
    p.h_state[(par ^ 1) * p.H + j] = h_new;
  }
}

// --------------------------------------------------------------------------- Philox4x32-10
__device__ __forceinline__ void philox(unsigned c0, unsigned c1, unsigned c2, unsigned c3, unsigned k0, unsigned k1,
                                       unsigned& o0) {
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
  o0 = c0;
}

__device__ __forceinline__ float gumbel(unsigned long long seed, int t, int j) {
  unsigned r;
  philox((unsigned)j, (unsigned)t, 0x5eedu, 0u, (unsigned)seed, (unsigned)(seed >> 32), r);
  const float u = ((r >> 8) + 0.5f) * (1.0f / 16777216.0f);  // (0, 1)
  return -__logf(-__logf(u));
}

// --------------------------------------------------------------------------- decoder GEMV
// logits = E . h + b over the tied embedding (bf16 [V][ldk]). Each wave takes 8 rows per
// iteration with all 8 x NCH 16-B loads in flight (NCH = ldk/512 is compile-time), then one
// 64-lane reduction per row. With `keys`, the epilogue also writes logit + Gumbel(seed,t,row)
// so the sampler only has to select (the Philox work is spread over the whole chip instead of
// one workgroup).
constexpr int DROWS = 8;
template <int NCH>
__global__ __launch_bounds__(256) void decoder_kernel(const HzDecoderParams p) {
  extern __shared__ __attribute__((aligned(16))) float hv[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int t = *p.step;
  const int par = t & 1;
  const float* h = p.h_state + (par ^ 1) * p.H;  // last layer's output of this step
  for (int i = tid; i < p.ldk; i += blockDim.x) hv[i] = i < p.H ? h[i] : 0.f;
  __syncthreads();
  const unsigned long long seed = p.keys ? *p.seed : 0ull;
  const int ngroups = (p.V + DROWS - 1) / DROWS;
  for (int g = blockIdx.x * 4 + wave; g < ngroups; g += gridDim.x * 4) {
    u32x4 wv[DROWS][NCH];
#pragma unroll
    for (int q = 0; q < DROWS; ++q) {
      const int r = min(g * DROWS + q, p.V - 1);
#pragma unroll
      for (int c = 0; c < NCH; ++c)
        wv[q][c] = *reinterpret_cast<const u32x4*>(p.w + (long)r * p.ldk + c * 512 + lane * 8);
    }
    float acc[DROWS];
#pragma unroll
    for (int q = 0; q < DROWS; ++q) acc[q] = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int k = c * 512 + lane * 8;
      const f32x4 v0 = *reinterpret_cast<const f32x4*>(hv + k);
      const f32x4 v1 = *reinterpret_cast<const f32x4*>(hv + k + 4);
#pragma unroll
      for (int q = 0; q < DROWS; ++q) {
        float f[8];
        unpack8(wv[q][c], f);
        acc[q] += f[0] * v0[0] + f[1] * v0[1] + f[2] * v0[2] + f[3] * v0[3] + f[4] * v1[0] + f[5] * v1[1] +
                  f[6] * v1[2] + f[7] * v1[3];
      }
    }
#pragma unroll
    for (int q = 0; q < DROWS; ++q) acc[q] = warp_sum(acc[q]);
    if (lane < DROWS) {
      const int r = g * DROWS + lane;
      float a = acc[0];
#pragma unroll
      for (int q = 1; q < DROWS; ++q) a = lane == q ? acc[q] : a;
      if (r < p.V) {
        const float lg = a + (p.bias ? p.bias[r] : 0.f);
        p.logits[r] = lg;
        if (p.keys) p.keys[r] = lg + gumbel(seed, t, r);
      }
    }
  }
}

constexpr int TOPK = 10;

// 64-lane argmax of (value, index) with ties to the lower index; every lane gets the result
__device__ __forceinline__ void wave_argmax(float& v, int& i) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(v, o, 64);
    const int oi = __shfl_xor(i, o, 64);
    if (ov > v || (ov == v && oi < i)) {
      v = ov;
      i = oi;
    }
  }
}

// Two-stage Gumbel top-10 (10 draws without replacement ∝ exp(logit)):
//   sampler_partial: ceil(V/1024) blocks; each thread loads its 4 keys unconditionally (one
//     round trip), sorts them, the wave merges its lanes' lists by 10 rounds of shuffle argmax,
//     wave 0 merges the 4 wave lists -> the block's top-10 into the candidate buffer;
//   sampler_final: one wave merges all candidates (loaded 8 at a time) and applies the
//     reference's selection rule (main.py:63-68), writes the token and advances the step.
// The previous single-workgroup version read the V keys through a data-dependent branch per
// element (a dependent L2 round trip each): 110 us per token, ~60 % of the whole decode step.
constexpr int SPB = 1024;  // keys per partial block (256 threads x 4)

__device__ __forceinline__ void cswap(float& va, int& ia, float& vb, int& ib) {  // descending
  if (vb > va || (vb == va && ib < ia)) {
    const float tv = va;
    const int ti = ia;
    va = vb;
    ia = ib;
    vb = tv;
    ib = ti;
  }
}

// 10 rounds of wave argmax over per-lane sorted lists of length L (head = next unpopped entry).
template <int L>
__device__ __forceinline__ void wave_topk(const float (&v)[L], const int (&id)[L], float (&ov)[TOPK],
                                          int (&oi)[TOPK]) {
  int head = 0;
#pragma unroll
  for (int r = 0; r < TOPK; ++r) {
    float hv = -INFINITY;
    int hi = 0x7fffffff;
#pragma unroll
    for (int q = 0; q < L; ++q)
      if (q == head) {
        hv = v[q];
        hi = id[q];
      }
    float bv = hv;
    int bi = hi;
    wave_argmax(bv, bi);
    if (hv == bv && hi == bi && head < L) ++head;  // indices are unique: one lane pops
    ov[r] = bv;
    oi[r] = bi;
  }
}

__global__ __launch_bounds__(256) void sampler_partial_kernel(const HzSamplerParams p) {
  __shared__ float w_val[4 * TOPK];
  __shared__ int w_idx[4 * TOPK];
  const int t = *p.step;
  if ((t + 1) < *p.n_forced) return;  // prompt step: the next token is given
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const unsigned long long seed = *p.seed;
  float v[4];
  int id[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int j = blockIdx.x * SPB + r * 256 + tid;
    id[r] = j;
    v[r] = p.logits[min(j, p.V - 1)];
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (!p.keyed) v[r] += gumbel(seed, t, id[r]);
    if (id[r] >= p.V) v[r] = -INFINITY;
  }
  cswap(v[0], id[0], v[1], id[1]);
  cswap(v[2], id[2], v[3], id[3]);
  cswap(v[0], id[0], v[2], id[2]);
  cswap(v[1], id[1], v[3], id[3]);
  cswap(v[1], id[1], v[2], id[2]);
  float wv[TOPK];
  int wi[TOPK];
  wave_topk<4>(v, id, wv, wi);
  if (lane == 0) {
#pragma unroll
    for (int r = 0; r < TOPK; ++r) {
      w_val[wave * TOPK + r] = wv[r];
      w_idx[wave * TOPK + r] = wi[r];
    }
  }
  __syncthreads();
  if (wave == 0) {
    float cv[1] = {lane < 4 * TOPK ? w_val[lane] : -INFINITY};
    int ci[1] = {lane < 4 * TOPK ? w_idx[lane] : 0x7fffffff};
    float bv[TOPK];
    int bi[TOPK];
    wave_topk<1>(cv, ci, bv, bi);
    if (lane < TOPK) {
      float o = bv[0];
      int oi = bi[0];
#pragma unroll
      for (int r = 1; r < TOPK; ++r) {
        o = lane == r ? bv[r] : o;
        oi = lane == r ? bi[r] : oi;
      }
      p.cand_val[blockIdx.x * TOPK + lane] = o;
      p.cand_idx[blockIdx.x * TOPK + lane] = oi;
    }
  }
}

__global__ __launch_bounds__(64) void sampler_final_kernel(const HzSamplerParams p) {
  const int lane = threadIdx.x;
  const int t = *p.step;
  if ((t + 1) >= *p.n_forced) {
    const int ncand = ((p.V + SPB - 1) / SPB) * TOPK;
    float v[TOPK];
    int id[TOPK];
#pragma unroll
    for (int q = 0; q < TOPK; ++q) {
      v[q] = -INFINITY;
      id[q] = 0x7fffffff;
    }
    for (int c0 = 0; c0 < ncand; c0 += 64 * 8) {
      float cv[8];
      int ci[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {  // 8 candidates in flight per lane
        const int c = min(c0 + u * 64 + lane, ncand - 1);
        cv[u] = p.cand_val[c];
        ci[u] = p.cand_idx[c];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        float x = c0 + u * 64 + lane < ncand ? cv[u] : -INFINITY;
        int xi = ci[u];
#pragma unroll
        for (int q = 0; q < TOPK; ++q) cswap(v[q], id[q], x, xi);  // insertion into the sorted list
      }
    }
    float dv[TOPK];
    int draws[TOPK];
    wave_topk<TOPK>(v, id, dv, draws);
    if (lane == 0) {
      int tok = draws[0];
      for (int r = 0; r < TOPK && r < p.V; ++r) {
        const int d = draws[r];
        bool ex = d <= 0;
        for (int e = 0; e < p.n_exclude; ++e) ex |= (d == p.exclude[e]);
        if (!ex) {
          tok = d;
          break;
        }
      }
      p.tok_seq[t + 1] = tok;
      if (p.draws) {
        for (int r = 0; r < TOPK; ++r) p.draws[(long)t * TOPK + r] = draws[r];
      }
    }
  }
  if (lane == 0) *p.step = t + 1;
}

}  // namespace

extern "C" int hz_lstm_cell_launch(const HzLstmParams* pp, hipStream_t st) {
  const HzLstmParams& p = *pp;
  if (p.ldk % 512 || p.ldk < p.In + p.H) return -1;
  const dim3 grid((p.H + 3) / 4), block(256);
  const size_t lds = p.ldk * sizeof(float);
  switch (p.ldk / 512) {
    case 1: hipLaunchKernelGGL(lstm_cell_kernel<1>, grid, block, lds, st, p); break;
    case 2: hipLaunchKernelGGL(lstm_cell_kernel<2>, grid, block, lds, st, p); break;
    case 3: hipLaunchKernelGGL(lstm_cell_kernel<3>, grid, block, lds, st, p); break;
    case 4: hipLaunchKernelGGL(lstm_cell_kernel<4>, grid, block, lds, st, p); break;
    case 5: hipLaunchKernelGGL(lstm_cell_kernel<5>, grid, block, lds, st, p); break;
    case 6: hipLaunchKernelGGL(lstm_cell_kernel<6>, grid, block, lds, st, p); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

extern "C" int hz_decoder_launch(const HzDecoderParams* pp, hipStream_t st) {
  const HzDecoderParams& p = *pp;
  if (p.ldk % 512 || p.ldk < p.H || (p.keys && !p.seed)) return -1;
  const int groups = (p.V + DROWS - 1) / DROWS;
  const dim3 grid(min(2048, (groups + 3) / 4)), block(256);
  const size_t lds = p.ldk * sizeof(float);
  switch (p.ldk / 512) {
    case 1: hipLaunchKernelGGL(decoder_kernel<1>, grid, block, lds, st, p); break;
    case 2: hipLaunchKernelGGL(decoder_kernel<2>, grid, block, lds, st, p); break;
    case 3: hipLaunchKernelGGL(decoder_kernel<3>, grid, block, lds, st, p); break;
    case 4: hipLaunchKernelGGL(decoder_kernel<4>, grid, block, lds, st, p); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

extern "C" int hz_sampler_launch(const HzSamplerParams* pp, hipStream_t st) {
  const HzSamplerParams& p = *pp;
  if (p.n_exclude > 8 || !p.cand_val || !p.cand_idx || p.V < 1) return -1;
  hipLaunchKernelGGL(sampler_partial_kernel, dim3((p.V + SPB - 1) / SPB), dim3(256), 0, st, p);
  hipLaunchKernelGGL(sampler_final_kernel, dim3(1), dim3(64), 0, st, p);
  return (int)hipGetLastError();
}
