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
__global__ __launch_bounds__(256) void lstm_cell_kernel(const HzLstmParams p) {
  extern __shared__ __attribute__((aligned(16))) float vin[];  // [ldk] = [x ; h_prev ; 0-pad]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int t = *p.step;
  const int par = t & 1;
  const float* h_prev = p.h_state + par * p.H;
  // ---- stage the input vector in LDS (fp32) ----
  for (int i = tid; i < p.ldk; i += blockDim.x) {
    float v = 0.f;
    if (i < p.In) {
      if (p.emb) {
        const int tok = p.tok_seq[t];
        v = bf2f(p.emb[(long)tok * p.lde + i]);
      } else {
        v = p.x_state[(par ^ 1) * p.In + i];  // previous layer's output of THIS step
      }
    } else if (i < p.In + p.H) {
      v = h_prev[i - p.In];
    }
    vin[i] = v;
  }
  __syncthreads();
  const int j = blockIdx.x * 4 + wave;  // hidden unit of this wave
  if (j >= p.H) return;
  const bf16_t* w = p.w + (long)(4 * j) * p.ldk;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  const int nchunk = p.ldk / (64 * CHUNK);
  for (int c = 0; c < nchunk; ++c) {
    const int k = (c * 64 + lane) * CHUNK;
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(vin + k);
    const f32x4 v1 = *reinterpret_cast<const f32x4*>(vin + k + 4);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float f[8];
      unpack8(*reinterpret_cast<const u32x4*>(w + (long)q * p.ldk + k), f);
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

// --------------------------------------------------------------------------- decoder GEMV
__global__ __launch_bounds__(256) void decoder_kernel(const HzDecoderParams p) {
  extern __shared__ __attribute__((aligned(16))) float hv[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int par = (*p.step) & 1;
  const float* h = p.h_state + (par ^ 1) * p.H;  // last layer's output of this step
  for (int i = tid; i < p.ldk; i += blockDim.x) hv[i] = i < p.H ? h[i] : 0.f;
  __syncthreads();
  const int nchunk = p.ldk / (64 * CHUNK);
  const int nquads = (p.V + 3) >> 2;
  for (int qd = blockIdx.x * 4 + wave; qd < nquads; qd += gridDim.x * 4) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < nchunk; ++c) {
      const int k = (c * 64 + lane) * CHUNK;
      const f32x4 v0 = *reinterpret_cast<const f32x4*>(hv + k);
      const f32x4 v1 = *reinterpret_cast<const f32x4*>(hv + k + 4);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = min(qd * 4 + q, p.V - 1);
        float f[8];
        unpack8(*reinterpret_cast<const u32x4*>(p.w + (long)r * p.ldk + k), f);
        acc[q] += f[0] * v0[0] + f[1] * v0[1] + f[2] * v0[2] + f[3] * v0[3] + f[4] * v1[0] + f[5] * v1[1] +
                  f[6] * v1[2] + f[7] * v1[3];
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = warp_sum(acc[q]);
    if (lane < 4) {
      const int r = qd * 4 + lane;
      const float a = lane == 0 ? acc[0] : lane == 1 ? acc[1] : lane == 2 ? acc[2] : acc[3];
      if (r < p.V) p.logits[r] = a + (p.bias ? p.bias[r] : 0.f);
    }
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

constexpr int TOPK = 10;

__global__ __launch_bounds__(1024) void sampler_kernel(const HzSamplerParams p) {
  __shared__ float s_val[32];
  __shared__ int s_idx[32];
  __shared__ int s_draw[TOPK];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  const int t = *p.step;
  const bool forced = (t + 1) < *p.n_forced;
  const unsigned long long seed = *p.seed;
  if (!forced) {
    // local top-K of perturbed logits (sorted descending, insertion)
    float v[TOPK];
    int id[TOPK];
#pragma unroll
    for (int q = 0; q < TOPK; ++q) {
      v[q] = -INFINITY;
      id[q] = -1;
    }
    for (int j = tid; j < p.V; j += blockDim.x) {
      const float key = p.logits[j] + gumbel(seed, t, j);
      if (key > v[TOPK - 1]) {
        float cv = key;
        int ci = j;
#pragma unroll
        for (int q = 0; q < TOPK; ++q) {
          if (cv > v[q]) {
            const float tv = v[q];
            const int ti = id[q];
            v[q] = cv;
            id[q] = ci;
            cv = tv;
            ci = ti;
          }
        }
      }
    }
    // K rounds of block-wide argmax over the per-thread heads
    int head = 0;
    for (int r = 0; r < TOPK; ++r) {
      float hv = -INFINITY;
      int hi = -1;
#pragma unroll
      for (int q = 0; q < TOPK; ++q)
        if (q == head) {
          hv = v[q];
          hi = id[q];
        }
      float bv = hv;
      int bt = tid;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int ot = __shfl_xor(bt, o, 64);
        if (ov > bv || (ov == bv && ot < bt)) {
          bv = ov;
          bt = ot;
        }
      }
      if (lane == 0) {
        s_val[wave] = bv;
        s_idx[wave] = bt;
      }
      __syncthreads();
      if (tid == 0) {
        float best = s_val[0];
        int bth = s_idx[0];
        for (int w = 1; w < nw; ++w)
          if (s_val[w] > best || (s_val[w] == best && s_idx[w] < bth)) {
            best = s_val[w];
            bth = s_idx[w];
          }
        s_idx[31] = bth;
      }
      __syncthreads();
      const int winner = s_idx[31];
      if (tid == winner) {
        s_draw[r] = hi;
        ++head;
      }
      __syncthreads();
    }
    if (tid == 0) {
      int tok = s_draw[0];
      for (int r = 0; r < TOPK && r < p.V; ++r) {
        const int d = s_draw[r];
        bool ex = d <= 0;
        for (int e = 0; e < p.n_exclude; ++e) ex |= (d == p.exclude[e]);
        if (!ex) {
          tok = d;
          break;
        }
      }
      p.tok_seq[t + 1] = tok;
      if (p.draws) {
        for (int r = 0; r < TOPK; ++r) p.draws[(long)t * TOPK + r] = s_draw[r];
      }
    }
  }
  __syncthreads();
  if (tid == 0) *p.step = t + 1;
}

}  // namespace

extern "C" int hz_lstm_cell_launch(const HzLstmParams* pp, hipStream_t st) {
  const HzLstmParams& p = *pp;
  if (p.ldk % 512 || p.ldk < p.In + p.H) return -1;
  hipLaunchKernelGGL(lstm_cell_kernel, dim3((p.H + 3) / 4), dim3(256), p.ldk * sizeof(float), st, p);
  return (int)hipGetLastError();
}

extern "C" int hz_decoder_launch(const HzDecoderParams* pp, hipStream_t st) {
  const HzDecoderParams& p = *pp;
  if (p.ldk % 512 || p.ldk < p.H) return -1;
  const int quads = (p.V + 3) / 4;
  const int blocks = min(2048, (quads + 3) / 4);
  hipLaunchKernelGGL(decoder_kernel, dim3(blocks), dim3(256), p.ldk * sizeof(float), st, p);
  return (int)hipGetLastError();
}

extern "C" int hz_sampler_launch(const HzSamplerParams* pp, hipStream_t st) {
  const HzSamplerParams& p = *pp;
  if (p.n_exclude > 8) return -1;
  hipLaunchKernelGGL(sampler_kernel, dim3(1), dim3(1024), 0, st, p);
  return (int)hipGetLastError();
}
