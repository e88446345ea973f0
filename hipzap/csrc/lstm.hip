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
#include <cstdlib>

#include "common.h"
#include "hipzap.h"

HZ_DEBUG_UNIT(lstm)

namespace {

constexpr int CHUNK = 8;  // bf16 per 16-B lane load

// total order of sampler keys: larger value first, ties to the lower row
__device__ __forceinline__ bool better(float av, int ai, float bv, int bi) {
  return av > bv || (av == bv && ai < bi);
}

// 16-B weight load at column k of a row of ld bf16, clamped into the row instead of predicated:
// `k < ld ? load : 0` compiles to an exec-masked branch whose zero write in the other lanes is a
// write-after-write hazard on the destination VGPRs of a load in flight, so the compiler put an
// s_waitcnt vmcnt(0) after the first loads -- the weight stream of every LSTM kernel was issued
// in two serialised halves. Columns past ld re-read the row's last 16 B; every caller multiplies
// them with a vector operand that is zero there.
__device__ __forceinline__ u32x4 ld_row(const bf16_t* row, int k, int ld) {
  return *reinterpret_cast<const u32x4*>(row + min(k, ld - 8));
}

// LDS-only workgroup barrier: unlike __syncthreads() it does not wait for the caller's
// outstanding global loads (the LSTM weight stream stays in flight across it)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int WAVES>
__device__ __forceinline__ void block_reduce_best(float* sv, int* si, float& v, int& i);

// best (value, row) of n entries, reduced by the calling workgroup (WAVES waves); every thread
// gets the result. Slots: 2*WAVES floats / ints of LDS.
template <int WAVES>
__device__ __forceinline__ void block_best(const float* val, const int* idx, int n, float* sv, int* si, float& v,
                                           int& i) {
  v = -INFINITY;
  i = 0x7fffffff;
  for (int j = threadIdx.x; j < n; j += WAVES * 64) {
    const float a = val[j];
    const int b = idx[j];
    if (better(a, b, v, i)) {
      v = a;
      i = b;
    }
  }
  block_reduce_best<WAVES>(sv, si, v, i);
}

// workgroup-wide best of every thread's (v, i); every thread gets it
template <int WAVES>
__device__ __forceinline__ void block_reduce_best(float* sv, int* si, float& v, int& i) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(v, o, 64);
    const int oi = __shfl_xor(i, o, 64);
    if (better(ov, oi, v, i)) {
      v = ov;
      i = oi;
    }
  }
  if (lane == 0) {
    sv[wave] = v;
    si[wave] = i;
  }
  lds_barrier();
  v = sv[0];
  i = si[0];
#pragma unroll
  for (int w = 1; w < WAVES; ++w)
    if (better(sv[w], si[w], v, i)) {
      v = sv[w];
      i = si[w];
    }
}

// The argmax sampler's token (exactness argument at sample_argmax): the best key over the
// ACCEPTABLE rows from the decoder's per-workgroup maxima, or, when no row is acceptable at all
// (V <= 9), the best key overall. Uniform control flow; every thread gets the token.
template <int WAVES>
__device__ __forceinline__ int block_token(const float* bacc_val, const int* bacc_idx, const float* bmax_val,
                                           const int* bmax_idx, int nblk, int V) {
  __shared__ float sv[2][WAVES];
  __shared__ int si[2][WAVES];
  float v;
  int i;
  block_best<WAVES>(bacc_val, bacc_idx, nblk, sv[0], si[0], v, i);
  if (i == 0x7fffffff) block_best<WAVES>(bmax_val, bmax_idx, nblk, sv[1], si[1], v, i);
  return min(max(i, 0), V - 1);
}

// --------------------------------------------------------------------------- LSTM cell
// NCH = ceil(ldk / 512) is a template parameter so every weight load of a wave (4 gate rows x
// its chunks) is issued before the first use. ldk is In + H padded to 64 only (v1 padded to
// 512: 2150 -> 2560 streamed 16 % zeros); lanes past ldk in the last chunk are predicated off.
// KW waves split one unit's K range (v1: one wave per unit, H/4 = 288 workgroups of 4.5 waves per
// CU) so twice as many independent load streams are in flight; the KW partial gate sums meet in
// LDS and the first wave of the unit applies the cell update.
template <int NCH, int KW>
__global__ __launch_bounds__(256) void lstm_cell_kernel(const HzLstmParams p) {
  extern __shared__ __attribute__((aligned(16))) float vin[];  // [NCH*512] = [x ; h_prev ; 0-pad]
  __shared__ float part[4][4];                                  // [wave][gate] partial sums
  constexpr int UPW = 4 / KW;                 // units per workgroup
  constexpr int NC = (NCH + KW - 1) / KW;     // chunks per wave
  constexpr int PER = NCH * 512 / 256;        // staged elements per thread
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int slot = wave / KW, kw = wave - slot * KW;
  const int t = *p.step + p.step_off;
  const int par = t & 1;
  const float* h_prev = p.h_state + par * p.H;
  if (!HZ_DCHECK(p.In + p.H <= p.ldk && p.ldk <= NCH * 512 && p.ldk % 8 == 0)) return;
  const float* xprev = p.x_state + (par ^ 1) * p.In;  // previous layer's output of THIS step
  // weights do not depend on the input vector: issue them first so their latency overlaps
  // the token selection and the staging loads (inactive tail units read row H-1, write nothing)
  // fused sampler: load the previous decoder's acceptable maxima FIRST (vmcnt retires in issue
  // order: a wait for loads issued after the weight stream would wait for the weights too)
  const bool fused = p.emb && p.bacc_val && t >= *p.n_forced;
  constexpr int TPT = 8;  // maxima per thread: nblk <= 2048 (hz_decoder_geometry)
  float tv[TPT];
  int ti[TPT];
  if (fused) {
#pragma unroll
    for (int r = 0; r < TPT; ++r) {
      const int e = tid + r * 256;
      const int ec = min(e, p.nblk - 1);  // unconditional load (see ld_row); duplicates do not change the max
      tv[r] = p.bacc_val[ec];
      ti[r] = p.bacc_idx[ec];
    }
  }
  const int j = blockIdx.x * UPW + slot;  // hidden unit of this wave
  const bf16_t* w = p.w + (long)(4 * min(j, p.H - 1)) * p.ldk;
  u32x4 wv[4][NC];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int c = 0; c < NC; ++c) wv[q][c] = ld_row(w + (long)q * p.ldk, (kw * NC + c) * 512 + lane * 8, p.ldk);
  __builtin_amdgcn_sched_barrier(0);  // the whole weight stream issued before anything waits
  int tok = 0;
  if (fused) {  // this step's token from the last decoder (the argmax sampler's rule)
    __shared__ float sv[4];
    __shared__ int si[4];
    float v = tv[0];
    int i = ti[0];
#pragma unroll
    for (int r = 1; r < TPT; ++r)
      if (better(tv[r], ti[r], v, i)) {
        v = tv[r];
        i = ti[r];
      }
    block_reduce_best<4>(sv, si, v, i);
    if (i == 0x7fffffff) {  // no acceptable row anywhere (V <= 9): the best key overall
      __shared__ float sv2[4];
      __shared__ int si2[4];
      block_best<4>(p.bmax_val, p.bmax_idx, p.nblk, sv2, si2, v, i);
    }
    tok = min(max(i, 0), p.V - 1);
    if (blockIdx.x == 0 && tid == 0) p.tok_seq[t] = tok;
  } else if (p.emb) {
    tok = p.tok_seq[t];
  }
  if (!HZ_DCHECK(tok >= 0)) return;
  const bf16_t* erow = p.emb ? p.emb + (long)tok * p.lde : nullptr;
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
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int k = (kw * NC + c) * 512 + lane * 8;
    if ((kw * NC + c) >= NCH) break;
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
  if (KW > 1) {
    if (lane == 0 && kw > 0)
#pragma unroll
      for (int q = 0; q < 4; ++q) part[wave][q] = acc[q];
    __syncthreads();
    if (kw == 0)
#pragma unroll
      for (int o = 1; o < KW; ++o)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] += part[wave + o][q];
  }
  if (lane == 0 && kw == 0 && j < p.H) {
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

// --------------------------------------------------------------------------- split-mode LSTM
// W_ih . x only: the recurrent half W_hh . h_{t-1} + b was computed by the previous step's
// decoder kernel (hh_rows below), where it streams at the decoder's full HBM rate instead of
// inside these short latency-bound kernels -> each layer kernel streams half the bytes.
// FUSE0: this is the layer-1 kernel and layer 0 is folded into it. Layer 0's input projection is
// a table lookup, xtab[tok] = W_ih^0 . emb[tok] (fp32 [V][4 H0], built once at pack time from the
// fp32 weights: 1.1 GB at the reference dims, cheap in 288 GB), so h0_t needs no GEMV at all:
// every workgroup rebuilds all H0 units from xtab[tok] + pre0 and c0_{t-1} straight into LDS
// (workgroup 0 publishes h0_t / c0_t), and the token selection of the fused sampler runs first.
// 8 waves: 4 units x 2 K-halves per workgroup.
template <int NCH, bool FUSE0>
__global__ __launch_bounds__(512) void lstm_x_kernel(const HzLstmParams p) {
  extern __shared__ __attribute__((aligned(16))) float vin[];  // [NCH*512] input vector, fp32
  __shared__ float part[8][4];
  constexpr int WAVES = 8, KW = 2, UPW = WAVES / KW;
  constexpr int NC = (NCH + KW - 1) / KW;  // 512-chunks per wave
  constexpr int TPT = 4;                    // decoder maxima per thread (nblk <= 2048)
  constexpr int U0 = 3;                     // layer-0 units per thread (H0 <= 1536)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int slot = wave / KW, kw = wave - slot * KW;
  const int j = blockIdx.x * UPW + slot;  // hidden unit of this wave
  const int jc = min(j, p.H - 1);
  // ---- every load that does not need the step counter, before anything waits: the step is a
  // global counter (an L2 miss across XCDs), so step-dependent (parity) operands are loaded for
  // BOTH parities and selected later; the weight stream goes last (vmcnt retires in issue order)
  float tv[TPT];
  int ti[TPT];
  if (FUSE0) {  // decoder maxima (clamped: duplicates do not change the argmax). Unconditional
    // loads: a branch on bacc_val made the compiler zero these registers on the other path,
    // a write-after-write hazard that cost a vmcnt(0) before the weight stream.
    const float* bv = p.bacc_val ? p.bacc_val : p.pre0;
    const int* bi = p.bacc_val ? p.bacc_idx : reinterpret_cast<const int*>(p.pre0);
    const int nb = p.bacc_val ? p.nblk : 1;
#pragma unroll
    for (int r = 0; r < TPT; ++r) {
      const int ec = min(tid + r * 512, nb - 1);
      tv[r] = bv[ec];
      ti[r] = bi[ec];
    }
  }
  f32x4 g0[U0];
  float c0[2][U0];
  float xs[2][NCH];
  if (FUSE0) {
#pragma unroll
    for (int r = 0; r < U0; ++r) {
      const int u = min(tid + r * 512, p.H0 - 1);
      g0[r] = *reinterpret_cast<const f32x4*>(p.pre0 + 4 * u);
      c0[0][r] = p.c0_state[u];
      c0[1][r] = p.c0_state[p.H0 + u];
    }
  } else {  // the previous layer's h of this step, both parity halves
#pragma unroll
    for (int r = 0; r < NCH; ++r) {
      const int i = min(tid + r * 512, p.In - 1);
      xs[0][r] = p.x_state[i];
      xs[1][r] = p.x_state[p.In + i];
    }
  }
  const f32x4 pj = *reinterpret_cast<const f32x4*>(p.pre + 4 * jc);
  const float cj0 = p.c_state[jc], cj1 = p.c_state[p.H + jc];
  const bf16_t* w = p.w + (long)(4 * jc) * p.ldk;
  u32x4 wv[4][NC];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int c = 0; c < NC; ++c) wv[q][c] = ld_row(w + (long)q * p.ldk, (kw * NC + c) * 512 + lane * 8, p.ldk);
  __builtin_amdgcn_sched_barrier(0);  // the whole weight stream issued before anything waits
  const int t = *p.step + p.step_off;
  const int par = t & 1;
  if (!HZ_DCHECK(p.In <= p.ldk && p.ldk <= NCH * 512 && (!FUSE0 || (p.H0 == p.In && p.H0 <= U0 * 512)))) return;
  // ---- the input vector in LDS ----
  if (FUSE0) {
    int tok;
    if (p.bacc_val && t >= *p.n_forced) {  // this step's token from the last decoder's maxima
      __shared__ float sv[WAVES];
      __shared__ int si[WAVES];
      float v = tv[0];
      int i = ti[0];
#pragma unroll
      for (int r = 1; r < TPT; ++r)
        if (better(tv[r], ti[r], v, i)) {
          v = tv[r];
          i = ti[r];
        }
      block_reduce_best<WAVES>(sv, si, v, i);
      if (i == 0x7fffffff) {  // no acceptable row anywhere (V <= 9): the best key overall
        __shared__ float sv2[WAVES];
        __shared__ int si2[WAVES];
        block_best<WAVES>(p.bmax_val, p.bmax_idx, p.nblk, sv2, si2, v, i);
      }
      tok = min(max(i, 0), p.V - 1);
      if (blockIdx.x == 0 && tid == 0) p.tok_seq[t] = tok;
    } else {
      tok = p.tok_seq[t];
    }
    const float* xr = p.xtab + (long)tok * 4 * p.H0;
    f32x4 xg[U0];
#pragma unroll
    for (int r = 0; r < U0; ++r) xg[r] = *reinterpret_cast<const f32x4*>(xr + 4 * min(tid + r * 512, p.H0 - 1));
#pragma unroll
    for (int r = 0; r < U0; ++r) {
      const int u = tid + r * 512;
      if (u < p.H0) {
        const f32x4 g = xg[r] + g0[r];
        const float si = 1.f / (1.f + __expf(-g[0]));
        const float sf = 1.f / (1.f + __expf(-g[1]));
        const float so = 1.f / (1.f + __expf(-g[3]));
        const float c_new = sf * (par ? c0[1][r] : c0[0][r]) + si * tanhf(g[2]);
        const float h_new = so * tanhf(c_new);
        vin[u] = h_new;
        if (blockIdx.x == 0) {
          p.c0_state[(par ^ 1) * p.H0 + u] = c_new;
          p.h0_state[(par ^ 1) * p.H0 + u] = h_new;
        }
      } else if (u < NCH * 512) {
        vin[u] = 0.f;
      }
    }
  } else {  // the previous layer's output of THIS step: parity half par ^ 1
#pragma unroll
    for (int r = 0; r < NCH; ++r) {
      const int i = tid + r * 512;
      vin[i] = i < p.In ? (par ? xs[0][r] : xs[1][r]) : 0.f;
    }
  }
  lds_barrier();  // LDS only: the weight loads stay in flight
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int k = (kw * NC + c) * 512 + lane * 8;
    if ((kw * NC + c) >= NCH) break;
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
  if (lane == 0 && kw > 0)
#pragma unroll
    for (int q = 0; q < 4; ++q) part[wave][q] = acc[q];
  lds_barrier();
  if (lane == 0 && kw == 0 && j < p.H) {
#pragma unroll
    for (int o = 1; o < KW; ++o)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] += part[wave + o][q];
    const float si = 1.f / (1.f + __expf(-(acc[0] + pj[0])));
    const float sf = 1.f / (1.f + __expf(-(acc[1] + pj[1])));
    const float so = 1.f / (1.f + __expf(-(acc[3] + pj[3])));
    const float c_new = sf * (par ? cj1 : cj0) + si * tanhf(acc[2] + pj[2]);
    const float h_new = so * tanhf(c_new);
    p.c_state[(par ^ 1) * p.H + j] = c_new;
    p.h_state[(par ^ 1) * p.H + j] = h_new;
  }
}

// Philox4x32-10 Gumbel noise: common.h (shared with the batched engine, csrc/lmbatch.hip)

// --------------------------------------------------------------------------- decoder GEMV
// logits = E . h + b over the tied embedding (bf16 [V][ldk]). Workgroup b owns the contiguous
// rows [b*rpb, (b+1)*rpb); each wave takes 8 rows per iteration with all 8 x NCH 16-B loads in
// flight (NCH = ldk/512 is compile-time), then one 64-lane reduction per row. With `keys`, the
// epilogue also writes logit + Gumbel(seed,t,row) (the Philox work is spread over the whole chip)
// and the workgroup's largest key (value, row) for the sampler's pruning.
constexpr int DROWS = 8;

constexpr int TOPK = 10;

// Bitonic sort of NC independent (value, row) vectors (one pair per lane each) across the
// wave into descending `better` order (lane 0 = best): 21 compare-exchange steps of one
// shuffle pair per vector; the NC chains interleave so the shuffle latency is hidden.
template <int NC>
__device__ __forceinline__ void wave_sort64(float (&v)[NC], int (&i)[NC]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const bool keep_better = ((lane & k) == 0) == ((lane & j) == 0);
      float ov[NC];
      int oi[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        ov[c] = __shfl_xor(v[c], j, 64);
        oi[c] = __shfl_xor(i[c], j, 64);
      }
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (keep_better == better(ov[c], oi[c], v[c], i[c])) {
          v[c] = ov[c];
          i[c] = oi[c];
        }
    }
  }
}

// Sampler: 10 draws without replacement ∝ exp(logit) = the 10 largest Gumbel keys
// (Plackett-Luce), selected exactly with pruning instead of a scan of all V keys:
//   1. the decoder left each workgroup's max key; every global top-10 key lies in one of the
//      10 workgroups with the largest maxima (a key in any other workgroup has >= 10 larger
//      keys: those 10 maxima), and within them it is among the rpb rows of the workgroup;
//   2. top-10 of the nblk maxima, then top-10 of the 10*rpb keys of the selected workgroups.
// Each top-10 is a tournament over 64-item chunks: the 16 waves bitonic-sort their chunks
// (CPW chunks per pass, all loads issued before the first sort), the 10 best of each chunk go
// to LDS, repeat until one chunk remains. One launch, one workgroup, no atomics. Then the
// reference's selection rule (main.py:63-68) via a ballot.
constexpr int SAMPLER_LDS = 1024;  // candidate slots per LDS buffer
constexpr int SAMPLER_WAVES = 16;  // standalone sampler_kernel: 1024 threads
constexpr int CPW = 2;             // chunks per wave per pass

template <int WAVES, int CPWT, class Load>
__device__ __forceinline__ void block_top10(int n, Load load, float* bv, int* bi, float* cv, int* ci, float& ov,
                                            int& oi) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  bool first = true;
  float* in_v = cv;
  int* in_i = ci;
  float* out_v = bv;
  int* out_i = bi;
  while (true) {
    const int nch = (n + 63) / 64;
    if (nch == 1) break;
    for (int c0 = wave; c0 < nch; c0 += WAVES * CPWT) {
      float v[CPWT];
      int i[CPWT];
#pragma unroll
      for (int u = 0; u < CPWT; ++u) {  // all of this pass's loads first
        const int j = (c0 + u * WAVES) * 64 + lane;
        v[u] = -INFINITY;
        i[u] = 0x7fffffff;
        if (j < n) {
          if (first) {
            load(j, v[u], i[u]);
          } else {
            v[u] = in_v[j];
            i[u] = in_i[j];
          }
        }
      }
      wave_sort64<CPWT>(v, i);
#pragma unroll
      for (int u = 0; u < CPWT; ++u) {
        const int c = c0 + u * WAVES;
        if (lane < TOPK && c < nch) {
          out_v[c * TOPK + lane] = v[u];
          out_i[c * TOPK + lane] = i[u];
        }
      }
    }
    __syncthreads();
    n = nch * TOPK;
    first = false;
    float* tv = in_v;
    int* ti = in_i;
    in_v = out_v;
    in_i = out_i;
    out_v = tv;
    out_i = ti;
  }
  // one chunk left: every wave sorts it (wave 0's result is used; no extra barrier needed)
  float v[1] = {-INFINITY};
  int i[1] = {0x7fffffff};
  if (lane < n) {
    if (first) {
      load(lane, v[0], i[0]);
    } else {
      v[0] = in_v[lane];
      i[0] = in_i[lane];
    }
  }
  wave_sort64<1>(v, i);
  ov = v[0];
  oi = i[0];
  __syncthreads();  // the LDS buffers are reused by the caller's next top-10
}

// Fast path (no draw record requested): the reference keeps the first of its 10 draws that is
// acceptable (not id 0, not excluded), else the first draw (main.py:63-68). At most 9 ids are
// unacceptable, so at most 9 keys can rank above the best ACCEPTABLE key: it is always among
// the 10 draws, hence always the one kept. The token is therefore exactly the argmax of the
// acceptable keys (per-workgroup maxima from the decoder epilogue -> one block reduction); only
// when no acceptable id exists at all (V <= 9) does the reference fall back to the first draw.
template <int WAVES>
__device__ __forceinline__ void sample_argmax(const HzSamplerParams& p, int t) {
  if ((t + 1) >= *p.n_forced) {
    const int tok = block_token<WAVES>(p.bacc_val, p.bacc_idx, p.bmax_val, p.bmax_idx, p.nblk, p.V);
    if (threadIdx.x == 0) p.tok_seq[t + 1] = tok;
  }
}

// one sampling step with the calling workgroup (WAVES waves): top-10 keys -> draws -> token
template <int WAVES, int CPWT>
__device__ __forceinline__ void sample_step(const HzSamplerParams& p, int t) {
  __shared__ float buf_v[2][SAMPLER_LDS];
  __shared__ int buf_i[2][SAMPLER_LDS];
  __shared__ int sel[TOPK];
  const int lane = threadIdx.x & 63;
  if ((t + 1) >= *p.n_forced) {
    float v;
    int i;
    // 1. the 10 decoder workgroups with the largest maxima
    block_top10<WAVES, CPWT>(p.nblk, [&](int j, float& a, int& b) { a = p.bmax_val[j]; b = p.bmax_idx[j]; },
                             buf_v[0], buf_i[0], buf_v[1], buf_i[1], v, i);
    const int nsel = min(TOPK, p.nblk);
    if (threadIdx.x < nsel) sel[threadIdx.x] = min(i / p.rpb, p.nblk - 1);  // (NaN keys: stay in range)
    __syncthreads();
    // 2. the 10 largest keys among their rows
    const int rpb = p.rpb;
    block_top10<WAVES, CPWT>(nsel * rpb, [&](int j, float& a, int& b) {
                               const int q = j / rpb;
                               const int r = sel[q] * rpb + (j - q * rpb);
                               a = r < p.V ? p.keys[r] : -INFINITY;
                               b = r;
                             }, buf_v[0], buf_i[0], buf_v[1], buf_i[1], v, i);
    if (threadIdx.x < 64) {  // wave 0: lanes 0..9 hold the draws in order
      const int nd = min(TOPK, p.V);
      bool ok = lane < nd && i > 0;
      for (int e = 0; e < p.n_exclude; ++e) ok = ok && i != p.exclude[e];
      const unsigned long long m = __ballot(ok);
      const int src = m ? __ffsll((long long)m) - 1 : 0;  // first acceptable draw, else the first
      const int tok = __shfl(i, src, 64);
      if (lane == 0) p.tok_seq[t + 1] = tok;
      if (p.draws && lane < TOPK) p.draws[(long)t * TOPK + lane] = i;
    }
  }
}

// 4 waves x 8 chunks per pass: the 1875 decoder maxima of V=60000 fit one pass, and barriers
// synchronise 4 waves instead of 16
template <int WAVES, int CPWT>
__global__ __launch_bounds__(WAVES * 64) void sampler_kernel(const HzSamplerParams p) {
  sample_step<WAVES, CPWT>(p, *p.step + p.step_off);
}

__global__ __launch_bounds__(1024) void argmax_sampler_kernel(const HzSamplerParams p) {
  sample_argmax<16>(p, *p.step + p.step_off);
}

// x[k .. k+8) for k = c*512 + lane*8 of every 512-chunk c (zero past n; n even, x 8-B aligned):
// the vector operand of a GEMV row loaded straight into registers. Issued BEFORE the weight
// loads, so waiting for it does not wait for the weight stream (vmcnt retires in issue order),
// and no LDS staging / workgroup barrier stands between the kernel start and the weight stream.
// Loads are clamped into [0, n) like ld_row (positions past n hold duplicates: callers zero the
// matching weights with wmask).
template <int NC>
__device__ __forceinline__ void load_vec(const float* x, int n, int lane, f32x4 (&v)[NC][2]) {
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const int k = c * 512 + lane * 8 + hf * 4 + pr * 2;
        const float2 e = *reinterpret_cast<const float2*>(x + min(k, n - 2));
        v[c][hf][2 * pr] = e.x;
        v[c][hf][2 * pr + 1] = e.y;
      }
}

// The clamped columns past ld are zeroed on the WEIGHT side, at use (a mask on the register
// vector operand is loop-invariant: the compiler hoisted it, and its wait, above the weight loads).
__device__ __forceinline__ u32x4 wmask(const u32x4 w, int k, int ld) { return k < ld ? w : u32x4{0u, 0u, 0u, 0u}; }

template <class T>
__device__ __forceinline__ T pick4(const T (&a)[4], int l) {  // uniform select, no dynamic kernarg index
  return l == 0 ? a[0] : l == 1 ? a[1] : l == 2 ? a[2] : a[3];
}

#ifndef HZ_HH_RR
#define HZ_HH_RR 2  // 70 VGPRs with the register vector operand (4 rows: 98, 4 waves/SIMD)
#endif
// Split LSTM mode: rows [r0, r0 + HZ_HH_ROWS) of layer l's next-step recurrent gate partials
// W_hh^l . h^l_t + b^l. 4 waves x RR rows per round, every 16-B load of a round in flight.
template <int NCHH>
__device__ __forceinline__ void hh_rows(const HzDecoderParams& p, int b, int par) {
  constexpr int RR = HZ_HH_RR;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int l = 0;
#pragma unroll
  for (int k = 1; k < 4; ++k) l += (k < p.n_hh && b >= p.hh_blk[k]);
  const int H = pick4(p.hh_H, l), ld = pick4(p.hh_ld, l), rows = 4 * H;
  const bf16_t* W = reinterpret_cast<const bf16_t*>(pick4(p.hh_w, l));
  const float* bias = pick4(p.hh_b, l);
  const float* h = pick4(p.hh_h, l) + (par ^ 1) * H;  // h^l of this step
  float* out = pick4(p.hh_out, l);
  const int r0 = (b - (l == 0 ? p.hh_blk[0] : l == 1 ? p.hh_blk[1] : l == 2 ? p.hh_blk[2] : p.hh_blk[3])) * HZ_HH_ROWS;
  if (!HZ_DCHECK(H <= ld && ld <= NCHH * 512)) return;
#pragma unroll
  for (int rr = 0; rr < HZ_HH_ROWS; rr += 4 * RR) {
    u32x4 wv[RR][NCHH];
#pragma unroll
    for (int q = 0; q < RR; ++q) {
      const int r = min(r0 + rr + wave * RR + q, rows - 1);
#pragma unroll
      for (int c = 0; c < NCHH; ++c) {
        const int k = c * 512 + lane * 8;
        wv[q][c] = ld_row(W + (long)r * ld, k, ld);
      }
    }
    f32x4 hr[NCHH][2];  // h after the weights: its address needs the step counter, theirs does not
    load_vec<NCHH>(h, H, lane, hr);
    __builtin_amdgcn_sched_barrier(0);
    float acc[RR];
#pragma unroll
    for (int q = 0; q < RR; ++q) acc[q] = 0.f;
#pragma unroll
    for (int c = 0; c < NCHH; ++c) {
      const int k = c * 512 + lane * 8;
      const f32x4 v0 = hr[c][0], v1 = hr[c][1];
#pragma unroll
      for (int q = 0; q < RR; ++q) {
        float f[8];
        unpack8(wmask(wv[q][c], k, ld), f);
        acc[q] += f[0] * v0[0] + f[1] * v0[1] + f[2] * v0[2] + f[3] * v0[3] + f[4] * v1[0] + f[5] * v1[1] +
                  f[6] * v1[2] + f[7] * v1[3];
      }
    }
#pragma unroll
    for (int q = 0; q < RR; ++q) acc[q] = warp_sum(acc[q]);
    if (lane < RR) {
      const int r = r0 + rr + wave * RR + lane;
      float a = acc[0];
#pragma unroll
      for (int q = 1; q < RR; ++q) a = lane == q ? acc[q] : a;
      if (r < rows) out[r] = a + bias[r];
    }
  }
}

template <int NCH, int R, int NCHH>
__global__ __launch_bounds__(256) void decoder_kernel(const HzDecoderParams p) {
  __shared__ float w_best[4];
  __shared__ int w_besti[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int t = *p.step + p.step_off;
  const int par = t & 1;
  if constexpr (NCHH > 0) {
    if ((int)blockIdx.x < p.hh_blocks) {  // split LSTM mode: next step's W_hh partials
      hh_rows<NCHH>(p, blockIdx.x, par);
      return;
    }
  }
  const int blk = blockIdx.x - (NCHH > 0 ? p.hh_blocks : 0);
  const float* h = p.h_state + (par ^ 1) * p.H;  // last layer's output of this step
  // R rows per wave round (R <= DROWS): fewer registers -> more resident waves
  if (!HZ_DCHECK(p.H <= p.ldk && p.ldk <= NCH * 512 && p.rpb % DROWS == 0)) return;
  const int ngroups = (p.V + R - 1) / R;
  const int gpb = p.rpb / R;
  const int g_end = min(ngroups, (blk + 1) * gpb);
  // h is not staged through LDS (v2 staged it first, then issued the weights: a load latency and
  // a barrier ahead of every workgroup's weight stream); each lane loads its own K positions
  const unsigned long long seed = p.keys ? *p.seed : 0ull;
  float best = -INFINITY, abest = -INFINITY;
  int besti = 0x7fffffff, abesti = 0x7fffffff;
  for (int g = blk * gpb + wave; g < g_end; g += 4) {
    u32x4 wv[R][NCH];
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int r = min(g * R + q, p.V - 1);
#pragma unroll
      for (int c = 0; c < NCH; ++c) wv[q][c] = ld_row(p.w + (long)r * p.ldk, c * 512 + lane * 8, p.ldk);
    }
    f32x4 hr[NCH][2];  // after the weights: h's address needs the step counter, theirs does not
    load_vec<NCH>(h, p.H, lane, hr);
    __builtin_amdgcn_sched_barrier(0);  // every load of the round issued before the first use
    float acc[R];
#pragma unroll
    for (int q = 0; q < R; ++q) acc[q] = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int k = c * 512 + lane * 8;
      const f32x4 v0 = hr[c][0], v1 = hr[c][1];
#pragma unroll
      for (int q = 0; q < R; ++q) {
        float f[8];
        unpack8(wmask(wv[q][c], k, p.ldk), f);
        acc[q] += f[0] * v0[0] + f[1] * v0[1] + f[2] * v0[2] + f[3] * v0[3] + f[4] * v1[0] + f[5] * v1[1] +
                  f[6] * v1[2] + f[7] * v1[3];
      }
    }
#pragma unroll
    for (int q = 0; q < R; ++q) acc[q] = warp_sum(acc[q]);
    if (lane < R) {
      const int r = g * R + lane;
      float a = acc[0];
#pragma unroll
      for (int q = 1; q < R; ++q) a = lane == q ? acc[q] : a;
      if (r < p.V) {
        const float lg = a + (p.bias ? p.bias[r] : 0.f);
        p.logits[r] = lg;
        if (p.keys) {
          const float key = lg + gumbel(seed, t, r);
          p.keys[r] = key;
          if (better(key, r, best, besti)) {
            best = key;
            besti = r;
          }
          bool acc = r != 0;
          for (int e = 0; e < p.n_exclude; ++e) acc = acc && r != p.exclude[e];
          if (acc && better(key, r, abest, abesti)) {
            abest = key;
            abesti = r;
          }
        }
      }
    }
  }
  if (p.keys) {  // workgroup max keys: lanes 0..R-1 hold the candidates, xor 1..R/2 stays inside them
    __shared__ float a_best[4];
    __shared__ int a_besti[4];
#pragma unroll
    for (int o = 1; o < R; o <<= 1) {
      const float ov = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(besti, o, 64);
      const float av = __shfl_xor(abest, o, 64);
      const int ai = __shfl_xor(abesti, o, 64);
      if (better(ov, oi, best, besti)) {
        best = ov;
        besti = oi;
      }
      if (better(av, ai, abest, abesti)) {
        abest = av;
        abesti = ai;
      }
    }
    if (lane == 0) {
      w_best[wave] = best;
      w_besti[wave] = besti;
      a_best[wave] = abest;
      a_besti[wave] = abesti;
    }
    __syncthreads();
    if (tid == 0) {
      for (int w = 1; w < 4; ++w) {
        if (better(w_best[w], w_besti[w], best, besti)) {
          best = w_best[w];
          besti = w_besti[w];
        }
        if (better(a_best[w], a_besti[w], abest, abesti)) {
          abest = a_best[w];
          abesti = a_besti[w];
        }
      }
      p.bmax_val[blk] = best;
      p.bmax_idx[blk] = besti;
      if (p.bacc_val) {
        p.bacc_val[blk] = abest;
        p.bacc_idx[blk] = abesti;
      }
    }
  }
}

}  // namespace

static int lstm_x_launch(const HzLstmParams& p, hipStream_t st) {
  if (p.ldk % 64 || p.ldk < p.In || p.In <= 0 || p.H <= 0 || p.ldk > 6 * 512) return -1;
  const bool fuse0 = p.xtab != nullptr;
  if (fuse0 && (p.H0 != p.In || p.H0 > 3 * 512 || !p.pre0 || !p.h0_state || !p.c0_state || !p.tok_seq)) return -1;
  if (!fuse0 && !p.x_state) return -1;
  if (p.bacc_val && (!fuse0 || !p.n_forced || !p.bacc_idx || !p.bmax_val || !p.bmax_idx || p.nblk < 1 || p.nblk > 2048 ||
                     p.V < 1))
    return -1;
  const int nch = (p.ldk + 511) / 512;
  const dim3 grid((p.H + 3) / 4), block(512);
  const size_t lds = (size_t)nch * 512 * sizeof(float);
#define HZ_LX(N)                                                                          \
  case N:                                                                                 \
    if (fuse0) hipLaunchKernelGGL((lstm_x_kernel<N, true>), grid, block, lds, st, p);     \
    else hipLaunchKernelGGL((lstm_x_kernel<N, false>), grid, block, lds, st, p);          \
    break;
  switch (nch) {
    HZ_LX(1) HZ_LX(2) HZ_LX(3) HZ_LX(4) HZ_LX(5) HZ_LX(6)
    default: return -1;
  }
#undef HZ_LX
  return (int)hipGetLastError();
}

extern "C" int hz_lstm_cell_launch(const HzLstmParams* pp, hipStream_t st) {
  const HzLstmParams& p = *pp;
  if (p.pre) return lstm_x_launch(p, st);
  if (p.ldk % 64 || p.ldk < p.In + p.H || p.In <= 0 || p.H <= 0) return -1;
  if (p.bacc_val && (!p.emb || !p.n_forced || !p.bacc_idx || !p.bmax_val || !p.bmax_idx || p.nblk < 1 || p.nblk > 2048 || p.V < 1))
    return -1;
  // waves per unit (K split): 2 (per-layer us at the reference dims, KW = 1 / 2 / 4: layer 0
  // 7.73 / 7.71 / 8.30, layer 1 5.64 / 5.48 / 5.58; profiles/r2_awd_lstm/v2/lstm_kw_ab)
  constexpr int KW = 2;
  const int nch = (p.ldk + 511) / 512;
  const dim3 grid((p.H + 4 / KW - 1) / (4 / KW)), block(256);
  const size_t lds = (size_t)nch * 512 * sizeof(float);
  switch (nch) {
    case 1: hipLaunchKernelGGL((lstm_cell_kernel<1, KW>), grid, block, lds, st, p); break;
    case 2: hipLaunchKernelGGL((lstm_cell_kernel<2, KW>), grid, block, lds, st, p); break;
    case 3: hipLaunchKernelGGL((lstm_cell_kernel<3, KW>), grid, block, lds, st, p); break;
    case 4: hipLaunchKernelGGL((lstm_cell_kernel<4, KW>), grid, block, lds, st, p); break;
    case 5: hipLaunchKernelGGL((lstm_cell_kernel<5, KW>), grid, block, lds, st, p); break;
    case 6: hipLaunchKernelGGL((lstm_cell_kernel<6, KW>), grid, block, lds, st, p); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

namespace {
__global__ void step_bump_kernel(int* step, int n) {
  if (threadIdx.x == 0) *step += n;
}
}  // namespace

extern "C" int hz_step_bump_launch(int* step, int n, hipStream_t st) {
  if (!step) return -1;
  hipLaunchKernelGGL(step_bump_kernel, dim3(1), dim3(64), 0, st, step, n);
  return (int)hipGetLastError();
}

extern "C" void hz_decoder_geometry(int V, int* nblk, int* rpb) {
  const int groups = (V + DROWS - 1) / DROWS;
  int nb = min(2048, (groups + 3) / 4);
  int gpb = (groups + nb - 1) / nb;
  gpb = (gpb + 3) / 4 * 4;  // whole wave rounds per workgroup
  *nblk = (groups + gpb - 1) / gpb;
  *rpb = gpb * DROWS;
}

extern "C" int hz_decoder_launch(const HzDecoderParams* pp, hipStream_t st) {
  const HzDecoderParams& p = *pp;
  if (p.ldk % 8 || p.ldk < p.H || p.H % 2 || (p.keys && (!p.seed || !p.bmax_val || !p.bmax_idx))) return -1;
  int nblk, rpb;
  hz_decoder_geometry(p.V, &nblk, &rpb);
  if (p.nblk != nblk || p.rpb != rpb) return -1;
  // split LSTM mode: recurrent-partial workgroups ahead of the decoder's (hh_rows)
  constexpr int NCHH = 3;
  if (p.n_hh < 0 || p.n_hh > 4) return -1;
  if (p.n_hh > 0) {
    if (p.hh_blk[0] != 0 || p.hh_blk[p.n_hh] != p.hh_blocks) return -1;
    for (int l = 0; l < p.n_hh; ++l)
      if (!p.hh_w[l] || !p.hh_b[l] || !p.hh_h[l] || !p.hh_out[l] || p.hh_H[l] < 1 || p.hh_H[l] % 2 || p.hh_ld[l] % 64 ||
          p.hh_ld[l] < p.hh_H[l] || p.hh_ld[l] > NCHH * 512 ||
          p.hh_blk[l + 1] - p.hh_blk[l] != (4 * p.hh_H[l] + HZ_HH_ROWS - 1) / HZ_HH_ROWS)
        return -1;
  }
  const int hh = p.n_hh > 0 ? p.hh_blocks : 0;
  const dim3 grid(nblk + hh), block(256);
  const int nch = (p.ldk + 511) / 512;
  const size_t lds = 0;  // the vector operand lives in registers (load_vec)
  // 4 rows per wave round: 72 VGPRs, 7 waves/SIMD (8 rows: 104 VGPRs, 4 waves/SIMD; 22.7 vs 23.3 us
  // at V = 60000). Non-temporal weight loads measured slower for the decoder and the LSTM cells; so
  // was a streaming variant (a wave walks 1/2/4 whole blocks with the next 4 rows in flight, h
  // staged once per workgroup): 23.8 / 29.9 / 53.1 vs 22.3 us -- one short round per workgroup
  // with every load of the chip in flight at once is what reaches ~5.5 TB/s.
  constexpr int R = 4;
#define HZ_DEC(N)                                                                       \
  case N:                                                                               \
    if (hh) hipLaunchKernelGGL((decoder_kernel<N, R, NCHH>), grid, block, lds, st, p);  \
    else hipLaunchKernelGGL((decoder_kernel<N, R, 0>), grid, block, lds, st, p);        \
    break;
  switch (nch) {
    HZ_DEC(1) HZ_DEC(2) HZ_DEC(3) HZ_DEC(4)
    default: return -1;
  }
#undef HZ_DEC
  return (int)hipGetLastError();
}

extern "C" int hz_sampler_launch(const HzSamplerParams* pp, hipStream_t st) {
  const HzSamplerParams& p = *pp;
  int nblk, rpb;
  hz_decoder_geometry(p.V, &nblk, &rpb);
  if (p.n_exclude > 8 || p.V < 1 || !p.keys || !p.bmax_val || !p.bmax_idx || p.nblk != nblk || p.rpb != rpb)
    return -1;
  // LDS tournament capacity: first-round chunks of either top-10 must fit one buffer
  if ((nblk + 63) / 64 * TOPK > SAMPLER_LDS || (TOPK * rpb + 63) / 64 * TOPK > SAMPLER_LDS) return -1;
  if (p.bacc_val && p.bacc_idx && !p.draws && !getenv("HIPZAP_SAMPLER_TOURNAMENT"))
    hipLaunchKernelGGL(argmax_sampler_kernel, dim3(1), dim3(1024), 0, st, p);
  else  // draws recorded (tests, diagnostics): the exact top-10 tournament
    hipLaunchKernelGGL((sampler_kernel<SAMPLER_WAVES, CPW>), dim3(1), dim3(64 * SAMPLER_WAVES), 0, st, p);
  return (int)hipGetLastError();
}
