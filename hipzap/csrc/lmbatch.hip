// Batched AWD-LSTM decode: continuous batching of concurrent GET /inference requests
// (/root/reference/main.py:40-81,84-112 decode loop; VERDICT r2 "next round" #3).
//
// The single-request engine (csrc/lstm.hip) streams all ~150 MB of weights for every token of
// every request. Here Bp request rows (16 or 32) share each decode step, so one pass over the
// weights serves all of them: every layer and the decoder are skinny GEMMs on the matrix cores
// (mfma_f32_16x16x32_bf16, A = weight fragment, B = request rows), memory-bound on the weight
// stream like the GEMV they replace. A step is 1 + L launches:
//   layer 0   token of every row (forced prompt token, or the argmax of the previous decoder's
//             per-workgroup maxima -- the exact main.py:63-68 rule, csrc/lstm.hip sample_argmax)
//             and its embedding as the x operand; gates = W0 [h0_prev ; emb(tok)] + b; cell update
//   layer l   gates = Wl [hl_prev ; h(l-1)_t] + b; cell update
//   decoder   logits = E h(L-1)_t + b -> key = logit + Gumbel(seed_r, t_r, v) (common.h, the same
//             noise as the single-request engine) -> per (workgroup, row) max over acceptable ids
// Numerics: weights bf16 (as in the single-request engine); the recurrent state is fp32 and
// enters the MFMAs as a bf16 hi/lo pair (two MFMAs, ~16 mantissa bits), accumulation fp32. Each
// output element depends only on its own row's operands, so a request's tokens do not depend on
// which other requests share the batch (tests/test_lmbatch_gpu.py checks bitwise).
#include <cstdlib>
#include <cstring>

#include "common.h"
#include "hipzap.h"

HZ_DEBUG_UNIT(lmbatch)

namespace {

constexpr int LW = 8;      // waves per layer workgroup (K split over them)
constexpr int SPW = 9;     // k-steps (of 32) per wave: K <= 8 * 9 * 32 = 2304
constexpr int DW = 8;      // decoder tile slots per workgroup / 2 (8 waves x 2 tiles or 4 x 4)
constexpr int DROWS = DW * 32;  // vocabulary rows per decoder workgroup
constexpr int DKMAX = 32;  // decoder k-steps (K <= 1024, a multiple of 256)


typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// order-preserving (key, row) -> u64; larger is better, ties to the lower row; 0 = nothing
__device__ __forceinline__ unsigned long long pack_key(float v, int row) {
  unsigned u = __float_as_uint(v);
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ((unsigned long long)u << 32) | (unsigned)(0xffffffffu - (unsigned)row);
}
__device__ __forceinline__ int key_row(unsigned long long k) { return (int)(0xffffffffu - (unsigned)k); }
__device__ __forceinline__ unsigned long long umax64(unsigned long long a, unsigned long long b) { return a > b ? a : b; }
__device__ __forceinline__ unsigned long long shfl_xor64(unsigned long long v, int o) {
  const unsigned lo = __shfl_xor((unsigned)v, o, 64), hi = __shfl_xor((unsigned)(v >> 32), o, 64);
  return ((unsigned long long)hi << 32) | lo;
}

__device__ __forceinline__ bf16x8 as_frag(const u32x4 v) { return __builtin_bit_cast(bf16x8, v); }

// element offset of (unit/k = j, request row = r) in one [K/32][Bp/16][64][8] state image
__device__ __forceinline__ int st_off(int j, int r, int NB) {
  return ((j >> 5) * NB + (r >> 4)) * 512 + ((((j & 31) >> 3) << 4) + (r & 15)) * 8 + (j & 7);
}

// ------------------------------------------------------------------------ layer kernel
// One workgroup per TPW 16-row tiles (4 hidden units x 4 gates each) x NBW row blocks of 16
// request rows; the 8 waves split K. Every load of a wave (its weight fragments, its state
// fragments) is issued before the first MFMA; partial tiles meet in LDS and TPW x NBW x 64 threads
// apply the cell update.
// NBW = NB: every workgroup reads all Bp rows' state (128 B per k at Bp 32 against 32 B of weights
// per tile): the layer is bound by what each CU fetches, not by HBM. NBW = 1 (Bp 32): twin
// workgroups b and b + 8 (one XCD under round-robin placement: the twin's weight read hits L2)
// take one row block each, so a CU fetches TPW * 32 + 64 B per k instead of TPW * 32 + 128.
// EP (first layer, p.embproj): the embedding half of the layer's K is precomputed per vocabulary
// id (lmb_embproj_kernel: P[v] = W_ih E[v], fp32), so the workgroup multiplies W_hh h only and the
// cell update adds P[token] -- half the weight bytes on the step's critical path.
// SOLO (p.nb_act == -1, the one-request program): request row 0 alone is busy; the other rows'
// state is neither read (their operand lanes are zero) nor written, so a wave fetches 1/16 of
// each 1 KiB state fragment (the lanes of row 0: 0, 16, 32, 48). Each MFMA output column depends
// on its own row's operand only: row 0 is bitwise the full program's.
template <int NB, bool FIRST, int TPW, int NBW, bool EP = false, bool SOLO = false>
__global__ __launch_bounds__(512) void lmb_layer_kernel(const HzLmbLayerParams p) {
  static_assert(NBW == NB || NBW == 1, "row blocks per workgroup");
  static_assert(!SOLO || NBW == NB, "the one-request program uses the all-row-block shape");
  static_assert(!EP || FIRST, "the projected embedding is the first layer's input");
  __shared__ f32x4 part[LW][TPW][NBW][64];
  __shared__ int s_tok[32];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int grp = blockIdx.x, cb0 = 0;  // tile group, first row block
  if constexpr (NBW != NB) {
    const int idx = blockIdx.x >> 3;
    grp = (idx >> 1) * 8 + (blockIdx.x & 7);
    cb0 = idx & 1;
  }
  const int tile0 = grp * TPW;  // this workgroup's row tiles tile0 .. tile0 + TPW - 1
  const int ntile = p.R >> 4;
  const int nba = SOLO ? 1 : p.nb_act > 0 ? p.nb_act : NB;  // row blocks computed (wave-uniform)
  if (tile0 >= ntile || cb0 >= nba) return;      // (grid padding of the twin mapping; low-load program)
  const bool row_lane = !SOLO || (lane & 15) == 0;  // this lane carries a busy row's operand
  const int nbw = min(NBW, nba - cb0);           // row blocks this workgroup computes
  const int KSH = p.Kh >> 5, KSX = p.Kx >> 5, KS = KSH + KSX;  // KS: the packed row stride
  const int KSE = EP ? KSH : KS;                                  // k-steps multiplied here
  const int spw = (KSE + LW - 1) / LW;
  const int k0 = wave * spw;
  const int cnt = max(0, min(spw, KSE - k0));
  const int Bp = NB * 16;
  if (!HZ_DCHECK(spw <= SPW && p.Bp == Bp && p.R % 16 == 0 && nba <= NB)) return;
  // ---- loads that need nothing: this sub-step's control + the decoder maxima (FIRST), then the
  // weight stream; vmcnt retires in issue order, so what the token selection waits for goes first
  HzLmbCtl cl = {};
  f32x4 pe = f32x4{0.f, 0.f, 0.f, 0.f};  // EP: this thread's unit's projected embedding (4 gates)
  unsigned long long best0 = 0, best1 = 0;  // both parities: no wait on the step parity before the weight stream
  if constexpr (FIRST) {
    if (tid < Bp) {
      cl = p.ctl[p.step_off * Bp + tid];
      best0 = p.dbest[tid];
      best1 = p.dbest[Bp + tid];
    }
  }
  const auto kcl = [&](int s) { return min(k0 + min(s, max(cnt - 1, 0)), KSE - 1); };
  u32x4 wf[TPW][SPW];
#pragma unroll
  for (int tt = 0; tt < TPW; ++tt) {
    const bf16_t* wt = p.w + (size_t)min(tile0 + tt, ntile - 1) * KS * 512 + lane * 8;
#pragma unroll
    for (int s = 0; s < SPW; ++s)  // (slots past this wave's cnt re-load its own last k-step, not the
                                   // next wave's: straight-line loads keep the counted vmcnt waits)
      wf[tt][s] = *reinterpret_cast<const u32x4*>(wt + (size_t)kcl(s) * 512);
  }
  __builtin_amdgcn_sched_barrier(0);
  const int par = (*p.gpar + p.step_off) & 1;
  // state operands: h_prev (own, parity par) for k < Kh; x for k >= Kh (previous layer's output
  // of this step, parity par ^ 1; FIRST: the embedding rows of the tokens, after selection)
  u32x4 ah[SPW][NBW], al[SPW][NBW];
#pragma unroll
  for (int s = 0; s < SPW; ++s) {
    const int ks = kcl(s);
    // FIRST: k-steps past Kh are the embedding, loaded after the token selection (a harmless
    // in-range h fragment here keeps the loop branch-free)
    const bool hk = FIRST || ks < KSH;
    const int kh = min(ks, KSH - 1);
    const bf16_t* src = hk ? p.h + ((size_t)(par * 2) * KSH + kh) * NB * 512
                           : p.x + ((size_t)((par ^ 1) * 2) * KSX + (ks - KSH)) * NB * 512;
    const size_t lo_off = (size_t)(hk ? KSH : KSX) * NB * 512;
#pragma unroll
    for (int cb = 0; cb < NBW; ++cb) {
      if (cb < nbw) {
        if (row_lane) {
          ah[s][cb] = *reinterpret_cast<const u32x4*>(src + (cb0 + cb) * 512 + lane * 8);
          al[s][cb] = *reinterpret_cast<const u32x4*>(src + lo_off + (cb0 + cb) * 512 + lane * 8);
        } else {
          ah[s][cb] = al[s][cb] = u32x4{0u, 0u, 0u, 0u};
        }
      }
    }
  }
  // the cell update's own operands (folded bias, previous cell state) need nothing computed here:
  // the cell-update threads fetch them now, behind the weight and state loads, instead of after
  // the MFMAs and the LDS reduction (one more memory round trip on the layer's critical path)
  const bool upd = tid < TPW * NBW * 64 && (tid >> 6) % NBW < nbw && row_lane;
  const int u_tt = tid / (NBW * 64), u_cb = (tid >> 6) % NBW, u_l = tid & 63;
  const int u_j = (tile0 + u_tt) * 4 + (u_l >> 4), u_r = (cb0 + u_cb) * 16 + (u_l & 15);
  const bool u_ok = upd && tile0 + u_tt < ntile && u_j < p.H;
  f32x4 u_b = f32x4{0.f, 0.f, 0.f, 0.f};
  float u_c = 0.f;
  if (u_ok) {
    u_b = *reinterpret_cast<const f32x4*>(p.bias + 4 * u_j);
    u_c = p.c[(size_t)u_r * p.H + u_j];
  }
  if constexpr (FIRST) {
    // ---- token of every row: the argmax of the acceptable keys of the last decoder (its
    // workgroups' atomic maxima, buffer of the other parity); the first workgroup clears this
    // parity's buffer for this step's decoder
    if (tid < Bp) {
      // (measured: sharding these maxima over 8 atomic slots made this kernel 1.3 us slower and
      // the decoder no faster, profiles/r3_lmbatch)
      const unsigned long long best = par ? best0 : best1;
      int tok = cl.tok >= 0 ? cl.tok : (cl.tok == -1 && best ? key_row(best) : 0);
      tok = min(max(tok, 0), p.V - 1);
      s_tok[tid] = tok;
      if (tile0 == 0 && cb0 == 0) {
        p.dbest[(size_t)par * Bp + tid] = 0ull;  // for this step's decoder
        if (p.tok) p.tok[tid] = tok;
        if (cl.tok == -1 && cl.out >= 0 && p.outp[tid]) p.outp[tid][cl.out] = tok;
      }
    }
    lds_barrier();  // LDS only: the weight and state loads stay in flight
    if constexpr (EP) {
      // the cell-update threads fetch their rows' projected embedding now (consumed after the MFMAs)
      if (tid < TPW * NBW * 64 && (tid >> 6) % NBW < nbw && row_lane) {
        const int tt = tid / (NBW * 64), cb = (tid >> 6) % NBW, l = tid & 63;
        const int j = min((tile0 + tt) * 4 + (l >> 4), p.R / 4 - 1);
        pe = *reinterpret_cast<const f32x4*>(p.embproj + (size_t)s_tok[(cb0 + cb) * 16 + (l & 15)] * p.R + 4 * j);
      }
    }
#pragma unroll
    for (int s = 0; s < SPW && !EP; ++s) {
      const int ks = min(k0 + s, KS - 1);
      if (ks >= KSH) {  // wave-uniform
#pragma unroll
        for (int cb = 0; cb < NBW; ++cb) {
          if (cb >= nbw || !row_lane) continue;  // (SOLO: the other lanes stay zero)
          const int tk = s_tok[(cb0 + cb) * 16 + (lane & 15)];
          ah[s][cb] = *reinterpret_cast<const u32x4*>(
              p.emb + ((size_t)(tk >> 4) * KSX + (ks - KSH)) * 512 + ((lane >> 4) * 16 + (tk & 15)) * 8);
        }
      }
    }
  }
  // ---- MFMAs over this wave's k-steps
  f32x4 acc[TPW][NBW];
#pragma unroll
  for (int tt = 0; tt < TPW; ++tt)
#pragma unroll
    for (int cb = 0; cb < NBW; ++cb) acc[tt][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < SPW; ++s) {
    if (s < cnt) {  // wave-uniform
      const bool lo = !FIRST || (k0 + s) < KSH;  // the embedding is exact bf16: no lo half
#pragma unroll
      for (int tt = 0; tt < TPW; ++tt)
#pragma unroll
        for (int cb = 0; cb < NBW; ++cb) {
          if (cb >= nbw) continue;
          acc[tt][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(wf[tt][s]), as_frag(ah[s][cb]), acc[tt][cb], 0, 0, 0);
          if (lo)
            acc[tt][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(wf[tt][s]), as_frag(al[s][cb]), acc[tt][cb], 0, 0, 0);
        }
    }
  }
#pragma unroll
  for (int tt = 0; tt < TPW; ++tt)
#pragma unroll
    for (int cb = 0; cb < NBW; ++cb) part[wave][tt][cb][lane] = acc[tt][cb];
  __syncthreads();
  // ---- cell update: thread (tt, cb, l) owns unit 4*(tile0+tt) + (l >> 4) of request row
  // (cb0+cb)*16 + (l & 15); its 4 accumulator registers ARE the unit's gates i, f, g, o (C/D rows
  // 4(l>>4) .. +3)
  if (upd) {
    const int tt = u_tt, cb = u_cb, l = u_l;
    f32x4 g = part[0][tt][cb][l];
#pragma unroll
    for (int w = 1; w < LW; ++w) g += part[w][tt][cb][l];  // fixed order: deterministic
    const int j = u_j, r = u_r;
    if (u_ok) {
      g += u_b;
      if constexpr (EP) g += pe;
      const float si = 1.f / (1.f + __expf(-g[0]));
      const float sf = 1.f / (1.f + __expf(-g[1]));
      const float so = 1.f / (1.f + __expf(-g[3]));
      const float c_new = sf * u_c + si * tanhf(g[2]);
      const float h_new = so * tanhf(c_new);
      p.c[(size_t)r * p.H + j] = c_new;
      const __bf16 hi = (__bf16)h_new;
      const __bf16 lo = (__bf16)(h_new - (float)hi);
      bf16_t* dst = p.h + (size_t)((par ^ 1) * 2) * KSH * NB * 512 + st_off(j, r, NB);
      dst[0] = __builtin_bit_cast(bf16_t, hi);
      dst[(size_t)KSH * NB * 512] = __builtin_bit_cast(bf16_t, lo);
    }
  }
}

// ------------------------------------------------------------------------ projected embedding
// P[v][r] = sum_k W0[r][Kh + k] E[v][k] (fp32, [Vp][R]): the first layer's input half for every
// vocabulary id, once per engine build. Workgroup = 8 vocabulary tiles (one per wave, its 16 ids'
// embedding fragments held in registers); the W_ih fragments of each 16-row gate tile are staged
// once per workgroup in LDS (double-buffered, global_load_lds) and shared by the 8 waves.
constexpr int EPKS = 32;  // Kx / 32 <= 32 (K <= 1024, the batched engine's embedding limit)

__global__ __launch_bounds__(512) void lmb_embproj_kernel(const HzLmbEmbProjParams p) {
  __shared__ __attribute__((aligned(16))) bf16_t A[2][EPKS * 512];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int KSX = p.Kx >> 5, KS = (p.Kh + p.Kx) >> 5, KSH = p.Kh >> 5;
  const int nvt = p.Vp >> 4, ngt = p.R >> 4;
  const int vt = blockIdx.x * 8 + wave;
  if (!HZ_DCHECK(KSX <= EPKS && KSX >= 1)) return;
  const bool live = vt < nvt;  // (waves past the vocabulary keep the barriers)
  bf16x8 b[EPKS];
#pragma unroll
  for (int s = 0; s < EPKS; ++s)
    if (s < KSX) b[s] = as_frag(*reinterpret_cast<const u32x4*>(p.emb + ((size_t)min(vt, nvt - 1) * KSX + s) * 512 + lane * 8));
  // stage gate tile g's KSX fragments: fragment s = 1 KiB, wave w takes s = w, w + 8, ...
  auto stage = [&](int buf, int g) {
    const bf16_t* src = p.w + ((size_t)g * KS + KSH) * 512 + lane * 8;
    for (int s = wave; s < KSX; s += 8)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + (size_t)s * 512),
                                       (lds_void*)(&A[buf][s * 512]), 16, 0, 0);
  };
  stage(0, 0);
  for (int g = 0; g < ngt; ++g) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // tile g staged by every wave; buffer (g + 1) & 1 free (tile g - 1 read)
    if (g + 1 < ngt) stage((g + 1) & 1, g + 1);
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    const bf16_t* a = &A[g & 1][lane * 8];
#pragma unroll
    for (int s = 0; s < EPKS; ++s)
      if (s < KSX) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(*reinterpret_cast<const u32x4*>(a + s * 512)), b[s], acc, 0, 0, 0);
    // lane l: gate rows 16g + 4(l>>4) .. +3 of vocabulary id 16vt + (l&15)
    if (live)
      *reinterpret_cast<f32x4*>(p.out + (size_t)(vt * 16 + (lane & 15)) * p.R + g * 16 + 4 * (lane >> 4)) = acc;
  }
}

// ------------------------------------------------------------------------ decoder kernel
// Workgroup = 256 vocabulary rows x all Bp request rows. The whole last-layer state (hi/lo, K <=
// 1024) is staged once into LDS (fragment-major, lane-linear: 16-B global_load_lds per lane) while
// the first weight chunk streams in; each wave owns 2 vocabulary tiles and walks K in chunks of CH
// k-steps through a ring of R register chunks: chunk c + R is issued into chunk c's registers as
// soon as chunk c is multiplied, so R - 1 chunks stream during every chunk's MFMAs (the
// compiler's vmcnt counts retire in issue order). (CH, R) = (8, 2) is the round-3 schedule.

// s_waitcnt vmcnt(N) with expcnt / lgkmcnt left alone (gfx9 encoding)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// TW vocabulary tiles per wave, 16 / TW waves per workgroup (the 16 tile slots of a workgroup
// either way): every wave reads each state fragment from LDS once per k-step, so TW = 4 halves
// the LDS reads per tile of TW = 2 (128 KiB of ds_read_b128 per wave at Bp 32) with half the waves
// DIAG (experiments build, timing only -- the tokens are garbage): 1 skips the state staging,
// 2 skips the lo-half MFMAs and LDS reads; what each costs at Bp 32 (profiles/r4_lmb)
template <int NB, int KS, int CH, int R, bool NT = false, bool SOLO = false, int TW = 2, int DIAG = 0>
__global__ __launch_bounds__(64 * (16 / TW)) void lmb_dec_kernel(const HzLmbDecParams p) {
  constexpr int NCH = KS / CH;  // K = 32 * KS
  constexpr int RR = R < NCH ? R : NCH;  // chunks issued before the first MFMA
  constexpr int NW = 16 / TW;            // waves
  static_assert(KS % CH == 0, "k-steps per chunk");
  static_assert(TW == 2 || TW == 4, "tiles per wave");
  static_assert((RR - 1) * TW * CH < 64, "vmcnt range");
  constexpr int Bp = NB * 16;
  const int nba = SOLO ? 1 : p.nb_act > 0 ? p.nb_act : NB;  // row blocks computed (wave-uniform)
  __shared__ __attribute__((aligned(16))) bf16_t act[KS * 2 * NB * 512];  // [KS][2 hi/lo][NB][512]: 128 KiB at Bp 32, K 1024
  __shared__ unsigned long long s_best[NW][32];
  __shared__ __attribute__((aligned(16))) HzLmbCtl s_ctl[32];
  __shared__ __attribute__((aligned(16))) unsigned long long s_seed[32];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int blk = blockIdx.x;
  if (!HZ_DCHECK(p.K == KS * 32 && p.Bp == Bp)) return;
  // this workgroup's vocabulary tiles [t_lo, t_hi) (<= 16: TW per wave)
  const int ntile = p.Vp >> 4;
  const int t_lo = (int)((long)blk * ntile / p.nblk), t_hi = (int)((long)(blk + 1) * ntile / p.nblk);
  const int tile0 = t_lo + wave * TW;
  // A workgroup owns 14-15 tiles (3750 over 256 at V = 60000) but has 16 tile slots: a slot past
  // t_hi loads through a range-checked buffer descriptor at an out-of-range offset -- no memory
  // traffic, zeros in the registers, and the load still counts in vmcnt, so the counted waits
  // below hold for every wave (these slots used to re-read the next workgroup's tiles: 8 % of
  // the decoder's bytes)
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0, (int)((long)ntile * KS * 1024), 0x00020000);
  constexpr int kOOB = 0x7ff00000;  // > every descriptor's size (the launcher bounds it)
  int woff[TW];
#pragma unroll
  for (int t = 0; t < TW; ++t) woff[t] = (tile0 + t < t_hi ? (tile0 + t) * KS * 1024 : kOOB) + lane * 16;
  // the epilogue's bias, fetched first (it needs nothing, and retiring first it never holds up the
  // counted weight-chunk waits below): one memory round trip less after the last chunk
  f32x4 bias_t[TW];
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    const int v0 = (tile0 + t) * 16 + (lane >> 4) * 4;
    bias_t[t] = p.bias && tile0 + t < t_hi && v0 < p.V ? *reinterpret_cast<const f32x4*>(p.bias + v0)
                                                       : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  u32x4 wr[TW][RR][CH];
  auto issue = [&](int slot, int c) {
#pragma unroll
    for (int s = 0; s < CH; ++s) {
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        if constexpr (NT) {  // non-temporal weight stream (MI355X_MICROARCH.md "nt-weights")
          const bf16_t* wt = p.w + (size_t)min(tile0 + t, ntile - 1) * KS * 512 + lane * 8;
          wr[t][slot][s] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wt + (size_t)(c * CH + s) * 512));
        } else {
          wr[t][slot][s] =
              __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wrs, woff[t] + (c * CH + s) * 1024, 0, 0));
        }
      }
    }
  };
  issue(0, 0);
  const int par = (*p.gpar + p.step_off) & 1;
  // stage the state: KS * 2 * NB fragments of 1 KiB, wave w takes fragments w, w + NW, ...
  {
    const bf16_t* src = p.h + (size_t)((par ^ 1) * 2) * KS * NB * 512;  // this step's output of the last layer
    constexpr int NFRAG = KS * 2 * NB;
    static_assert(NFRAG % NW == 0, "state fragments per wave");
#pragma unroll
    for (int f0 = 0; f0 < NFRAG; f0 += NW) {
      const int f = f0 + wave;
      const int ks = f / (2 * NB), rem = f - ks * 2 * NB, hl = rem / NB, cb = rem - hl * NB;
      const bf16_t* g = src + ((size_t)hl * KS * NB + (size_t)ks * NB + cb) * 512 + lane * 8;
      // (the vmcnt wait below counts only the weight chunks issued after the staging; SOLO: the
      // lanes of row 0 only -- the other rows' logits are garbage nobody reads: their dec_t is -1)
      if (cb < nba && (!SOLO || (lane & 15) == 0) && DIAG != 1)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(g), (lds_void*)(act + (size_t)f * 512), 16, 0, 0);
    }
  }
  // the rows' control and seeds go to LDS the same way (an ordinary load here would make hipcc
  // wait for vmcnt(0) at its first use while the global_load_lds are in flight)
  if (wave == NW - 1) {
    if (lane < Bp)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(p.ctl + p.step_off * Bp + lane), (lds_void*)s_ctl,
                                       16, 0, 0);
    if (lane < Bp / 2)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(p.seed + 2 * lane), (lds_void*)s_seed, 16, 0, 0);
  }
#pragma unroll
  for (int c = 1; c < RR; ++c) issue(c, c);
  __builtin_amdgcn_sched_barrier(0);
  // the staged state is complete once everything issued before chunk 1 has landed (every wave);
  // chunks 1 .. RR - 1 keep streaming across the barrier
  wait_vmcnt<(RR - 1) * TW * CH>();
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  // the Gumbel noise of this wave's rows does not depend on the logits: compute it (VALU) while
  // the chunks stream (after the barrier: with a global_load_lds in flight hipcc would wait for
  // vmcnt(0) at the first use of the control loads)
  int dt[NB];
  bool rec[NB];
  f32x4 gn[TW][NB];
#pragma unroll
  for (int cb = 0; cb < NB; ++cb) {
    const int r = cb * 16 + (lane & 15);
    const HzLmbCtl cl = s_ctl[r];
    dt[cb] = cl.dec_t;
    rec[cb] = cl.rec != 0;
    const unsigned long long sd = s_seed[r];
#pragma unroll
    for (int t = 0; t < TW; ++t)
      gn[t][cb] = dt[cb] >= 0 ? gumbel4(sd, dt[cb], (tile0 + t) * 16 + (lane >> 4) * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  f32x4 acc[TW][NB];
#pragma unroll
  for (int t = 0; t < TW; ++t)
#pragma unroll
    for (int cb = 0; cb < NB; ++cb) acc[t][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int cur = c % RR;  // compile-time after unrolling: register arrays stay registers
#pragma unroll
    for (int s = 0; s < CH; ++s) {
      const int ks = c * CH + s;
#pragma unroll
      for (int cb = 0; cb < NB; ++cb) {
        if (cb >= nba) continue;
        const bf16x8 hi = as_frag(*reinterpret_cast<const u32x4*>(act + ((size_t)(ks * 2 + 0) * NB + cb) * 512 + lane * 8));
#pragma unroll
        for (int t = 0; t < TW; ++t)
          acc[t][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(wr[t][cur][s]), hi, acc[t][cb], 0, 0, 0);
        if constexpr (DIAG != 2) {
          const bf16x8 lo = as_frag(*reinterpret_cast<const u32x4*>(act + ((size_t)(ks * 2 + 1) * NB + cb) * 512 + lane * 8));
#pragma unroll
          for (int t = 0; t < TW; ++t)
            acc[t][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(wr[t][cur][s]), lo, acc[t][cb], 0, 0, 0);
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // chunk c's MFMAs are done with its registers
    if (c + RR < NCH) issue(cur, c + RR);  // refill them with chunk c + RR
    __builtin_amdgcn_sched_barrier(0);
  }
  // ---- epilogue: lane l holds vocabulary rows 16*tile + 4(l>>4) + i of request row cb*16 + (l&15)
  // (4 consecutive ids: one Philox block gives their noise)
  unsigned long long bst[NB];
#pragma unroll
  for (int cb = 0; cb < NB; ++cb) {
    const int r = cb * 16 + (lane & 15);
    unsigned long long b = 0;
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      const int v0 = (tile0 + t) * 16 + (lane >> 4) * 4;
      if (cb >= nba || tile0 + t >= t_hi || v0 >= p.V) continue;
      f32x4 lg = acc[t][cb];
      if (p.bias) lg += bias_t[t];
      if (p.logits && rec[cb])
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (v0 + i < p.V) p.logits[(size_t)r * p.V + v0 + i] = lg[i];
      if (dt[cb] >= 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int v = v0 + i;
          bool ok = v != 0 && v < p.V;
          for (int e = 0; e < p.n_exclude; ++e) ok = ok && v != p.exclude[e];
          if (ok) b = umax64(b, pack_key(lg[i] + gn[t][cb][i], v));
        }
      }
    }
    b = umax64(b, shfl_xor64(b, 16));
    b = umax64(b, shfl_xor64(b, 32));
    bst[cb] = b;
  }
  if (lane < 16)
#pragma unroll
    for (int cb = 0; cb < NB; ++cb) s_best[wave][cb * 16 + lane] = bst[cb];
  __syncthreads();
  if (tid < Bp) {  // this workgroup's best per request row -> the row's running maximum
    unsigned long long b = s_best[0][tid];
#pragma unroll
    for (int w = 1; w < NW; ++w) b = umax64(b, s_best[w][tid]);
    if (b) atomicMax(p.dbest + (size_t)par * Bp + tid, b);
  }
}

// ------------------------------------------------------------------------ admit kernel
// First node of every replay: workgroup r copies row r's control for the U sub-steps from the
// pinned host block and, for a newly admitted request, zeroes the row's recurrent state.
// Host block (ints): [0] parity of sub-step 0; row r at 8 + r * (8 + 4U): admit flag, seed lo/hi,
// out pointer lo/hi, 3 spare, then U HzLmbCtl.
__global__ __launch_bounds__(256) void lmb_admit_kernel(const HzLmbAdmitParams p) {
  const int r = blockIdx.x, tid = threadIdx.x;
  const int RS = 8 + 4 * p.U;
  const int* row = p.block + 8 + (size_t)r * RS;
  __shared__ int s_hdr[8];
  if (tid < 8) s_hdr[tid] = row[tid];
  if (tid < 4 * p.U) reinterpret_cast<int*>(p.ctl)[(size_t)(tid >> 2) * p.Bp * 4 + r * 4 + (tid & 3)] = row[8 + tid];
  if (r == 0 && tid == 0) *p.gpar = p.block[0] & 1;
  __syncthreads();
  if (tid == 0) {
    p.seed[r] = (unsigned long long)(unsigned)s_hdr[1] | ((unsigned long long)(unsigned)s_hdr[2] << 32);
    p.outp[r] = reinterpret_cast<int*>((unsigned long long)(unsigned)s_hdr[3] | ((unsigned long long)(unsigned)s_hdr[4] << 32));
  }
  if (!s_hdr[0]) return;
  const int NB = p.Bp >> 4;
  for (int l = 0; l < p.n_layers; ++l) {
    const int H = p.H[l], Kh = p.Kh[l];
    for (int j = tid; j < H; j += 256) p.c[l][(size_t)r * H + j] = 0.f;
    const size_t img = (size_t)Kh * p.Bp;  // elements of one [Kh/32][NB][64][8] image
    for (int e = tid; e < 4 * Kh; e += 256) {
      const int im = e / Kh, j = e - im * Kh;  // 4 images: parity x hi/lo
      p.h[l][im * img + st_off(j, r, NB)] = 0;
    }
  }
}

}  // namespace

// decoder grid: every CU streams a share (<= 256 workgroups), at most 16 tiles per workgroup
extern "C" int hz_lmb_dec_blocks(int V) {
  const int ntile = (V + 15) / 16;
  return max((ntile + DROWS / 16 - 1) / (DROWS / 16), min(256, (ntile + 1) / 2));
}

extern "C" int hz_lmb_layer_launch(const HzLmbLayerParams* pp, hipStream_t st) {
  const HzLmbLayerParams& p = *pp;
  const bool first = p.emb != nullptr;
  // nb_act: 0 all row blocks, 1 the first one (low-load program), -1 request row 0 only (SOLO)
  if ((p.Bp != 16 && p.Bp != 32) || p.nb_act < -1 || p.nb_act > p.Bp / 16) return -1;
  if (p.Kh % 32 || p.Kx % 32 || p.Kh < p.H || p.R % 16 || p.R < 4 * p.H || !p.w || !p.bias || !p.h || !p.c || !p.gpar)
    return -1;
  const int KS = (p.Kh + p.Kx) / 32;
  if ((KS + LW - 1) / LW > SPW) return -1;
  if (first && (!p.ctl || !p.dbest || !p.outp || p.V < 16)) return -1;
  if (!first && !p.x) return -1;
  // workgroup shape: HIPZAP_LMB_LAYER = "t2" (round 3: 2 tiles x all rows), "t1" (1 tile x all
  // rows) or, at Bp 32, "t3h" (default: 3 tiles x one row block, twin workgroups)
  static const int shape = [] {
    const char* e = getenv("HIPZAP_LMB_LAYER");
    if (e && !strcmp(e, "t1")) return 1;
    if (e && !strcmp(e, "t2")) return 2;
    return 3;
  }();
  const int ntile = p.R / 16;
#define HZ_LMBL(NB, T, NBW, S)                                                                       \
  do {                                                                                               \
    const int groups = (ntile + T - 1) / T;                                                          \
    const dim3 grid(NBW == NB ? groups : 2 * ((groups + 7) / 8 * 8)), block(512);                    \
    if (first && p.embproj) hipLaunchKernelGGL((lmb_layer_kernel<NB, true, T, NBW, true, S>), grid, block, 0, st, p); \
    else if (first) hipLaunchKernelGGL((lmb_layer_kernel<NB, true, T, NBW, false, S>), grid, block, 0, st, p); \
    else hipLaunchKernelGGL((lmb_layer_kernel<NB, false, T, NBW, false, S>), grid, block, 0, st, p); \
  } while (0)
  // one tile per workgroup when the tiles fit the CUs (the last layer, R = 4000: 250 tiles): at low
  // load a workgroup's fetch is its weight tiles plus one row block of state, so fewer tiles per
  // CU is a shorter step
  const bool one = ntile <= 256;
  if (p.nb_act == -1) {
    if (p.Bp == 16) {
      if (one) HZ_LMBL(1, 1, 1, true);
      else HZ_LMBL(1, 2, 1, true);
    } else {
      if (one) HZ_LMBL(2, 1, 2, true);
      else HZ_LMBL(2, 2, 2, true);
    }
  } else if (p.Bp == 16) {
    if (shape == 1) HZ_LMBL(1, 1, 1, false);
    else HZ_LMBL(1, 2, 1, false);
  } else if (p.nb_act == 1) {
    // low-load program: the first row block (64 B of state per k)
    if (one) HZ_LMBL(2, 1, 2, false);
    else HZ_LMBL(2, 2, 2, false);
  } else {
    if (shape == 1) HZ_LMBL(2, 1, 2, false);
    else if (shape == 2) HZ_LMBL(2, 2, 2, false);
    else HZ_LMBL(2, 3, 1, false);
  }
#undef HZ_LMBL
  return (int)hipGetLastError();
}

// decoder weight pipeline: HIPZAP_LMB_DEC_PIPE = "8x2" (default: 8 k-steps per chunk, 2 chunks in
// the ring); experiments build only (measured negatives, profiles/r4_lmb): "4x5" or "4x6" (K = 1024)
// and "8x2nt" (the default ring with non-temporal weight loads)
// HIPZAP_LMB_DEC_TW = 4 (experiments build, measured slower: profiles/r4_lmb): four vocabulary
// tiles per wave, four waves (K = 1024); default 2
static int lmb_dec_tw() {
  static const int v = [] {
    const char* e = getenv("HIPZAP_LMB_DEC_TW");
    return e && !strcmp(e, "4") ? 4 : 2;
  }();
  return v;
}

static int lmb_dec_diag() {
  static const int v = [] {
    const char* e = getenv("HIPZAP_LMB_DEC_DIAG");
    return e ? atoi(e) : 0;
  }();
  return v;
}

static int lmb_dec_pipe() {
  static const int v = [] {
    const char* e = getenv("HIPZAP_LMB_DEC_PIPE");
    if (!e) return 0;
    if (!strcmp(e, "4x5")) return 1;
    if (!strcmp(e, "4x6")) return 2;
    if (!strcmp(e, "8x2nt")) return 3;
    return 0;
  }();
  return v;
}

extern "C" int hz_lmb_dec_launch(const HzLmbDecParams* pp, hipStream_t st) {
  const HzLmbDecParams& p = *pp;
  if ((p.Bp != 16 && p.Bp != 32) || p.nb_act < -1 || p.nb_act > p.Bp / 16) return -1;
  if (p.K % 256 || p.K < 256 || p.K > DKMAX * 32 || p.Vp % 16 || p.Vp < p.V || p.n_exclude < 0 || p.n_exclude > 8)
    return -1;
  if (!p.w || !p.h || !p.gpar || !p.ctl || !p.seed || !p.dbest || p.nblk != hz_lmb_dec_blocks(p.V)) return -1;
  if ((long)p.Vp * p.K * 2 > 0x70000000L) return -1;  // the weight descriptor's 32-bit range (see the kernel)
  const dim3 grid(p.nblk), block(512);
  const int pipe = p.K == 1024 ? lmb_dec_pipe() : 0;
  const int tw = lmb_dec_tw();
  (void)pipe;
  (void)tw;
#define HZ_LMBD(NB, KS, CH, R, ...) hipLaunchKernelGGL((lmb_dec_kernel<NB, KS, CH, R, ##__VA_ARGS__>), grid, block, 0, st, p)
#if HZ_EXPERIMENTS  // measured negatives (profiles/r4_lmb): deeper rings, non-temporal weight loads
#define HZ_LMBD_EXP(NB)                                                   \
  if (pipe == 1) { HZ_LMBD(NB, 32, 4, 5); break; }                         \
  if (pipe == 2) { HZ_LMBD(NB, 32, 4, 6); break; }                         \
  if (pipe == 3) { HZ_LMBD(NB, 32, 8, 2, true); break; }
// four tiles per wave, four waves: +5 us per step (fewer waves hide less of the weight stream);
// HIPZAP_LMB_DEC_DIAG = 1 / 2: the timing-only variants of the kernel's DIAG parameter
#define HZ_LMBD_TW4(NB, S)                                                                          \
  if (tw == 4) {                                                                                   \
    hipLaunchKernelGGL((lmb_dec_kernel<NB, 32, 4, 2, false, S, 4>), grid, dim3(256), 0, st, p);    \
    break;                                                                                         \
  }                                                                                                \
  if (lmb_dec_diag() == 1) {                                                                       \
    hipLaunchKernelGGL((lmb_dec_kernel<NB, 32, 8, 2, false, S, 2, 1>), grid, dim3(512), 0, st, p); \
    break;                                                                                         \
  }                                                                                                \
  if (lmb_dec_diag() == 2) {                                                                       \
    hipLaunchKernelGGL((lmb_dec_kernel<NB, 32, 8, 2, false, S, 2, 2>), grid, dim3(512), 0, st, p); \
    break;                                                                                         \
  }
#else
#define HZ_LMBD_EXP(NB)
#define HZ_LMBD_TW4(NB, S)
#endif
#define HZ_LMBD_K(NB, S)                            \
  switch (p.K / 256) {                              \
    case 1: HZ_LMBD(NB, 8, 8, 2, false, S); break;  \
    case 2: HZ_LMBD(NB, 16, 8, 2, false, S); break; \
    case 3: HZ_LMBD(NB, 24, 8, 2, false, S); break; \
    case 4:                                         \
      if (!S) { HZ_LMBD_EXP(NB) }                   \
      HZ_LMBD_TW4(NB, S)                            \
      HZ_LMBD(NB, 32, 8, 2, false, S);              \
      break;                                        \
    default: return -1;                             \
  }
  if (p.nb_act == -1) {  // the one-request program
    if (p.Bp == 16) {
      HZ_LMBD_K(1, true)
    } else {
      HZ_LMBD_K(2, true)
    }
  } else if (p.Bp == 16) {
    HZ_LMBD_K(1, false)
  } else {
    HZ_LMBD_K(2, false)
  }
#undef HZ_LMBD_K
#undef HZ_LMBD_EXP
#undef HZ_LMBD_TW4
#undef HZ_LMBD
  return (int)hipGetLastError();
}

extern "C" int hz_lmb_embproj_launch(const HzLmbEmbProjParams* pp, hipStream_t st) {
  const HzLmbEmbProjParams& p = *pp;
  if (!p.w || !p.emb || !p.out || p.Kh % 32 || p.Kx % 32 || p.Kx < 32 || p.Kx > EPKS * 32 || p.R % 16 || p.Vp % 16 ||
      p.Vp < 16)
    return -1;
  hipLaunchKernelGGL(lmb_embproj_kernel, dim3((p.Vp / 16 + 7) / 8), dim3(512), 0, st, p);
  return (int)hipGetLastError();
}

extern "C" int hz_lmb_admit_launch(const HzLmbAdmitParams* pp, hipStream_t st) {
  const HzLmbAdmitParams& p = *pp;
  if ((p.Bp != 16 && p.Bp != 32) || p.U < 1 || p.U > HZ_LMB_MAXU || p.n_layers < 1 || p.n_layers > 4) return -1;
  if (!p.block || !p.ctl || !p.seed || !p.outp || !p.gpar) return -1;
  for (int l = 0; l < p.n_layers; ++l)
    if (!p.h[l] || !p.c[l] || p.Kh[l] % 32 || p.H[l] > p.Kh[l]) return -1;
  hipLaunchKernelGGL(lmb_admit_kernel, dim3(p.Bp), dim3(256), 0, st, p);
  return (int)hipGetLastError();
}
