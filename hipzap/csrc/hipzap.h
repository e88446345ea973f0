// hipzap native C ABI (consumed from Python through ctypes: hipzap/_native.py).
// Every struct here is mirrored field-for-field by a ctypes.Structure; keep them in sync.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { HZ_ACT_NONE = 0, HZ_ACT_RELU = 1, HZ_ACT_GELU = 2, HZ_ACT_TANH = 3 };

typedef struct HzConvParams {
  const unsigned short* x;   // input: channel-blocked [N][C/32][H][W][32] (C%32==0) or NHWC (C in {8,16})
  const unsigned short* w;   // fragment-major bf16 weights [Cout_pad/16][ksteps][64][8]; k = (r*S + s)*C + c
  const float* bias;         // fp32 [Cout] or NULL
  const unsigned short* res; // bf16 residual, same layout as out, or NULL
  void* out;                 // bf16 or fp32; channel-blocked, or row-major [M][ldo] if out_rowmajor
  int N, H, W, C;
  int Cout, R, S, stride, pad, P, Q;
  int M, K, ksteps;          // M = N*P*Q; ksteps = ceil(K/32)
  int act, out_f32, out_rowmajor, ldo;
  int x_rowmajor, ldx;        // GEMM mode: activations row-major [M][ldx] (M = N*H*W, 1x1 only)
  int tiles_n;               // filled by the launcher
  int kw;                    // waves per workgroup splitting K
  const struct HzLnFold* lnf; // LDS GEMM only: LayerNorm folded into this GEMM (device memory), or NULL
  // ResNet 1x1 -> 1x1 seams (block.hip seam_kernel; register-ring 3x3 convs only):
  int x_f32;                 // 1: x is fp32 in the same channel-blocked layout (a seam's conv1 sum, its
                             //    folded-BN bias included): ReLU + bf16 applied at the operand load
  int z_C;                   // channels of zinit
  float* zinit;              // or NULL: after its tiles the launch fills zinit [N][z_C/32][z_HW][32] fp32
                             //   with zbias[c] (the NEXT seam's accumulator, before its atomic adds)
  const float* zbias;        // [z_C]
  int z_HW, pad_z;
} HzConvParams;

// Post-LN transformer LayerNorm folded into the neighbouring GEMMs (gemm.hip, BERT). A GEMM
// whose input is LN(y) runs on the raw y with gamma folded into its weights (W' = W diag(gamma),
// c1[n] = sum_k W'[n][k], bias' = bias + W beta) and corrects in the epilogue:
//   out = rstd * (y.W'^T - mean * c1) + bias'
// A GEMM whose residual is LN(y) normalises the residual elementwise. The producing GEMM writes
// per-row partial (sum, sumsq) of its bf16-rounded output, one float2 slab per (N tile, wave
// column): deterministic, no atomics; consumers sum the slabs of a row.
typedef struct HzLnFold {
  const float* stats_in;   // [nslab_in][ld_stats] float2 of the GEMM input rows, or NULL
  const float* c1;         // [Cout] (with stats_in)
  const float* res_stats;  // [nslab_res][ld_stats] float2 of the residual rows, or NULL
  const float* res_gamma;  // [Cout] (with res_stats)
  const float* res_beta;
  float* stats_out;        // [2 * tiles_n][ld_stats] float2 of this GEMM's output rows, or NULL
  int nslab_in, nslab_res, ld_stats;
  float inv_d, eps_in, eps_res;  // inv_d = 1 / LayerNorm width
} HzLnFold;

// cfg 0..8: register-ring tile (FC*16 channels x FP*16 pixels), cfg = log2(FC)*3 + log2(FP);
// cfg 16..19: LDS-tiled GEMM (gemm.hip; row-major activations, K % 64 == 0, weight rows % 128 == 0)
int hz_conv_launch(const HzConvParams* p, int cfg, hipStream_t st);
int hz_gemm_lds_launch(const HzConvParams* p, int cfg, hipStream_t st);
// two independent convs with one shared (cfg, kw) in one launch (grouped; conv.hip conv2_kernel)
int hz_conv2_launch(const HzConvParams* a, const HzConvParams* b, int cfg, hipStream_t st);

// (kind 17, the persistent dependent-conv chain, was removed in round 5: measured negative in
// round 3, profiles/r3_chain)

typedef struct HzPoolParams {
  const unsigned short* x;  // NHWC bf16
  unsigned short* out;      // NHWC bf16
  int N, H, W, C, P, Q, k, stride, pad;
} HzPoolParams;
int hz_maxpool_launch(const HzPoolParams* p, hipStream_t st);
// global average pool NHWC [N,H,W,C] -> [N,C] bf16
// blocked: x is [N][C/32][HW][32] instead of NHWC
int hz_avgpool_launch(const unsigned short* x, unsigned short* out, int N, int HW, int C, int blocked, hipStream_t st);

// fused global-average-pool + classifier (ResNet head):
//   out[b][n] = bias[n] + sum_c W[n][c] * mean_hw x[b][c][hw]
typedef struct HzPoolFcParams {
  const unsigned short* x;  // channel-blocked bf16 [B][C/32][HW][32]
  const unsigned short* w;  // fragment-major bf16 [N_pad/16][C/32][64][8] (pack_linear)
  const float* bias;        // [N]
  float* out;               // fp32 [B][ldo]
  int B, C, HW, N, ldo;
  int pooled, pad_;         // pooled: x is already the fp32 [B][C] channel means (a tail seam's output)
} HzPoolFcParams;
int hz_pool_fc_launch(const HzPoolFcParams* p, hipStream_t st);

// image pre-processing: src NCHW fp32 (mode 0) or NHWC uint8 (mode 1) -> NHWC bf16 with Cpad channels;
// mode 2: src NCHW fp32 -> bf16 patch rows [N * H/P * W/P][Cin * P * P] in (c, ky, kx) order, with
// P = Cpad (16; the ViT patch embedding as a row-major GEMM)
int hz_preprocess_launch(const void* src, unsigned short* dst, int N, int Cin, int H, int W, int Cpad,
                         int mode, const float* mean, const float* inv_std, hipStream_t st);

// elementwise helpers
int hz_cast_f32_bf16(const float* x, unsigned short* y, long n, hipStream_t st);
int hz_cast_bf16_f32(const unsigned short* x, float* y, long n, hipStream_t st);

typedef void* HzProgram;

// ---- AWD-LSTM decode (csrc/lstm.hip) ----
typedef struct HzLstmParams {
  const unsigned short* w;    // [4H][ldk] bf16, gate-interleaved rows (4j+q = gate q of unit j; i,f,g,o)
  const float* bias;          // [4H] fp32 (b_ih + b_hh, same interleave)
  const unsigned short* emb;  // layer 0: embedding [V][lde] bf16 (input gathered by token); else NULL
  int lde;
  int* tok_seq;               // token sequence; step t consumes tok_seq[t]
  const float* x_state;       // layers > 0: previous layer's h_state [2][In]
  float* h_state;             // [2][H] fp32, ping-pong by step parity
  float* c_state;             // [2][H] fp32
  const int* step;            // device step counter: this op runs step t = *step + step_off
  int In, H, ldk;             // ldk = padded In + H (multiple of 64; chunks of 512 are predicated)
  int step_off;
  // layer 0 only, optional (fused sampler): for t >= *n_forced the token of step t is the argmax
  // of the previous step's decoder maxima (the argmax sampler's rule, computed redundantly by
  // every workgroup); workgroup 0 records it in tok_seq[t]. NULL bacc_val: tok_seq[t] is read.
  const int* n_forced;
  const float* bacc_val;      // [nblk] decoder per-workgroup maxima over acceptable rows
  const int* bacc_idx;
  const float* bmax_val;      // [nblk] overall maxima (fallback when no row is acceptable)
  const int* bmax_idx;
  int nblk, V;
  // split mode (pre != NULL; csrc/lstm.hip lstm_x_kernel): w holds W_ih only ([4H][ldk], ldk =
  // In padded to 64) and the recurrent half arrives precomputed by the previous step's decoder
  // kernel: pre[4H] = W_hh . h_{t-1} + b (bias is then unused)
  const float* pre;
  // split mode, layer 0 folded into the layer-1 kernel (xtab != NULL; In = H0): h0_t is rebuilt
  // in every workgroup from xtab[tok] (= W_ih^0 . emb[tok], fp32 [V][4*H0]), pre0 and c0_{t-1};
  // token selection as above (emb unused); workgroup 0 publishes h0_t / c0_t
  const float* xtab;
  const float* pre0;          // [4*H0]
  float* h0_state;            // [2][H0]
  float* c0_state;            // [2][H0]
  int H0, pad0;
} HzLstmParams;
typedef struct HzSamplerParams {
  const float* keys;          // [V] Gumbel-perturbed logits (decoder epilogue)
  int* tok_seq;               // writes tok_seq[t+1] when t+1 >= n_forced
  const int* step;            // this op samples after step t = *step + step_off (no increment:
  int step_off;               //   hz_step_bump_launch advances the counter once per graph)
  int* draws;                 // optional [steps][10] record of the draws
  const int* n_forced;        // device: prompt length (tokens 0..n_forced-1 are given)
  int V, n_exclude;
  int exclude[8];
  const float* bmax_val;      // [nblk] decoder workgroup maxima (value, row)
  const int* bmax_idx;
  int nblk, rpb;              // decoder geometry: workgroup b owns rows [b*rpb, (b+1)*rpb)
  // with draws == NULL: the token is the argmax of the ACCEPTABLE keys (row != 0, not excluded),
  // from the decoder's per-workgroup acceptable maxima; exact for the reference rule (see lstm.hip)
  const float* bacc_val;      // [nblk] or NULL (then the top-10 tournament always runs)
  const int* bacc_idx;
} HzSamplerParams;
typedef struct HzDecoderParams {
  const unsigned short* w;    // [V][ldk] bf16 (tied embedding, K padded)
  const float* bias;          // [V] or NULL
  const float* h_state;       // last layer [2][H]
  const int* step;            // step t = *step + step_off
  int step_off;
  float* logits;              // [V]
  int V, H, ldk;
  float* keys;                // optional [V]: logits + Gumbel(seed, step, row) for the sampler
  const unsigned long long* seed;
  float* bmax_val;            // with keys: [nblk] per-workgroup max key (value, row) -> sampler
  int* bmax_idx;
  int nblk, rpb;              // workgroups and rows per workgroup (hz_decoder_geometry)
  float* bacc_val;            // optional [nblk]: per-workgroup max key over ACCEPTABLE rows
  int* bacc_idx;              //   (row != 0 and not in exclude[]), -inf/INT_MAX if none
  int n_exclude;
  int exclude[8];
  // split LSTM mode: hh_blocks extra workgroups (blockIdx < hh_blocks, before the decoder's)
  // compute the NEXT step's recurrent gate partials hh_out[l] = W_hh^l . h^l_t + b^l, layer l
  // owning workgroups [hh_blk[l], hh_blk[l+1]) of HZ_HH_ROWS rows each
  int n_hh, hh_blocks;
  const unsigned short* hh_w[4];  // [4H][ld] bf16, gate-interleaved like HzLstmParams.w
  const float* hh_b[4];           // [4H]
  const float* hh_h[4];           // the layer's h_state [2][H]
  float* hh_out[4];               // [4H] -> HzLstmParams.pre / pre0
  int hh_H[4], hh_ld[4];
  int hh_blk[5];
} HzDecoderParams;
#define HZ_HH_ROWS 16
// decoder launch geometry for vocabulary V: workgroups and rows per workgroup (contiguous)
void hz_decoder_geometry(int V, int* nblk, int* rpb);
int hz_lstm_cell_launch(const HzLstmParams* p, hipStream_t st);
int hz_decoder_launch(const HzDecoderParams* p, hipStream_t st);
int hz_sampler_launch(const HzSamplerParams* p, hipStream_t st);
// *step += n (one thread): closes a captured run of decode steps
int hz_step_bump_launch(int* step, int n, hipStream_t st);

// ---- batched AWD-LSTM decode (csrc/lmbatch.hip + csrc/lmserve.cpp) ----
// Continuous batching for concurrent GET /inference: Bp (16 or 32) request rows share every
// decode step, so each weight byte is read once per step for all of them. Weights and the
// recurrent state are fragment-major for mfma_f32_16x16x32_bf16: W as the A operand
// ([R/16][K/32][64 lanes][8], lane l = row l&15, k 8(l>>4)..+7) and h as the B operand
// ([K/32][Bp/16][64][8], lane l = request row l&15). h is kept as a bf16 hi/lo pair (hi = bf16(h),
// lo = bf16(h - hi)): two MFMAs per fragment give ~16 mantissa bits of the fp32 state.
// Per-step control comes from the host scheduler (row step, forced prompt token or sample, where
// the token goes): the admit kernel copies it from a pinned host block at each replay start.
#define HZ_LMB_MAXU 32
typedef struct HzLmbCtl {     // one (sub-step u, row r) entry, computed by the host
  int tok;                    // >= 0: forced (prompt) token; -1: sample from the last decoder; -2: idle row
  int out;                    // sampled token's index in the request's output (-1: none)
  int dec_t;                  // decoder: step t whose next token is sampled (noise counter), -1: no keys
  int rec;                    // decoder: 1 = record this row's logits (tests)
} HzLmbCtl;
typedef struct HzLmbLayerParams {
  const unsigned short* w;    // [R/16][(Kh+Kx)/32][64][8] bf16, K order [h_prev | x], rows 4j+q (gate q of unit j)
  const float* bias;          // [R] fp32 (b_ih + b_hh, same interleave)
  unsigned short* h;          // this layer's state [2 parity][2 hi/lo][Kh/32][Bp/16][64][8] bf16
  const unsigned short* x;    // layers > 0: the previous layer's h buffers (its Kh = this Kx)
  float* c;                   // [Bp][H] fp32 cell state
  const int* gpar;            // device: h parity of the graph's first sub-step
  const HzLmbCtl* ctl;        // [U][Bp] (first layer)
  int H, Kh, Kx, R, Bp, step_off;
  // first layer: the token of each row (forced, or the argmax of the previous decoder's maxima)
  // and its embedding as the x operand
  const unsigned short* emb;  // [Vp/16][Kx/32][64][8] fragment-major embedding (NULL: not first)
  unsigned long long* dbest;  // [2 parity][Bp] running maxima (packed key, row) of the decoder; the
  int V;                      //   first layer reads the other parity and clears its own
  int nb_act;                 // row blocks (of 16) computed: 0 = all Bp/16; 1 = rows 0..15 only (the
                              //   low-load program: every busy row is below 16); -1 = request row 0
                              //   only (the one-request program: no other row's state read or written)
  int* const* outp;           // [Bp] request output arrays (pinned host, written by workgroup 0)
  int* tok;                   // [Bp] this step's tokens (device, diagnostics)
  const float* embproj;       // first layer: [Vp][R] fp32 W_ih E[v] (hz_lmb_embproj_launch) or NULL
} HzLmbLayerParams;
typedef struct HzLmbEmbProjParams {  // P[v][r] = sum_k W[r][Kh + k] emb[v][k]
  const unsigned short* w;    // the first layer's packed weights [R/16][(Kh+Kx)/32][64][8]
  const unsigned short* emb;  // [Vp/16][Kx/32][64][8]
  float* out;                 // [Vp][R]
  int R, Kh, Kx, Vp;
} HzLmbEmbProjParams;
typedef struct HzLmbDecParams {
  const unsigned short* w;    // [Vp/16][K/32][64][8] bf16 (tied embedding when untied weights are absent)
  const float* bias;          // [Vp] or NULL
  const unsigned short* h;    // last layer's h buffers (Kh = K)
  const int* gpar;
  const HzLmbCtl* ctl;        // [U][Bp]
  const unsigned long long* seed;  // [Bp]
  unsigned long long* dbest;  // [2 parity][Bp]: atomic max over acceptable ids -> the next first layer
  float* logits;              // [Bp][V] (recorded rows only) or NULL
  int V, Vp, K, Bp, nblk, step_off, n_exclude;
  int nb_act;                 // as HzLmbLayerParams::nb_act
  int exclude[8];
} HzLmbDecParams;
typedef struct HzLmbAdmitParams {
  const int* block;           // pinned host block (csrc/lmserve.cpp layout)
  HzLmbCtl* ctl;              // [U][Bp] device
  unsigned long long* seed;   // [Bp]
  int** outp;                 // [Bp]
  int* gpar;
  int Bp, U, n_layers, pad_;
  unsigned short* h[4];       // per layer: h buffers (zeroed for an admitted row)
  float* c[4];                // [Bp][H]
  int Kh[4], H[4];
} HzLmbAdmitParams;
int hz_lmb_layer_launch(const HzLmbLayerParams* p, hipStream_t st);
int hz_lmb_dec_launch(const HzLmbDecParams* p, hipStream_t st);
int hz_lmb_admit_launch(const HzLmbAdmitParams* p, hipStream_t st);
int hz_lmb_embproj_launch(const HzLmbEmbProjParams* p, hipStream_t st);
int hz_lmb_dec_blocks(int V);  // decoder workgroups (256 vocabulary rows each)
// scheduler: one worker thread replays the captured U-step program(s); requests join free rows
// at replay boundaries and leave when their last token is out (csrc/lmserve.cpp). Two programs
// (each reading its own host block and recording into its own logits buffer): pipelined replays.
void* hz_lmb_create(const HzProgram* progs, int nprog, hipStream_t st, int* const* blocks, int Bp, int U, int maxp,
                    int maxn, int* out_pool, float* const* logits, int V);
int hz_lmb_submit(void* s, const int* prompt, int P, int n, unsigned long long seed, int* out, float* logits_out,
                  double* lat_us);
void hz_lmb_stats(void* s, unsigned long long* out4);  // replays, served, row-steps used, row-steps total
int hz_lmb_set_lowload(void* s, const HzProgram* lo, int rows);  // programs for replays whose busy rows are < rows
unsigned long long hz_lmb_lo_replays(void* s);
int hz_lmb_set_solo(void* s, const HzProgram* solo);  // programs for replays whose only busy row is row 0
unsigned long long hz_lmb_solo_replays(void* s);
void hz_lmb_destroy(void* s);

// ---- device-side packing of raw checkpoint tensors (csrc/pack.hip; torch-free .pth cold start) ----
typedef struct HzPackConvParams {
  const float* w;             // OIHW fp32, contiguous (a Linear weight is [cout][cin] with r = s = 1)
  const float* gamma;         // eval BatchNorm (fp32 [cout]) to fold, or NULL
  const float* beta;
  const float* mean;
  const float* var;
  const float* bias_in;       // [cout] or NULL
  unsigned short* wf;         // packed bf16 [rows/16][ksteps][64][8]
  float* bias_out;            // [cout] fp32
  int cout, cin, r, s, cin_p, rows, ksteps, pad_;
  double eps;
} HzPackConvParams;
int hz_pack_conv_launch(const HzPackConvParams* p, hipStream_t st);
int hz_conv_code_warm(void);    // load conv.hip / vision.hip device code (no launch)
int hz_vision_code_warm(void);
int hz_gemm_code_warm(void);
int hz_transformer_code_warm(void);
int hz_fp8_code_warm(void);
int hz_pack_code_warm(void);
// fp32 row-major source(s) -> bf16 fragment-major [R/16][K/32][64][8] (+ an fp32 bias row), the
// batched AWD-LSTM packing (engine/lmbatch.py pack_lmb) on the device: output row r reads source
// row r, or (interleave_h = H > 0) row (r & 3) * H + (r >> 2) (unit-major gates); output column k
// reads a[src][k] for k < ka (zero at k >= acols) and b[src][k - ka] beyond (zero at >= bcols);
// source rows >= nrows and absent segments are zeros. out == NULL: bias only.
typedef struct HzFragPackParams {
  const float* a;
  const float* b;
  unsigned short* out;
  const float* bias_a;  // bias_out[r] = bias_a[src] (+ bias_b[src]), zero beyond the source rows
  const float* bias_b;
  float* bias_out;
  int R, K, nrows, interleave_h, ka, acols, lda, bcols, ldb, pad_;
} HzFragPackParams;
int hz_frag_pack_launch(const HzFragPackParams* p, hipStream_t st);
// file byte ranges -> device memory (csrc/plan.cpp): pread into two pinned staging buffers, DMA
// chunk i while reading chunk i+1; synchronous on `st`
int hz_upload_file(const char* path, int n, const uint64_t* file_off, const uint64_t* nbytes, void* const* dst,
                   void* st);

// ---- FP8 (OCP e4m3fn) path (csrc/fp8.hip) ----
typedef struct HzQuantParams {
  const unsigned short* x;    // [rows][ldx] bf16
  unsigned char* out;         // [rows][ldo] fp8 e4m3fn
  float* scale;               // [rows] fp32 (amax/448)
  int rows, D, ldx, ldo;
} HzQuantParams;
typedef struct HzGemmFp8Params {
  const unsigned char* x;     // [M][ldx] fp8
  const float* sx;            // [M] row scales
  const unsigned char* w;     // fragment-major fp8 [N_pad/16][ksteps][64][8]
  const float* sw;            // [N_pad] per-channel scales
  const float* bias;          // [N] or NULL
  const unsigned short* res;  // [M][ldo] bf16 or NULL
  void* out;                  // [M][ldo] bf16 or fp32
  int M, N, K, ksteps, ldx, ldo;
  int act, out_f32, cfg, kw;
  const unsigned char* wmx;   // MX-packed weights [N_pad/16][K/128][2][64][16] (cfg 16..23) or NULL
  // MX8 activations (OCP MX: e4m3 + one E8M0 power-of-two scale per 32 consecutive k), cfg >= 16:
  const unsigned char* xs;    // input block scales [M][K/32] (then sx may be NULL) or NULL
  unsigned char* out8;        // MX8 output instead of `out`: e4m3 [M][ldo] ...
  unsigned char* os8;         //   ... and E8M0 scales [M][ldo/32]
} HzGemmFp8Params;
int hz_quant_launch(const HzQuantParams* p, hipStream_t st);
int hz_gemm_fp8_launch(const HzGemmFp8Params* p, hipStream_t st);

// ---- transformer kernels (csrc/transformer.hip) ----
typedef struct HzLayerNormParams {
  const unsigned short* x;    // [rows][ldx] bf16
  const unsigned short* res;  // optional residual [rows][ldr] (added before the norm)
  unsigned short* out;        // [rows][ldo] bf16
  const float* gamma;
  const float* beta;
  int rows, D, ldx, ldr, ldo;
  float eps;
  unsigned char* out8;        // optional fused per-row fp8 quantisation of the output [rows][D]
  float* scale8;              //   and its row scales (amax / 448); out may then be NULL
} HzLayerNormParams;
typedef struct HzEmbedParams {
  const int* ids;             // [rows] token ids (rows = B*L)
  const int* types;           // [rows] token-type ids or NULL
  const unsigned short* word; // [V][D]
  const unsigned short* pos;  // [Lmax][D]
  const unsigned short* type; // [2][D]
  const float* gamma;
  const float* beta;
  unsigned short* out;        // [rows][D]
  int rows, L, D;
  float eps;
  int vocab, ntypes;          // table rows: ids / types are clamped into range (a bad request id
                              // cannot read outside the tables; the servers also reject it)
} HzEmbedParams;
typedef struct HzAttentionParams {
  const unsigned short* qkv;  // [B*L][ldqkv]: Q at col h*64, K at +k_off, V at +v_off
  const float* mask;          // additive per-key mask [B][L] or NULL
  unsigned short* out;        // [B*L][ldo], head h at col h*64
  int B, L, heads, head_dim, ldqkv, k_off, v_off, ldo;
  float scale;
  unsigned char* out8;        // optional MX8 output (e4m3 [B*L][ldo] + E8M0 [B*L][ldo/32]) instead of out
  unsigned char* os8;
} HzAttentionParams;
typedef struct HzVitTokensParams {
  const unsigned short* patches;  // [B*np][D]
  const unsigned short* cls;      // [D]
  const unsigned short* pos;      // [np+1][D]
  unsigned short* out;            // [B][np+1][D]
  int B, np, D;
} HzVitTokensParams;
int hz_layernorm_launch(const HzLayerNormParams* p, hipStream_t st);
int hz_embed_ln_launch(const HzEmbedParams* p, hipStream_t st);
int hz_attention_launch(const HzAttentionParams* p, hipStream_t st);
// QKV projection + self-attention in one launch (transformer.hip qkvatt_kernel): one workgroup per
// (sequence, head), L <= 128, head_dim 64; the QKV GEMM's own weight packing and bias
typedef struct HzQkvAttParams {
  const unsigned short* x;    // [B*L][ldx] bf16 (the layer input)
  const unsigned short* w;    // packed QKV weights [3D/16][D/32][64][8] (rows: Q 0..D-1, K D.., V 2D..)
  const float* bias;          // [3D]
  const float* mask;          // additive per-key mask [B][L] or NULL
  unsigned short* out;        // [B*L][ldo] context, head h at column h*64
  int B, L, heads, D, ksteps, ldx, ldo;
  float scale;
} HzQkvAttParams;
int hz_qkvatt_launch(const HzQkvAttParams* p, hipStream_t st);
int hz_vit_tokens_launch(const HzVitTokensParams* p, hipStream_t st);

// row softmax: out[r][i] = exp(s*x[r][i] + mask[i] - m_r) / sum_i(...), i < D
typedef struct HzSoftmaxParams {
  const void* x;       // [rows][ldx] fp32 (x_bf16 = 0) or bf16
  const float* mask;   // optional additive [D] mask
  float* out;          // [rows][ldo] fp32
  int rows, D, ldx, ldo, x_bf16;
  float scale;
} HzSoftmaxParams;
int hz_softmax_launch(const HzSoftmaxParams* p, hipStream_t st);

// ---- fused ResNet stages (csrc/block.hip; bs=1 dispatch count) ----
// stem: image -> normalise -> 7x7/2 conv (packed like conv1: cin_pad 8, 13 k-steps) + bias + ReLU ->
// 3x3/2 max-pool pad 1, channel-blocked output; one launch instead of preprocess + conv + maxpool
typedef struct HzStemParams {
  const void* src;            // uint8 NHWC [N][H][W][3] (mode 1), fp32 NCHW [N][3][H][W] (mode 0), or bf16
                              // NHWC [N][H][W][8] already normalised (mode 2: after the preprocess kernel)
  const unsigned short* w;    // fragment-major [4][13][64][8], k = (r*7 + s)*8 + c
  const float* bias;          // [64]
  unsigned short* out;        // [N][2][PH][PW][32]
  int N, H, W, mode;
  int SH, SW, PH, PW;         // stem output / pooled sizes
  int norm, pad_;             // norm: (x - mean) * inv_std (mode 1 scales bytes by 1/255 first)
  float mean[4], inv_std[4];
} HzStemParams;
// one bottleneck block at layer1 geometry (Cmid 64, Cout 256, stride 1): conv1 1x1 -> conv2 3x3 ->
// conv3 1x1 + residual (identity when wd == NULL, else the 1x1 downsample) + ReLU, each workgroup an
// 8x8 output tile recomputing its conv1 halo; H, W multiples of 8
typedef struct HzBneckParams {
  const unsigned short* x;    // [N][Cin/32][H][W][32]
  const unsigned short* w1;   // packed as the per-conv kernels (fragment-major, K order (r, s, c))
  const float* b1;
  const unsigned short* w2;
  const float* b2;
  const unsigned short* w3;
  const float* b3;
  const unsigned short* wd;   // downsample (layer1: Cin 64; layer2: Cin 256, stride 2) or NULL (identity)
  const float* bd;
  unsigned short* out;        // [N][Cout/32][H][W][32]
  int N, H, W, Cin, Cmid, Cout;  // H, W: the block's OUTPUT size (the input is 2H x 2W for the
                                 //   stride-2 first block of layer2)
  int tile_h;                 // layer1 output tile rows: 8 (default when 0) or 4 (twice the workgroups)
  int imgs;                   // layer2 images per workgroup: 0 auto (2 at an even N >= 8), 1, 2
} HzBneckParams;
// ResNet 1x1 -> 1x1 seam at 14x14 / 7x7 (layer3 / layer4, bs=1): conv3 of block i (1x1 CM -> 4CM,
// + residual + ReLU) and the K-split conv1 of block i+1 (1x1 4CM -> CM) in ONE launch. A workgroup
// owns (pixel tile <= 32, slice of cs of the 4CM channels): it computes that slice of y = relu(W3 t2
// + b3 + res) over the full K, stores it, and adds W1[:, slice] . y_slice into the fp32 accumulator z
// (no-return float atomics; z was set to conv1's bias by the launch before, see HzConvParams.zinit);
// block i+1's 3x3 conv reads z with ReLU at its operand load (HzConvParams.x_f32). No workgroup
// waits for another: the conv1 reduction happens in the memory-side atomic units.
typedef struct HzSeamParams {
  const unsigned short* t2;   // conv3 input [N][CM/32][HW][32] bf16
  const unsigned short* w3;   // conv3 weights, packed as the per-conv kernels ([4CM/16][CM/32][64][8])
  const float* b3;            // [4CM]
  const unsigned short* res;  // residual [N][4CM/32][HW][32]
  unsigned short* y;          // block output [N][4CM/32][HW][32]
  const unsigned short* w1;   // next conv1 weights [CM/16][4CM/32][64][8]
  float* z;                   // next conv1 accumulator [N][CM/32][HW][32] fp32, preset to its bias
  int N, HW, CM, cs;          // cs: slice width (64 or 128)
  int tiles, t2_f32;          // tiles: pixel tiles per image (launcher: ceil(HW / 32)); t2_f32: t2 is the
                              //   fp32 accumulator of a K-split 3x3 conv (ReLU applied at the load)
  float* zinit;               // or NULL: afterwards filled with zbias per channel ([N][z_C/32][z_HW][32]):
  const float* zbias;         //   the next K-split 3x3 conv's accumulator
  int z_C, z_HW;
  int tail, pad_;             // tail: the last block -- conv3 + global average pool, no conv1 half (w1, z
                              //   unused): fp32 [N][4CM] means into y's buffer (HW <= 64, CM 512)
  int cn;                     // conv1 outputs (0: CM); 512 at CM 256 = the layer3 -> layer4 seam
  int ds;                     // 1: the residual is the stride-2 1x1 downsample of xd (res unused):
  const unsigned short* xd;   //   [N][2CM/32][xd_H][xd_W][32] bf16, the stage input
  const unsigned short* wd;   //   packed like the per-conv kernels ([4CM/16][2CM/32][64][8])
  const float* bd;            //   [4CM]
  int xd_H, xd_W;
} HzSeamParams;
// K-split 3x3 conv (pad 1, stride 1 at <= 14 x 14 or stride 2 from <= 28 x 28) into an fp32
// accumulator (block.hip kconv_kernel):
// a workgroup owns (image, 32 output channels, a slice of ck input channels): it stages that slice of
// the whole image (+ zero halo) in LDS once -- bf16, or fp32 with the ReLU applied (x_f32: a seam's
// conv1 sum) -- multiplies all 9 taps from LDS (mfma 32x32x16, pixels on the A rows) and adds its
// partial into `out` by float atomics (out preset to the conv's bias by the launch before; the
// consumer applies the ReLU when it loads out). Each input byte is read from L2 once per workgroup
// instead of once per tap; the weight stream is split over C/ck workgroups per channel tile.
typedef struct HzKconvParams {
  const void* x;              // [N][C/32][H][W][32] fp32 (x_f32) or bf16
  const unsigned short* w;    // packed as the per-conv kernels: [Cout/16][9C/32][64][8], k = (r*3 + s)*C + c
  float* out;                 // [N][Cout/32][H][W][32] fp32, preset to the bias
  float* zinit;               // or NULL: filled with zbias per channel afterwards, as HzConvParams.zinit
  const float* zbias;
  int z_C, z_HW;
  int N, H, W, C, Cout, x_f32;  // H, W: the INPUT size (the output is H/stride x W/stride)
  int ck, stride;             // input channels per workgroup: 32, 64 or 128; stride 1 or 2
  // optional second job of the launch (dso != NULL): the block's stride-2 1x1 downsample, in its
  // own workgroups (32 output channels x <= 64 output pixels, full K): dso = dsw dsx(2y, 2x) + dsb
  const unsigned short* dsx;  // [N][ds_C/32][ds_H][ds_W][32] bf16
  const unsigned short* dsw;  // packed [ds_Cout/16][ds_C/32][64][8]
  const float* dsb;           // [ds_Cout]
  unsigned short* dso;        // [N][ds_Cout/32][ds_H/2][ds_W/2][32] bf16
  int ds_C, ds_Cout, ds_H, ds_W;
} HzKconvParams;
int hz_stem_launch(const HzStemParams* p, hipStream_t st);
int hz_bneck_launch(const HzBneckParams* p, hipStream_t st);
int hz_seam_launch(const HzSeamParams* p, hipStream_t st);
int hz_kconv_launch(const HzKconvParams* p, hipStream_t st);
int hz_block_code_warm(void);

// generic program op: kind selects the launcher, params are copied into the program
enum { HZ_K_CONV = 1, HZ_K_LAYERNORM = 2, HZ_K_EMBED = 3, HZ_K_ATTENTION = 4, HZ_K_VIT_TOKENS = 5,
       HZ_K_LSTM = 6, HZ_K_DECODER = 7, HZ_K_SAMPLER = 8, HZ_K_MAXPOOL = 9, HZ_K_QUANT = 10, HZ_K_GEMM_FP8 = 11,
       HZ_K_SOFTMAX = 12, HZ_K_POOL_FC = 13, HZ_K_LMB_LAYER = 14, HZ_K_LMB_DEC = 15,
       HZ_K_LMB_ADMIT = 16, /* 17: removed */ HZ_K_STEM = 18, HZ_K_BNECK = 19, HZ_K_SEAM = 20, HZ_K_KCONV = 21,
       HZ_K_QKVATT = 22 };
int hz_launch_kernel(int kind, const void* params, hipStream_t st);
int hz_experiments(void);  // 1: built with HZ_EXPERIMENTS (measured-negative kernel variants)
size_t hz_kernel_param_size(int kind);  // 0: unknown kind
int hz_prog_add_kernel(HzProgram p, int kind, const void* params, size_t size, int slot);

// ---- runtime: static op programs, graph capture / replay ----
HzProgram hz_prog_create(void);
void hz_prog_destroy(HzProgram p);
int hz_prog_num_ops(HzProgram p);
int hz_prog_add_conv(HzProgram p, const HzConvParams* cp, int cfg, int slot);
int hz_prog_add_conv2(HzProgram p, const HzConvParams* a, const HzConvParams* b, int cfg, int slot);
int hz_prog_add_maxpool(HzProgram p, const HzPoolParams* pp, int slot);
int hz_prog_add_avgpool(HzProgram p, const unsigned short* x, unsigned short* out, int N, int HW, int C, int blocked,
                        int slot);
int hz_prog_add_preprocess(HzProgram p, const void* src, unsigned short* dst, int N, int Cin, int H, int W,
                           int Cpad, int mode, const float* mean, const float* inv_std, int slot);
int hz_prog_add_memcpy(HzProgram p, void* dst, const void* src, size_t bytes, int slot);  // any direction (UVA)
int hz_prog_add_lstm(HzProgram p, const HzLstmParams* lp, int slot);
int hz_prog_add_decoder(HzProgram p, const HzDecoderParams* dp, int slot);
int hz_prog_add_sampler(HzProgram p, const HzSamplerParams* sp, int slot);
int hz_prog_add_step_bump(HzProgram p, int* step, int n, int slot);
int hz_prog_add_fork(HzProgram p, int slot);   // side stream `slot` waits for main
int hz_prog_add_join(HzProgram p, int slot);   // main waits for side stream `slot`
int hz_prog_run(HzProgram p, hipStream_t st);  // eager launch of every op
int hz_prog_capture(HzProgram p, hipStream_t st);
int hz_prog_replay(HzProgram p, hipStream_t st);
int hz_prog_is_captured(HzProgram p);
// make the side streams / fork events a run needs (before a lazy capture races a replay)
int hz_prog_prepare(HzProgram p);
int hz_prog_replay_n(HzProgram p, hipStream_t st, int n);  // n back-to-back replays, no sync
// replay `n` programs round-robin on `n` streams `iters` times from C++ and synchronize;
// returns elapsed microseconds (host wall, includes the final sync) or negative on error.
double hz_prog_bench(HzProgram* progs, hipStream_t* streams, int n, int iters);
int hz_prog_bench2(HzProgram* progs, hipStream_t* streams, int n, int iters, int threads, double* out);
// closed-loop serving benchmark (one host thread per context; per-request latency in lat_us[n*iters])
int hz_serve_bench(HzProgram* progs, hipStream_t* streams, void** in_dst, void** in_src, uint64_t in_bytes,
                   void** out_src, void** out_dst, uint64_t out_bytes, int n, int iters, double* lat_us,
                   double* wall_us);
// diagnostics (csrc/diag.hip): kind 0 = no-op kernel, 1 = copy `bytes` from a to b
int hz_diag_launch(int kind, int blocks, int threads, void* a, void* b, long bytes, hipStream_t st);
int hz_prog_add_diag(HzProgram p, int kind, int blocks, int threads, void* a, void* b, long bytes, int slot);

// ---- plan images (csrc/plan.cpp, engine/plan.py): serialised bound programs ----
// bump HZ_ABI_EPOCH when a kernel's parameter SEMANTICS change without a size change
#define HZ_ABI_EPOCH 2
enum { HZ_PLAN_OP_CONV = 1, HZ_PLAN_OP_CONV2 = 2, HZ_PLAN_OP_MAXPOOL = 3, HZ_PLAN_OP_AVGPOOL = 4,
       HZ_PLAN_OP_PREPROCESS = 5, HZ_PLAN_OP_MEMCPY = 6, HZ_PLAN_OP_KERNEL = 7, HZ_PLAN_OP_FORK = 8,
       HZ_PLAN_OP_JOIN = 9 };
// argument records of the ops whose hz_prog_add_* takes scalars
typedef struct HzAvgpoolArgs {
  const unsigned short* x;
  unsigned short* out;
  int N, HW, C, blocked;
} HzAvgpoolArgs;
typedef struct HzPreprocessArgs {
  const void* src;
  unsigned short* dst;
  const float* mean;
  const float* inv_std;
  int N, Cin, H, W, Cpad, mode;
} HzPreprocessArgs;
typedef struct HzMemcpyArgs {
  void* dst;
  const void* src;
  uint64_t bytes;
} HzMemcpyArgs;
// load-phase timings (ms) reported by hz_plan_open / hz_plan_timings
enum { HZ_PLAN_T_PARSE = 0, HZ_PLAN_T_HIP_INIT = 1, HZ_PLAN_T_UPLOAD = 2, HZ_PLAN_T_CTX_ALLOC = 3,
       HZ_PLAN_T_BIND = 4, HZ_PLAN_T_CAPTURE = 5, HZ_PLAN_T_BLOB_ALLOC = 6,
       HZ_PLAN_T_FIRST_COPY = 7,
       // sub-phases of HZ_PLAN_T_UPLOAD (cold-start phase table): stream creation, the blob's
       // read + DMA, the wait for the device-code warm thread; and that thread's own duration
       HZ_PLAN_T_STREAM = 8, HZ_PLAN_T_UPLOAD_DMA = 9, HZ_PLAN_T_WARM_WAIT = 10, HZ_PLAN_T_WARM_THREAD = 11,
       HZ_PLAN_NT = 12 };
uint64_t hz_abi_version(void);
const char* hz_plan_last_error(void);
// read_blob = 0: allocate the weight blob but leave it unfilled (an RCCL broadcast fills it)
void* hz_plan_open(const char* path, int device, int read_blob, double* timings);
int hz_plan_add_contexts(void* plan, int n, int capture);
int hz_plan_num_contexts(void* plan);
// contexts added after this call (except one on the upload stream) get highest-priority streams
void hz_plan_set_stream_priority(void* plan, int high);
void hz_plan_timings(void* plan, double* out);
void* hz_plan_blob(void* plan, uint64_t* bytes);
void* hz_plan_host(void* plan, int ctx);
void* hz_plan_device(void* plan, int ctx);
void* hz_plan_stream(void* plan, int ctx);
void* hz_plan_upload_stream(void* plan);
int hz_plan_replay(void* plan, int ctx);
int hz_plan_sync(void* plan, int ctx);
int hz_plan_infer(void* plan, int ctx, const void* in, uint64_t in_off, uint64_t in_bytes, void* out,
                  uint64_t out_off, uint64_t out_bytes);
double hz_plan_bench(void* plan, int iters);
HzProgram hz_plan_prog(void* plan, int ctx);
int hz_plan_capture_ctx(void* plan, int ctx);

// ---- request executor (csrc/executor.cpp): one worker thread submits + polls completions ----
// host_in[k * n + i] = context i's pinned input k (n_in <= 4); host_out[i] = its pinned output
void* hz_exec_create(HzProgram* progs, hipStream_t* streams, void** host_in, const uint64_t* in_bytes, int n_in,
                     void** host_out, uint64_t out_bytes, int n);
// blocking: one request (in[k] = payload of input k), result copied to out; latency in *lat_us
void* hz_exec_create_batched(HzProgram* progs, hipStream_t* streams, void** host_in, const uint64_t* in_bytes,
                             int n_in, void** host_out, uint64_t out_bytes, int n, int rows, double max_wait_us,
                             int min_inflight);
void hz_exec_batches(void* exec, uint64_t* batches);
int hz_exec_submit(void* exec, const void* const* in, void* out, double* lat_us);
int hz_exec_submit_rows(void* exec, const void* const* in, int m, void* out, double* lat_us);
void hz_exec_stats(void* exec, uint64_t* served, uint64_t* polls);
void hz_exec_destroy(void* exec);
int hz_exec_bench(void* exec, int clients, int iters, const void* const* in, double* lat_us, double* wall_us);

// ---- native HTTP/1.1 front end (csrc/http.cpp): POST /predict fast path + WSGI callback ----
typedef void (*HzHttpPyHandler)(void* req, const char* method, const char* target, const char* headers,
                                uint64_t hlen, const char* body, uint64_t blen);
void* hz_http_start(int listen_fd, HzHttpPyHandler py);
int hz_http_set_fast(void* srv, void* exec, int H, int W, int C, int out_floats, int classes, int probs,
                     const char* model);
// the native GET /inference route (csrc/http.cpp try_lm); sched = NULL removes it
int hz_http_set_lm(void* srv, void* sched, int V, int maxn, int dflt, int empty_id, const char* blob, uint64_t blen,
                   const uint8_t* flags);
void hz_http_respond(void* req, int status, const char* headers, uint64_t hlen, const char* body, uint64_t blen);
void hz_http_stats(void* srv, uint64_t* out4);
int hz_http_stop(void* srv);  // 1: all connections ended; 0: some still live (state leaked)
void hz_plan_close(void* plan);

#ifdef __cplusplus
}
#endif
