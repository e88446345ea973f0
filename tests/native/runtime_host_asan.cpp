// Host-side AddressSanitizer / UBSan check of the native runtime (csrc/runtime.cpp): the
// Program container, parameter capture by value, op ordering, slot validation and teardown.
// Every kernel launcher is replaced by a recording stub, so the test needs no GPU and runs in
// the CPU CI (tests/test_native_asan_cpu.py builds it with -Xarch_host -fsanitize=...).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "hipzap.h"

static std::vector<int> g_calls;  // launch kinds in execution order
static std::vector<int> g_vals;   // one identifying field per call

#define STUB(name, T, kind, field)                \
  extern "C" int name(const T* p, hipStream_t) { \
    g_calls.push_back(kind);                      \
    g_vals.push_back((int)p->field);              \
    return 0;                                     \
  }
STUB(hz_maxpool_launch, HzPoolParams, 2, C)
STUB(hz_pool_fc_launch, HzPoolFcParams, 3, N)
STUB(hz_lstm_cell_launch, HzLstmParams, 4, H)
STUB(hz_decoder_launch, HzDecoderParams, 5, V)
STUB(hz_sampler_launch, HzSamplerParams, 6, V)
STUB(hz_quant_launch, HzQuantParams, 7, rows)
STUB(hz_gemm_fp8_launch, HzGemmFp8Params, 8, M)
STUB(hz_layernorm_launch, HzLayerNormParams, 9, rows)
STUB(hz_embed_ln_launch, HzEmbedParams, 10, L)
STUB(hz_attention_launch, HzAttentionParams, 11, L)
STUB(hz_vit_tokens_launch, HzVitTokensParams, 12, B)
extern "C" int hz_softmax_launch(const HzSoftmaxParams* p, hipStream_t) {
  g_calls.push_back(13);
  g_vals.push_back(p->rows);
  return p->rows < 0 ? 7 : 0;  // a negative row count: a failing launch
}
STUB(hz_lmb_layer_launch, HzLmbLayerParams, 14, H)
STUB(hz_lmb_dec_launch, HzLmbDecParams, 15, V)
STUB(hz_lmb_admit_launch, HzLmbAdmitParams, 16, Bp)
STUB(hz_stem_launch, HzStemParams, 18, N)
STUB(hz_bneck_launch, HzBneckParams, 19, N)
STUB(hz_seam_launch, HzSeamParams, 20, N)
STUB(hz_kconv_launch, HzKconvParams, 21, N)
STUB(hz_qkvatt_launch, HzQkvAttParams, 22, B)
extern "C" int hz_step_bump_launch(int*, int n, hipStream_t) {
  g_calls.push_back(18);
  g_vals.push_back(n);
  return 0;
}
extern "C" int hz_conv_launch(const HzConvParams* p, int cfg, hipStream_t) {
  g_calls.push_back(1);
  g_vals.push_back(p->K * 100 + cfg);
  return 0;
}
extern "C" int hz_conv2_launch(const HzConvParams* a, const HzConvParams* b, int cfg, hipStream_t) {
  g_calls.push_back(14);
  g_vals.push_back(a->K + b->K + cfg);
  return 0;
}
extern "C" int hz_avgpool_launch(const unsigned short*, unsigned short*, int N, int, int, int, hipStream_t) {
  g_calls.push_back(15);
  g_vals.push_back(N);
  return 0;
}
extern "C" int hz_preprocess_launch(const void*, unsigned short*, int N, int, int, int, int, int, const float*,
                                    const float*, hipStream_t) {
  g_calls.push_back(16);
  g_vals.push_back(N);
  return 0;
}
extern "C" int hz_diag_launch(int kind, int, int, void*, void*, long, hipStream_t) {
  g_calls.push_back(17);
  g_vals.push_back(kind);
  return kind == 99 ? 7 : 0;  // kind 99: a failing launch
}

#define CHECK(c)                                                \
  do {                                                          \
    if (!(c)) {                                                 \
      fprintf(stderr, "CHECK failed line %d: %s\n", __LINE__, #c); \
      return 1;                                                 \
    }                                                           \
  } while (0)

int main() {
  for (int round = 0; round < 50; ++round) {  // repeated build/run/destroy: leaks and UAF show up
    g_calls.clear();
    g_vals.clear();
    HzProgram p = hz_prog_create();
    HzConvParams c;
    memset(&c, 0, sizeof(c));
    c.K = 576;
    CHECK(hz_prog_add_conv(p, &c, 3, 0) == 0);
    c.K = 1;  // the program captured the params by value at add time
    HzConvParams d = c;
    d.K = 64;
    CHECK(hz_prog_add_conv2(p, &c, &d, 2, 0) == 0);
    HzLstmParams l;
    memset(&l, 0, sizeof(l));
    l.H = 1150;
    CHECK(hz_prog_add_lstm(p, &l, 0) == 0);
    HzLayerNormParams ln;
    memset(&ln, 0, sizeof(ln));
    ln.rows = 2048;
    CHECK(hz_prog_add_kernel(p, HZ_K_LAYERNORM, &ln, sizeof(ln), 0) == 0);
    ln.rows = -5;  // generic kernels also copy their parameter block
    std::vector<char> big(4096, 0);  // a parameter block larger than any struct
    CHECK(hz_prog_add_kernel(p, 9999, big.data(), big.size(), 0) == -101);  // unknown kind: refused at add
    CHECK(hz_prog_add_kernel(p, HZ_K_LAYERNORM, &ln, sizeof(ln) - 8, 0) == -101);  // short record: refused
    HzSoftmaxParams sm;
    memset(&sm, 0, sizeof(sm));
    sm.rows = -7;
    CHECK(hz_prog_add_kernel(p, HZ_K_SOFTMAX, big.data(), big.size(), 0) == 0);  // a longer record is fine
    memcpy(big.data(), &sm, sizeof(sm));
    CHECK(hz_prog_num_ops(p) == 5);
    hz_prog_destroy(p);  // (discard: rebuild with the failing softmax as op 4)
    p = hz_prog_create();
    c.K = 576;
    CHECK(hz_prog_add_conv(p, &c, 3, 0) == 0);
    c.K = 1;
    CHECK(hz_prog_add_conv2(p, &c, &d, 2, 0) == 0);
    CHECK(hz_prog_add_lstm(p, &l, 0) == 0);
    ln.rows = 2048;
    CHECK(hz_prog_add_kernel(p, HZ_K_LAYERNORM, &ln, sizeof(ln), 0) == 0);
    CHECK(hz_prog_add_kernel(p, HZ_K_SOFTMAX, big.data(), big.size(), 0) == 0);  // fails at run
    CHECK(hz_prog_add_avgpool(p, nullptr, nullptr, 7, 49, 2048, 1, 0) == 0);
    CHECK(hz_prog_add_conv(p, &c, 0, -1) == -4);  // slot out of range
    CHECK(hz_prog_add_conv(p, &c, 0, 9) == -4);
    CHECK(hz_prog_add_fork(p, 0) == -4);
    CHECK(hz_prog_num_ops(p) == 6);
    CHECK(hz_prog_is_captured(p) == 0);
    g_calls.clear();
    g_vals.clear();
    const int rc = hz_prog_run(p, nullptr);  // op 4 (the failing softmax) -> run stops there
    CHECK(rc == 7);
    CHECK(g_calls.size() == 5 && g_calls[4] == 13);
    CHECK(g_calls[0] == 1 && g_vals[0] == 576 * 100 + 3);
    CHECK(g_calls[1] == 14 && g_vals[1] == 1 + 64 + 2);
    CHECK(g_calls[2] == 4 && g_vals[2] == 1150);
    CHECK(g_calls[3] == 9 && g_vals[3] == 2048);
    hz_prog_destroy(p);

    HzProgram q = hz_prog_create();
    for (int i = 0; i < 64; ++i) CHECK(hz_prog_add_avgpool(q, nullptr, nullptr, i, 1, 1, 0, 0) == 0);
    g_calls.clear();
    g_vals.clear();
    CHECK(hz_prog_replay_n(q, nullptr, 3) == 0);  // not captured: eager runs
    CHECK(g_calls.size() == 192 && g_vals[191] == 63);
    hz_prog_destroy(q);
  }
  printf("runtime host asan: ok\n");
  return 0;
}
