"""BERT-base / ViT-B/16 lowering vs the HF eager models (CPU, fp32 graph oracle)."""
import pytest
import torch

from hipzap.engine.graph import plan_memory
from hipzap.engine.reference import run_graph_reference
from hipzap.models import bert, registry, vit


def _small_bert():
    torch.manual_seed(0)
    m = bert.make_model(num_labels=3, num_hidden_layers=2, vocab_size=500, max_position_embeddings=64)
    with torch.no_grad():  # non-trivial LayerNorm affine params (HF init is gamma=1, beta=0)
        for name, p in m.named_parameters():
            if "LayerNorm" in name:
                p.add_(0.3 * torch.randn_like(p))
    return m


@pytest.mark.parametrize("ln_fold", [True, False])
def test_bert_graph_oracle_matches_hf(ln_fold):
    m = _small_bert()
    P, cfg = bert.pack_bert(m.state_dict(), ln_fold=ln_fold)
    assert cfg["layers"] == 2 and cfg["num_labels"] == 3 and cfg["ln_fold"] == ln_fold
    B, L = 2, 16
    g = bert.build_graph(B, L, layers=2, num_labels=3, ln_fold=ln_fold)
    assert [n.kind for n in g.nodes].count("layernorm") == (1 if ln_fold else 4)
    ids = torch.randint(0, 500, (B, L))
    tt = torch.randint(0, 2, (B, L))
    am = torch.ones(B, L, dtype=torch.long)
    am[1, 12:] = 0
    with torch.no_grad():
        ref = m(input_ids=ids, token_type_ids=tt, attention_mask=am).logits
    vals = run_graph_reference(g, P, bert.encode_inputs(ids, tt, am), bf16_acts=False)
    out = vals[g.outputs[0]][:, :3]
    assert (out - ref).abs().max() / ref.abs().max() < 3e-2, (out, ref)
    _, arena = plan_memory(g)
    assert arena > 0


def test_bert_base_shapes_meta():
    a = registry.get("bert-base")
    meta, cfg = a.meta_params()
    assert cfg["layers"] == 12 and cfg["hidden"] == 768 and cfg["ffn"] == 3072
    assert meta["l0.qkv"].cout == 2304 and meta["cls"].cout == 4  # 2 labels padded to 4
    g = a.build_graph(batch=16, **cfg)
    kinds = [n.kind for n in g.nodes]
    # LayerNorms folded into the GEMMs (cfg["ln_fold"], default): only the CLS-row LN for the pooler
    nln = 1 if cfg["ln_fold"] else 24
    assert kinds.count("gemm") == 12 * 4 + 2 and kinds.count("attention") == 12 and kinds.count("layernorm") == nln


@pytest.mark.parametrize("legacy_keys", [False, True])
def test_vit_graph_oracle_matches_hf(legacy_keys):
    torch.manual_seed(0)
    m = vit.make_model(num_labels=10, num_hidden_layers=2, image_size=64, patch_size=16)
    sd = m.state_dict()
    if legacy_keys:  # classic HF names (vit.encoder.layer.N.attention.attention.query ...)
        ren = {"attention.q_proj": "attention.attention.query", "attention.k_proj": "attention.attention.key",
               "attention.v_proj": "attention.attention.value", "attention.o_proj": "attention.output.dense",
               "mlp.fc1": "intermediate.dense", "mlp.fc2": "output.dense"}
        sd2 = {}
        for k, v in sd.items():
            nk = k.replace("vit.layers.", "vit.encoder.layer.")
            for a, b in ren.items():
                nk = nk.replace(a, b)
            sd2[nk] = v
        sd = sd2
    P, cfg = vit.pack_vit(sd)
    assert cfg["image"] == 64 and cfg["layers"] == 2
    g = vit.build_graph(2, **{k: cfg[k] for k in ("layers", "hidden", "heads", "ffn", "patch", "image", "num_labels")})
    x = torch.randn(2, 3, 64, 64)
    with torch.no_grad():
        ref = m(pixel_values=x).logits
    out = run_graph_reference(g, P, [x], bf16_acts=False)[g.outputs[0]][:, :10]
    assert (out - ref).abs().max() / ref.abs().max() < 3e-2


def test_vit_b16_meta():
    a = registry.get("vit-b16")
    meta, cfg = a.meta_params()
    assert cfg["image"] == 224 and cfg["patch"] == 16 and cfg["layers"] == 12
    g = a.build_graph(batch=8, **{k: cfg[k] for k in ("layers", "hidden", "heads", "ffn", "patch", "image", "num_labels")})
    assert g.shape(g.outputs[0]) == (8, 1000)


def test_vit_fp8_oracle_close_to_bf16():
    torch.manual_seed(0)
    m = vit.make_model(num_labels=10, num_hidden_layers=2, image_size=64, patch_size=16)
    sd = m.state_dict()
    kw = lambda cfg: {k: cfg[k] for k in ("layers", "hidden", "heads", "ffn", "patch", "image", "num_labels")}
    P16, cfg = vit.pack_vit(sd)
    P8, cfg8 = vit.pack_vit(sd, weights="fp8")
    g16 = vit.build_graph(2, **kw(cfg))
    g8 = vit.build_graph(2, **kw(cfg), weights="fp8")
    assert any(n.kind == "gemm_fp8" for n in g8.nodes) and any(n.kind == "quant" for n in g8.nodes)
    x = torch.randn(2, 3, 64, 64)
    a = run_graph_reference(g16, P16, [x], bf16_acts=False)[g16.outputs[0]][:, :10]
    b = run_graph_reference(g8, P8, [x], bf16_acts=False)[g8.outputs[0]][:, :10]
    assert (a - b).abs().max() / a.abs().max() < 0.15  # e4m3 has a 3-bit mantissa


def test_fp8_weight_roundtrip():
    from hipzap.ops.conv import pack_linear
    from hipzap.ops.fp8 import quantize_linear
    w = torch.randn(100, 96)
    pw = quantize_linear(pack_linear(w, torch.zeros(100)))
    err = (pw.dequant() - w).abs() / w.abs().amax(dim=1, keepdim=True)
    assert err.max() < 0.07 and pw.w8.dtype == torch.uint8 and pw.sw.shape[0] % 64 == 0


def test_mx_pack_layout():
    """MX packing (csrc/fp8.hip gemm_mx_kernel): lane l = 16*lg + row%16, register half h holds
    k%128 = 64*h + 16*lg + byte (the f8f6f4 MFMA's hardware K order); mx_unpack inverts it."""
    from hipzap.ops import fp8 as F8
    q = torch.randint(0, 256, (32, 256), dtype=torch.uint8)
    w = F8.mx_pack(q)
    assert w.shape == (2, 2, 2, 64, 16)
    assert torch.equal(F8.mx_unpack(w), q)
    g, kb, half, lane, byte = 1, 1, 1, 37, 5
    row, k = g * 16 + lane % 16, kb * 128 + half * 64 + (lane // 16) * 16 + byte
    assert w[g, kb, half, lane, byte] == q[row, k]


def test_quantize_linear_builds_mx_copy():
    from hipzap.ops import conv as C
    from hipzap.ops import fp8 as F8
    pw = F8.quantize_linear(C.pack_linear(torch.randn(200, 256), torch.zeros(200)))
    assert pw.w8mx is not None and pw.w8mx.shape == (256 // 16, 2, 2, 64, 16)
    # both packings carry the same bytes
    dense = pw.w8.reshape(16, 8, 4, 16, 8).permute(0, 3, 1, 2, 4).reshape(256, 256)
    assert torch.equal(F8.mx_unpack(pw.w8mx), dense)
    assert F8.choose_config_fp8(2048, pw)[0] in F8.MX_TILES
    assert F8.choose_config_fp8(8, pw)[0] not in F8.MX_TILES


def test_bert_fp8_graph_oracle_vs_hf():
    """bert-base-fp8 lowering on the CPU oracle: one quantisation kernel (after the embedding
    LayerNorm), every encoder LayerNorm but the last emits bf16 + e4m3 together, and the fp8
    logits stay near HF fp32."""
    import torch
    from hipzap.engine.reference import run_graph_reference
    from hipzap.models import bert, registry
    torch.manual_seed(0)
    a = registry.get("bert-base-fp8")
    m = a.make_model().eval()
    P, cfg = a.pack(m.state_dict(), "cpu")
    assert cfg["weights"] == "fp8" and not cfg["ln_fold"]
    g = a.build_graph(batch=2, **cfg)
    kinds = [n.kind for n in g.nodes]
    assert kinds.count("quant") == 1 and kinds.count("gemm_fp8") == 4 * cfg["layers"]
    assert sum(1 for n in g.nodes if n.kind == "layernorm" and len(n.outputs) == 3) == 2 * cfg["layers"] - 1
    ids = torch.randint(1000, 30000, (2, 128))
    out = run_graph_reference(g, P, bert.encode_inputs(ids))[g.outputs[0]].reshape(2, -1)[:, :2]
    with torch.no_grad():
        ref = m(input_ids=ids).logits
    assert ((out - ref).abs().max() / ref.abs().max()).item() < 0.25


def test_qkvatt_pairs(monkeypatch):
    """Every (QKV projection, attention) pair of BERT-base at L = 128 binds as one qkvatt launch
    (engine/program.py qkvatt_pairs); not ViT (L = 197 > 128), not a projection that reads folded
    LayerNorm statistics, not with HIPZAP_QKVATT=0."""
    from hipzap.engine.program import qkvatt_pairs
    a = registry.get("bert-base")
    meta, cfg = a.meta_params()
    g = a.build_graph(batch=16, **dict(cfg, ln_fold=False))
    pairs = qkvatt_pairs(g, meta)
    assert len(pairs) == 12
    for i, att in pairs.items():
        assert g.nodes[i].kind == "gemm" and g.nodes[i].attrs["w"].endswith("qkv") and att is g.nodes[i + 1]
    # with the fold only the first layer's projection (it reads the embedding LayerNorm's output)
    assert list(qkvatt_pairs(a.build_graph(batch=16, **dict(cfg, ln_fold=True)), meta)) == [1]
    v = registry.get("vit-b16")
    vmeta, vcfg = v.meta_params()
    assert not qkvatt_pairs(v.build_graph(batch=4, **vcfg), vmeta)
    monkeypatch.setenv("HIPZAP_QKVATT", "0")
    assert not qkvatt_pairs(g, meta)
