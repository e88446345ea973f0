"""ViT-B/16 image classification (HF ``ViTForImageClassification`` checkpoint layout).

North-star config 5 (BASELINE.json): ViT-B/16, bs=64 data-parallel over 8 GPUs (8 img/GPU),
with fp8 weights on the CDNA4 fp8 MFMA path (``weights="fp8"``; bf16 also supported).
Not in the reference.

* Checkpoint schema + fp32 oracle: ``transformers.ViTForImageClassification`` (random init from
  ``ViTConfig``). Both the transformers-5 key names (``vit.layers.{i}.attention.q_proj``,
  ``layernorm_before``, ``mlp.fc1``) and the classic ones
  (``vit.encoder.layer.{i}.attention.attention.query``, ``intermediate.dense``, ...) load.
* Lowering: patchify (fp32 NCHW -> bf16 patch rows [B*196][3*16*16], the flattened conv weight's
  K order) -> patch-embed as a plain row-major GEMM (K 768; the round-1..5 implicit-GEMM conv over
  8-channel padded pixels ran K 2048 at 112 us per bs64 forward) -> CLS + position add -> 12
  pre-LN blocks (LN -> QKV GEMM ->
  fused attention (L=197) -> O-proj GEMM + residual -> LN -> FC1 + GELU -> FC2 + residual)
  -> LN on the CLS rows only -> classifier GEMM (fp32 logits).
"""
from __future__ import annotations

import os

import torch

from ..engine.graph import Graph
from ..ops.conv import pack_conv
from ._tx import TxBuilder, norm, pack_linear_padded, pack_qkv


def _patch_lowering(patch: int = 16, image: int = 224) -> str:
    """How the patch embedding lowers: "gemm" (patchify + a row-major GEMM; the patchify kernel is
    built for 16 x 16 patches tiling the image) or "conv" (the implicit-GEMM conv over 8-channel
    padded pixels, rounds 1-5: any patch size). HIPZAP_VIT_PATCH=conv forces the conv (A/B runs).
    Chosen ONCE at pack time and recorded in the packed config (``patch_lowering``), which the
    graph builder follows, so packed weights and the graph cannot disagree."""
    if os.environ.get("HIPZAP_VIT_PATCH", "gemm") == "conv" or patch != 16 or image % patch:
        return "conv"
    return "gemm"


def make_model(num_labels: int = 1000, **cfg):
    from transformers import ViTConfig, ViTForImageClassification
    return ViTForImageClassification(ViTConfig(num_labels=num_labels, **cfg)).eval()


_NEW = {"q": "attention.q_proj", "k": "attention.k_proj", "v": "attention.v_proj", "o": "attention.o_proj",
        "ln1": "layernorm_before", "ln2": "layernorm_after", "fc1": "mlp.fc1", "fc2": "mlp.fc2"}
_OLD = {"q": "attention.attention.query", "k": "attention.attention.key", "v": "attention.attention.value",
        "o": "attention.output.dense", "ln1": "layernorm_before", "ln2": "layernorm_after",
        "fc1": "intermediate.dense", "fc2": "output.dense"}


def _layer_keys(sd: dict, i: int) -> dict:
    if f"vit.layers.{i}.attention.q_proj.weight" in sd:
        return {k: f"vit.layers.{i}.{v}" for k, v in _NEW.items()}
    if f"vit.encoder.layer.{i}.attention.attention.query.weight" in sd:
        return {k: f"vit.encoder.layer.{i}.{v}" for k, v in _OLD.items()}
    return {}


def config_from_sd(sd: dict) -> dict:
    layers = 0
    while _layer_keys(sd, layers):
        layers += 1
    pw = sd["vit.embeddings.patch_embeddings.projection.weight"]
    hidden, _, patch, _ = pw.shape
    npos = sd["vit.embeddings.position_embeddings"].shape[1]
    image = int(round((npos - 1) ** 0.5)) * patch
    fc1 = _layer_keys(sd, 0)["fc1"]
    return {"layers": layers, "hidden": hidden, "heads": hidden // 64, "patch": patch, "image": image,
            "ffn": sd[f"{fc1}.weight"].shape[0], "num_labels": sd["classifier.weight"].shape[0]}


def pack_vit(sd: dict, device="cpu", eps: float = 1e-12, weights: str = "bf16",
             patch_lowering: str | None = None) -> tuple[dict, dict]:
    """``patch_lowering``: the source rank's choice (broadcast metadata); default: decided here."""
    sd = {k: v.to(device) for k, v in sd.items()}
    cfg = config_from_sd(sd)
    pw = sd["vit.embeddings.patch_embeddings.projection.weight"]
    pb = sd["vit.embeddings.patch_embeddings.projection.bias"]
    cfg["patch_lowering"] = patch_lowering or _patch_lowering(cfg["patch"], cfg["image"])
    P = {"patch": (pack_conv(pw, pb, None, stride=cfg["patch"], pad=0, cin_pad=8) if cfg["patch_lowering"] == "conv"
                   else pack_linear_padded(pw.reshape(pw.shape[0], -1), pb)),
         "cls_token": sd["vit.embeddings.cls_token"].reshape(-1).to(torch.bfloat16).contiguous(),
         "pos": sd["vit.embeddings.position_embeddings"].reshape(-1, cfg["hidden"]).to(torch.bfloat16).contiguous(),
         "final_ln": norm(sd, "vit.layernorm", eps),
         "head": pack_linear_padded(sd["classifier.weight"], sd["classifier.bias"])}
    for i in range(cfg["layers"]):
        k = _layer_keys(sd, i)
        P[f"l{i}.qkv"] = pack_qkv(sd[f"{k['q']}.weight"], sd[f"{k['q']}.bias"], sd[f"{k['k']}.weight"],
                                  sd[f"{k['k']}.bias"], sd[f"{k['v']}.weight"], sd[f"{k['v']}.bias"])
        P[f"l{i}.o"] = pack_linear_padded(sd[f"{k['o']}.weight"], sd[f"{k['o']}.bias"])
        P[f"l{i}.ln1"] = norm(sd, k["ln1"], eps)
        P[f"l{i}.ln2"] = norm(sd, k["ln2"], eps)
        P[f"l{i}.fc1"] = pack_linear_padded(sd[f"{k['fc1']}.weight"], sd[f"{k['fc1']}.bias"])
        P[f"l{i}.fc2"] = pack_linear_padded(sd[f"{k['fc2']}.weight"], sd[f"{k['fc2']}.bias"])
    if weights == "fp8":
        from ..ops.fp8 import quantize_params
        P = quantize_params(P, [n for n in P if n.startswith("l") or n == "head"])
    cfg["weights"] = weights
    return P, cfg


def build_graph(batch: int, layers: int = 12, hidden: int = 768, heads: int = 12, ffn: int = 3072,
                patch: int = 16, image: int = 224, num_labels: int = 1000, weights: str = "bf16",
                patch_lowering: str | None = None, **_) -> Graph:
    B, D = batch, hidden
    n_side = image // patch
    npch = n_side * n_side
    T = npch + 1
    g = Graph(f"vit_bs{B}")
    x_in = g.tensor((B, 3, image, image), torch.float32, "input", external=True)
    g.inputs.append(x_in)
    tb = TxBuilder(g)
    if (patch_lowering or _patch_lowering(patch, image)) == "conv":  # any patch size; the A/B lowering
        nhwc = g.tensor((B, image, image, 8), name="nhwc")
        g.add("preprocess", [x_in], [nhwc], mean=None, std=None)
        patches = g.tensor((B * npch, D), torch.bfloat16, "patches")
        g.add("conv", [nhwc], [patches], w="patch", act="none", rowmajor=True, name="patch_embed")
    else:
        prow = g.tensor((B * npch, 3 * patch * patch), torch.bfloat16, "patch_rows")
        g.add("patchify", [x_in], [prow], patch=patch, mean=None, std=None)
        patches = tb.gemm(prow, "patch", D, name="patch_embed")
    tok = g.tensor((B * T, D), torch.bfloat16, "tokens")
    g.add("vit_tokens", [patches], [tok], cls="cls_token", pos="pos", B=B, np=npch)
    f8 = weights == "fp8"
    x = tok
    for i in range(layers):
        if f8:
            # every fp8 GEMM input is produced already quantised by its producer: the pre-LN
            # LayerNorms emit e4m3 + per-row scales, attention and FC1 emit MX8 (e4m3 + one E8M0
            # scale per 32 columns) consumed by the block-scaled MFMA — no quantisation kernels
            qkv = tb.gemm8q(tb.layernorm_q8(x, f"l{i}.ln1"), f"l{i}.qkv", 3 * D)
            x2 = tb.gemm8q(tb.attention(qkv, B, T, heads, out_mx=True), f"l{i}.o", D, res=x)
            f = tb.gemm8q(tb.layernorm_q8(x2, f"l{i}.ln2"), f"l{i}.fc1", ffn, act="gelu", out_mx=True)
            x = tb.gemm8q(f, f"l{i}.fc2", D, res=x2)
        else:
            qkv = tb.gemm(tb.layernorm(x, f"l{i}.ln1"), f"l{i}.qkv", 3 * D)
            ctx = tb.attention(qkv, B, T, heads)
            x2 = tb.gemm(ctx, f"l{i}.o", D, res=x)
            f = tb.gemm(tb.layernorm(x2, f"l{i}.ln2"), f"l{i}.fc1", ffn, act="gelu")
            x = tb.gemm(f, f"l{i}.fc2", D, res=x2)
    cls = tb.layernorm(x, "final_ln", rows=B, ldx=T * D, name="cls_ln")
    npad = (num_labels + 3) // 4 * 4
    logits = tb.linear(cls, "head", npad, fp8=f8, out_f32=True, ext=True)
    g.outputs.append(logits)
    g.meta = {"num_labels": num_labels}
    return g
