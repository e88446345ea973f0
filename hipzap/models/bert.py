"""BERT-base sequence classification (HF ``BertForSequenceClassification`` checkpoint layout).

North-star config 4 (BASELINE.json): BERT-base seq-cls bs=16 on one MI355X through the
Linear/LayerNorm/Softmax HIP path. Not in the reference.

* Checkpoint schema + fp32 oracle: ``transformers.BertForSequenceClassification`` (installed,
  random init from ``BertConfig`` — no network), keys ``bert.embeddings.*``,
  ``bert.encoder.layer.{i}.attention.self.{query,key,value}``, ``...attention.output.dense``,
  ``...intermediate.dense``, ``...output.dense``, ``bert.pooler.dense``, ``classifier``.
* Lowering per encoder layer (post-LN, 7 kernels): QKV GEMM (Q|K|V packed as one 2304-row
  matrix, bias fused) -> fused attention (softmax(QK^T/8 + mask)V) -> O-proj GEMM with the
  residual add fused in the epilogue -> LayerNorm -> FFN1 GEMM + GELU(erf) -> FFN2 GEMM +
  residual -> LayerNorm. Embeddings gather-sum + LN is one kernel; pooler = GEMM over the
  CLS rows (row stride L*768) + tanh; classifier GEMM writes fp32 logits.
"""
from __future__ import annotations

import os

import torch

from ..engine.graph import Graph
from ..ops.transformer import EmbedTables
from ._tx import TxBuilder, fold_ln_linear, norm, pack_linear_padded, pack_qkv


def ln_fold_default() -> bool:
    """HIPZAP_LN_FOLD=1 folds the encoder LayerNorms into the GEMMs. Off by default: measured on
    one MI355X (profiles/r1_ab/bert_lnfold.txt, interleaved A/B) it removes 23 LayerNorm launches
    but the GEMM epilogues' statistics work costs more (14.3k vs 14.9k seq/s, 1 context; equal at 4)."""
    return os.environ.get("HIPZAP_LN_FOLD", "0") == "1"


def make_model(num_labels: int = 2, **cfg):
    from transformers import BertConfig, BertForSequenceClassification
    m = BertForSequenceClassification(BertConfig(num_labels=num_labels, **cfg))
    return m.eval()


def config_from_sd(sd: dict) -> dict:
    layers = 0
    while f"bert.encoder.layer.{layers}.attention.self.query.weight" in sd:
        layers += 1
    hidden = sd["bert.embeddings.word_embeddings.weight"].shape[1]
    return {"layers": layers, "hidden": hidden, "heads": hidden // 64,
            "ffn": sd["bert.encoder.layer.0.intermediate.dense.weight"].shape[0],
            "num_labels": sd["classifier.weight"].shape[0],
            "max_pos": sd["bert.embeddings.position_embeddings.weight"].shape[0]}


def pack_bert(sd: dict, device="cpu", eps: float = 1e-12, ln_fold: bool | None = None,
              weights: str = "bf16") -> tuple[dict, dict]:
    """``ln_fold``: fold every encoder LayerNorm into its consumer GEMMs (see build_graph); the
    returned cfg records the choice so the graph is built to match the packed weights.
    ``weights="fp8"``: encoder projections as e4m3 + per-channel scales on the MX fp8 MFMA path
    (pooler and classifier stay bf16; no LayerNorm fold)."""
    sd = {k: v.to(device) for k, v in sd.items()}
    cfg = config_from_sd(sd)
    cfg["ln_fold"] = False if weights == "fp8" else (ln_fold_default() if ln_fold is None else bool(ln_fold))
    cfg["weights"] = weights
    P = {
        "emb": EmbedTables(sd["bert.embeddings.word_embeddings.weight"].to(torch.bfloat16).contiguous(),
                           sd["bert.embeddings.position_embeddings.weight"].to(torch.bfloat16).contiguous(),
                           sd["bert.embeddings.token_type_embeddings.weight"].to(torch.bfloat16).contiguous()),
        "emb_ln": norm(sd, "bert.embeddings.LayerNorm", eps),
    }
    for i in range(cfg["layers"]):
        pre = f"bert.encoder.layer.{i}"
        a = f"{pre}.attention.self"
        if cfg["ln_fold"] and i > 0:  # input = raw sum of layer i-1, normalised by its ln2
            P[f"l{i}.qkv"], P[f"l{i}.qkv.c1"] = fold_ln_linear(
                torch.cat([sd[f"{a}.query.weight"], sd[f"{a}.key.weight"], sd[f"{a}.value.weight"]]),
                torch.cat([sd[f"{a}.query.bias"], sd[f"{a}.key.bias"], sd[f"{a}.value.bias"]]), P[f"l{i - 1}.ln2"])
        else:
            P[f"l{i}.qkv"] = pack_qkv(sd[f"{a}.query.weight"], sd[f"{a}.query.bias"], sd[f"{a}.key.weight"],
                                      sd[f"{a}.key.bias"], sd[f"{a}.value.weight"], sd[f"{a}.value.bias"])
        P[f"l{i}.o"] = pack_linear_padded(sd[f"{pre}.attention.output.dense.weight"],
                                          sd[f"{pre}.attention.output.dense.bias"])
        P[f"l{i}.ln1"] = norm(sd, f"{pre}.attention.output.LayerNorm", eps)
        if cfg["ln_fold"]:
            P[f"l{i}.ffn1"], P[f"l{i}.ffn1.c1"] = fold_ln_linear(
                sd[f"{pre}.intermediate.dense.weight"], sd[f"{pre}.intermediate.dense.bias"], P[f"l{i}.ln1"])
        else:
            P[f"l{i}.ffn1"] = pack_linear_padded(sd[f"{pre}.intermediate.dense.weight"],
                                                 sd[f"{pre}.intermediate.dense.bias"])
        P[f"l{i}.ffn2"] = pack_linear_padded(sd[f"{pre}.output.dense.weight"], sd[f"{pre}.output.dense.bias"])
        P[f"l{i}.ln2"] = norm(sd, f"{pre}.output.LayerNorm", eps)
    P["pooler"] = pack_linear_padded(sd["bert.pooler.dense.weight"], sd["bert.pooler.dense.bias"])
    P["cls"] = pack_linear_padded(sd["classifier.weight"], sd["classifier.bias"])
    if weights == "fp8":
        from ..ops.fp8 import quantize_params
        P = quantize_params(P, [n for n in P if n.startswith("l") and n.rsplit(".", 1)[-1] in ("qkv", "o", "ffn1", "ffn2")])
    return P, cfg


def build_graph(batch: int, seq_len: int = 128, layers: int = 12, hidden: int = 768, heads: int = 12,
                ffn: int = 3072, num_labels: int = 2, ln_fold: bool = False, weights: str = "bf16", **_) -> Graph:
    """``ln_fold`` (must match pack_bert's cfg): no standalone encoder LayerNorm. The O-proj and
    FFN2 GEMMs emit per-row (sum, sumsq) slabs of their raw output y; FFN1 and the next layer's
    QKV run on y with gamma/beta folded into their weights and normalise in the epilogue; the
    residual reads of y are normalised in the epilogue too (HzLnFold, csrc/hipzap.h). Only the
    B CLS rows get a real LayerNorm, for the pooler. 5 kernels per layer instead of 7."""
    B, L, D = batch, seq_len, hidden
    T = B * L
    g = Graph(f"bert_bs{B}_L{L}")
    ids = g.tensor((T,), torch.int32, "input_ids", external=True)
    types = g.tensor((T,), torch.int32, "token_type_ids", external=True)
    mask = g.tensor((T,), torch.float32, "mask_add", external=True)
    g.inputs += [ids, types, mask]
    tb = TxBuilder(g)
    x = g.tensor((T, D), torch.bfloat16, "emb")
    g.add("embed_ln", [ids, types], [x], emb="emb", ln="emb_ln", L=L)
    ln_x = None  # (LayerNorm param, stats) while x is a raw pre-LN sum (ln_fold)
    xq = None  # fp8: (e4m3, per-row scales) of x, emitted by the LayerNorm that produced x
    for i in range(layers):
        if weights == "fp8":
            # post-LN: each LayerNorm emits bf16 (the next residual) AND e4m3 + row scales (the next
            # GEMM's input) in one pass; attention and FFN1 emit MX8 for O-proj / FFN2
            qkv = tb.gemm8q(xq, f"l{i}.qkv", 3 * D) if xq is not None else tb.gemm8(x, f"l{i}.qkv", 3 * D)
            y = tb.gemm8q(tb.attention(qkv, B, L, heads, mask, out_mx=True), f"l{i}.o", D, res=x)
            x1, x1q = tb.layernorm_q8(y, f"l{i}.ln1", keep_bf16=True)
            h = tb.gemm8q(x1q, f"l{i}.ffn1", ffn, act="gelu", out_mx=True)
            y2 = tb.gemm8q(h, f"l{i}.ffn2", D, res=x1)
            if i + 1 < layers:
                x, xq = tb.layernorm_q8(y2, f"l{i}.ln2", keep_bf16=True)
            else:
                x = tb.layernorm(y2, f"l{i}.ln2")
            continue
        qkv = tb.gemm(x, f"l{i}.qkv", 3 * D, ln_in=ln_x)
        ctx = tb.attention(qkv, B, L, heads, mask)
        if ln_fold:
            y, s1 = tb.gemm(ctx, f"l{i}.o", D, res=x, res_ln=ln_x, stats_out=True)
            h = tb.gemm(y, f"l{i}.ffn1", ffn, act="gelu", ln_in=(f"l{i}.ln1", s1))
            x, s2 = tb.gemm(h, f"l{i}.ffn2", D, res=y, res_ln=(f"l{i}.ln1", s1), stats_out=True)
            ln_x = (f"l{i}.ln2", s2)
            continue
        y = tb.gemm(ctx, f"l{i}.o", D, res=x)
        x1 = tb.layernorm(y, f"l{i}.ln1")
        h = tb.gemm(x1, f"l{i}.ffn1", ffn, act="gelu")
        y2 = tb.gemm(h, f"l{i}.ffn2", D, res=x1)
        x = tb.layernorm(y2, f"l{i}.ln2")
    if ln_x is not None:  # the pooler reads only the CLS rows: normalise just those B rows
        xc = tb.layernorm(x, ln_x[0], rows=B, ldx=L * D, name="cls_ln")
        pooled = tb.gemm(xc, "pooler", D, act="tanh", rows=B)
    else:
        pooled = tb.gemm(x, "pooler", D, act="tanh", rows=B, ldx=L * D)
    npad = (num_labels + 3) // 4 * 4
    logits = tb.gemm(pooled, "cls", npad, out_f32=True, ext=True)
    g.outputs.append(logits)
    g.meta = {"num_labels": num_labels}
    return g


def encode_inputs(input_ids: torch.Tensor, token_type_ids=None, attention_mask=None):
    """HF-style request tensors -> the graph's three int32/fp32 inputs."""
    ids = input_ids.to(torch.int32).reshape(-1)
    tt = (token_type_ids if token_type_ids is not None else torch.zeros_like(input_ids)).to(torch.int32).reshape(-1)
    am = attention_mask if attention_mask is not None else torch.ones_like(input_ids)
    madd = (1.0 - am.float()).reshape(-1) * -1e9
    return [ids, tt, madd]
