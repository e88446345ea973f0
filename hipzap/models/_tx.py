"""Shared helpers for lowering transformer encoders (BERT, ViT) to hipzap graphs."""
from __future__ import annotations

import torch

from ..engine.graph import Graph
from ..ops.conv import GEMM_ROW_PAD, pack_matrix
from ..ops.transformer import NormParams


def pack_linear_padded(weight: torch.Tensor, bias: torch.Tensor | None, out_multiple: int = 4):
    """Pack a Linear for the GEMM kernel; output rows padded to ``out_multiple`` (the epilogue
    stores 4 channels per lane) — logical width kept by the caller."""
    w = weight.detach().float()
    b = bias.detach().float() if bias is not None else torch.zeros(w.shape[0], device=w.device)
    n = w.shape[0]
    npad = (n + out_multiple - 1) // out_multiple * out_multiple
    if npad != n:
        w = torch.cat([w, w.new_zeros(npad - n, w.shape[1])])
        b = torch.cat([b, b.new_zeros(npad - n)])
    return pack_matrix(w, b, w.shape[1], row_pad=GEMM_ROW_PAD)


def pack_qkv(q_w, q_b, k_w, k_b, v_w, v_b):
    return pack_linear_padded(torch.cat([q_w, k_w, v_w]), torch.cat([q_b, k_b, v_b]))


def fold_ln_linear(weight: torch.Tensor, bias: torch.Tensor, ln: NormParams):
    """Linear whose input is LayerNorm(y), folded to run on the raw y (HzLnFold, csrc/hipzap.h):
    W' = W diag(gamma), bias' = bias + W beta, c1[n] = sum_k W'[n][k] of the bf16-packed W' (so
    the epilogue's mean * c1 cancels exactly what the MFMA accumulated). -> (packed W', c1)."""
    w = weight.detach().float()
    pc = pack_linear_padded(w * ln.gamma.float()[None, :], bias.detach().float() + w @ ln.beta.float())
    return pc, pc.dense().sum(1).contiguous()


def norm(sd, prefix, eps):
    return NormParams(sd[f"{prefix}.weight"].float().contiguous(), sd[f"{prefix}.bias"].float().contiguous(), eps)


class TxBuilder:
    """Adds transformer nodes to a Graph (row-major [rows, cols] bf16 activations)."""

    def __init__(self, g: Graph):
        self.g = g

    def gemm(self, x, w: str, cols: int, act="none", res=None, rows=None, ldx=None, out_f32=False, ext=False,
             name=None, ln_in=None, res_ln=None, stats_out=False):
        """``ln_in`` / ``res_ln`` = (LayerNorm param, stats tensor): the input / residual is the raw
        pre-LN sum and the LayerNorm is folded into this GEMM (``w`` packed by fold_ln_linear, its
        ``c1`` at ``w + ".c1"``). ``stats_out``: also emit the per-row (sum, sumsq) slabs of the
        output for folded consumers; returns (out, stats)."""
        g = self.g
        r = rows if rows is not None else g.shape(x)[0]
        out = g.tensor((r, cols), torch.float32 if out_f32 else torch.bfloat16, name or w, external=ext)
        ins = [x] if res is None else [x, res]
        attrs = dict(w=w, act=act, rows=r, ldx=ldx, out_f32=out_f32, name=name or w, has_res=res is not None)
        outs = [out]
        if ln_in is not None:
            attrs["ln_in"] = ln_in
            ins.append(ln_in[1])
        if res_ln is not None:
            assert res is not None
            attrs["res_ln"] = res_ln
            ins.append(res_ln[1])
        if stats_out:  # slabs for the smallest N tile (64 columns, 2 wave columns each): [2*ceil(cols/64), r, 2]
            st = g.tensor((2 * ((cols + 63) // 64), r, 2), torch.float32, f"{name or w}.stats")
            attrs["stats_out"] = st
            outs.append(st)
        g.add("gemm", ins, outs, **attrs)
        return (out, outs[1]) if stats_out else out

    def gemm8(self, x, w: str, cols: int, act="none", res=None, out_f32=False, ext=False, name=None):
        """fp8 GEMM: per-row dynamic quantisation of ``x`` then the fp8 MFMA GEMM."""
        g = self.g
        r, k = g.shape(x)
        x8 = g.tensor((r, k), torch.uint8, f"{w}.x8")
        sx = g.tensor((r,), torch.float32, f"{w}.sx")
        g.add("quant", [x], [x8, sx])
        return self.gemm8q((x8, sx), w, cols, act=act, res=res, out_f32=out_f32, ext=ext, name=name)

    def linear(self, x, w: str, cols: int, fp8: bool = False, **kw):
        return self.gemm8(x, w, cols, **kw) if fp8 else self.gemm(x, w, cols, **kw)

    def layernorm(self, x, p: str, res=None, rows=None, ldx=None, name=None):
        g = self.g
        r = rows if rows is not None else g.shape(x)[0]
        out = g.tensor((r, g.shape(x)[1]), torch.bfloat16, name or p)
        ins = [x] if res is None else [x, res]
        g.add("layernorm", ins, [out], p=p, rows=r, ldx=ldx)
        return out

    def layernorm_q8(self, x, p: str, res=None, keep_bf16=False):
        """LayerNorm whose output feeds fp8 GEMMs: fused per-row fp8 quantisation. ``keep_bf16``
        (post-LN residual stream): also the bf16 output, returned as ``(out, (x8, scales))``."""
        g = self.g
        r, d = g.shape(x)
        x8 = g.tensor((r, d), torch.uint8, f"{p}.x8")
        sx = g.tensor((r,), torch.float32, f"{p}.sx")
        ins = [x] if res is None else [x, res]
        if keep_bf16:
            out = g.tensor((r, d), torch.bfloat16, p)
            g.add("layernorm", ins, [out, x8, sx], p=p, rows=r, ldx=None)
            return out, (x8, sx)
        g.add("layernorm", ins, [x8, sx], p=p, rows=r, ldx=None)
        return x8, sx

    def gemm8q(self, xq, w: str, cols: int, act="none", res=None, out_f32=False, ext=False, name=None,
               out_mx=False):
        """fp8 GEMM on an already-quantised input ``xq = (x8, scales)``: per-row fp32 scales
        ``[rows]`` or MX8 E8M0 block scales ``[rows, K/32]`` (uint8). ``out_mx``: the output is
        MX8 too, returned as ``(o8, os8)`` for the next fp8 GEMM."""
        g = self.g
        x8, sx = xq
        r = g.shape(x8)[0]
        ins = [x8, sx] if res is None else [x8, sx, res]
        if out_mx:
            o8 = g.tensor((r, cols), torch.uint8, f"{name or w}.o8")
            os8 = g.tensor((r, cols // 32), torch.uint8, f"{name or w}.os8")
            g.add("gemm_fp8", ins, [o8, os8], w=w, act=act, rows=r, name=name or w)
            return o8, os8
        out = g.tensor((r, cols), torch.float32 if out_f32 else torch.bfloat16, name or w, external=ext)
        g.add("gemm_fp8", ins, [out], w=w, act=act, rows=r, out_f32=out_f32, name=name or w)
        return out

    def attention(self, qkv, B, L, heads, mask=None, out_mx=False):
        """Fused attention; ``out_mx``: MX8 output ``(ctx8, ctxs)`` for an fp8 consumer."""
        g = self.g
        ins = [qkv] if mask is None else [qkv, mask]
        if out_mx:
            o8 = g.tensor((B * L, heads * 64), torch.uint8, "ctx.o8")
            os8 = g.tensor((B * L, heads * 2), torch.uint8, "ctx.os8")
            g.add("attention", ins, [o8, os8], B=B, L=L, heads=heads)
            return o8, os8
        out = g.tensor((B * L, heads * 64), torch.bfloat16, "ctx")
        g.add("attention", ins, [out], B=B, L=L, heads=heads)
        return out
