"""Shared helpers for lowering transformer encoders (BERT, ViT) to hipzap graphs."""
from __future__ import annotations

import torch

from ..engine.graph import Graph
from ..ops.conv import GEMM_ROW_PAD, pack_matrix
from ..ops.transformer import NormParams


def _native_ok(*ts) -> bool:
    """Device packing (csrc/pack.hip hz_frag_pack_launch) for tensors on a GPU: one launch per
    matrix instead of ~6 torch ops whose first use in a fresh process is mostly kernel loading."""
    import os
    if os.environ.get("HIPZAP_NATIVE_PACK", "1") == "0":
        return False
    if not all(t is None or t.device.type == "cuda" for t in ts) or ts[0].device.type != "cuda":
        return False
    try:
        from .. import _native as N
        return hasattr(N.lib(), "hz_frag_pack_launch")
    except OSError:
        return False


def _pack_rows_native(parts: list, npad: int):
    """[(weight [n_j, K], bias [n_j] | None)] stacked by rows (each n_j % 16 == 0 but the last),
    padded to ``npad`` rows and then to GEMM_ROW_PAD -> PackedConv, bitwise pack_matrix of the
    row-concatenation (zero rows / columns, RNE bf16, fp32 bias)."""
    import ctypes as C
    import math
    from .. import _native as N
    from ..ops.conv import PackedConv
    K = parts[0][0].shape[1]
    dev = parts[0][0].device
    ksteps = int(math.ceil(K / 32))
    rows = int(math.ceil(npad / GEMM_ROW_PAD) * GEMM_ROW_PAD)
    wf = torch.empty(rows // 16, ksteps, 64, 8, dtype=torch.bfloat16, device=dev)
    bias = torch.empty(rows, dtype=torch.float32, device=dev)
    f32 = lambda t: None if t is None else (t.detach() if t.dtype == torch.float32 else t.detach().float()).contiguous()  # noqa: E731
    keep, r0 = [], 0
    for j, (w, b) in enumerate(parts):
        w, b = f32(w), f32(b)
        keep += [w, b]
        n = w.shape[0]
        R = rows - r0 if j == len(parts) - 1 else n  # the last part also writes the zero padding rows
        p = N.FragPackParams()
        p.a, p.out = w.data_ptr(), wf.data_ptr() + (r0 // 16) * ksteps * 1024
        p.bias_a, p.bias_out = (0 if b is None else b.data_ptr()), bias.data_ptr() + 4 * r0
        p.R, p.K, p.nrows, p.ka, p.acols, p.lda = R, ksteps * 32, n, ksteps * 32, K, K
        N.check(N.lib().hz_frag_pack_launch(C.byref(p), N.stream_ptr()), "hz_frag_pack_launch")
        r0 += n
    out_bias = bias[:npad].clone()  # its own storage (a D2D copy), as the torch path's bias
    torch.cuda.current_stream(dev).synchronize()  # the fp32 sources may be temporaries
    return PackedConv(wf, out_bias, K, npad, 1, 1, 1, 0)


def pack_linear_padded(weight: torch.Tensor, bias: torch.Tensor | None, out_multiple: int = 4):
    """Pack a Linear for the GEMM kernel; output rows padded to ``out_multiple`` (the epilogue
    stores 4 channels per lane) — logical width kept by the caller. On a GPU: the device packer
    (bitwise the torch ops, tests/test_transformers_gpu.py)."""
    if _native_ok(weight, bias):
        n = weight.shape[0]
        return _pack_rows_native([(weight, bias)], (n + out_multiple - 1) // out_multiple * out_multiple)
    w = weight.detach().float()
    b = bias.detach().float() if bias is not None else torch.zeros(w.shape[0], device=w.device)
    n = w.shape[0]
    npad = (n + out_multiple - 1) // out_multiple * out_multiple
    if npad != n:
        w = torch.cat([w, w.new_zeros(npad - n, w.shape[1])])
        b = torch.cat([b, b.new_zeros(npad - n)])
    return pack_matrix(w, b, w.shape[1], row_pad=GEMM_ROW_PAD)


def pack_qkv(q_w, q_b, k_w, k_b, v_w, v_b):
    if _native_ok(q_w, q_b, k_w, k_b, v_w, v_b) and q_w.shape[0] % 16 == 0 and k_w.shape[0] % 16 == 0:
        n = q_w.shape[0] + k_w.shape[0] + v_w.shape[0]
        return _pack_rows_native([(q_w, q_b), (k_w, k_b), (v_w, v_b)], (n + 3) // 4 * 4)
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
