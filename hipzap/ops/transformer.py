"""Transformer ops (LayerNorm, BERT embeddings, fused attention, ViT tokens): packed-parameter
types, native launch-parameter builders, eager wrappers and fp32 PyTorch oracles."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import torch
import torch.nn.functional as F

from .. import _native as N

K_LAYERNORM, K_EMBED, K_ATTENTION, K_VIT_TOKENS = 2, 3, 4, 5
K_SOFTMAX = 12
K_QKVATT = 22


class SoftmaxParams(C.Structure):
    _fields_ = [("x", C.c_void_p), ("mask", C.c_void_p), ("out", C.c_void_p), ("rows", C.c_int), ("D", C.c_int),
                ("ldx", C.c_int), ("ldo", C.c_int), ("x_bf16", C.c_int), ("scale", C.c_float)]


class LayerNormParams(C.Structure):
    _fields_ = [("x", C.c_void_p), ("res", C.c_void_p), ("out", C.c_void_p), ("gamma", C.c_void_p),
                ("beta", C.c_void_p), ("rows", C.c_int), ("D", C.c_int), ("ldx", C.c_int), ("ldr", C.c_int),
                ("ldo", C.c_int), ("eps", C.c_float), ("out8", C.c_void_p), ("scale8", C.c_void_p)]


class EmbedParams(C.Structure):
    _fields_ = [("ids", C.c_void_p), ("types", C.c_void_p), ("word", C.c_void_p), ("pos", C.c_void_p),
                ("type", C.c_void_p), ("gamma", C.c_void_p), ("beta", C.c_void_p), ("out", C.c_void_p),
                ("rows", C.c_int), ("L", C.c_int), ("D", C.c_int), ("eps", C.c_float),
                ("vocab", C.c_int), ("ntypes", C.c_int)]


class AttentionParams(C.Structure):
    _fields_ = [("qkv", C.c_void_p), ("mask", C.c_void_p), ("out", C.c_void_p), ("B", C.c_int), ("L", C.c_int),
                ("heads", C.c_int), ("head_dim", C.c_int), ("ldqkv", C.c_int), ("k_off", C.c_int),
                ("v_off", C.c_int), ("ldo", C.c_int), ("scale", C.c_float), ("out8", C.c_void_p),
                ("os8", C.c_void_p)]


class QkvAttParams(C.Structure):  # HzQkvAttParams: QKV projection + attention in one launch
    _fields_ = [("x", C.c_void_p), ("w", C.c_void_p), ("bias", C.c_void_p), ("mask", C.c_void_p), ("out", C.c_void_p),
                ("B", C.c_int), ("L", C.c_int), ("heads", C.c_int), ("D", C.c_int), ("ksteps", C.c_int),
                ("ldx", C.c_int), ("ldo", C.c_int), ("scale", C.c_float)]


class VitTokensParams(C.Structure):
    _fields_ = [("patches", C.c_void_p), ("cls", C.c_void_p), ("pos", C.c_void_p), ("out", C.c_void_p),
                ("B", C.c_int), ("np", C.c_int), ("D", C.c_int)]


def launch(kind: int, prm, stream=None):
    N.check(N.lib().hz_launch_kernel(kind, C.byref(prm), N.stream_ptr(stream)), f"kernel {kind}")


def prog_add(prog, kind: int, prm=None, slot: int = 0, lib=None):
    lib = lib if lib is not None else N.lib()
    N.check(lib.hz_prog_add_kernel(prog, kind, C.byref(prm), C.sizeof(prm), slot), f"prog_add {kind}")


@dataclass
class NormParams:
    gamma: torch.Tensor  # fp32 [D]
    beta: torch.Tensor   # fp32 [D]
    eps: float = 1e-12

    def to(self, device):
        return NormParams(self.gamma.to(device), self.beta.to(device), self.eps)


@dataclass
class EmbedTables:
    word: torch.Tensor   # bf16 [V, D]
    pos: torch.Tensor    # bf16 [Lmax, D]
    type: torch.Tensor   # bf16 [T, D]


def norm_from(sd, prefix, eps) -> NormParams:
    return NormParams(sd[f"{prefix}.weight"].float().contiguous(), sd[f"{prefix}.bias"].float().contiguous(), eps)


# ----------------------------------------------------------------------------- eager
def layernorm(x: torch.Tensor, np_: NormParams, residual: torch.Tensor | None = None, out=None) -> torch.Tensor:
    rows, D = x.shape
    out = out if out is not None else torch.empty_like(x)
    prm = LayerNormParams(x.data_ptr(), N.ptr(residual), out.data_ptr(), np_.gamma.data_ptr(), np_.beta.data_ptr(),
                          rows, D, x.stride(0), residual.stride(0) if residual is not None else 0, out.stride(0),
                          np_.eps)
    launch(K_LAYERNORM, prm)
    return out


def layernorm_q8(x: torch.Tensor, np_: NormParams, residual: torch.Tensor | None = None, keep_bf16: bool = False):
    """LayerNorm with the per-row fp8 quantisation of its output fused in:
    returns (x8 uint8 [rows, D], row scales fp32 [rows]) and, with ``keep_bf16``, the bf16 output."""
    rows, D = x.shape
    out = torch.empty_like(x) if keep_bf16 else None
    x8 = torch.empty(rows, D, dtype=torch.uint8, device=x.device)
    sx = torch.empty(rows, dtype=torch.float32, device=x.device)
    prm = LayerNormParams(x.data_ptr(), N.ptr(residual), N.ptr(out), np_.gamma.data_ptr(), np_.beta.data_ptr(),
                          rows, D, x.stride(0), residual.stride(0) if residual is not None else 0, D, np_.eps,
                          x8.data_ptr(), sx.data_ptr())
    launch(K_LAYERNORM, prm)
    return (x8, sx, out) if keep_bf16 else (x8, sx)


def softmax(x: torch.Tensor, cols: int | None = None, scale: float = 1.0, mask: torch.Tensor | None = None,
            out: torch.Tensor | None = None) -> torch.Tensor:
    """Row softmax over the first ``cols`` columns of a 2-D fp32/bf16 tensor -> fp32."""
    rows, ld = x.shape
    D = cols or ld
    assert x.dtype in (torch.float32, torch.bfloat16) and x.stride(1) == 1
    out = out if out is not None else torch.empty(rows, D, device=x.device, dtype=torch.float32)
    prm = SoftmaxParams(x.data_ptr(), N.ptr(mask), out.data_ptr(), rows, D, x.stride(0), out.stride(0),
                        int(x.dtype == torch.bfloat16), scale)
    launch(K_SOFTMAX, prm)
    return out


def softmax_ref(x: torch.Tensor, cols: int | None = None, scale: float = 1.0, mask=None) -> torch.Tensor:
    D = cols or x.shape[-1]
    v = x[..., :D].float() * scale
    if mask is not None:
        v = v + mask.float()
    return torch.softmax(v, dim=-1)


def attention(qkv: torch.Tensor, B: int, L: int, heads: int, mask: torch.Tensor | None = None,
              out: torch.Tensor | None = None) -> torch.Tensor:
    D = heads * 64
    out = out if out is not None else torch.empty(B * L, D, dtype=torch.bfloat16, device=qkv.device)
    prm = AttentionParams(qkv.data_ptr(), N.ptr(mask), out.data_ptr(), B, L, heads, 64, qkv.stride(0), D, 2 * D,
                          out.stride(0), 1.0 / 8.0)
    launch(K_ATTENTION, prm)
    return out


# ----------------------------------------------------------------------------- oracles
def layernorm_ref(x, np_: NormParams, residual=None):
    x = x.float() + (residual.float() if residual is not None else 0)
    return F.layer_norm(x, (x.shape[-1],), np_.gamma.float(), np_.beta.float(), np_.eps)


def attention_ref(qkv, B, L, heads, mask=None):
    D = heads * 64
    q, k, v = qkv.float().reshape(B, L, 3, heads, 64).permute(2, 0, 3, 1, 4)
    s = q @ k.transpose(-1, -2) / 8.0
    if mask is not None:
        s = s + mask.float().reshape(B, 1, 1, L)
    return (torch.softmax(s, -1) @ v).permute(0, 2, 1, 3).reshape(B * L, D)


def embed_ref(ids, types, tab: EmbedTables, np_: NormParams, L):
    pos = torch.arange(ids.numel(), device=ids.device) % L
    x = tab.word.float()[ids.long().reshape(-1)] + tab.pos.float()[pos] + tab.type.float()[types.long().reshape(-1)]
    return F.layer_norm(x, (x.shape[-1],), np_.gamma, np_.beta, np_.eps)
