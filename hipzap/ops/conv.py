"""Conv2d + folded BatchNorm + residual + activation on the native MFMA implicit-GEMM kernel.

Weights are packed ONCE at load time (``pack_conv``): BN folded in fp32, OIHW -> O,R,S,C
(K contiguous, NHWC-matching), input channels padded to a multiple of 8, K padded to a
multiple of 32 and output-channel rows padded to 128 so that every tile config reads in
bounds. A Linear layer is the 1x1 case on a 1x1 image (``pack_linear``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from .. import _native as N

# Mirrors the switch in csrc/conv.hip: (WC, WP, FC, FP); tile = WC*FC*16 ch x WP*FP*16 px
CONV_CONFIGS = [
    (2, 2, 2, 2), (4, 1, 1, 1), (4, 1, 2, 1), (1, 4, 1, 1), (2, 2, 1, 1), (2, 2, 4, 4),
    (2, 2, 2, 4), (2, 2, 4, 2), (4, 1, 1, 2), (1, 4, 2, 1), (4, 1, 2, 2), (1, 4, 1, 2),
]
ROW_PAD = 128
ACT = {"none": 0, "relu": 1, "gelu": 2, "tanh": 3}
NUM_CUS = 256


def tile_dims(cfg: int) -> tuple[int, int]:
    wc, wp, fc, fp = CONV_CONFIGS[cfg]
    return wc * fc * 16, wp * fp * 16


@dataclass
class PackedConv:
    w: torch.Tensor          # bf16 [Cout_pad, ldw]
    bias: torch.Tensor       # fp32 [Cout]
    cin: int                 # padded input channels (multiple of 8)
    cout: int
    r: int
    s: int
    stride: int
    pad: int

    @property
    def K(self) -> int:
        return self.r * self.s * self.cin

    @property
    def ldw(self) -> int:
        return self.w.shape[1]

    def to(self, device) -> "PackedConv":
        return PackedConv(self.w.to(device), self.bias.to(device), self.cin, self.cout, self.r, self.s,
                          self.stride, self.pad)


def fold_bn(weight: torch.Tensor, bias: torch.Tensor | None, bn: dict | None, eps: float = 1e-5):
    """Fold eval-mode BatchNorm into conv weight/bias (fp32)."""
    w = weight.detach().float()
    b = bias.detach().float() if bias is not None else torch.zeros(w.shape[0], device=w.device)
    if bn is not None:
        scale = bn["weight"].float() / torch.sqrt(bn["running_var"].float() + eps)
        w = w * scale.view(-1, *([1] * (w.dim() - 1)))
        b = (b - bn["running_mean"].float()) * scale + bn["bias"].float()
    return w, b


def pack_conv(weight, bias=None, bn=None, stride=1, pad=0, eps=1e-5, cin_pad: int | None = None) -> PackedConv:
    w, b = fold_bn(weight, bias, bn, eps)
    cout, cin, r, s = w.shape
    cin_p = cin_pad or int(math.ceil(cin / 8) * 8)
    w = w.permute(0, 2, 3, 1)  # O,R,S,C
    if cin_p != cin:
        w = torch.nn.functional.pad(w, (0, cin_p - cin))
    K = r * s * cin_p
    ldw = int(math.ceil(K / 32) * 32)
    rows = int(math.ceil(cout / ROW_PAD) * ROW_PAD)
    wp = torch.zeros(rows, ldw, dtype=torch.bfloat16, device=w.device)
    wp[:cout, :K] = w.reshape(cout, K).to(torch.bfloat16)
    return PackedConv(wp, b.contiguous(), cin_p, cout, r, s, stride, pad)


def pack_linear(weight, bias=None) -> PackedConv:
    return pack_conv(weight[:, :, None, None], bias)


KW_TILES = [(fc, fp) for fc in (1, 2, 4) for fp in (1, 2, 4)]  # cfg = 100 + index


def kw_max_threads(nf: int) -> int:
    return 256 if nf >= 16 else 512 if nf >= 8 else 1024


def kw_cfg(fc: int, fp: int) -> int:
    return 100 + KW_TILES.index((fc, fp))


def tile_of(cfg: int) -> tuple[int, int]:
    """(channels, pixels) per workgroup for any cfg."""
    if cfg >= 100:
        fc, fp = KW_TILES[cfg - 100]
        return fc * 16, fp * 16
    return tile_dims(cfg)


def candidates(M: int, cout: int, K: int) -> list[tuple[int, int, int]]:
    """All legal (cfg, splitk, kw) launch choices worth timing for one conv shape."""
    steps = max(1, math.ceil(K / 32))
    out = []
    for (fc, fp) in KW_TILES:
        if (fc > 1 and fc * 16 > cout) or (fp > 1 and fp * 16 > M):
            continue
        for kw in (1, 2, 4, 8, 16):
            if kw * fc * fp > 64 or 64 * kw > kw_max_threads(fc * fp):
                continue
            if kw > 1 and steps / kw < 2:
                continue
            out.append((kw_cfg(fc, fp), 1, kw))
    for cfg in range(len(CONV_CONFIGS)):  # v1 (cross-workgroup split-K) kept as candidates
        c, sk = _v1_choice(M, cout, K, cfg)
        out.append((cfg, sk, 1))
    return out


def _v1_choice(M, cout, K, cfg):
    steps = max(1, math.ceil(K / 32))
    bnc, bmp = tile_dims(cfg)
    tiles = math.ceil(cout / bnc) * math.ceil(M / bmp)
    want = max(1, math.ceil(NUM_CUS / tiles))
    return cfg, max(1, min(want, steps // 4, 32))


def choose_config(M: int, cout: int, K: int, tuned: dict | None = None, key: str | None = None):
    """Pick (cfg, splitk, kw) for an implicit GEMM of M pixels x cout channels x K.

    A measured table (``tuned``, produced on the GPU by ``hipzap.engine.tune``) wins. The
    fallback heuristic uses the K-across-waves kernel: the smallest output tile that still
    yields >= 1 workgroup per CU, then enough waves per workgroup that each wave streams
    ~6 K-steps.
    """
    if tuned is not None and key is not None and key in tuned:
        v = tuned[key]
        return int(v[0]), int(v[1]), int(v[2]) if len(v) > 2 else 1
    steps = max(1, math.ceil(K / 32))
    fc, fp = 1, 1
    full = []
    for (a, b) in KW_TILES:
        tiles = math.ceil(cout / (16 * a)) * math.ceil(M / (16 * b))
        waste = tiles * 256 * a * b / max(1, M * cout)
        if tiles >= NUM_CUS and waste < 1.3:
            full.append((a * b, -waste, a, b))
    if full:
        _, _, fc, fp = max(full)
    kw = 1
    while kw * 2 <= 16 and steps / (kw * 2) >= 6 and kw * 2 * fc * fp <= 64 and 128 * kw <= kw_max_threads(fc * fp):
        kw *= 2
    return kw_cfg(fc, fp), 1, kw


def split_k_slice(K: int, splitk: int) -> int:
    steps = math.ceil(K / 32)
    return int(math.ceil(steps / splitk) * 32)


def workspace_bytes(M: int, cout: int, cfg: int, splitk: int) -> tuple[int, int]:
    """(slab bytes, counter ints) for a split-K launch."""
    if splitk <= 1 or cfg >= 100:
        return 0, 0
    wc, wp, fc, fp = CONV_CONFIGS[cfg]
    bnc, bmp = tile_dims(cfg)
    tiles = math.ceil(cout / bnc) * math.ceil(M / bmp)
    return tiles * splitk * fc * fp * 256 * 16, tiles


def make_params(x_ptr, pc: PackedConv, n, h, w, out_ptr, res_ptr=0, act="relu", out_f32=False,
                cfg=0, splitk=1, ws_ptr=0, cnt_ptr=0, ldo=None, ldr=None, kw=1) -> tuple[N.ConvParams, int, int]:
    p_out = (h + 2 * pc.pad - pc.r) // pc.stride + 1
    q_out = (w + 2 * pc.pad - pc.s) // pc.stride + 1
    M = n * p_out * q_out
    prm = N.ConvParams()
    prm.x, prm.w, prm.bias, prm.res, prm.out = x_ptr, pc.w.data_ptr(), pc.bias.data_ptr(), res_ptr, out_ptr
    prm.ws, prm.cnt = ws_ptr, cnt_ptr
    prm.N, prm.H, prm.W, prm.C = n, h, w, pc.cin
    prm.Cout, prm.R, prm.S, prm.stride, prm.pad, prm.P, prm.Q = pc.cout, pc.r, pc.s, pc.stride, pc.pad, p_out, q_out
    prm.M, prm.K, prm.ldw = M, pc.K, pc.ldw
    prm.ldo = ldo if ldo is not None else pc.cout
    prm.ldr = ldr if ldr is not None else pc.cout
    prm.act, prm.out_f32 = ACT[act], int(out_f32)
    prm.splitk, prm.kslice = splitk, split_k_slice(pc.K, splitk)
    prm.tiles_n = 0
    prm.kw = kw
    return prm, p_out, q_out


def conv2d_nhwc(x: torch.Tensor, pc: PackedConv, residual: torch.Tensor | None = None, act: str = "relu",
                out_f32: bool = False, cfg: int | None = None, splitk: int | None = None,
                kw: int | None = None) -> torch.Tensor:
    """Eager launch: x NHWC bf16 [N,H,W,Cin_pad] -> NHWC [N,P,Q,Cout] (bf16 or fp32)."""
    assert x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and x.shape[-1] == pc.cin
    n, h, w, _ = x.shape
    p_out = (h + 2 * pc.pad - pc.r) // pc.stride + 1
    q_out = (w + 2 * pc.pad - pc.s) // pc.stride + 1
    M = n * p_out * q_out
    if cfg is None:
        cfg, splitk, kw = choose_config(M, pc.cout, pc.K)
    splitk = 1 if splitk is None else splitk
    kw = 1 if kw is None else kw
    out = torch.empty(n, p_out, q_out, pc.cout, device=x.device,
                      dtype=torch.float32 if out_f32 else torch.bfloat16)
    ws_b, n_cnt = workspace_bytes(M, pc.cout, cfg, splitk)
    ws = torch.empty(max(ws_b, 16), dtype=torch.uint8, device=x.device)
    cnt = torch.zeros(max(n_cnt, 1), dtype=torch.int32, device=x.device)
    if residual is not None:
        assert residual.dtype == torch.bfloat16 and residual.is_contiguous()
        assert residual.numel() == M * pc.cout
    prm, _, _ = make_params(x.data_ptr(), pc, n, h, w, out.data_ptr(), N.ptr(residual), act, out_f32,
                            cfg, splitk, ws.data_ptr(), cnt.data_ptr(), kw=kw)
    N.check(N.lib().hz_conv_launch(prm, cfg, N.stream_ptr()), "hz_conv_launch")
    return out


def conv2d_reference(x_nchw: torch.Tensor, weight, bias=None, bn=None, stride=1, pad=0, residual=None,
                     act="relu", eps=1e-5) -> torch.Tensor:
    """fp32 PyTorch oracle of the fused op (NCHW in/out)."""
    w, b = fold_bn(weight, bias, bn, eps)
    y = torch.nn.functional.conv2d(x_nchw.float(), w, b, stride=stride, padding=pad)
    if residual is not None:
        y = y + residual.float()
    if act == "relu":
        y = torch.relu(y)
    elif act == "gelu":
        y = torch.nn.functional.gelu(y)
    elif act == "tanh":
        y = torch.tanh(y)
    return y
