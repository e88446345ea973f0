"""FP8 (OCP e4m3fn) weight packing, activation quantisation and the fp8 MFMA GEMM.

Weights: per-output-channel scale ``s_n = amax_n / 448``, ``w8 = e4m3(w / s_n)``, packed
fragment-major ``[N_pad/16][K/32][64][8]`` bytes (csrc/fp8.hip). Activations: per-row dynamic
scale computed on device by ``quant_rows`` right before each GEMM.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass

import torch

from .. import _native as N
from .conv import PackedConv, choose_config, fragment_major

K_QUANT, K_GEMM_FP8 = 10, 11
FP8_MAX = 448.0


class QuantParams(C.Structure):
    _fields_ = [("x", C.c_void_p), ("out", C.c_void_p), ("scale", C.c_void_p), ("rows", C.c_int), ("D", C.c_int),
                ("ldx", C.c_int), ("ldo", C.c_int)]


class GemmFp8Params(C.Structure):
    _fields_ = [("x", C.c_void_p), ("sx", C.c_void_p), ("w", C.c_void_p), ("sw", C.c_void_p), ("bias", C.c_void_p),
                ("res", C.c_void_p), ("out", C.c_void_p), ("M", C.c_int), ("N", C.c_int), ("K", C.c_int),
                ("ksteps", C.c_int), ("ldx", C.c_int), ("ldo", C.c_int), ("act", C.c_int), ("out_f32", C.c_int),
                ("cfg", C.c_int), ("kw", C.c_int), ("wmx", C.c_void_p), ("xs", C.c_void_p), ("out8", C.c_void_p),
                ("os8", C.c_void_p)]


@dataclass
class PackedFp8:
    w8: torch.Tensor     # uint8 (e4m3fn bits) fragment-major [rows_pad/16, ksteps, 64, 8]
    sw: torch.Tensor     # fp32 [rows_pad] per-output-channel scales
    bias: torch.Tensor   # fp32 [cout]
    cin: int             # K
    cout: int
    w8mx: torch.Tensor | None = None  # MX-packed copy [rows_pad/16, K/128, 2, 64, 16] for the LDS GEMM

    @property
    def K(self) -> int:
        return self.cin

    @property
    def ksteps(self) -> int:
        return self.w8.shape[1]

    def dequant(self) -> torch.Tensor:
        g, ks = self.w8.shape[0], self.w8.shape[1]
        w = self.w8.view(torch.float8_e4m3fn).float()
        w = w.reshape(g, ks, 4, 16, 8).permute(0, 3, 1, 2, 4).reshape(g * 16, ks * 32)
        w = w * self.sw.float().reshape(-1, 1)
        return w[: self.cout, : self.K]


def quantize_weight(w2d: torch.Tensor, rows_pad: int | None = None):
    """[N, K] float -> (e4m3fn bits [N_pad, K_pad] uint8, scales [N_pad])."""
    n, k = w2d.shape
    rows = rows_pad or n
    kp = int(math.ceil(k / 32) * 32)
    amax = w2d.float().abs().amax(dim=1).clamp_min(1e-12)
    s = amax / FP8_MAX
    q = torch.zeros(rows, kp, dtype=torch.float8_e4m3fn, device=w2d.device)
    q[:n, :k] = (w2d.float() / s.reshape(-1, 1)).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn)
    sw = torch.ones(rows, device=w2d.device)
    sw[:n] = s
    return q.view(torch.uint8), sw


def mx_pack(q: torch.Tensor) -> torch.Tensor:
    """[rows, K] e4m3 bytes (rows % 16 == 0, K % 128 == 0) -> [rows/16, K/128, 2, 64, 16]:
    lane l = 16*lg + row%16, register half h holds k%128 = 64*h + 16*lg + byte — the hardware K
    order of v_mfma_scale_f32_16x16x128_f8f6f4, which the E8M0 block scales follow (pinned by
    tests/test_fp8_gpu.py::test_mfma_block_scale_kblock_map)."""
    rows, K = q.shape
    t = q.reshape(rows // 16, 16, K // 128, 2, 4, 16)          # g, r, kb, half, lg, byte
    return t.permute(0, 2, 3, 4, 1, 5).reshape(rows // 16, K // 128, 2, 64, 16)


def mx_unpack(w: torch.Tensor) -> torch.Tensor:
    g, kb = w.shape[0], w.shape[1]
    return w.reshape(g, kb, 2, 4, 16, 16).permute(0, 4, 1, 2, 3, 5).reshape(g * 16, kb * 128)


def quantize_linear(pc: PackedConv) -> PackedFp8:
    if pc.r != 1 or pc.s != 1:
        raise ValueError("fp8 path is for Linear layers")
    rows = pc.wf.shape[0] * 16
    q, sw = quantize_weight(pc.dense(), rows)
    mx = mx_pack(q).contiguous() if (pc.K % 128 == 0 and rows % 128 == 0) else None
    return PackedFp8(fragment_major(q).contiguous(), sw.contiguous(), pc.bias.float().contiguous(), pc.K, pc.cout, mx)


# cfg -> (BM, BN), csrc/fp8.hip gemm_mx_kernel; 16-19: 3 LDS stages, 20-23: 2 stages
MX_TILES = {16: (128, 128), 17: (64, 128), 18: (128, 64), 19: (64, 64),
            20: (128, 128), 21: (64, 128), 22: (128, 64), 23: (64, 64),
            # 24-29: 8-wave workgroups (2 / 3 stages); N must be a multiple of BN
            24: (128, 128), 25: (256, 128), 26: (128, 256), 27: (128, 128), 28: (256, 128), 29: (128, 256),
            # 30-32: 4 LDS stages (8-wave 128x128; 4-wave 64x128, 128x64)
            30: (128, 128), 31: (64, 128), 32: (128, 64),
            # 33: 8-wave 256x256 (plain). Removed in round 5 with their negatives committed: 34-36
            # (ping-pong, profiles/r4_mx), 43-47 (256-row tiles, profiles/r3_mx256, r3_mxk)
            33: (256, 256),
            # 40 / 41 / 42: role-split 128x128 (8 MFMA waves + 2 loader waves, LDS FULL / FREE counters), 4 / 3 / 2
            # stages (profiles/r6_mx: 1.2-1.5x slower than cfg 24)
            40: (128, 128), 41: (128, 128), 42: (128, 128)}
MX_WIDE = (24, 25, 26, 27, 28, 29, 30, 33, 40, 41, 42)
MX_PERROW_ONLY = ()
MX_EXPERIMENTS = ()  # MX tiles that exist only in the HZ_EXPERIMENTS library: none left


def mx_fits(cfg: int, n: int) -> bool:
    return cfg not in MX_WIDE or n % MX_TILES[cfg][1] == 0


def mx_ok(M: int, pw: PackedFp8, ldx: int | None = None) -> bool:
    return pw.w8mx is not None and M >= 64 and pw.K % 128 == 0 and (ldx or pw.K) % 16 == 0


def candidates_fp8(M: int, pw: PackedFp8, mx_io: bool = False) -> list:
    from .conv import candidates
    exp = N.experiments()
    out = [(cfg, 1) for cfg in MX_TILES if mx_fits(cfg, pw.cout) and (exp or cfg not in MX_EXPERIMENTS)
           and not (mx_io and cfg in MX_PERROW_ONLY)] if mx_ok(M, pw) else []
    # the fp8 launcher reads cfg >= 16 as an MX tile: the bf16-only 32x32 LDS tiles do not exist there
    return out if mx_io else out + [c for c in candidates(M, pw.cout, pw.K) if c[0] < 64]


def choose_config_fp8(M: int, pw: PackedFp8, tuned: dict | None = None, key: str | None = None, mx_io=False):
    """``mx_io``: MX8 input or output -> only the MX LDS kernel can run it."""
    if tuned is not None and key is not None and key in tuned:
        cfg, kw = int(tuned[key][0]), int(tuned[key][1])
        if (cfg not in MX_TILES and not mx_io) or (cfg in MX_TILES and mx_ok(M, pw) and mx_fits(cfg, pw.cout)):
            return cfg, kw
    if mx_ok(M, pw) and (M >= 512 or mx_io):
        for cfg in (16, 17, 18, 19):
            bm, bn = MX_TILES[cfg]
            if math.ceil(M / bm) * math.ceil(pw.cout / bn) >= 256:
                return cfg, 1
        return 19, 1
    return choose_config(M, pw.cout, pw.K)


def quantize_params(P: dict, names) -> dict:
    out = dict(P)
    for n in names:
        if isinstance(P[n], PackedConv):
            out[n] = quantize_linear(P[n])
    return out


def quant_mx_ref(x: torch.Tensor, block: int = 32):
    """fp32 oracle of MX8 (OCP MX e4m3, one E8M0 scale per ``block`` columns): returns
    (dequantised x, exponents [rows, cols/block]) with 2^e the smallest power of two such
    that amax / 2^e <= 448 (frexp rule, csrc/common.h mx_exp)."""
    x = x.float()
    r, c = x.shape
    xb = x.reshape(r, c // block, block)
    amax = xb.abs().amax(-1)
    _, e = torch.frexp(amax / FP8_MAX)
    e = torch.where(amax > 0, e, torch.full_like(e, -127)).clamp(-127, 127)
    sc = torch.ldexp(torch.ones_like(amax), e)
    q = (xb / sc.unsqueeze(-1)).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn).float()
    return (q * sc.unsqueeze(-1)).reshape(r, c), e


def quant_rows_ref(x: torch.Tensor):
    """fp32 oracle of quant_rows: returns (dequantised x, scales)."""
    x = x.float()
    s = x.abs().amax(dim=-1).clamp_min(1e-12) / FP8_MAX
    q = (x / s.unsqueeze(-1)).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn).float()
    return q * s.unsqueeze(-1), s


# ----------------------------------------------------------------------------- eager
def quant_rows(x: torch.Tensor):
    rows, D = x.shape
    out = torch.empty(rows, D, dtype=torch.uint8, device=x.device)
    sc = torch.empty(rows, dtype=torch.float32, device=x.device)
    prm = QuantParams(x.data_ptr(), out.data_ptr(), sc.data_ptr(), rows, D, x.stride(0), out.stride(0))
    N.check(N.lib().hz_launch_kernel(K_QUANT, C.byref(prm), N.stream_ptr()), "quant_rows")
    return out, sc


def gemm_params(x8_ptr, sx_ptr, pw: PackedFp8, M, out_ptr, res_ptr=0, act="none", out_f32=False, cfg=0, kw=1,
                ldx=None, ldo=None, xs_ptr=0, out8_ptr=0, os8_ptr=0) -> GemmFp8Params:
    """``sx_ptr``: per-row fp32 activation scales, or ``xs_ptr``: MX8 block scales [M][K/32];
    ``out8_ptr``/``os8_ptr``: write MX8 (e4m3 + E8M0 per 32 columns) instead of ``out_ptr``."""
    from .conv import ACT
    if cfg in MX_TILES and not mx_ok(M, pw, ldx):
        raise ValueError(f"MX fp8 GEMM config {cfg} not legal for M={M} K={pw.K}")
    if (xs_ptr or out8_ptr) and cfg not in MX_TILES:
        raise ValueError("MX8 activations need an MX (LDS) GEMM config")
    return GemmFp8Params(x8_ptr, sx_ptr, pw.w8.data_ptr(), pw.sw.data_ptr(), pw.bias.data_ptr(), res_ptr, out_ptr, M,
                         pw.cout, pw.K, pw.ksteps, ldx if ldx is not None else pw.K,
                         ldo if ldo is not None else pw.cout, ACT[act], int(out_f32), cfg, kw,
                         pw.w8mx.data_ptr() if pw.w8mx is not None else 0, xs_ptr, out8_ptr, os8_ptr)


def gemm_fp8(x8: torch.Tensor, sx: torch.Tensor, pw: PackedFp8, residual=None, act="none", out_f32=False,
             cfg=None, kw=None) -> torch.Tensor:
    M = x8.shape[0]
    if cfg is None:
        cfg, kw = choose_config_fp8(M, pw)
    out = torch.empty(M, pw.cout, device=x8.device, dtype=torch.float32 if out_f32 else torch.bfloat16)
    prm = gemm_params(x8.data_ptr(), sx.data_ptr(), pw, M, out.data_ptr(), N.ptr(residual), act, out_f32, cfg,
                      kw or 1, x8.stride(0), out.stride(0))
    N.check(N.lib().hz_launch_kernel(K_GEMM_FP8, C.byref(prm), N.stream_ptr()), "gemm_fp8")
    return out
