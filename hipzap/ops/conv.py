"""Conv2d + folded BatchNorm + residual + activation on the native MFMA implicit-GEMM kernel.

Weights are packed ONCE at load time (``pack_conv``): BN folded in fp32, OIHW -> O,R,S,C
(K contiguous), input channels padded to a multiple of 8, K padded to a multiple of 32,
output rows padded to a multiple of 64, then re-ordered fragment-major
``[Cout_pad/16][K/32][64 lanes][8]`` so each wave's MFMA A-fragment load is one contiguous
1 KiB (csrc/conv.hip). A Linear layer is the 1x1 case on a 1x1 image (``pack_linear``).

Activation layout on device: channel-blocked ``[N][C/32][H][W][32]`` when C % 32 == 0,
plain NHWC otherwise (the 8-channel stem input). ``to_blocked``/``from_blocked`` convert.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from .. import _native as N

TILES = [(fc, fp) for fc in (1, 2, 4) for fp in (1, 2, 4)]  # cfg index -> (FC, FP)
ROW_PAD = 64        # conv weights: rows padded to the largest register-ring tile (64 channels)
GEMM_ROW_PAD = 128  # linear weights: rows padded to the largest LDS-tiled GEMM tile (csrc/gemm.hip)
# cfg >= 16: LDS-tiled GEMM (csrc/gemm.hip), row-major activations, K % 64 == 0 -> (BM, BN);
# 16-19 use 3 LDS stages, 20-23 the same tiles with 2 (half the LDS: more workgroups per CU)
LDS_TILES = {16: (128, 128), 17: (64, 128), 18: (128, 64), 19: (64, 64),
             20: (128, 128), 21: (64, 128), 22: (128, 64), 23: (64, 64),
             24: (128, 128), 25: (64, 128), 26: (128, 64), 27: (64, 64),  # 3 / 2 / 4 LDS stages
             28: (128, 128), 29: (128, 128), 30: (256, 128), 31: (128, 64), 32: (64, 128),
             33: (256, 64),  # 28-33: 8-wave workgroups
             34: (64, 96), 35: (128, 192), 36: (128, 192), 37: (64, 288), 38: (64, 288), 39: (256, 96),
             40: (64, 96)}  # 34-40: one tile per CU at M = 2048 (BERT) projection widths
# (cfg 64-77, the same LDS image read as 32x32x16 MFMA operands, were a measured negative,
# profiles/r3_m32, and were deleted in round 5; source: git history)
# the folded-LayerNorm epilogue (HzLnFold, experiments build) writes its statistics slabs per
# (feature tile, wave column) of a 2-column wave grid: LDS tiles with 4 wave columns map to the
# same tile with 2 (128x192 has none: 128x128)
LNF_REMAP = {28: 16, 29: 20, 32: 17, 35: 16, 36: 16}
# LDS tiles that also run as an implicit-GEMM conv on channel-blocked activations (csrc/gemm.hip CV
# mode; ResNet at batch >= 4): C % 64 == 0, Cout % BN == 0
LDS_CONV_CFGS = (16, 17, 18, 19, 20, 21, 22, 23, 28, 29, 30, 31, 32, 33)
LDS_CONV_MIN_M = 4096  # heuristic: below this the register-ring conv kernel (bs=1 shapes) stays
ACT = {"none": 0, "relu": 1, "gelu": 2, "tanh": 3}
NUM_CUS = 256


@dataclass
class PackedConv:
    wf: torch.Tensor         # bf16 fragment-major [rows_pad/16, ksteps, 64, 8]
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
    def ksteps(self) -> int:
        return self.wf.shape[1]

    def dense(self) -> torch.Tensor:
        """Row-major [cout, K] view of the packed weights (fp32; for oracles/tests)."""
        g, ks = self.wf.shape[0], self.wf.shape[1]
        w = self.wf.float().reshape(g, ks, 4, 16, 8).permute(0, 3, 1, 2, 4).reshape(g * 16, ks * 32)
        return w[: self.cout, : self.K]

    def to(self, device) -> "PackedConv":
        return PackedConv(self.wf.to(device), self.bias.to(device), self.cin, self.cout, self.r, self.s,
                          self.stride, self.pad)


def fold_bn(weight: torch.Tensor, bias: torch.Tensor | None, bn: dict | None, eps: float = 1e-5):
    """Fold eval-mode BatchNorm into conv weight/bias (fp32).

    The per-channel scale gamma / sqrt(var + eps) is computed in float64 and rounded once: torch's
    CPU sqrt is not correctly rounded (SLEEF), so a float32 scale would differ by an ulp from the
    torch-free packers (engine/nppack.py, the device pack kernel in csrc/pack.hip) in ~1 % of
    channels; the rest (w * scale, (b - mean) * scale + beta) is plain IEEE float32 everywhere."""
    w = weight.detach().float()
    b = bias.detach().float() if bias is not None else torch.zeros(w.shape[0], device=w.device)
    if bn is not None:
        scale = (bn["weight"].double() / torch.sqrt(bn["running_var"].double() + eps)).float()
        w = w * scale.view(-1, *([1] * (w.dim() - 1)))
        b = (b - bn["running_mean"].float()) * scale + bn["bias"].float()
    return w, b


def fragment_major(w2d: torch.Tensor) -> torch.Tensor:
    """[rows, K] (rows % 16 == 0, K % 32 == 0) -> [rows/16, K/32, 64, 8]; lane = kc*16 + row."""
    rows, K = w2d.shape
    return w2d.reshape(rows // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).reshape(rows // 16, K // 32, 64, 8)


def pack_matrix(w2d: torch.Tensor, bias: torch.Tensor, cin: int, r: int = 1, s: int = 1, stride: int = 1,
                pad: int = 0, row_pad: int = ROW_PAD) -> PackedConv:
    cout, K = w2d.shape
    ksteps = int(math.ceil(K / 32))
    rows = int(math.ceil(cout / row_pad) * row_pad)
    wp = torch.zeros(rows, ksteps * 32, dtype=torch.bfloat16, device=w2d.device)
    wp[:cout, :K] = w2d.to(torch.bfloat16)
    return PackedConv(fragment_major(wp).contiguous(), bias.float().contiguous(), cin, cout, r, s, stride, pad)


def pack_conv(weight, bias=None, bn=None, stride=1, pad=0, eps=1e-5, cin_pad: int | None = None) -> PackedConv:
    w, b = fold_bn(weight, bias, bn, eps)
    cout, cin, r, s = w.shape
    cin_p = cin_pad or int(math.ceil(cin / 8) * 8)
    w = w.permute(0, 2, 3, 1)  # O,R,S,C
    if cin_p != cin:
        w = torch.nn.functional.pad(w, (0, cin_p - cin))
    return pack_matrix(w.reshape(cout, r * s * cin_p), b, cin_p, r, s, stride, pad)


def pack_linear(weight, bias=None) -> PackedConv:
    b = bias if bias is not None else torch.zeros(weight.shape[0], device=weight.device)
    cin = weight.shape[1]
    assert cin % 8 == 0
    return pack_matrix(weight.detach().float(), b.detach().float(), cin, row_pad=GEMM_ROW_PAD)


# ----------------------------------------------------------------------------- layouts
def is_blocked(c: int) -> bool:
    return c % 32 == 0


def to_blocked(x_nhwc: torch.Tensor) -> torch.Tensor:
    """[N,H,W,C] -> [N, C/32, H, W, 32] (contiguous) when C % 32 == 0, else unchanged."""
    n, h, w, c = x_nhwc.shape
    if not is_blocked(c):
        return x_nhwc.contiguous()
    return x_nhwc.reshape(n, h, w, c // 32, 32).permute(0, 3, 1, 2, 4).contiguous()


def from_blocked(t: torch.Tensor, shape) -> torch.Tensor:
    """Inverse of :func:`to_blocked` for a logical NHWC ``shape``."""
    n, h, w, c = shape
    if not is_blocked(c):
        return t.reshape(n, h, w, c)
    return t.reshape(n, c // 32, h, w, 32).permute(0, 2, 3, 1, 4).reshape(n, h, w, c)


# ----------------------------------------------------------------------------- configs
def max_threads(nf: int) -> int:
    return 256 if nf >= 16 else 512 if nf >= 8 else 1024


def cfg_of(fc: int, fp: int) -> int:
    return TILES.index((fc, fp))


def tile_of(cfg: int) -> tuple[int, int]:
    """(channels, pixels) of one output tile."""
    if cfg in LDS_TILES:
        bm, bn = LDS_TILES[cfg]
        return bn, bm
    fc, fp = TILES[cfg]
    return fc * 16, fp * 16


def lds_ok(M: int, K: int, rowmajor: bool, pc: PackedConv | None = None) -> bool:
    """Can the LDS-tiled GEMM run this shape? (row-major activations, K % 64, rows padded to 128)."""
    if not rowmajor or K % 64 or M < 64:
        return False
    return pc is None or (pc.wf.shape[0] % (GEMM_ROW_PAD // 16) == 0 and pc.ksteps * 32 == K)


def lds_conv_ok(M: int, pc: PackedConv | None, n_in_bytes: int | None = None) -> bool:
    """Can the LDS tile run this conv as an implicit GEMM (csrc/gemm.hip CV mode)?"""
    if pc is None or M < 64 or pc.cin % 64 or pc.cout % 32 or pc.ksteps * 32 != pc.K:
        return False
    return n_in_bytes is None or n_in_bytes < 2 ** 31


def lds_conv_fits(cfg: int, cout: int) -> bool:
    return cfg in LDS_CONV_CFGS and cout % LDS_TILES[cfg][1] == 0


def lds_fits(cfg: int, cout: int) -> bool:
    """The last BN-wide feature tile stays inside the GEMM_ROW_PAD-padded weight rows."""
    bn = LDS_TILES[cfg][1]
    return math.ceil(cout / bn) * bn <= math.ceil(cout / GEMM_ROW_PAD) * GEMM_ROW_PAD


def legal(cfg: int, kw: int) -> bool:
    if cfg in LDS_TILES:
        return kw == 1
    fc, fp = TILES[cfg]
    return 1 <= kw <= 16 and kw & (kw - 1) == 0 and kw * fc * fp <= 64 and 64 * kw <= max_threads(fc * fp)


def candidates(M: int, cout: int, K: int, rowmajor: bool = False, pc: PackedConv | None = None) -> list[tuple[int, int]]:
    """All legal (cfg, kw) launch choices worth timing for one conv / GEMM shape."""
    steps = max(1, math.ceil(K / 32))
    out = []
    if lds_ok(M, K, rowmajor, pc):
        out += [(cfg, 1) for cfg in LDS_TILES if lds_fits(cfg, cout)]
    elif not rowmajor and lds_conv_ok(M, pc):
        out += [(cfg, 1) for cfg in LDS_CONV_CFGS if lds_conv_fits(cfg, cout)]
    for cfg, (fc, fp) in enumerate(TILES):
        if (fc > 1 and fc * 16 > cout) or (fp > 1 and fp * 16 > M):
            continue
        for kw in (1, 2, 4, 8, 16):
            if not legal(cfg, kw) or (kw > 1 and steps / kw < 2):
                continue
            out.append((cfg, kw))
    return out


def choose_config(M: int, cout: int, K: int, tuned: dict | None = None, key: str | None = None,
                  rowmajor: bool = False, pc: PackedConv | None = None):
    """Pick (cfg, kw) for an implicit GEMM of M pixels x cout channels x K.

    A measured table (``tuned``, produced on the GPU by ``hipzap.engine.tune``) wins. The
    fallback heuristic: the largest output tile that still yields >= 1 workgroup per CU
    with < 30 % padding waste (else 16x16 tiles), then enough waves per workgroup that each
    wave streams ~6 K-steps.
    """
    if tuned is not None and key is not None and key in tuned:
        v = tuned[key]
        c = int(v[0])
        if (c not in LDS_TILES or (lds_ok(M, K, rowmajor, pc) and lds_fits(c, cout))
                or (not rowmajor and lds_conv_ok(M, pc) and lds_conv_fits(c, cout))):
            return c, int(v[1])
    if not rowmajor and M >= LDS_CONV_MIN_M and K >= 256 and lds_conv_ok(M, pc):
        # large-M conv (batched ResNet): the biggest LDS tile that still gives every CU a workgroup,
        # 8-wave tiles first (the bs=32 tuner's winners, profiles/r2_conv_lds); K = 64 1x1 convs are
        # store-bound and stay on the register-ring kernel
        for cfg in (29, 32, 33, 31, 19):
            bm, bn = LDS_TILES[cfg]
            if lds_conv_fits(cfg, cout) and math.ceil(M / bm) * (cout // bn) >= NUM_CUS:
                return cfg, 1
        return 19, 1
    if lds_ok(M, K, rowmajor, pc) and M >= 512:
        # large-M GEMM: the biggest LDS tile that still gives every CU a workgroup
        for cfg in (16, 17, 18, 19):
            bm, bn = LDS_TILES[cfg]
            if math.ceil(M / bm) * math.ceil(cout / bn) >= NUM_CUS:
                return cfg, 1
        return 19, 1
    steps = max(1, math.ceil(K / 32))
    fc, fp = 1, 1
    full = []
    for (a, b) in TILES:
        tiles = math.ceil(cout / (16 * a)) * math.ceil(M / (16 * b))
        waste = tiles * 256 * a * b / max(1, M * cout)
        if tiles >= NUM_CUS and waste < 1.3:
            full.append((a * b, -waste, a, b))
    if full:
        _, _, fc, fp = max(full)
    cfg = cfg_of(fc, fp)
    kw = 1
    while steps / (kw * 2) >= 6 and legal(cfg, kw * 2):
        kw *= 2
    return cfg, kw


def conv_key(M: int, pc: PackedConv) -> str:
    return f"{M}x{pc.cout}x{pc.K}x{pc.r}{pc.s}s{pc.stride}"


def make_params(x_ptr, pc: PackedConv, n, h, w, out_ptr, res_ptr=0, act="relu", out_f32=False,
                cfg=0, kw=1, out_rowmajor=False, ldo=None, x_rowmajor=False, ldx=None) -> tuple[N.ConvParams, int, int]:
    p_out = (h + 2 * pc.pad - pc.r) // pc.stride + 1
    q_out = (w + 2 * pc.pad - pc.s) // pc.stride + 1
    prm = N.ConvParams()
    prm.x, prm.w, prm.bias, prm.res, prm.out = x_ptr, pc.wf.data_ptr(), pc.bias.data_ptr(), res_ptr, out_ptr
    prm.N, prm.H, prm.W, prm.C = n, h, w, pc.cin
    prm.Cout, prm.R, prm.S, prm.stride, prm.pad, prm.P, prm.Q = pc.cout, pc.r, pc.s, pc.stride, pc.pad, p_out, q_out
    prm.M, prm.K, prm.ksteps = n * p_out * q_out, pc.K, pc.ksteps
    prm.act, prm.out_f32 = ACT[act], int(out_f32)
    rowmajor = out_rowmajor or not is_blocked(pc.cout)
    prm.out_rowmajor, prm.ldo = int(rowmajor), ldo if ldo is not None else pc.cout
    prm.x_rowmajor, prm.ldx = int(x_rowmajor), ldx if ldx is not None else pc.cin
    prm.tiles_n, prm.kw = 0, kw
    return prm, p_out, q_out


def linear(x: torch.Tensor, pc: PackedConv, residual: torch.Tensor | None = None, act: str = "none",
           out_f32: bool = False, cfg: int | None = None, kw: int | None = None, out: torch.Tensor | None = None,
           ldx: int | None = None, rows: int | None = None) -> torch.Tensor:
    """Eager GEMM: y[M,N] = act(x[M,K] @ W^T + b (+ residual)); x row-major (stride ``ldx``)."""
    M = rows if rows is not None else x.shape[0]
    if cfg is None:
        cfg, kw = choose_config(M, pc.cout, pc.K, rowmajor=True, pc=pc)
    if cfg in LDS_TILES:
        assert lds_ok(M, pc.K, True, pc) and (ldx if ldx is not None else x.stride(0)) % 8 == 0
    kw = kw or 1
    if out is None:
        out = torch.empty(M, pc.cout, device=x.device, dtype=torch.float32 if out_f32 else torch.bfloat16)
    prm, _, _ = make_params(x.data_ptr(), pc, M, 1, 1, out.data_ptr(), N.ptr(residual), act, out_f32, cfg, kw,
                            out_rowmajor=True, ldo=out.stride(0), x_rowmajor=True,
                            ldx=ldx if ldx is not None else x.stride(0))
    N.check(N.lib().hz_conv_launch(prm, cfg, N.stream_ptr()), "hz_conv_launch(linear)")
    return out


def conv2d_nhwc(x: torch.Tensor, pc: PackedConv, residual: torch.Tensor | None = None, act: str = "relu",
                out_f32: bool = False, cfg: int | None = None, kw: int | None = None) -> torch.Tensor:
    """Eager launch on logical NHWC tensors (converted to/from the device layout)."""
    assert x.is_cuda and x.dtype == torch.bfloat16 and x.shape[-1] == pc.cin
    n, h, w, _ = x.shape
    p_out = (h + 2 * pc.pad - pc.r) // pc.stride + 1
    q_out = (w + 2 * pc.pad - pc.s) // pc.stride + 1
    M = n * p_out * q_out
    if cfg is None:
        cfg, kw = choose_config(M, pc.cout, pc.K, pc=pc if is_blocked(pc.cin) else None)
    kw = kw or 1
    xb = to_blocked(x)
    oshape = (n, p_out, q_out, pc.cout)
    out = torch.empty(M * pc.cout, device=x.device, dtype=torch.float32 if out_f32 else torch.bfloat16)
    rb = None
    if residual is not None:
        assert residual.dtype == torch.bfloat16 and tuple(residual.shape) == oshape
        rb = to_blocked(residual) if is_blocked(pc.cout) else residual.contiguous()
    prm, _, _ = make_params(xb.data_ptr(), pc, n, h, w, out.data_ptr(), N.ptr(rb), act, out_f32, cfg, kw)
    N.check(N.lib().hz_conv_launch(prm, cfg, N.stream_ptr()), "hz_conv_launch")
    if prm.out_rowmajor:
        return out.reshape(oshape)
    return from_blocked(out, oshape)


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
