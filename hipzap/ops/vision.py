"""Eager wrappers + fp32 oracles for the vision helper kernels (csrc/vision.hip)."""
from __future__ import annotations

import ctypes as C

import torch

from .. import _native as N

K_POOL_FC = 13


class PoolFcParams(C.Structure):
    _fields_ = [("x", C.c_void_p), ("w", C.c_void_p), ("bias", C.c_void_p), ("out", C.c_void_p), ("B", C.c_int),
                ("C", C.c_int), ("HW", C.c_int), ("N", C.c_int), ("ldo", C.c_int),
                ("pooled", C.c_int), ("pad_", C.c_int)]

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def maxpool_nhwc(x: torch.Tensor, k=3, stride=2, pad=1) -> torch.Tensor:
    n, h, w, c = x.shape
    p = (h + 2 * pad - k) // stride + 1
    q = (w + 2 * pad - k) // stride + 1
    out = torch.empty(n, p, q, c, device=x.device, dtype=torch.bfloat16)
    prm = N.PoolParams(x.data_ptr(), out.data_ptr(), n, h, w, c, p, q, k, stride, pad)
    N.check(N.lib().hz_maxpool_launch(prm, N.stream_ptr()), "maxpool")
    return out


def avgpool_nhwc(x: torch.Tensor, blocked: bool = False) -> torch.Tensor:
    """x: logical [N,H,W,C]; ``blocked`` stores it channel-blocked on device first."""
    from .conv import to_blocked
    n, h, w, c = x.shape
    src = to_blocked(x) if blocked else x.contiguous()
    out = torch.empty(n, c, device=x.device, dtype=torch.bfloat16)
    N.check(N.lib().hz_avgpool_launch(src.data_ptr(), out.data_ptr(), n, h * w, c, int(blocked), N.stream_ptr()),
            "avgpool")
    return out


def pool_fc(x: torch.Tensor, pc, blocked_input: bool = False) -> torch.Tensor:
    """Fused global-average-pool + Linear: x logical [B,H,W,C] bf16 -> fp32 logits [B, cout]."""
    from .conv import to_blocked
    b, h, w, c = x.shape
    assert c == pc.K == pc.ksteps * 32 and c % 32 == 0
    src = x if blocked_input else to_blocked(x)
    out = torch.empty(b, pc.cout, device=x.device, dtype=torch.float32)
    prm = PoolFcParams(src.data_ptr(), pc.wf.data_ptr(), pc.bias.data_ptr(), out.data_ptr(), b, c, h * w, pc.cout,
                       pc.cout)
    N.check(N.lib().hz_launch_kernel(K_POOL_FC, C.byref(prm), N.stream_ptr()), "pool_fc")
    return out


def pool_fc_ref(x: torch.Tensor, pc) -> torch.Tensor:
    """fp32 oracle: x logical [B,H,W,C]."""
    pooled = x.float().mean(dim=(1, 2))
    return pooled @ pc.dense().float().t() + pc.bias.float()


def preprocess(src: torch.Tensor, cpad: int = 8, mean=None, std=None) -> torch.Tensor:
    """fp32 NCHW (mode 0) or uint8 NHWC (mode 1) -> bf16 NHWC with ``cpad`` channels."""
    if src.dtype == torch.uint8:
        n, h, w, cin = src.shape
        mode = 1
    else:
        n, cin, h, w = src.shape
        mode = 0
    out = torch.empty(n, h, w, cpad, device=src.device, dtype=torch.bfloat16)
    mean_t = inv_t = None
    if mean is not None:
        mean_t = torch.tensor(mean, dtype=torch.float32, device=src.device)
        inv_t = 1.0 / torch.tensor(std, dtype=torch.float32, device=src.device)
    N.check(N.lib().hz_preprocess_launch(src.data_ptr(), out.data_ptr(), n, cin, h, w, cpad, mode,
                                         N.ptr(mean_t), N.ptr(inv_t), N.stream_ptr()), "preprocess")
    return out


def patchify(src: torch.Tensor, patch: int = 16, mean=None, std=None) -> torch.Tensor:
    """fp32 NCHW -> bf16 patch rows [N*(H/P)*(W/P)][C*P*P], columns in (c, ky, kx) order (preprocess
    mode 2, csrc/vision.hip patchify_kernel: the ViT patch embedding's GEMM operand)."""
    n, cin, h, w = src.shape
    out = torch.empty(n * (h // patch) * (w // patch), cin * patch * patch, device=src.device, dtype=torch.bfloat16)
    mean_t = inv_t = None
    if mean is not None:
        mean_t = torch.tensor(mean, dtype=torch.float32, device=src.device)
        inv_t = 1.0 / torch.tensor(std, dtype=torch.float32, device=src.device)
    N.check(N.lib().hz_preprocess_launch(src.data_ptr(), out.data_ptr(), n, cin, h, w, patch, 2,
                                         N.ptr(mean_t), N.ptr(inv_t), N.stream_ptr()), "patchify")
    return out


def patchify_reference(src: torch.Tensor, patch: int = 16) -> torch.Tensor:
    n, c, h, w = src.shape
    x = src.float().reshape(n, c, h // patch, patch, w // patch, patch).permute(0, 2, 4, 1, 3, 5)
    return x.reshape(n * (h // patch) * (w // patch), c * patch * patch).to(torch.bfloat16)


def preprocess_reference(src: torch.Tensor, cpad: int = 8, mean=None, std=None) -> torch.Tensor:
    if src.dtype == torch.uint8:
        x = src.float() / 255.0
    else:
        x = src.float().permute(0, 2, 3, 1)
    if mean is not None:
        x = (x - torch.tensor(mean, device=x.device)) / torch.tensor(std, device=x.device)
    return torch.nn.functional.pad(x, (0, cpad - x.shape[-1]))
