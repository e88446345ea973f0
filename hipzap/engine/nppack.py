"""Torch-free packing of a ResNet state_dict for the plan runtime (numpy only).

The same transformation as ``ops/conv.py`` ``pack_conv`` / ``pack_linear`` and
``models/resnet.py`` ``pack_resnet`` -- eval BatchNorm folded into each conv in fp32, OIHW ->
O,R,S,C with input channels padded to 8, K padded to 32, rows padded to 64 (conv) / 128 (linear),
bf16 (round to nearest even), fragment-major ``[rows/16][K/32][64][8]`` -- written with numpy so a
``.pth`` checkpoint (read by :mod:`hipzap.pthreader`) can be packed and served without importing
torch. Every float32 operation is the one torch performs, in the same order, so the packed bytes
are bitwise those of the torch path (``tests/test_pth_lite_cpu.py``).

numpy is imported only by the packing functions: ``pack_sources`` / ``conv_geometry`` /
``infer_resnet`` (the recipe side, used by the torch-free cold start) need no third-party module.

The result maps each packed parameter to ``{"wf": uint16 array, "bias": float32 array}``, the
two tensor fields of :class:`hipzap.ops.conv.PackedConv`, which a weightless plan template
(``engine/plan.py`` ``export_template``) places in its device blob by name.
"""
from __future__ import annotations

import math

ROW_PAD = 64        # ops/conv.py ROW_PAD
GEMM_ROW_PAD = 128  # ops/conv.py GEMM_ROW_PAD
ARCHS = {"resnet18": ("basic", [2, 2, 2, 2]), "resnet34": ("basic", [3, 4, 6, 3]),
         "resnet50": ("bottleneck", [3, 4, 6, 3]), "resnet101": ("bottleneck", [3, 4, 23, 3])}


def bf16_bits(x: np.ndarray) -> np.ndarray:
    """float32 -> bfloat16 bit patterns, round to nearest even (torch's conversion; NaN -> 0x7FC0)."""
    import numpy as np
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32)
    out = ((u + (np.uint32(0x7FFF) + ((u >> np.uint32(16)) & np.uint32(1)))) >> np.uint32(16)).astype(np.uint16)
    nan = np.isnan(x)
    if nan.any():
        out[nan] = 0x7FC0
    return out


def fragment_major(w2d: np.ndarray) -> np.ndarray:
    import numpy as np
    rows, K = w2d.shape
    return np.ascontiguousarray(w2d.reshape(rows // 16, 16, K // 32, 4, 8).transpose(0, 2, 3, 1, 4)).reshape(
        rows // 16, K // 32, 64, 8)


def pack_matrix(w2d: np.ndarray, bias: np.ndarray, row_pad: int = ROW_PAD) -> dict:
    import numpy as np
    cout, K = w2d.shape
    ksteps = int(math.ceil(K / 32))
    rows = int(math.ceil(cout / row_pad) * row_pad)
    wp = np.zeros((rows, ksteps * 32), np.uint16)
    wp[:cout, :K] = bf16_bits(w2d)
    return {"wf": fragment_major(wp), "bias": np.ascontiguousarray(bias, dtype=np.float32)}


def fold_bn(weight: np.ndarray, bn: dict | None, eps: float = 1e-5):
    import numpy as np
    w = np.asarray(weight, np.float32)
    b = np.zeros(w.shape[0], np.float32)
    if bn is not None:
        # float64 scale rounded once (ops/conv.py fold_bn)
        scale = (np.asarray(bn["weight"], np.float64) /
                 np.sqrt(np.asarray(bn["running_var"], np.float32).astype(np.float64) + eps)).astype(np.float32)
        w = w * scale.reshape((-1,) + (1,) * (w.ndim - 1))
        b = (b - np.asarray(bn["running_mean"], np.float32)) * scale + np.asarray(bn["bias"], np.float32)
    return w, b


def pack_conv(weight, bn=None, eps: float = 1e-5, cin_pad: int | None = None) -> dict:
    import numpy as np
    w, b = fold_bn(weight, bn, eps)
    cout, cin, r, s = w.shape
    cin_p = cin_pad or int(math.ceil(cin / 8) * 8)
    w = w.transpose(0, 2, 3, 1)  # O,R,S,C
    if cin_p != cin:
        w = np.pad(w, ((0, 0), (0, 0), (0, 0), (0, cin_p - cin)))
    return pack_matrix(np.ascontiguousarray(w).reshape(cout, r * s * cin_p), b)


def pack_linear(weight, bias=None) -> dict:
    import numpy as np
    w = np.asarray(weight, np.float32)
    b = np.zeros(w.shape[0], np.float32) if bias is None else np.asarray(bias, np.float32)
    assert w.shape[1] % 8 == 0
    return pack_matrix(w, b, row_pad=GEMM_ROW_PAD)


def infer_resnet(sd: dict) -> tuple[str, int]:
    """(arch, num_classes) from the key layout (models/resnet.py infer_arch, without torch)."""
    nblk = [len({k.split(".")[1] for k in sd if k.startswith(f"layer{i}.")}) for i in range(1, 5)]
    kind = "bottleneck" if any(k.endswith("conv3.weight") for k in sd) else "basic"
    for name, (blk, layers) in ARCHS.items():
        if layers == nblk and blk == kind:
            return name, int(sd["fc.weight"].shape[0])
    raise ValueError(f"unrecognised ResNet state_dict (blocks {nblk})")


def _bn(sd, prefix):
    return {k: sd[f"{prefix}.{k}"] for k in ("weight", "bias", "running_mean", "running_var")}


def pack_sources(sd: dict) -> list:
    """[(packed name, kind, weight key, BN prefix or None, bias key or None)] of a ResNet
    state_dict, in packing order -- the one mapping the torch packer (models/resnet.py
    pack_resnet), this numpy packer and the device packer (plan templates) all follow."""
    arch, _ = infer_resnet(sd)
    kind, layers = ARCHS[arch]
    out = [("conv1", "conv", "conv1.weight", "bn1", None)]
    for li, nb in enumerate(layers, start=1):
        for b in range(nb):
            pre = f"layer{li}.{b}"
            for c in (("conv1", "conv2", "conv3") if kind == "bottleneck" else ("conv1", "conv2")):
                out.append((f"{pre}.{c}", "conv", f"{pre}.{c}.weight", f"{pre}.bn{c[-1]}", None))
            if f"{pre}.downsample.0.weight" in sd:
                out.append((f"{pre}.downsample", "conv", f"{pre}.downsample.0.weight", f"{pre}.downsample.1", None))
    out.append(("fc", "linear", "fc.weight", None, "fc.bias" if "fc.bias" in sd else None))
    return out


def conv_geometry(name: str, kind: str, wshape: tuple) -> dict:
    """Packed geometry of one parameter from its weight shape (ops/conv.py pack_conv /
    pack_linear): the stem's 3 input channels pad to 8, others to a multiple of 8."""
    if kind == "linear":
        cout, cin = wshape
        r = s = 1
        cin_p, row_pad = cin, GEMM_ROW_PAD
    else:
        cout, cin, r, s = wshape
        cin_p, row_pad = (8 if name == "conv1" else int(math.ceil(cin / 8) * 8)), ROW_PAD
    return {"cout": cout, "cin": cin, "r": r, "s": s, "cin_p": cin_p,
            "rows": int(math.ceil(cout / row_pad) * row_pad), "ksteps": int(math.ceil(r * s * cin_p / 32))}


def pack_resnet_jobs(sd: dict) -> list:
    """[(name, thunk)]: one packing job per parameter (numpy releases the GIL in the large
    array operations, so they can run on a thread pool)."""
    jobs = []
    for name, kind, w, bn, b in pack_sources(sd):
        if kind == "linear":
            jobs.append((name, lambda w=w, b=b: pack_linear(sd[w], sd[b] if b else None)))
        else:
            jobs.append((name, lambda name=name, w=w, bn=bn: pack_conv(sd[w], _bn(sd, bn),
                                                                     cin_pad=8 if name == "conv1" else None)))
    return jobs


def pack_resnet(sd: dict, threads: int = 8) -> dict:
    jobs = pack_resnet_jobs(sd)
    if threads <= 1:
        return {k: f() for k, f in jobs}
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(threads) as ex:
        futs = [(k, ex.submit(f)) for k, f in jobs]
        return {k: fu.result() for k, fu in futs}
