"""Bind-time fusion of ResNet stages into single launches (csrc/block.hip).

The graph IR keeps one node per conv (the fp32 oracle, ``engine/reference.py``, interprets it
unchanged); :class:`~hipzap.engine.program.ExecContext` asks :func:`plan` which node runs it may
bind as ONE fused kernel instead:

* ``stem``: preprocess -> conv1 (7x7/2, BN folded, ReLU) -> maxpool 3x3/2 -> ``hz_stem_launch``;
* ``convpool``: the same kernel after a standalone preprocess (conv1 + maxpool only, bf16 NHWC8
  input): the default, since a zero-copy request read inside the 98-workgroup stem cost served
  throughput (profiles/r4_fuse/README.md);
* ``bneck``: a layer1-geometry bottleneck (1x1 Cin -> 64, 3x3 64 -> 64, 1x1 64 -> 256 + residual,
  optionally with its 1x1 downsample) -> ``hz_bneck_launch``;
* ``bneck2``: a layer2 bottleneck (1x1 512 -> 128, 3x3 128 -> 128, 1x1 128 -> 512 + residual;
  or the first block: 1x1 256 -> 128, 3x3/2, 1x1 -> 512 + the 1x1/2 downsample) ->
  ``hz_bneck_launch`` (the weight-streaming ``bneck2_kernel`` / ``bneck2d_kernel``);
* ``seam``: layer3 / layer4 -- conv3 of block i and conv1 of block i+1 (1x1 CM -> 4CM + residual,
  1x1 4CM -> CM; CM 256 or 512) -> ``hz_seam_launch`` (``seam_kernel``): conv1's K is split over
  the workgroups and summed by float atomics into an fp32 accumulator that block i's 3x3 conv
  presets to conv1's bias (``HzConvParams.zinit``) and block i+1's 3x3 conv reads with the ReLU
  at its operand load (``HzConvParams.x_f32``). The accumulator is conv1's output tensor, planned
  as fp32 (:func:`planning_graph`). Atomic accumulation order varies run to run: a seam program is
  numerically equal to the per-conv one within fp32 rounding, not bitwise reproducible.
* ``kconv``: a seam's 3x3 neighbours as K-split 3x3 launches into fp32 accumulators
  (``kconv_kernel``; :func:`match_kconvs`).
* ``tail``: the last block's conv3 + the global average pool (the seam kernel's tail mode): the
  classifier's ``pool_fc`` then reads fp32 channel means (``HzPoolFcParams.pooled``).
* ``dsseam``: layer3's downsample as more K of layer3's first seam (its node skipped), so the
  stage's downsample + conv1 pair launch becomes conv1 alone (:func:`match_dsseam`).
* ``xseam``: the layer3 -> layer4 boundary -- layer3's last conv3 + layer4's first conv1 as one
  seam (:func:`match_xseam`), layer4's stride-2 3x3 as its K-split consumer, and layer4's
  downsample computed inside the next seam's conv3 (``HzSeamParams.ds``): the pair launch is gone.

Both reuse the per-conv packed weights, so plan images / templates need no new parameters; the
fused kernels' intermediate tensors simply stay unwritten in the arena. ``HIPZAP_FUSE`` selects
(comma list of ``stem``, ``convpool``, ``bneck``, ``bneck2``; ``none`` disables; default
``convpool,bneck,bneck2``) -- the A/B switch of
``profiles/r4_fuse``. Reference: the per-conv contract these replace is SURVEY.md §2e N1/N2/N14.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

from .. import _native as N

HZ_K_STEM, HZ_K_BNECK, HZ_K_SEAM, HZ_K_KCONV = 18, 19, 20, 21
KINDS = ("stem", "convpool", "bneck", "bneck2", "seam", "kconv", "tail", "xseam", "dsseam")
# measured default (profiles/r4_fuse/README.md: served 11.3k -> 13.4k inf/s on one box; round 5
# adds the layer3/layer4 seams + K-split 3x3 convs: 13.5-13.6k -> 14.2k same box, and the pooling
# tail: pool_fc 7.5 -> 4.6 us, sustained 13.2-13.9k -> 14.4k same box; the layer3 -> layer4
# cross-stage + downsample seams: 29 dispatches, 14.36-14.41k -> 14.51-14.57k, profiles/r5_seam)
DEFAULT = "convpool,bneck,bneck2,seam,kconv,tail,xseam"


class StemParams(C.Structure):  # HzStemParams (csrc/hipzap.h)
    _fields_ = [("src", C.c_void_p), ("w", C.c_void_p), ("bias", C.c_void_p), ("out", C.c_void_p),
                ("N", C.c_int), ("H", C.c_int), ("W", C.c_int), ("mode", C.c_int),
                ("SH", C.c_int), ("SW", C.c_int), ("PH", C.c_int), ("PW", C.c_int),
                ("norm", C.c_int), ("pad_", C.c_int), ("mean", C.c_float * 4), ("inv_std", C.c_float * 4)]


class BneckParams(C.Structure):  # HzBneckParams
    _fields_ = [("x", C.c_void_p), ("w1", C.c_void_p), ("b1", C.c_void_p), ("w2", C.c_void_p),
                ("b2", C.c_void_p), ("w3", C.c_void_p), ("b3", C.c_void_p), ("wd", C.c_void_p),
                ("bd", C.c_void_p), ("out", C.c_void_p), ("N", C.c_int), ("H", C.c_int), ("W", C.c_int),
                ("Cin", C.c_int), ("Cmid", C.c_int), ("Cout", C.c_int), ("tile_h", C.c_int), ("imgs", C.c_int)]


class SeamParams(C.Structure):  # HzSeamParams
    _fields_ = [("t2", C.c_void_p), ("w3", C.c_void_p), ("b3", C.c_void_p), ("res", C.c_void_p),
                ("y", C.c_void_p), ("w1", C.c_void_p), ("z", C.c_void_p), ("N", C.c_int), ("HW", C.c_int),
                ("CM", C.c_int), ("cs", C.c_int), ("tiles", C.c_int), ("t2_f32", C.c_int), ("zinit", C.c_void_p),
                ("zbias", C.c_void_p), ("z_C", C.c_int), ("z_HW", C.c_int), ("tail", C.c_int), ("pad_", C.c_int),
                ("cn", C.c_int), ("ds", C.c_int), ("xd", C.c_void_p), ("wd", C.c_void_p), ("bd", C.c_void_p),
                ("xd_H", C.c_int), ("xd_W", C.c_int)]


class KconvParams(C.Structure):  # HzKconvParams
    _fields_ = [("x", C.c_void_p), ("w", C.c_void_p), ("out", C.c_void_p), ("zinit", C.c_void_p),
                ("zbias", C.c_void_p), ("z_C", C.c_int), ("z_HW", C.c_int), ("N", C.c_int), ("H", C.c_int),
                ("W", C.c_int), ("C", C.c_int), ("Cout", C.c_int), ("x_f32", C.c_int), ("ck", C.c_int),
                ("stride", C.c_int), ("dsx", C.c_void_p), ("dsw", C.c_void_p), ("dsb", C.c_void_p), ("dso", C.c_void_p),
                ("ds_C", C.c_int), ("ds_Cout", C.c_int), ("ds_H", C.c_int), ("ds_W", C.c_int)]


@dataclass
class Fused:
    kind: str
    start: int
    end: int      # exclusive node index
    nodes: list   # the graph nodes it replaces
    init: int | None = None      # seam: the conv that presets the accumulator (block i's 3x3 conv)
    consumer: int | None = None  # seam: the conv that reads it (block i+1's 3x3 conv)
    # kconv (a seam's consumer bound as the K-split 3x3 kernel): the seam that presets its fp32 output,
    # the seam whose accumulator it presets (or None), the 1x1 conv that reads its output when that
    # conv is not in a seam (the last block of a stage)
    seam: int | None = None
    next_seam: int | None = None
    reader: int | None = None
    preset: int | None = None  # kconv: node whose launch presets its accumulator (a seam's conv1, or conv1 of a pair)
    # cross-stage seam (xseam: the last block's conv3 + the next stage's first conv1, the downsample
    # node between them skipped) and the seam that computes that downsample as its residual
    ds: object | None = None       # seam: the downsample node whose output is this seam's residual
    ds_from: int | None = None     # seam: the cross-stage seam that skipped it


def enabled_kinds(spec: str | None = None) -> set:
    v = os.environ.get("HIPZAP_FUSE", DEFAULT) if spec is None else spec
    v = v.strip().lower()
    if v in ("", "0", "none", "off"):
        return set()
    if v in ("1", "all", "on"):
        return {"stem", "bneck", "bneck2"}
    return {k for k in v.split(",") if k in KINDS}


def _conv(n, kind="conv"):
    return n is not None and n.kind == kind


def _geom(pc, cin, cout, k, stride, pad) -> bool:
    return (pc.cin == cin and pc.cout == cout and pc.r == k and pc.s == k and pc.stride == stride
            and pc.pad == pad)


def _internal_only(g, grp) -> bool:
    """The fused kernel writes only the run's last output: every other output of the run must be
    read inside the run alone (and not be a graph output)."""
    inner = {t for n in grp[:-1] for t in n.outputs}
    if inner & set(g.outputs):
        return False
    ids = {id(n) for n in grp}
    return not any(t in inner for n in g.nodes if id(n) not in ids for t in n.inputs)


def match_stem(g, params, i: int) -> Fused | None:
    nodes = g.nodes
    if i + 3 > len(nodes):
        return None
    pre, cv, mp = nodes[i:i + 3]
    if pre.kind != "preprocess" or not _conv(cv) or mp.kind != "maxpool":
        return None
    if cv.inputs != [pre.outputs[0]] or mp.inputs != [cv.outputs[0]] or len({pre.slot, cv.slot, mp.slot}) != 1:
        return None
    pc = params.get(cv.attrs.get("w"))
    if pc is None or not _geom(pc, 8, 64, 7, 2, 3) or pc.ksteps != 13 or cv.attrs.get("act", "relu") != "relu":
        return None
    if cv.attrs.get("out_f32") or (mp.attrs.get("k"), mp.attrs.get("stride"), mp.attrs.get("pad")) != (3, 2, 1):
        return None
    src = g.tensors[pre.inputs[0]]
    import torch
    if src.dtype == torch.uint8:
        if src.shape[-1] != 3 or (src.shape[1] * src.shape[2] * 3) % 4:
            return None
    elif src.dtype != torch.float32 or src.shape[1] != 3:
        return None
    return Fused("stem", i, i + 3, [pre, cv, mp]) if _internal_only(g, [pre, cv, mp]) else None


def match_convpool(g, params, i: int) -> Fused | None:
    nodes = g.nodes
    if i + 2 > len(nodes):
        return None
    cv, mp = nodes[i:i + 2]
    if not _conv(cv) or mp.kind != "maxpool" or mp.inputs != [cv.outputs[0]] or cv.slot != mp.slot:
        return None
    pc = params.get(cv.attrs.get("w"))
    if pc is None or not _geom(pc, 8, 64, 7, 2, 3) or pc.ksteps != 13 or cv.attrs.get("act", "relu") != "relu":
        return None
    if cv.attrs.get("out_f32") or (mp.attrs.get("k"), mp.attrs.get("stride"), mp.attrs.get("pad")) != (3, 2, 1):
        return None
    if len(cv.inputs) != 1 or g.shape(cv.inputs[0])[-1] != 8:
        return None
    return Fused("convpool", i, i + 2, [cv, mp]) if _internal_only(g, [cv, mp]) else None


def match_bneck(g, params, i: int, layer2: bool = False) -> Fused | None:
    """layer1 geometry (``bneck``: Cmid 64, Cout 256, optional downsample) or, with ``layer2``,
    the identity blocks of layer2 (``bneck2``: Cin = Cout = 512, Cmid 128)."""
    nodes = g.nodes
    run = nodes[i:i + 4]
    if len(run) < 3 or not all(_conv(n) for n in run[:3]):
        return None
    ds = None
    if len(run) == 4 and _conv(run[3]) and run[0].inputs == run[1].inputs and len(run[0].inputs) == 1:
        ds, c1, c2, c3 = run
    else:
        c1, c2, c3 = run[:3]
    x = c1.inputs[0]
    if len(c1.inputs) != 1 or c2.inputs != [c1.outputs[0]]:
        return None
    res = ds.outputs[0] if ds is not None else x
    if c3.inputs != [c2.outputs[0], res]:
        return None
    grp = [n for n in (ds, c1, c2, c3) if n is not None]
    if not _internal_only(g, grp):
        return None
    if len({n.slot for n in grp}) != 1 or any(n.attrs.get("out_f32") or n.attrs.get("rowmajor") for n in grp):
        return None
    if any(n.attrs.get("act", "relu") != "relu" for n in (c1, c2, c3)):
        return None
    p1, p2, p3 = (params.get(n.attrs.get("w")) for n in (c1, c2, c3))
    if p1 is None or p2 is None or p3 is None:
        return None
    if layer2:
        if ds is None:
            if not (_geom(p1, 512, 128, 1, 1, 0) and _geom(p2, 128, 128, 3, 1, 1) and _geom(p3, 128, 512, 1, 1, 0)):
                return None
        else:  # the first block: stride-2 3x3 and the stride-2 downsample
            pd = params.get(ds.attrs.get("w"))
            if pd is None or ds.attrs.get("act", "relu") != "none" or not (
                    _geom(pd, 256, 512, 1, 2, 0) and _geom(p1, 256, 128, 1, 1, 0) and _geom(p2, 128, 128, 3, 2, 1)
                    and _geom(p3, 128, 512, 1, 1, 0)):
                return None
        nb, h, w, c = g.shape(c3.outputs[0])
        if c != 512 or h % 4 or w % 4 or g.shape(x)[1:3] != ((h, w) if ds is None else (2 * h, 2 * w)):
            return None  # (4x4 output tiles)
        return Fused("bneck2", i, i + len(grp), grp)
    cin = 64 if ds is not None else 256
    if not (_geom(p1, cin, 64, 1, 1, 0) and _geom(p2, 64, 64, 3, 1, 1) and _geom(p3, 64, 256, 1, 1, 0)):
        return None
    if ds is not None:
        pd = params.get(ds.attrs.get("w"))
        if pd is None or not _geom(pd, 64, 256, 1, 1, 0) or ds.attrs.get("act", "relu") != "none":
            return None
    nb, h, w, c = g.shape(x)
    if c != cin or h % 8 or w % 8:  # (8x8 or 4x8 output tiles)
        return None
    return Fused("bneck", i, i + len(grp), grp)


def match_seam(g, params, i: int) -> Fused | None:
    """nodes[i] = conv3 of a layer3/layer4 block, nodes[i+1] = the next block's conv1 reading its
    output, nodes[i-1] / nodes[i+2] = the two 3x3 convs around them (accumulator preset / reader)."""
    nodes = g.nodes
    if i < 1 or i + 3 > len(nodes):
        return None
    c2a, c3, c1, c2b = nodes[i - 1:i + 3]
    if not all(_conv(n) for n in (c2a, c3, c1, c2b)):
        return None
    if len({n.slot for n in (c2a, c3, c1, c2b)}) != 1:
        return None
    if any(n.attrs.get("out_f32") or n.attrs.get("rowmajor") for n in (c2a, c3, c1, c2b)):
        return None
    if any(n.attrs.get("act", "relu") != "relu" for n in (c3, c1, c2b)):
        return None
    pa, p3, p1, pb = (params.get(n.attrs.get("w")) for n in (c2a, c3, c1, c2b))
    if None in (pa, p3, p1, pb):
        return None
    cm = p1.cout
    if cm not in (256, 512):
        return None
    if not (_geom(p3, cm, 4 * cm, 1, 1, 0) and _geom(p1, 4 * cm, cm, 1, 1, 0) and _geom(pb, cm, cm, 3, 1, 1)
            and pa.cout == cm and pa.r == 3):
        return None
    if len(c3.inputs) != 2 or c3.inputs[0] != c2a.outputs[0] or c1.inputs != [c3.outputs[0]]:
        return None
    if c2b.inputs != [c1.outputs[0]]:
        return None
    t1 = c1.outputs[0]
    if t1 in g.outputs or g.tensors[t1].external:
        return None
    if any(t1 in n.inputs for j, n in enumerate(nodes) if j != i + 2):  # read by the 3x3 conv alone
        return None
    if len(g.shape(c3.outputs[0])) != 4 or g.shape(c3.outputs[0])[1:3] != g.shape(t1)[1:3]:
        return None
    return Fused("seam", i, i + 2, [c3, c1], init=i - 1, consumer=i + 2)


def match_tail(g, params, i: int) -> Fused | None:
    """nodes[i] = conv3 of the network's last bottleneck (1x1 512 -> 2048 + residual, <= 64 pixels),
    nodes[i+1] = the pooled classifier (``pool_fc``) reading its output alone: conv3 binds as the
    seam kernel's tail mode, which writes the channel means instead of the block output, and the
    pool_fc launch reads them (``reader``)."""
    nodes = g.nodes
    if i + 2 > len(nodes):
        return None
    c3, pf = nodes[i:i + 2]
    if not _conv(c3) or pf.kind != "pool_fc" or pf.inputs != [c3.outputs[0]] or c3.slot != pf.slot:
        return None
    if c3.attrs.get("out_f32") or c3.attrs.get("rowmajor") or c3.attrs.get("act", "relu") != "relu":
        return None
    p3 = params.get(c3.attrs.get("w"))
    if p3 is None or not _geom(p3, 512, 2048, 1, 1, 0) or len(c3.inputs) != 2:
        return None
    y = c3.outputs[0]
    if y in g.outputs or g.tensors[y].external or any(y in n.inputs for j, n in enumerate(nodes) if j != i + 1):
        return None
    sh = g.shape(y)
    # (>= 2 pixels: the fp32 channel means must fit the block output's bf16 buffer they are written to)
    if len(sh) != 4 or not 2 <= sh[1] * sh[2] <= 64 or g.shape(c3.inputs[1]) != sh:
        return None
    return Fused("tail", i, i + 1, [c3], reader=i + 1)


def match_xseam(g, params, i: int, seams: dict) -> Fused | None:
    """The layer3 -> layer4 boundary: nodes[i] = conv3 of layer3's last block (1x1 256 -> 1024 +
    residual), nodes[i+1] = layer4's downsample (1x1/2 1024 -> 2048), nodes[i+2] = layer4's first
    conv1 (1x1 1024 -> 512), nodes[i+3] = its stride-2 3x3, nodes[i+4] = its conv3 (+ the
    downsample) starting a seam. The cross-stage seam binds conv3 + conv1 (conv1's K split over the
    workgroups into an fp32 accumulator, as every seam); the downsample becomes more K of the
    nodes[i+4] seam (its residual computed from the block input), so the pair launch is gone."""
    nodes = g.nodes
    if i < 1 or i + 5 > len(nodes) or (i + 4) not in seams:
        return None
    c2a, c3, ds, c1, c2b, c3b = nodes[i - 1:i + 5]
    if not all(_conv(n) for n in (c2a, c3, ds, c1, c2b, c3b)) or len({n.slot for n in (c3, ds, c1, c2b, c3b)}) != 1:
        return None
    if any(n.attrs.get("out_f32") or n.attrs.get("rowmajor") for n in (c3, ds, c1, c2b, c3b)):
        return None
    if any(n.attrs.get("act", "relu") != "relu" for n in (c3, c1, c2b, c3b)) or ds.attrs.get("act", "relu") != "none":
        return None
    p2a, p3, pd, p1, p2b = (params.get(n.attrs.get("w")) for n in (c2a, c3, ds, c1, c2b))
    if None in (p2a, p3, pd, p1, p2b):
        return None
    if not (_geom(p3, 256, 1024, 1, 1, 0) and _geom(pd, 1024, 2048, 1, 2, 0) and _geom(p1, 1024, 512, 1, 1, 0)
            and _geom(p2b, 512, 512, 3, 2, 1) and p2a.r == 3 and p2a.cout == 256):
        return None
    y = c3.outputs[0]
    if len(c3.inputs) != 2 or c3.inputs[0] != c2a.outputs[0] or ds.inputs != [y] or c1.inputs != [y]:
        return None
    if c2b.inputs != [c1.outputs[0]] or c3b.inputs != [c2b.outputs[0], ds.outputs[0]]:
        return None
    for t, reader in ((ds.outputs[0], i + 4), (c1.outputs[0], i + 3)):
        if t in g.outputs or any(t in n.inputs for j, n in enumerate(nodes) if j != reader):
            return None
    if y in g.outputs or any(y in n.inputs for j, n in enumerate(nodes) if j not in (i + 1, i + 2)):
        return None
    nb, h, w, _ = g.shape(y)
    if h % 2 or w % 2 or h * w > 196:  # the stride-2 K-split consumer stages (h+2)(w+2) <= 256 pixels
        return None
    return Fused("seam", i, i + 3, [c3, c1], init=i - 1, consumer=i + 3)


def match_dsseam(g, params, f: Fused, covered: set) -> Fused | None:
    """A stage's first block whose conv3 opens a seam (layer3: 1x1 256 -> 1024 + the downsample
    1x1/2 512 -> 1024 of the stage input): nodes [ds, conv1, 3x3/2, conv3 ...]. The downsample then
    runs inside that seam (HzSeamParams.ds, more phase-1 K from the stage input) and its own node is
    skipped (a ``skip`` run: no launch), so layer3's downsample + conv1 pair becomes conv1 alone.
    Returns the skip run."""
    nodes = g.nodes
    c3 = f.nodes[0]
    if f.end - f.start != 2 or len(c3.inputs) != 2 or f.init is None or f.init < 2:
        return None
    d, c1, c2 = nodes[f.init - 2], nodes[f.init - 1], nodes[f.init]
    if not all(_conv(n) for n in (d, c1, c2)) or f.init - 2 in covered or c3.inputs[1] != d.outputs[0]:
        return None
    if d.attrs.get("act", "relu") != "none" or d.attrs.get("out_f32") or d.slot != c3.slot:
        return None
    pd, p3 = params.get(d.attrs.get("w")), params.get(c3.attrs.get("w"))
    if pd is None or p3 is None or p3.cin != 256 or not _geom(pd, 2 * p3.cin, p3.cout, 1, 2, 0):
        return None
    if d.outputs[0] in g.outputs or any(d.outputs[0] in n.inputs for n in nodes if n is not c3):
        return None
    if c1.inputs != d.inputs or c2.inputs != [c1.outputs[0]]:
        return None
    return Fused("skip", f.init - 2, f.init - 1, [d], seam=f.start)


def plan(g, params, kinds: set | None = None) -> dict[int, Fused]:
    """{first node index: Fused} for every fusible run of ``g`` (non-overlapping, in order)."""
    kinds = enabled_kinds() if kinds is None else kinds
    out: dict[int, Fused] = {}
    if not kinds:
        return out
    i = 0
    while i < len(g.nodes):
        f = None
        if "stem" in kinds:
            f = match_stem(g, params, i)
        if f is None and "convpool" in kinds:
            f = match_convpool(g, params, i)
        if f is None and "bneck" in kinds:
            f = match_bneck(g, params, i)
        if f is None and "bneck2" in kinds:
            f = match_bneck(g, params, i, layer2=True)
        if f is not None:
            out[i] = f
            i = f.end
        else:
            i += 1
    if "seam" in kinds:  # over the nodes the block fusions left, their 3x3 neighbours included
        covered = {j for f in out.values() for j in range(f.start, f.end)}
        seams = {}
        for i in range(len(g.nodes)):
            f = match_seam(g, params, i)
            if f is not None and not covered & set(range(f.init, f.consumer + 1)):
                seams[i] = f
        if "xseam" in kinds and "kconv" in kinds:
            for i in range(len(g.nodes)):
                f = match_xseam(g, params, i, seams)
                if f is not None and not covered & set(range(f.init, f.consumer + 1)) and \
                        not any(j in seams for j in range(f.init, f.consumer + 1)):
                    seams[i] = f
                    seams[i + 4].ds, seams[i + 4].ds_from = g.nodes[i + 1], i
        out.update(seams)
        if "dsseam" in kinds and "kconv" in kinds:  # layer3's downsample inside its first seam
            for s0, f in seams.items():
                sk = match_dsseam(g, params, f, covered | set(out) | {j for x in seams.values()
                                                                     for j in range(x.start, x.end)})
                if sk is not None:
                    out[sk.start] = sk
                    f.ds, f.ds_from = g.nodes[sk.start], sk.start
        if "kconv" in kinds:
            out.update(match_kconvs(g, params, seams, covered))
            # where layer4's downsample runs (HIPZAP_XSEAM_DS): "seam" (default) = more K of the next
            # seam; "kconv" = extra workgroups of the stride-2 K-split launch (measured slower served:
            # the full-chip launch costs CU-time, profiles/r5_seam)
            if os.environ.get("HIPZAP_XSEAM_DS", "seam") == "kconv":
                for f in seams.values():
                    kc = out.get(f.start - 1)
                    if f.ds is not None and seams.get(f.ds_from) is not None and kc is not None and \
                            kc.kind == "kconv" and kc.start == f.init:
                        kc.ds, kc.ds_from, f.ds, f.ds_from = f.ds, f.ds_from, None, None
    if "tail" in kinds:
        covered = {j for f in out.values() for j in range(f.start, f.end)}
        for i in range(len(g.nodes)):
            f = match_tail(g, params, i)
            if f is not None and i not in covered and i + 1 not in covered:
                out[i] = f
    return dict(sorted(out.items()))


def match_kconvs(g, params, seams: dict, covered: set = frozenset()) -> dict:
    """Each seam's consumer (block i+1's 3x3 conv, stride 1, 14 x 14 / 7 x 7) as a K-split 3x3
    launch whose output is an fp32 accumulator: preset by that seam, read with the ReLU at the load
    by the next seam's conv3 half (or, at a stage's last block, by a plain 1x1 conv3 with x_f32).
    Also a stage's first 3x3 conv (stride 2, 28 x 28 -> 14 x 14 / 14 x 14 -> 7 x 7) when it is the
    first seam's init: preset by the launch before it (its block's conv1, usually paired with the
    downsample), read by that seam's conv3 half."""
    out = {}
    by_init = {f.init: s for s, f in seams.items()}
    for s, f in seams.items():  # the first block of a stage: its stride-2 3x3 conv
        k = f.init
        n = g.nodes[k]
        pk = params.get(n.attrs.get("w"))
        if pk is None or k < 1 or not _conv(n) or k - 1 in covered:
            continue
        nb, h, w, c = g.shape(n.inputs[0])
        prev = g.nodes[k - 1]
        if not (_geom(pk, c, c, 3, 2, 1) and c in (256, 512) and h % 2 == 0 and w % 2 == 0
                and (h + 2) * (w + 2) <= (900 if c == 256 else 256)):
            continue
        if not _conv(prev) or prev.outputs[0] != n.inputs[0] or prev.attrs.get("act", "relu") != "relu":
            continue
        if any(s2 != s and f2.consumer == k for s2, f2 in seams.items()):
            continue  # (a seam consumer: handled below)
        if not kconv_launchable(h, w, c, 2):
            continue
        out[k] = Fused("kconv", k, k + 1, [n], seam=None, next_seam=s, reader=None, preset=k - 1)
    for s, f in seams.items():
        k = f.consumer
        n = g.nodes[k]
        pk = params.get(n.attrs.get("w"))
        nb, h, w, c = g.shape(n.inputs[0])
        cross = f.end - f.start == 3  # a cross-stage seam's consumer: the next stage's stride-2 3x3
        if cross:
            if pk is None or not _geom(pk, c, c, 3, 2, 1) or c != 512 or (h + 2) * (w + 2) > 256:
                continue
        elif pk is None or not _geom(pk, c, c, 3, 1, 1) or c not in (256, 512) or h * w > (196 if c == 256 else 64):
            continue
        if not kconv_launchable(h, w, c, pk.stride):
            continue
        if k + 1 >= len(g.nodes):
            continue
        c3 = g.nodes[k + 1]
        a = n.outputs[0]
        if not _conv(c3) or c3.inputs[0] != a or a in g.outputs:
            continue
        if any(a in m.inputs for j, m in enumerate(g.nodes) if j != k + 1):
            continue
        nxt = by_init.get(k)  # the seam this conv presets (its own block's conv3 + the next conv1)
        if nxt is not None and nxt != k + 1:
            continue
        p3 = params.get(c3.attrs.get("w"))
        if nxt is None and (p3 is None or not _geom(p3, c, 4 * c, 1, 1, 0)):
            continue
        out[k] = Fused("kconv", k, k + 1, [n], seam=s, next_seam=nxt, reader=None if nxt is not None else k + 1,
                       preset=f.end - 1)  # (the seam's conv1 node)
    return out


def planning_graph(g, fused: dict):
    """The graph the arena planner sees: a seam's accumulator (conv1's output) and a K-split 3x3
    conv's output are fp32, and each is live from the launch that presets it (an extra output of
    that launch's node: the 3x3 conv before a seam, the seam before a K-split conv)."""
    accs = [f for f in fused.values() if f.kind in ("seam", "kconv")]
    if not accs:
        return g
    import copy

    import torch
    gp = copy.copy(g)
    gp.tensors = list(g.tensors)
    gp.nodes = list(g.nodes)

    def fp32(t):
        spec = g.tensors[t]
        gp.tensors[t] = type(spec)(spec.shape, torch.float32, spec.name, spec.external)

    def preset_by(j, t):
        n = gp.nodes[j]
        gp.nodes[j] = type(n)(n.kind, list(n.inputs), list(n.outputs) + [t], n.slot, n.attrs)

    for f in accs:
        if f.kind == "seam":
            t1 = f.nodes[1].outputs[0]
            fp32(t1)
            preset_by(f.init, t1)
            if f.ds is not None:  # the downsample's input stays live until this seam reads it
                j = f.start
                n = gp.nodes[j]
                gp.nodes[j] = type(n)(n.kind, list(n.inputs) + [f.ds.inputs[0]], list(n.outputs), n.slot, n.attrs)
        else:
            a = f.nodes[0].outputs[0]
            fp32(a)
            preset_by(f.preset, a)  # a seam's conv1 half, or the conv before a stage's stride-2 3x3
            if f.ds is not None:  # the launch also computes the downsample: its input and output
                n = gp.nodes[f.start]
                gp.nodes[f.start] = type(n)(n.kind, list(n.inputs) + [f.ds.inputs[0]],
                                            list(n.outputs) + [f.ds.outputs[0]], n.slot, n.attrs)
    return gp


def seam_cs(cm: int) -> int:
    """Slice width of the seam kernel per geometry (HIPZAP_SEAM_CS="<cs for CM 256>,<cs for CM 512>")."""
    v = [int(x) for x in os.environ.get("HIPZAP_SEAM_CS", "128,128").split(",")]
    return v[0] if cm == 256 else v[-1]


def seam_params(g, params, f: Fused, addr, fused: dict | None = None) -> SeamParams:
    fused = fused or {}
    kc = fused.get(f.start - 1)  # t2 is a K-split conv's fp32 accumulator
    if f.kind == "tail":
        c3 = f.nodes[0]
        p3 = params[c3.attrs["w"]]
        p = SeamParams()
        p.t2, p.res, p.y = addr(c3.inputs[0]), addr(c3.inputs[1]), addr(c3.outputs[0])
        p.w3, p.b3 = p3.wf.data_ptr(), p3.bias.data_ptr()
        nb, h, w, _ = g.shape(c3.outputs[0])
        p.N, p.HW, p.CM, p.tail = nb, h * w, p3.cin, 1
        p.cs = int(os.environ.get("HIPZAP_TAIL_CS", "64"))  # 32 workgroups at bs=1 (128: 16, measured slower)
        p.t2_f32 = int(kc is not None and kc.kind == "kconv")
        return p
    c3, c1 = f.nodes
    p3, p1 = params[c3.attrs["w"]], params[c1.attrs["w"]]
    p = SeamParams()
    p.t2, p.res, p.y, p.z = addr(c3.inputs[0]), addr(c3.inputs[1]), addr(c3.outputs[0]), addr(c1.outputs[0])
    p.w3, p.b3, p.w1 = p3.wf.data_ptr(), p3.bias.data_ptr(), p1.wf.data_ptr()
    nb, h, w, _ = g.shape(c3.outputs[0])
    p.N, p.HW, p.CM = nb, h * w, p3.cin
    p.cn = p1.cout if p1.cout != p3.cin else 0
    # slice widths of the cross-stage seam and of the downsample seam: HIPZAP_XSEAM_CS="<xseam>,<ds seam>"
    xcs = [int(v) for v in os.environ.get("HIPZAP_XSEAM_CS", "128,128").split(",")]
    p.cs = xcs[0] if p.cn else xcs[-1] if f.ds is not None else seam_cs(p.CM)
    if f.ds is not None:
        pd = params[f.ds.attrs["w"]]
        p.ds, p.xd, p.wd, p.bd = 1, addr(f.ds.inputs[0]), pd.wf.data_ptr(), pd.bias.data_ptr()
        _, p.xd_H, p.xd_W, _ = g.shape(f.ds.inputs[0])
    p.t2_f32 = int(kc is not None and kc.kind == "kconv")
    kn = fused.get(f.consumer)  # this seam presets its consumer's accumulator
    if kn is not None and kn.kind == "kconv":
        kcv = kn.nodes[0]
        _, kh, kw_, kcout = g.shape(kcv.outputs[0])
        p.zinit, p.zbias = addr(kcv.outputs[0]), params[kcv.attrs["w"]].bias.data_ptr()
        p.z_C, p.z_HW = kcout, kh * kw_
    return p


def kconv_launchable(h: int, w: int, c: int, stride: int) -> bool:
    """The geometry ``hz_kconv_launch`` (csrc/block.hip) accepts, mirrored on the host so a graph at
    another image size binds its 3x3 convs per conv instead of failing at the first replay: an
    output of 7 (14 x 14) or 2 (<= 64 px) 32-pixel groups, a channel slice the kernel is
    instantiated for at that group count, and the padded input within the kernel's LDS image."""
    st = 2 if stride == 2 else 1
    if st == 2 and (h % 2 or w % 2):
        return False
    pg = ((h // st) * (w // st) + 31) // 32
    ck = kconv_ck(c, st)
    if c % 32 or ck <= 0 or c % ck:
        return False
    if not ((pg == 7 and ck in (32, 64)) or (pg == 2 and ck in (64, 128))):
        return False
    npmax = (256 if pg == 7 else 100) if st == 1 else (900 if pg == 7 else 256)
    return (h + 2) * (w + 2) <= npmax


def kconv_ck(c: int, stride: int = 1) -> int:
    """Input-channel slice of the K-split 3x3 conv: HIPZAP_KCONV_CK="<C 256>,<C 512>[,<C 256 stride 2>,
    <C 512 stride 2>]" (stride-2 entries default to the stride-1 ones); defaults from the microbenchmark
    (scripts/bench_kconv.py) and the served A/B (profiles/r5_seam)."""
    v = [int(x) for x in os.environ.get("HIPZAP_KCONV_CK", "32,64").split(",")]
    if stride == 2 and len(v) >= 4:
        return v[2] if c == 256 else v[3]
    return v[0] if c == 256 else v[1 if len(v) > 1 else 0]


def kconv_params(g, params, f: Fused, addr, fused: dict) -> KconvParams:
    n = f.nodes[0]
    pk = params[n.attrs["w"]]
    p = KconvParams()
    nb, h, w, c = g.shape(n.inputs[0])
    p.x, p.w, p.out = addr(n.inputs[0]), pk.wf.data_ptr(), addr(n.outputs[0])
    p.N, p.H, p.W, p.C, p.Cout, p.ck, p.stride = nb, h, w, c, pk.cout, kconv_ck(c, pk.stride), pk.stride
    p.x_f32 = int(f.seam is not None)  # a seam's fp32 conv1 sum; a stage's first 3x3 reads bf16
    if f.ds is not None:  # layer4's downsample in extra workgroups of this launch
        pd = params[f.ds.attrs["w"]]
        p.dsx, p.dsw, p.dsb, p.dso = addr(f.ds.inputs[0]), pd.wf.data_ptr(), pd.bias.data_ptr(), addr(f.ds.outputs[0])
        _, p.ds_H, p.ds_W, p.ds_C = g.shape(f.ds.inputs[0])
        p.ds_Cout = pd.cout
    if f.next_seam is not None:  # preset the next seam's conv1 accumulator
        nf = fused[f.next_seam]
        t1 = nf.nodes[1].outputs[0]
        _, th, tw, tc = g.shape(t1)
        p.zinit, p.zbias = addr(t1), params[nf.nodes[1].attrs["w"]].bias.data_ptr()
        p.z_C, p.z_HW = tc, th * tw
    return p


def stem_params(g, params, f: Fused, addr) -> StemParams:
    if f.kind == "convpool":
        cv, mp = f.nodes
        pc = params[cv.attrs["w"]]
        p = StemParams()
        p.src, p.w, p.bias, p.out = addr(cv.inputs[0]), pc.wf.data_ptr(), pc.bias.data_ptr(), addr(mp.outputs[0])
        p.N, p.H, p.W, _ = g.shape(cv.inputs[0])
        p.mode = 2
        _, p.SH, p.SW, _ = g.shape(cv.outputs[0])
        _, p.PH, p.PW, _ = g.shape(mp.outputs[0])
        return p
    pre, cv, mp = f.nodes
    import torch
    src = g.tensors[pre.inputs[0]]
    pc = params[cv.attrs["w"]]
    p = StemParams()
    p.src, p.w, p.bias, p.out = addr(pre.inputs[0]), pc.wf.data_ptr(), pc.bias.data_ptr(), addr(mp.outputs[0])
    if src.dtype == torch.uint8:
        p.N, p.H, p.W, _ = src.shape
        p.mode = 1
    else:
        p.N, _, p.H, p.W = src.shape
        p.mode = 0
    _, p.SH, p.SW, _ = g.shape(cv.outputs[0])
    _, p.PH, p.PW, _ = g.shape(mp.outputs[0])
    mean, std = pre.attrs.get("mean"), pre.attrs.get("std")
    p.norm = int(mean is not None)
    if mean is not None:
        # the same float32 constants as the standalone preprocess kernel (inv_std = 1/std in fp32)
        inv = (np.float32(1.0) / np.asarray(std, dtype=np.float32)).astype(np.float32)
        for c in range(3):
            p.mean[c] = float(np.float32(mean[c]))
            p.inv_std[c] = float(inv[c])
    return p


def bneck_params(g, params, f: Fused, addr) -> BneckParams:
    grp = f.nodes
    ds = grp[0] if len(grp) == 4 else None
    c1, c2, c3 = grp[-3:]
    p1, p2, p3 = (params[n.attrs["w"]] for n in (c1, c2, c3))
    p = BneckParams()
    p.x, p.out = addr(c1.inputs[0]), addr(c3.outputs[0])
    p.w1, p.b1 = p1.wf.data_ptr(), p1.bias.data_ptr()
    p.w2, p.b2 = p2.wf.data_ptr(), p2.bias.data_ptr()
    p.w3, p.b3 = p3.wf.data_ptr(), p3.bias.data_ptr()
    if ds is not None:
        pd = params[ds.attrs["w"]]
        p.wd, p.bd = pd.wf.data_ptr(), pd.bias.data_ptr()
    p.N, p.H, p.W, p.Cin = g.shape(c1.inputs[0])
    p.Cmid, p.Cout = p1.cout, p3.cout
    if p.Cmid == 128:  # layer2 kernels take the block's OUTPUT size (the first block halves it)
        _, p.H, p.W, _ = g.shape(c3.outputs[0])
    p.tile_h = 0 if p.Cmid == 128 else int(os.environ.get("HIPZAP_BNECK_TH", "8"))  # layer1 tile rows
    # layer2 images per workgroup (batched programs): 0 = auto (2 at an even batch >= 8: the weight
    # stream is paid once per image pair, bitwise the one-image kernel), HIPZAP_B2_IMG=1 / 2: forced
    p.imgs = int(os.environ.get("HIPZAP_B2_IMG", "0")) if p.Cmid == 128 else 0
    return p


def add_fused(prog, g, params, f: Fused, addr, lib, fused: dict | None = None) -> tuple:
    """Bind ``f`` as one program op; returns the (name, key, cfg, kw) record ExecContext.configs keeps."""
    if f.kind == "skip":  # computed inside another launch (a downsample seam): no op of its own
        return (str(f.nodes[0].attrs.get("name", "")), "fused:skip", -1, 0)
    if f.kind in ("stem", "convpool"):
        prm, kind = stem_params(g, params, f, addr), HZ_K_STEM
    elif f.kind in ("seam", "tail"):
        prm, kind = seam_params(g, params, f, addr, fused), HZ_K_SEAM
    elif f.kind == "kconv":
        prm, kind = kconv_params(g, params, f, addr, fused or {}), HZ_K_KCONV
    else:
        prm, kind = bneck_params(g, params, f, addr), HZ_K_BNECK
    N.check(lib.hz_prog_add_kernel(prog, kind, C.byref(prm), C.sizeof(prm), f.nodes[0].slot), f"add_{f.kind}")
    names = "+".join(str(n.attrs.get("name", n.kind)) for n in f.nodes)
    return (names, f"fused:{f.kind}", -1, 0)


def launch(kind: str, prm, stream=None) -> None:
    """Eager launch of a fused kernel (tests)."""
    k = {"stem": HZ_K_STEM, "seam": HZ_K_SEAM, "tail": HZ_K_SEAM, "kconv": HZ_K_KCONV}.get(kind, HZ_K_BNECK)
    N.check(N.lib().hz_launch_kernel(k, C.byref(prm), N.stream_ptr(stream)), f"launch_{kind}")
