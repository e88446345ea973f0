"""Bind a planned :class:`~hipzap.engine.graph.Graph` to device memory as a native Program.

An :class:`ExecContext` owns one activation arena, static input/output buffers, split-K
workspaces and a native ``HzProgram`` whose ops are fully bound launches. It is the unit of
concurrency: a serving engine keeps several contexts per GPU (one per in-flight request
stream), all sharing one packed weight set. ``capture()`` records the program into a
hipGraph; ``replay()`` is the warm path.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

from .. import _native as N
from ..ops import conv as conv_ops
from ..ops import fp8
from ..ops import transformer as tx
from ..ops import vision
from . import fusion
from .graph import Graph, plan_memory


def pair_key(ka: str, kb: str) -> str:
    return f"pair:{ka}|{kb}"


def conv_pairs(g: Graph) -> dict:
    """{i: i+1} for adjacent conv nodes that can share one launch: both single-input, same
    input tensor, same stream slot, not row-major (e.g. ResNet's downsample + conv1)."""
    out = {}
    i = 0
    while i + 1 < len(g.nodes):
        a, b = g.nodes[i], g.nodes[i + 1]
        if (a.kind == b.kind == "conv" and len(a.inputs) == 1 and len(b.inputs) == 1 and a.inputs[0] == b.inputs[0]
                and a.slot == b.slot and not a.attrs.get("rowmajor") and not b.attrs.get("rowmajor")):
            out[i] = i + 1
            i += 2
            continue
        i += 1
    return out


def qkvatt_pairs(g: Graph, params: dict) -> dict:
    """{index of a QKV gemm node: its attention node} for every (QKV projection, attention) pair
    that binds as ONE qkvatt launch: bf16 in / out, head_dim 64, L <= 128, the projection's output
    read by the attention alone. ``HIPZAP_QKVATT=0``: never."""
    if os.environ.get("HIPZAP_QKVATT", "1") == "0":
        return {}
    out = {}
    nodes = g.nodes
    for i in range(len(nodes) - 1):
        gm, att = nodes[i], nodes[i + 1]
        if gm.kind != "gemm" or att.kind != "attention" or att.inputs[0] != gm.outputs[0] or gm.slot != att.slot:
            continue
        if len(att.outputs) != 1 or _ln_folded(gm) or len(gm.outputs) != 1:
            continue
        a = gm.attrs
        if a.get("act", "none") != "none" or a.get("out_f32") or a.get("has_res", len(gm.inputs) > 1):
            continue
        L, heads, B = att.attrs["L"], att.attrs["heads"], att.attrs["B"]
        pc = params.get(a.get("w"))
        D = heads * 64
        if pc is None or L > 128 or pc.cout != 3 * D or pc.ksteps * 32 != D or pc.bias is None:
            continue
        qkv = gm.outputs[0]
        if qkv in g.outputs or g.shape(qkv) != (B * L, 3 * D) or (a.get("ldx") or g.shape(gm.inputs[0])[-1]) % 8:
            continue
        if any(qkv in n.inputs for j, n in enumerate(nodes) if j != i + 1):
            continue
        if g.tensors[att.outputs[0]].dtype != torch.bfloat16 or g.tensors[gm.inputs[0]].dtype != torch.bfloat16:
            continue
        out[i] = att
    return out


def _ln_folded(n) -> bool:
    a = n.attrs
    return n.kind == "gemm" and bool(a.get("ln_in") or a.get("res_ln") or a.get("stats_out") is not None)


class ExecContext:
    def __init__(self, g: Graph, params: dict, device: torch.device, tuned: dict | None = None,
                 host_io: bool = False, pair_convs: bool | None = None, zero_copy: str | None = None,
                 lib=None, fuse: str | None = None):
        """``lib``: the native library (default) or a recorder with the same ``hz_prog_add_*``
        surface (engine/plan.py ``PlanRecorder``: binds against CPU tensors and serialises the
        program as a plan image instead of launching it). ``fuse``: which ResNet stage fusions to
        bind (engine/fusion.py; default: env ``HIPZAP_FUSE``, else all)."""
        self.graph = g
        self.recording = lib is not None and getattr(lib, "recording", False)
        self.device = torch.device(device)
        self.params = params
        self._keep: list = []
        self._nslab: dict[int, int] = {}  # stats tensor -> slabs written by its producer (HzLnFold)
        lib = lib if lib is not None else N.lib()
        self._lib = lib
        # fused ResNet stages (engine/fusion.py, csrc/block.hip): runs of nodes bound as ONE launch;
        # the arena plan keeps each run's tensors live over the whole run
        self.fused = fusion.plan(g, params, fusion.enabled_kinds(fuse) if fuse is not None else None)
        conv_plans = self._conv_plans(g, params, tuned)
        if pair_convs is None:
            pair_convs = os.environ.get("HIPZAP_PAIR_CONVS", "1") != "0"
        self.pairs = conv_pairs(g) if pair_convs else {}
        paired = set(self.pairs) | set(self.pairs.values())
        # a seam's 3x3 neighbours must bind as single register-ring convs (zinit / x_f32 live there)
        self.fused = {k: f for k, f in self.fused.items() if f.kind != "seam" or (
            f.init not in paired and f.consumer not in paired and conv_plans[f.init][0] < 16
            and conv_plans[f.consumer][0] < 16)}
        # a K-split 3x3 conv needs the seam that presets its output and, when it presets one, the next
        # (and a cross-stage seam needs its K-split consumer: a fixed point over the two rules)
        while True:
            n0 = len(self.fused)
            self.fused = {k: f for k, f in self.fused.items() if f.kind != "kconv" or (
                (f.seam is None or f.seam in self.fused) and (f.next_seam is None or f.next_seam in self.fused)
                and (f.seam is not None or conv_plans[f.preset][0] < 16))}
            self.fused = {k: f for k, f in self.fused.items() if f.kind != "seam" or f.end - f.start == 2 or (
                f.consumer in self.fused and self.fused[f.consumer].kind == "kconv")}
            # a skipped downsample node needs the seam that computes it (and a K-split conv before that
            # seam: the downsample seam reads an fp32 t2)
            self.fused = {k: f for k, f in self.fused.items() if f.kind != "skip" or (
                f.seam in self.fused and self.fused.get(self.fused[f.seam].init) is not None
                and self.fused[self.fused[f.seam].init].kind == "kconv")}
            if len(self.fused) == n0:
                break
        for f in self.fused.values():  # a launch computing the downsample needs the seam that skipped its node
            if f.ds is not None and f.ds_from not in self.fused:
                f.ds = f.ds_from = None
        self.seam_init = {id(g.nodes[f.init]): f for f in self.fused.values() if f.kind == "seam"}
        self.seam_consumer = {id(g.nodes[f.consumer]) for f in self.fused.values() if f.kind == "seam"}
        self.f32_readers = {id(g.nodes[f.reader]) for f in self.fused.values() if f.kind == "kconv" and f.reader}
        # a kconv's reader bound as a tail seam instead reads its accumulator through HzSeamParams.t2_f32
        self.pooled_readers = {id(g.nodes[f.reader]) for f in self.fused.values() if f.kind == "tail"}
        # K-split 3x3 convs preset by a plain (or paired) conv launch: a stage's first block
        self.kconv_preset = {id(g.nodes[f.preset]): f for f in self.fused.values()
                             if f.kind == "kconv" and f.seam is None}
        # QKV projection + attention as one launch (HIPZAP_QKVATT, csrc/transformer.hip qkvatt_kernel)
        self.qkvatt = qkvatt_pairs(g, params)
        offsets, arena_bytes = plan_memory(fusion.planning_graph(g, self.fused),
                                           groups=[(f.start, f.end) for f in self.fused.values()] +
                                           [(i, i + 2) for i in self.qkvatt])
        self.arena_bytes = arena_bytes
        self.arena = torch.empty(max(arena_bytes, 256), dtype=torch.uint8, device=self.device)
        base = self.arena.data_ptr()
        self.ext: dict[int, torch.Tensor] = {}
        for tid, spec in enumerate(g.tensors):
            if spec.external:
                self.ext[tid] = torch.zeros(spec.shape, dtype=spec.dtype, device=self.device)

        def addr(tid):
            if tid is None:
                return 0
            if tid in self.ext:
                return self.ext[tid].data_ptr()
            return base + offsets[tid]

        self._addr = addr
        self.tensor_offsets = offsets
        self.prog = lib.hz_prog_create()
        self.configs: list = []
        # host_io: the request's PCIe transfers are part of the program (and of the graph):
        # pinned host inputs -> device inputs ... device output -> pinned host output.
        # zero_copy ("in", "out", "all"): the first/last kernels read the request from / write the
        # result to the pinned host buffers directly (UVA), replacing the copy node(s) and their
        # kernel boundaries; HIPZAP_ZERO_COPY picks the default.
        self.host_io = host_io
        zc = zero_copy if zero_copy is not None else os.environ.get("HIPZAP_ZERO_COPY", "")
        self.zc_in, self.zc_out = host_io and zc in ("in", "all", "1"), host_io and zc in ("out", "all", "1")
        if host_io:
            pin = (lambda t: t) if self.recording else (lambda t: t.pin_memory())
            self.host_inputs = [pin(torch.zeros(self.ext[t].shape, dtype=self.ext[t].dtype)) for t in g.inputs]
            self.host_input = self.host_inputs[0]
            self.host_output = pin(torch.zeros(self.output.shape, dtype=self.output.dtype))
            for t, hbuf in zip(g.inputs, self.host_inputs):
                if self.zc_in:
                    self.ext[t] = hbuf
                    continue
                d = self.ext[t]
                N.check(lib.hz_prog_add_memcpy(self.prog, d.data_ptr(), hbuf.data_ptr(), d.numel() * d.element_size(),
                                               0), "h2d")
            if self.zc_out:
                self.ext[g.outputs[0]] = self.host_output
        i = 0
        while i < len(g.nodes):
            n = g.nodes[i]
            if i in self.fused:
                f = self.fused[i]
                self.configs.append(fusion.add_fused(self.prog, g, params, f, addr, lib, self.fused))
                i = f.end
                continue
            if i in self.qkvatt:
                self._add_qkvatt(lib, n, g.nodes[i + 1])
                i += 2
                continue
            if i in self.pairs:
                self._add_conv_pair(lib, n, g.nodes[i + 1], conv_plans[i], conv_plans[i + 1], tuned)
                i += 2
                continue
            self._add_node(lib, n, conv_plans[i])
            i += 1
        if host_io and not self.zc_out:
            N.check(lib.hz_prog_add_memcpy(self.prog, self.host_output.data_ptr(), self.output.data_ptr(),
                                           self.output.numel() * self.output.element_size(), 0), "d2h")

    # ------------------------------------------------------------------
    def _add_qkvatt(self, lib, gm, att) -> None:
        g, a = self.graph, att.attrs
        pc = self.params[gm.attrs["w"]]
        mask = att.inputs[1] if len(att.inputs) > 1 else None
        D = a["heads"] * 64
        prm = tx.QkvAttParams(self._addr(gm.inputs[0]), pc.wf.data_ptr(), pc.bias.data_ptr(), self._addr(mask),
                              self._addr(att.outputs[0]), a["B"], a["L"], a["heads"], D, pc.ksteps,
                              gm.attrs.get("ldx") or g.shape(gm.inputs[0])[-1], g.shape(att.outputs[0])[-1], 0.125)
        self.configs.append((f"{gm.attrs.get('name', '')}+attention", "fused:qkvatt", -1, 0))
        tx.prog_add(self.prog, tx.K_QKVATT, prm, gm.slot, lib=lib)

    def _conv_plans(self, g: Graph, params: dict, tuned: dict | None) -> list:
        """(cfg, kw, tuning key) of every conv / GEMM node, None for other nodes."""
        conv_plans = []
        for n in g.nodes:
            if n.kind not in ("conv", "gemm", "gemm_fp8"):
                conv_plans.append(None)
                continue
            pc = params[n.attrs["w"]]
            if n.kind == "gemm_fp8":
                M = n.attrs["rows"]
                key = f"f8r{M}x{pc.cout}x{pc.K}"
            elif n.kind == "conv":
                nb, h, w, _ = g.shape(n.inputs[0])
                p_out = (h + 2 * pc.pad - pc.r) // pc.stride + 1
                q_out = (w + 2 * pc.pad - pc.s) // pc.stride + 1
                M = nb * p_out * q_out
                key = conv_ops.conv_key(M, pc)
            else:
                M = n.attrs["rows"]
                key = "r" + conv_ops.conv_key(M, pc)
            if n.attrs.get("cfg") is not None:
                cfg, kw = n.attrs["cfg"], n.attrs.get("kw", 1)
            elif n.kind == "gemm_fp8":
                mx_io = g.tensors[n.inputs[1]].dtype == torch.uint8 or len(n.outputs) == 2
                cfg, kw = fp8.choose_config_fp8(M, pc, tuned, key, mx_io=mx_io)
            else:
                # a conv with row-major output (ViT patch embedding) never runs as the LDS implicit GEMM
                lds_pc = None if n.kind == "conv" and n.attrs.get("rowmajor") else pc
                cfg, kw = conv_ops.choose_config(M, pc.cout, pc.K, tuned, key, rowmajor=n.kind == "gemm", pc=lds_pc)
            # HzLnFold lives in the LDS GEMM epilogue with 2 wave columns, and only in the
            # experiments build
            if _ln_folded(n):
                if not self.recording and not N.experiments():
                    raise RuntimeError("the folded-LayerNorm GEMMs (HIPZAP_LN_FOLD=1) are a measured negative "
                                       "built only into the experiments library: python -m hipzap.build "
                                       "--experiments, HIPZAP_LIB=hipzap/_lib/libhipzap_exp.so")
                cfg = conv_ops.LNF_REMAP.get(cfg, cfg)
                if cfg not in conv_ops.LDS_TILES:
                    if not conv_ops.lds_ok(M, pc.K, True, pc):
                        raise ValueError(f"{n.attrs.get('name')}: folded LayerNorm needs the LDS GEMM (M={M} < 64?)")
                    cfg, kw = 19, 1
            conv_plans.append((cfg, kw, key))
        return conv_plans

    def _conv_params(self, n, cfg, kw):
        g, addr = self.graph, self._addr
        pc = self.params[n.attrs["w"]]
        nb, h, w, _ = g.shape(n.inputs[0])
        res = n.inputs[1] if len(n.inputs) > 1 else None
        prm, _, _ = conv_ops.make_params(
            addr(n.inputs[0]), pc, nb, h, w, addr(n.outputs[0]), addr(res), n.attrs.get("act", "relu"),
            n.attrs.get("out_f32", False), cfg, kw, out_rowmajor=n.attrs.get("rowmajor", False))
        return prm

    def _add_conv_pair(self, lib, a, b, plan_a, plan_b, tuned):
        """Two independent convs reading the same input -> one grouped launch (conv2_kernel).
        Convs planned on the LDS tile (large-M implicit GEMM, gemm.hip CV mode) launch alone."""
        if plan_a[0] in conv_ops.LDS_TILES or plan_b[0] in conv_ops.LDS_TILES:
            self._add_node(lib, a, plan_a)
            self._add_node(lib, b, plan_b)
            return
        key = pair_key(plan_a[2], plan_b[2])
        if tuned is not None and key in tuned:
            cfg, kw = int(tuned[key][0]), int(tuned[key][1])
        else:  # the larger problem's own choice
            fa = self._conv_flops(a)
            cfg, kw = (plan_a if fa >= self._conv_flops(b) else plan_b)[:2]
        pa, pb = self._conv_params(a, cfg, kw), self._conv_params(b, cfg, kw)
        kf = self.kconv_preset.get(id(a)) or self.kconv_preset.get(id(b))
        if kf is not None:  # the pair presets the stage's first K-split 3x3 conv's accumulator
            self._set_kconv_preset(pa, kf)
        self.configs.append((a.attrs.get("name", "") + "+" + b.attrs.get("name", ""), key, cfg, kw))
        N.check(lib.hz_prog_add_conv2(self.prog, C.byref(pa), C.byref(pb), cfg, a.slot), "add_conv2")

    def _ln_fold(self, n, pc, cfg: int, M: int) -> int:
        """Device copy of this GEMM's HzLnFold (csrc/hipzap.h); returns its address. Producers run
        before their consumers, so each stats tensor's slab count is known when it is read."""
        g, a = self.graph, n.attrs
        if self.recording:  # HzLnFold holds arena pointers in device memory: not relocatable
            raise NotImplementedError("plan images do not support the folded-LayerNorm GEMMs (HIPZAP_LN_FOLD)")
        f = N.LnFold()
        if a.get("ln_in"):
            pname, st = a["ln_in"]
            f.stats_in, f.c1 = self._addr(st), self.params[a["w"] + ".c1"].data_ptr()
            f.nslab_in, f.eps_in = self._nslab[st], self.params[pname].eps
            f.ld_stats, f.inv_d = g.shape(st)[1], 1.0 / pc.K
        if a.get("res_ln"):
            pname, st = a["res_ln"]
            npar = self.params[pname]
            f.res_stats, f.res_gamma, f.res_beta = self._addr(st), npar.gamma.data_ptr(), npar.beta.data_ptr()
            f.nslab_res, f.eps_res = self._nslab[st], npar.eps
            f.ld_stats, f.inv_d = g.shape(st)[1], 1.0 / pc.cout
        if a.get("stats_out") is not None:
            st = a["stats_out"]
            bn = conv_ops.LDS_TILES[cfg][1]
            self._nslab[st] = 2 * ((pc.cout + bn - 1) // bn)
            assert self._nslab[st] <= g.shape(st)[0] and g.shape(st)[1] == M
            f.stats_out, f.ld_stats, f.inv_d = self._addr(st), M, 1.0 / pc.cout
        assert f.ld_stats == M, "stats slabs are indexed by this GEMM's rows"
        assert max(f.nslab_in, f.nslab_res) <= 24, "rows_stats reads at most 4 * HZ_LNF_MAXT slabs (gemm.hip)"
        buf = torch.frombuffer(bytearray(bytes(f)), dtype=torch.uint8).to(self.device)
        self._keep.append(buf)
        return buf.data_ptr()

    def _set_kconv_preset(self, prm, f) -> None:
        k = f.nodes[0]
        _, h, w, c = self.graph.shape(k.outputs[0])
        prm.zinit, prm.zbias = self._addr(k.outputs[0]), self.params[k.attrs["w"]].bias.data_ptr()
        prm.z_C, prm.z_HW = c, h * w

    def _conv_flops(self, n) -> int:
        pc = self.params[n.attrs["w"]]
        nb, p, q, _ = self.graph.shape(n.outputs[0])
        return nb * p * q * pc.cout * pc.K

    def _add_node(self, lib, n, plan):
        g, addr = self.graph, self._addr
        if n.kind == "conv":
            pc = self.params[n.attrs["w"]]
            cfg, kw, key = plan
            nb, h, w, _ = g.shape(n.inputs[0])
            res = n.inputs[1] if len(n.inputs) > 1 else None
            prm, _, _ = conv_ops.make_params(
                addr(n.inputs[0]), pc, nb, h, w, addr(n.outputs[0]), addr(res), n.attrs.get("act", "relu"),
                n.attrs.get("out_f32", False), cfg, kw, out_rowmajor=n.attrs.get("rowmajor", False))
            if id(n) in self.seam_consumer or id(n) in self.f32_readers:  # reads an fp32 accumulator
                prm.x_f32 = 1  # (a seam's conv1 sum or a K-split 3x3 conv's output; ReLU at the load)
            if id(n) in self.kconv_preset:
                self._set_kconv_preset(prm, self.kconv_preset[id(n)])
            if id(n) in self.seam_init:  # presets the next seam's accumulator to conv1's bias
                f = self.seam_init[id(n)]
                t1 = f.nodes[1].outputs[0]
                nb1, h1, w1, c1 = g.shape(t1)
                prm.zinit, prm.zbias = addr(t1), self.params[f.nodes[1].attrs["w"]].bias.data_ptr()
                prm.z_C, prm.z_HW = c1, h1 * w1
                assert nb1 == nb
            self.configs.append((n.attrs.get("name", ""), key, cfg, kw))
            N.check(lib.hz_prog_add_conv(self.prog, C.byref(prm), cfg, n.slot), "add_conv")
        elif n.kind == "maxpool":
            nb, h, w, c = g.shape(n.inputs[0])
            _, p, q, _ = g.shape(n.outputs[0])
            a = n.attrs
            if conv_ops.is_blocked(c):  # [N][C/32][H][W][32] == NHWC with N*C/32 images of 32 ch
                nb, c = nb * c // 32, 32
            prm = N.PoolParams(addr(n.inputs[0]), addr(n.outputs[0]), nb, h, w, c, p, q, a["k"], a["stride"], a["pad"])
            N.check(lib.hz_prog_add_maxpool(self.prog, C.byref(prm), n.slot), "add_maxpool")
        elif n.kind == "avgpool":
            nb, h, w, c = g.shape(n.inputs[0])
            N.check(lib.hz_prog_add_avgpool(self.prog, addr(n.inputs[0]), addr(n.outputs[0]), nb, h * w, c,
                                            int(conv_ops.is_blocked(c)), n.slot), "add_avgpool")
        elif n.kind == "preprocess":
            src = g.tensors[n.inputs[0]]
            if src.dtype == torch.uint8:
                nb, h, w, cin = src.shape
                mode = 1
            else:
                nb, cin, h, w = src.shape
                mode = 0
            cpad = g.shape(n.outputs[0])[-1]
            mean = std = None
            if n.attrs.get("mean") is not None:
                mean = torch.tensor(n.attrs["mean"], dtype=torch.float32, device=self.device)
                std = 1.0 / torch.tensor(n.attrs["std"], dtype=torch.float32, device=self.device)
                self._keep += [mean, std]
            N.check(lib.hz_prog_add_preprocess(self.prog, addr(n.inputs[0]), addr(n.outputs[0]), nb, cin, h, w,
                                               cpad, mode, N.ptr(mean), N.ptr(std), n.slot), "add_preprocess")
        elif n.kind == "patchify":  # preprocess mode 2: fp32 NCHW -> bf16 patch rows (Cpad = patch)
            nb, cin, h, w = g.tensors[n.inputs[0]].shape
            mean = std = None
            if n.attrs.get("mean") is not None:
                mean = torch.tensor(n.attrs["mean"], dtype=torch.float32, device=self.device)
                std = 1.0 / torch.tensor(n.attrs["std"], dtype=torch.float32, device=self.device)
                self._keep += [mean, std]
            N.check(lib.hz_prog_add_preprocess(self.prog, addr(n.inputs[0]), addr(n.outputs[0]), nb, cin, h, w,
                                               n.attrs["patch"], 2, N.ptr(mean), N.ptr(std), n.slot), "add_patchify")
        elif n.kind == "gemm":
            pc = self.params[n.attrs["w"]]
            cfg, kw, key = plan
            M = n.attrs["rows"]
            res = n.inputs[1] if n.attrs.get("has_res", len(n.inputs) > 1) else None
            out_spec = g.tensors[n.outputs[0]]
            ldx = n.attrs.get("ldx") or g.shape(n.inputs[0])[-1]
            prm, _, _ = conv_ops.make_params(addr(n.inputs[0]), pc, M, 1, 1, addr(n.outputs[0]), addr(res),
                                             n.attrs.get("act", "none"), n.attrs.get("out_f32", False), cfg, kw,
                                             out_rowmajor=True, ldo=out_spec.shape[-1], x_rowmajor=True, ldx=ldx)
            if _ln_folded(n):
                prm.lnf = self._ln_fold(n, pc, cfg, M)
            self.configs.append((n.attrs.get("name", ""), key, cfg, kw))
            N.check(lib.hz_prog_add_conv(self.prog, C.byref(prm), cfg, n.slot), "add_gemm")
        elif n.kind == "quant":
            rows, D = g.shape(n.inputs[0])
            prm = fp8.QuantParams(addr(n.inputs[0]), addr(n.outputs[0]), addr(n.outputs[1]), rows, D, D, D)
            tx.prog_add(self.prog, fp8.K_QUANT, prm, n.slot, lib=lib)
        elif n.kind == "gemm_fp8":
            pw = self.params[n.attrs["w"]]
            cfg, kw, key = plan
            res = n.inputs[2] if len(n.inputs) > 2 else None
            xs_mx = g.tensors[n.inputs[1]].dtype == torch.uint8  # MX8 block scales, not per-row fp32
            o_mx = len(n.outputs) == 2
            prm = fp8.gemm_params(addr(n.inputs[0]), 0 if xs_mx else addr(n.inputs[1]), pw, n.attrs["rows"],
                                  0 if o_mx else addr(n.outputs[0]), addr(res), n.attrs.get("act", "none"),
                                  n.attrs.get("out_f32", False), cfg, kw, ldx=g.shape(n.inputs[0])[-1],
                                  ldo=g.shape(n.outputs[0])[-1], xs_ptr=addr(n.inputs[1]) if xs_mx else 0,
                                  out8_ptr=addr(n.outputs[0]) if o_mx else 0,
                                  os8_ptr=addr(n.outputs[1]) if o_mx else 0)
            self.configs.append((n.attrs.get("name", ""), key, cfg, kw))
            tx.prog_add(self.prog, fp8.K_GEMM_FP8, prm, n.slot, lib=lib)
        elif n.kind == "layernorm":
            npar = self.params[n.attrs["p"]]
            res = n.inputs[1] if len(n.inputs) > 1 else None
            D = g.shape(n.outputs[0])[-1]
            # fused fp8 quantisation: outputs (x8, scales), or (bf16, x8, scales) when both are kept
            outs = list(n.outputs)
            bf = outs.pop(0) if g.tensors[outs[0]].dtype != torch.uint8 else None
            q8 = len(outs) == 2
            prm = tx.LayerNormParams(addr(n.inputs[0]), addr(res), addr(bf) if bf is not None else 0,
                                     npar.gamma.data_ptr(), npar.beta.data_ptr(), n.attrs["rows"], D,
                                     n.attrs.get("ldx") or D, D, D, npar.eps, addr(outs[0]) if q8 else 0,
                                     addr(outs[1]) if q8 else 0)
            tx.prog_add(self.prog, tx.K_LAYERNORM, prm, n.slot, lib=lib)
        elif n.kind == "attention":
            a = n.attrs
            qkv = n.inputs[0]
            mask = n.inputs[1] if len(n.inputs) > 1 else None
            D = a["heads"] * 64
            mx = len(n.outputs) == 2  # MX8 output (e4m3 + E8M0 per 32 columns)
            prm = tx.AttentionParams(addr(qkv), addr(mask), 0 if mx else addr(n.outputs[0]), a["B"], a["L"],
                                     a["heads"], 64, g.shape(qkv)[-1], D, 2 * D, D, 0.125,
                                     addr(n.outputs[0]) if mx else 0, addr(n.outputs[1]) if mx else 0)
            tx.prog_add(self.prog, tx.K_ATTENTION, prm, n.slot, lib=lib)
        elif n.kind == "embed_ln":
            tab, ln = self.params[n.attrs["emb"]], self.params[n.attrs["ln"]]
            rows, D = g.shape(n.outputs[0])
            prm = tx.EmbedParams(addr(n.inputs[0]), addr(n.inputs[1]), tab.word.data_ptr(), tab.pos.data_ptr(),
                                 tab.type.data_ptr(), ln.gamma.data_ptr(), ln.beta.data_ptr(), addr(n.outputs[0]),
                                 rows, n.attrs["L"], D, ln.eps, tab.word.shape[0], tab.type.shape[0])
            tx.prog_add(self.prog, tx.K_EMBED, prm, n.slot, lib=lib)
        elif n.kind == "vit_tokens":
            a = n.attrs
            D = g.shape(n.outputs[0])[-1]
            prm = tx.VitTokensParams(addr(n.inputs[0]), self.params[a["cls"]].data_ptr(),
                                     self.params[a["pos"]].data_ptr(), addr(n.outputs[0]), a["B"], a["np"], D)
            tx.prog_add(self.prog, tx.K_VIT_TOKENS, prm, n.slot, lib=lib)
        elif n.kind == "pool_fc":
            pc = self.params[n.attrs["w"]]
            nb, h, w, c = g.shape(n.inputs[0])
            assert conv_ops.is_blocked(c) and pc.K == c and pc.ksteps * 32 == c
            prm = vision.PoolFcParams(addr(n.inputs[0]), pc.wf.data_ptr(), pc.bias.data_ptr(), addr(n.outputs[0]),
                                      nb, c, h * w, pc.cout, g.shape(n.outputs[0])[-1],
                                      int(id(n) in self.pooled_readers))
            tx.prog_add(self.prog, vision.K_POOL_FC, prm, n.slot, lib=lib)
        elif n.kind == "softmax":
            ishape = g.shape(n.inputs[0])
            rows, ld = ishape[0], int(torch.tensor(ishape[1:]).prod())
            src = g.tensors[n.inputs[0]]
            D = n.attrs.get("D") or ld
            prm = tx.SoftmaxParams(addr(n.inputs[0]), 0, addr(n.outputs[0]), rows, D, ld, g.shape(n.outputs[0])[-1],
                                   int(src.dtype == torch.bfloat16), float(n.attrs.get("scale", 1.0)))
            tx.prog_add(self.prog, tx.K_SOFTMAX, prm, n.slot, lib=lib)
        elif n.kind == "fork":
            N.check(lib.hz_prog_add_fork(self.prog, n.slot), "fork")
        elif n.kind == "join":
            N.check(lib.hz_prog_add_join(self.prog, n.slot), "join")
        else:
            raise NotImplementedError(f"node kind {n.kind}")

    # ------------------------------------------------------------------
    @property
    def input(self) -> torch.Tensor:
        return self.ext[self.graph.inputs[0]]

    @property
    def inputs(self) -> list:
        return [self.ext[t] for t in self.graph.inputs]

    @property
    def output(self) -> torch.Tensor:
        return self.ext[self.graph.outputs[0]]

    def view(self, tid: int) -> torch.Tensor:
        """Debug view of any tensor of the graph (arena-backed)."""
        if tid in self.ext:
            return self.ext[tid]
        spec = self.graph.tensors[tid]
        off = self.tensor_offsets[tid]
        return self.arena[off: off + spec.nbytes].view(spec.dtype).view(spec.shape)

    def run(self, stream=None):
        N.check(N.lib().hz_prog_run(self.prog, N.stream_ptr(stream)), "prog_run")

    def capture(self, stream=None):
        N.check(N.lib().hz_prog_capture(self.prog, N.stream_ptr(stream)), "prog_capture")

    @property
    def captured(self) -> bool:
        return bool(N.lib().hz_prog_is_captured(self.prog))

    def replay(self, stream=None):
        N.check(N.lib().hz_prog_replay(self.prog, N.stream_ptr(stream)), "prog_replay")

    def num_ops(self) -> int:
        return N.lib().hz_prog_num_ops(self.prog)

    def __del__(self):
        try:
            if getattr(self, "prog", None):
                self._lib.hz_prog_destroy(self.prog)
                self.prog = None
        except Exception:
            pass


def bench_contexts(ctxs: list, streams: list, iters: int, threads: bool | None = None) -> float:
    """Replay every context on its own stream ``iters`` times from C++; returns seconds.
    ``threads`` (default: env ``HIPZAP_SUBMIT_THREADS=1``): one host submission thread per
    stream instead of one thread round-robining over all streams."""
    n = len(ctxs)
    progs = (C.c_void_p * n)(*[c.prog for c in ctxs])
    strs = (C.c_void_p * n)(*[s.cuda_stream for s in streams])
    if threads is None:
        threads = os.environ.get("HIPZAP_SUBMIT_THREADS", "0") == "1"
    if threads and n > 1:
        out = (C.c_double * 2)()
        rc = N.lib().hz_prog_bench2(progs, strs, n, iters, 1, out)
        if rc:
            raise RuntimeError(f"hz_prog_bench2 failed ({rc})")
        return out[1] * 1e-6
    us = N.lib().hz_prog_bench(progs, strs, n, iters)
    if us < 0:
        raise RuntimeError(f"hz_prog_bench failed ({us})")
    return us * 1e-6


def serve_bench_contexts(ctxs: list, streams: list, iters: int, payloads: list | None = None) -> tuple[float, list]:
    """Closed-loop serving benchmark over host-I/O contexts (csrc/runtime.cpp hz_serve_bench):
    one native thread per context, each request = copy its payload into the pinned input,
    replay, wait, copy the logits out. Returns (seconds, per-request latencies in ms)."""
    n = len(ctxs)
    assert all(c.host_io for c in ctxs), "serve_bench needs host-I/O contexts"
    in_bytes = ctxs[0].host_input.numel() * ctxs[0].host_input.element_size()
    out_bytes = ctxs[0].host_output.numel() * ctxs[0].host_output.element_size()
    if payloads is None:
        payloads = [c.host_input.clone() for c in ctxs]
    outs = [c.host_output.clone() for c in ctxs]
    V = C.c_void_p * n
    lat = (C.c_double * (n * iters))()
    wall = C.c_double()
    rc = N.lib().hz_serve_bench(V(*[c.prog for c in ctxs]), V(*[s.cuda_stream for s in streams]),
                                V(*[c.host_input.data_ptr() for c in ctxs]), V(*[p.data_ptr() for p in payloads]),
                                in_bytes, V(*[c.host_output.data_ptr() for c in ctxs]),
                                V(*[o.data_ptr() for o in outs]), out_bytes, n, iters, lat, C.byref(wall))
    if rc:
        raise RuntimeError(f"hz_serve_bench failed ({rc})")
    return wall.value * 1e-6, [v * 1e-3 for v in lat]
