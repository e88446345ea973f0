"""Plan images: serialise a bound native Program for the torch-free cold start.

``export_plan`` builds the same :class:`~hipzap.engine.program.ExecContext` a GPU engine would
(same graph, same tuned launch configs, same zero-copy request I/O), but against CPU tensors
and a :class:`PlanRecorder` instead of the native library. Every pointer field of every
recorded launch is then resolved to (region, offset):

* region 0 — the shared device blob: every parameter/constant storage a launch references,
  256-B aligned; its bytes are stored in the file (4 KiB aligned, so it can be mmapped and
  DMA'd as is);
* region 1 — the per-context device block: the activation arena + static device I/O;
* region 2 — the per-context pinned host block: the request input(s) and the logits.

``csrc/plan.cpp`` loads the file with no Python tensor library at all (``hipzap/lite.py``):
mmap, one H2D (or an RCCL broadcast) of the blob, patch relocations, capture. The format is
tied to the native parameter layouts by ``hz_abi_version()``; a stale plan is refused and the
caller falls back to the ``.pth`` path. Reference parity: the plan is a deploy-time artifact
derived from the public ``torch.load`` state_dict (``/root/reference/main.py:99``), the way
Zappa's slim handler ships a pre-built package (``zappa_settings.rename.json:10``).
"""
from __future__ import annotations

import ctypes as C
import dataclasses
import json
import os
import struct

import torch

from .. import _native as N
from ..models import registry
from .engine import add_softmax_head, load_tuning
from .program import ExecContext

PLAN_SUFFIX = ".hzplan"
MAGIC = b"HZPLAN01"
VERSION = 1
HEADER = struct.Struct("<8s15Q")  # csrc/plan.cpp FileHeader
OPHDR = struct.Struct("<IiiIII")   # OpHeader
RELOC = struct.Struct("<IIQ")      # Reloc
OP_CONV, OP_CONV2, OP_MAXPOOL, OP_AVGPOOL, OP_PREPROCESS, OP_MEMCPY, OP_KERNEL, OP_FORK, OP_JOIN = range(1, 10)
BLOB_ALIGN = 4096
FLAG_WEIGHTLESS = 1  # csrc/plan.cpp kFlagWeightless


class AvgpoolArgs(C.Structure):
    _fields_ = [("x", C.c_void_p), ("out", C.c_void_p), ("N", C.c_int), ("HW", C.c_int), ("C", C.c_int),
                ("blocked", C.c_int)]


class PreprocessArgs(C.Structure):
    _fields_ = [("src", C.c_void_p), ("dst", C.c_void_p), ("mean", C.c_void_p), ("inv_std", C.c_void_p),
                ("N", C.c_int), ("Cin", C.c_int), ("H", C.c_int), ("W", C.c_int), ("Cpad", C.c_int),
                ("mode", C.c_int)]


class MemcpyArgs(C.Structure):
    _fields_ = [("dst", C.c_void_p), ("src", C.c_void_p), ("bytes", C.c_uint64)]


def plan_path(ckpt_path: str, tag: str = "") -> str:
    """``m.pth`` -> ``m.pth.hzplan`` (``tag`` distinguishes batch/concurrency variants)."""
    return ckpt_path + (f".{tag}" if tag else "") + PLAN_SUFFIX


def _obj(ref):
    """ctypes.byref(x) -> x."""
    return getattr(ref, "_obj", ref)


class PlanRecorder:
    """Stands in for the native library while an ExecContext binds: records every op with its
    parameter struct (pointer fields found from the ctypes field types)."""
    recording = True

    def __init__(self):
        self.ops: list = []  # (type, arg, slot, [ctypes structs])

    def hz_prog_create(self):
        return 1

    def hz_prog_destroy(self, prog):
        pass

    def hz_prog_num_ops(self, prog):
        return len(self.ops)

    def _add(self, t, arg, slot, *structs):
        self.ops.append((t, int(arg), int(slot), [_obj(s) for s in structs]))
        return 0

    def hz_prog_add_conv(self, prog, prm, cfg, slot):
        return self._add(OP_CONV, cfg, slot, prm)

    def hz_prog_add_conv2(self, prog, a, b, cfg, slot):
        return self._add(OP_CONV2, cfg, slot, a, b)

    def hz_prog_add_maxpool(self, prog, prm, slot):
        return self._add(OP_MAXPOOL, 0, slot, prm)

    def hz_prog_add_avgpool(self, prog, x, out, n, hw, c, blocked, slot):
        return self._add(OP_AVGPOOL, 0, slot, AvgpoolArgs(x, out, n, hw, c, blocked))

    def hz_prog_add_preprocess(self, prog, src, dst, n, cin, h, w, cpad, mode, mean, inv_std, slot):
        return self._add(OP_PREPROCESS, 0, slot, PreprocessArgs(src, dst, mean, inv_std, n, cin, h, w, cpad, mode))

    def hz_prog_add_memcpy(self, prog, dst, src, nbytes, slot):
        return self._add(OP_MEMCPY, 0, slot, MemcpyArgs(dst, src, nbytes))

    def hz_prog_add_kernel(self, prog, kind, prm, size, slot):
        s = _obj(prm)
        assert C.sizeof(s) == size
        return self._add(OP_KERNEL, kind, slot, s)

    def hz_prog_add_fork(self, prog, slot):
        return self._add(OP_FORK, 0, slot)

    def hz_prog_add_join(self, prog, slot):
        return self._add(OP_JOIN, 0, slot)


def _pointer_fields(st) -> list[tuple[int, int]]:
    """[(byte offset, value)] of every pointer-typed field of a ctypes struct."""
    out = []
    for name, ty in st._fields_:
        if ty is C.c_void_p or (isinstance(ty, type) and issubclass(ty, C._Pointer)):
            v = getattr(st, name)
            v = v if isinstance(v, int) or v is None else C.cast(v, C.c_void_p).value
            out.append((getattr(type(st), name).offset, v or 0))
    return out


def _tensors(obj):
    """(field name, tensor) of a packed parameter (None for a bare tensor)."""
    if torch.is_tensor(obj):
        yield None, obj
    elif dataclasses.is_dataclass(obj):
        for f in dataclasses.fields(obj):
            v = getattr(obj, f.name)
            if torch.is_tensor(v):
                yield f.name, v


class _Regions:
    """Address -> (region, offset) over the storages a context references."""

    def __init__(self):
        self.spans: list = []  # (start, end, region, region_offset_of_start, storage tensor)
        self.size = [0, 0, 0]
        self.blob_items: list = []  # (offset, storage bytes as uint8 tensor)
        self._seen: set = set()

    def add(self, t: torch.Tensor, region: int, keep_bytes: bool, label=None):
        """``label``: (parameter name, field) of a packed-parameter storage (weightless templates
        place it by name), None for a constant (its bytes travel in the template)."""
        st = t.untyped_storage()
        ptr, nb = st.data_ptr(), st.nbytes()
        if nb == 0 or (ptr, region) in self._seen:
            return
        self._seen.add((ptr, region))
        off = (self.size[region] + 255) // 256 * 256
        self.size[region] = off + nb
        self.spans.append((ptr, ptr + nb, region, off))
        if keep_bytes:
            if label is not None and nb != t.numel() * t.element_size():
                label = None  # a view into a larger storage: ship its bytes instead
            self.blob_items.append((off, torch.empty(0, dtype=torch.uint8).set_(st, 0, (nb,), (1,)), label))

    def resolve(self, v: int) -> tuple[int, int] | None:
        for start, end, region, off in self.spans:
            if start <= v < end:
                return region, off + (v - start)
        return None


def _dtype_name(dt: torch.dtype) -> str:
    return str(dt).replace("torch.", "")


def export_plan(model: str, params: dict, arch_kw: dict, path: str, batch: int = 1, contexts: int = 1,
                zero_copy: str = "all", probs: bool = False, tuned: dict | None = None,
                source: dict | None = None, host_io: bool = True, weightless: bool = False,
                extra_meta: dict | None = None) -> dict:
    """Write a plan image for ``model`` with CPU-resident packed ``params`` (``adapter.pack(sd,
    "cpu")``). ``contexts``: the request concurrency the launch configs are tuned for (the conv
    tables differ for 1 vs 24 streams); any number of contexts can be instantiated at load.
    ``host_io``: request I/O in pinned host memory (serving, zero-copy by default); False: the
    inputs/outputs live in the context's device block (a DP shard fed by an RCCL scatter).
    ``weightless``: a TEMPLATE -- no weight bytes in the file; ``meta["blob_map"]`` says where each
    packed parameter's storage goes in the blob (its name and field), ``meta["blob_consts"]`` carries
    the few constant storages (preprocess mean/std) inline; the loader fills the blob itself
    (hipzap/lite.py ``PlanEngine.from_checkpoint``: device-side packing of a .pth).
    Returns the metadata dict stored in the file."""
    adapter = registry.get(model)
    g = adapter.build_graph(batch=batch, **arch_kw)
    if probs:
        add_softmax_head(g)
    if tuned is None:
        tuned = load_tuning(model, batch, contexts)
    rec = PlanRecorder()
    ctx = ExecContext(g, params, torch.device("cpu"), tuned, host_io=host_io, zero_copy=zero_copy if host_io else "",
                      lib=rec)
    regs = _Regions()
    for key, obj in params.items():
        for field, t in _tensors(obj):
            regs.add(t, 0, True, label=(key, field))
    for t in ctx._keep:
        regs.add(t, 0, True)
    host = (list(ctx.host_inputs) + [ctx.host_output]) if host_io else []
    host_ptrs = {h.untyped_storage().data_ptr() for h in host}
    regs.add(ctx.arena, 1, False)
    for tid, t in ctx.ext.items():
        if t.untyped_storage().data_ptr() not in host_ptrs:
            regs.add(t, 1, False)
    for h in host:
        regs.add(h, 2, False)

    # ops: params bytes + relocations; only blob storages some launch references are kept
    used_blob: set = set()
    recs = []
    for (t, arg, slot, structs) in rec.ops:
        raw, rels, base = b"", [], 0
        for st in structs:
            for off, v in _pointer_fields(st):
                if not v:
                    continue
                hit = regs.resolve(v)
                if hit is None:
                    raise ValueError(f"plan export: op {len(recs)} ({type(st).__name__}) points outside every "
                                     f"known buffer")
                rels.append((base + off, hit[0], hit[1]))
                if hit[0] == 0:
                    used_blob.add(hit)
            raw += bytes(st)
            base += C.sizeof(st)
        recs.append((t, arg, slot, raw, rels))

    # compact the blob to the referenced storages
    keep = []
    for off, data, label in regs.blob_items:
        if any(off <= r_off < off + max(1, data.numel()) for (_, r_off) in used_blob):
            keep.append((off, data, label))
    remap, blob_len = {}, 0
    for off, data, _ in keep:
        new = (blob_len + 255) // 256 * 256
        remap[off] = (new, data.numel())
        blob_len = new + data.numel()

    def blob_off(r_off):
        for old, (new, nb) in remap.items():
            if old <= r_off < old + max(1, nb):
                return new + (r_off - old)
        raise AssertionError("unreferenced blob storage")

    ops_bytes = bytearray()
    for (t, arg, slot, raw, rels) in recs:
        ops_bytes += OPHDR.pack(t, arg, slot, len(raw), len(rels), 0)
        ops_bytes += raw + b"\0" * ((-len(raw)) % 8)
        for (off, region, r_off) in rels:
            ops_bytes += RELOC.pack(off, region, blob_off(r_off) if region == 0 else r_off)

    def io(t):
        region, off = regs.resolve(t.data_ptr())
        return {"region": region, "off": off, "shape": list(t.shape), "dtype": _dtype_name(t.dtype),
                "bytes": t.numel() * t.element_size()}

    out_spec = ctx.host_output if host_io else ctx.output
    meta = {
        "format": "hzplan", "version": VERSION, "model": model, "batch": batch, "arch_kw": arch_kw,
        "tuned_contexts": contexts, "zero_copy": zero_copy if host_io else "", "probs": probs, "host_io": host_io,
        "inputs": [io(h) for h in (ctx.host_inputs if host_io else ctx.inputs)],
        "output": {**io(out_spec),
                   "num_labels": (getattr(g, "meta", None) or {}).get("num_labels",
                                                                       (getattr(g, "meta", None) or {}).get(
                                                                           "num_classes"))},
        "configs": [list(c) for c in ctx.configs], "n_ops": len(recs), "source": source,
        "ctx_dev_bytes": regs.size[1], "ctx_host_bytes": regs.size[2], "blob_bytes": blob_len,
        "arena_bytes": ctx.arena_bytes,
    }
    emb = params.get("emb")
    if emb is not None and hasattr(emb, "word"):  # BERT-style text plan: inputs ids / types / additive mask
        meta.update({"kind": "text", "seq_len": int(g.shape(g.inputs[0])[0]) // batch,
                     "vocab": int(emb.word.shape[0]), "type_vocab": int(emb.type.shape[0])})
    import hashlib
    h = hashlib.sha256()
    for old, data, _ in keep:  # digest of the blob exactly as written (offsets + bytes)
        h.update(remap[old][0].to_bytes(8, "little"))
        h.update(data.numpy().tobytes())
    meta["blob_sha256"] = h.hexdigest()
    if weightless:
        import base64
        meta["weightless"] = True
        meta["blob_map"] = {f"{label[0]}/{label[1]}": [remap[old][0], remap[old][1]]
                            for old, data, label in keep if label is not None}
        meta["blob_consts"] = [[remap[old][0], base64.b64encode(data.numpy().tobytes()).decode()]
                               for old, data, label in keep if label is None]
        del meta["blob_sha256"]  # no weights: nothing to digest
    if extra_meta:
        meta.update(extra_meta)
    meta_b = json.dumps(meta).encode()
    meta_off = HEADER.size
    ops_off = (meta_off + len(meta_b) + 7) // 8 * 8
    b_off = (ops_off + len(ops_bytes) + BLOB_ALIGN - 1) // BLOB_ALIGN * BLOB_ALIGN
    abi = N.lib().hz_abi_version()
    hdr = HEADER.pack(MAGIC, VERSION, abi, len(recs), meta_off, len(meta_b), ops_off, len(ops_bytes), b_off, blob_len,
                      regs.size[1], regs.size[2], FLAG_WEIGHTLESS if weightless else 0, 0, 0, 0)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = f"{path}.tmp{os.getpid()}"
    with open(tmp, "wb") as f:
        f.write(hdr)
        f.write(meta_b)
        f.write(b"\0" * (ops_off - meta_off - len(meta_b)))
        f.write(ops_bytes)
        f.write(b"\0" * (b_off - ops_off - len(ops_bytes)))
        pos = 0
        for old, data, _ in ([] if weightless else keep):
            new, nb = remap[old]
            f.write(b"\0" * (new - pos))
            f.write(data.numpy().tobytes())
            pos = new + nb
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)
    del ctx
    return meta


def export_from_checkpoint(model: str, ckpt: str, path: str | None = None, batch: int = 1, contexts: int = 1,
                           input_uint8: bool | None = None, dp_shard: int | None = None, **kw) -> str:
    """``torch.load`` the checkpoint, pack it on the CPU and write its plan image (deploy time,
    ``hipzap plan``); the plan is keyed to the checkpoint's identity (size, mtime, sampled hash)."""
    from .packfile import source_stamp
    sd = torch.load(ckpt, map_location="cpu", weights_only=True)
    if isinstance(sd, dict) and "state_dict" in sd and isinstance(sd["state_dict"], dict):
        sd = sd["state_dict"]
    adapter = registry.get(model)
    params, arch_kw = adapter.pack(sd, "cpu")
    arch_kw = dict(arch_kw)
    if input_uint8 is None:
        input_uint8 = model.startswith("resnet")
    if input_uint8 and model.startswith("resnet"):
        arch_kw["input_uint8"] = True
    stamp = source_stamp(ckpt)
    if dp_shard:  # device-I/O shard program of a DP cluster (serve/cluster.py PlanShardRunner)
        shard_path = plan_path(ckpt, f"dp{dp_shard}")
        export_plan(model, params, arch_kw, shard_path, batch=dp_shard, contexts=1, source=stamp, host_io=False)
    path = path or plan_path(ckpt)
    export_plan(model, params, arch_kw, path, batch=batch, contexts=contexts, source=stamp, **kw)
    return path


def export_template(model: str, num_classes: int = 1000, batch: int = 1, contexts: int = 1,
                    input_uint8: bool = True, path: str | None = None) -> str:
    """Write the weightless plan TEMPLATE of an architecture (no checkpoint involved): the bound
    program, launch configs and arena layout of ``model`` at ``batch`` / ``contexts``, plus the
    packing recipe -- which checkpoint tensors (by state_dict key) produce each packed parameter,
    its geometry and where it goes in the blob. ``hipzap.lite.PlanEngine.from_checkpoint`` then
    cold-starts ANY checkpoint of that architecture straight from its ``.pth`` without torch: the
    raw tensors are copied to the device and packed there (csrc/pack.hip). Templates are built
    with the native library (``hipzap.build``), keyed to the lowering code (``lite.code_stamp``)."""
    from ..lite import code_stamp, template_path
    from .nppack import conv_geometry, pack_sources
    if not model.startswith("resnet"):
        raise ValueError("plan templates cover the ResNet family (device packer: conv + linear)")
    adapter = registry.get(model)
    torch.manual_seed(0)
    m = adapter.make_model(num_classes).eval()
    sd = m.state_dict()
    params, arch_kw = adapter.pack(sd, "cpu")
    arch_kw = dict(arch_kw, input_uint8=bool(input_uint8))
    recipe = {}
    for name, kind, w, bn, b in pack_sources(sd):
        recipe[name] = {"kind": kind, "w": w, "bn": bn, "b": b, **conv_geometry(name, kind, tuple(sd[w].shape))}
    path = path or template_path(model, batch, contexts, num_classes, input_uint8)
    meta = export_plan(model, params, arch_kw, path, batch=batch, contexts=contexts, weightless=True,
                       extra_meta={"code_stamp": code_stamp(), "pack": recipe})
    missing = [n for n in recipe if f"{n}/wf" not in meta["blob_map"] or f"{n}/bias" not in meta["blob_map"]]
    if missing:
        os.unlink(path)
        raise ValueError(f"template: packed parameters without a blob slot: {missing}")
    return path
