"""Torch-free serving runtime over plan images (``.hzplan``, engine/plan.py + csrc/plan.cpp).

The serverless cold path: process start -> ctypes load of
``libhipzap.so`` -> mmap the plan -> HIP init -> one DMA of the packed weights -> bind +
capture -> first request. Nothing here imports torch (``import torch`` alone is ~1.5 s of a
~2 s cold process); requests are plain byte buffers (a decoded uint8 HWC image for the vision
models) and results come back as ``array.array`` (or numpy, if the caller asks and has it).

Concurrency mirrors :class:`hipzap.engine.engine.Engine`: N contexts (own arena, pinned I/O,
stream and captured graph) over one weight blob; ``infer`` releases the GIL inside the native
call, so request threads overlap.
"""
from __future__ import annotations

import array
import ctypes as C
import json
import os
import struct
import threading
import time

from . import _native as N

HEADER = struct.Struct("<8s15Q")
PHASES = ("parse_ms", "hip_init_ms", "upload_ms", "ctx_alloc_ms", "bind_ms", "capture_ms", "blob_alloc_ms",
          "first_copy_ms",
          # upload_ms = stream_ms + upload_dma_ms + warm_wait_ms; warm_thread_ms runs beside them
          "stream_ms", "upload_dma_ms", "warm_wait_ms", "warm_thread_ms")
_TYPECODE = {"float32": "f", "uint8": "B", "int32": "i", "int64": "q", "bfloat16": "H", "float16": "H"}


class PlanError(RuntimeError):
    pass


def lib():
    """The native library (plan prototypes are registered by hipzap._native)."""
    return N.lib()


def read_meta(path: str) -> dict:
    """The plan's JSON metadata (model, I/O offsets and shapes, launch configs, source stamp)."""
    with open(path, "rb") as f:
        hdr = f.read(HEADER.size)
        if len(hdr) < HEADER.size or hdr[:8] != b"HZPLAN01":
            raise PlanError(f"{path}: not a hipzap plan image")
        fields = HEADER.unpack(hdr)
        meta_off, meta_len = fields[4], fields[5]
        f.seek(meta_off)
        meta = json.loads(f.read(meta_len))
    meta["abi"] = fields[2]
    return meta


def plan_usable(path: str) -> bool:
    """True if ``path`` is a plan image this library build can load (same native ABI)."""
    try:
        return read_meta(path)["abi"] == lib().hz_abi_version()
    except (OSError, PlanError, ValueError, KeyError):
        return False


def _in_buffer(x):
    """(address, nbytes, keepalive) of a host buffer: bytes, bytearray, memoryview, numpy array
    or CPU torch tensor (duck-typed: torch is never imported here)."""
    if hasattr(x, "data_ptr") and hasattr(x, "element_size"):  # torch.Tensor
        x = x.contiguous()
        return x.data_ptr(), x.numel() * x.element_size(), x
    if hasattr(x, "__array_interface__") and hasattr(x, "ctypes"):  # numpy
        if not x.flags["C_CONTIGUOUS"]:
            x = x.copy(order="C")
        return x.ctypes.data, x.nbytes, x
    if isinstance(x, bytes):
        return C.cast(C.c_char_p(x), C.c_void_p).value, len(x), x
    mv = memoryview(x).cast("B")
    if mv.readonly:
        b = bytes(mv)
        return C.cast(C.c_char_p(b), C.c_void_p).value, len(b), b
    buf = (C.c_char * mv.nbytes).from_buffer(mv)
    return C.addressof(buf), mv.nbytes, buf


_PKG = os.path.dirname(os.path.abspath(__file__))
_STAMP_DIRS = ("engine", "models", "ops", "tuning")


def code_stamp() -> str:
    """Identity of the code that lowers a model to a plan (graph building, arena planning, launch
    configs, tuning tables): a plan TEMPLATE (weightless) is valid only for the code that wrote
    it, beyond the native ABI the loader already checks. Hashes file bytes; no imports."""
    import hashlib
    h = hashlib.sha256()
    for d in _STAMP_DIRS:
        root = os.path.join(_PKG, d)
        for name in sorted(os.listdir(root)):
            if name.endswith((".py", ".json")):
                h.update(name.encode())
                with open(os.path.join(root, name), "rb") as f:
                    h.update(f.read())
    return h.hexdigest()[:16]


def template_dir() -> str:
    return os.environ.get("HIPZAP_TEMPLATE_DIR") or os.path.join(_PKG, "_lib", "templates")


def template_path(model: str, batch: int = 1, contexts: int = 1, num_classes: int = 1000,
                  input_uint8: bool = True) -> str:
    """Where the weightless plan template of an architecture lives (built by ``hipzap.build``)."""
    return os.path.join(template_dir(), f"{model}-b{batch}-c{contexts}-n{num_classes}{'-u8' if input_uint8 else ''}"
                                        ".hztmpl")


def no_sdma_default() -> None:
    """Copies through blit kernels instead of the SDMA engines (``HSA_ENABLE_SDMA=0``), unless the
    deployment chose (or ``HIPZAP_KEEP_SDMA=1``): the plan's 51-MB weight upload is faster that way
    and the process's first queue is cheaper -- fresh-process cold start 262 -> 237 ms p50,
    interleaved on one box (``profiles/r2_coldstart/sdma_ab``). The serving path has no copies
    (zero-copy request I/O). Takes effect only before the process's first HIP call."""
    if os.environ.get("HIPZAP_KEEP_SDMA", "0") != "1":
        os.environ.setdefault("HSA_ENABLE_SDMA", "0")


_fill_tls = threading.local()


def upload_stream() -> int | None:
    """Inside a ``fill_blob`` callback: the plan's upload stream, which becomes the first
    context's stream (a fill that runs on it creates no stream of its own, ~10-20 ms of lazy
    runtime work in a fresh process); None outside a fill."""
    return getattr(_fill_tls, "stream", None)


class PlanEngine:
    """One plan image on one GPU. ``read_blob=False`` + ``fill_blob(address, nbytes)`` lets a DP
    rank receive the weights by RCCL broadcast instead of reading the file."""

    def __init__(self, path: str, device: int = 0, contexts: int = 1, eager_contexts: int | None = None,
                 capture: bool | str = True, read_blob: bool = True, fill_blob=None):
        """``capture="lazy"``: the eager contexts are NOT captured at load; their first requests
        run the bound program launch by launch and :meth:`ensure_contexts` captures them (cold
        start -> first response without the graph instantiation on the critical path)."""
        t0 = time.perf_counter()
        self.path = path
        self.meta = read_meta(path)
        self.device = device
        L = lib()
        if self.meta["abi"] != L.hz_abi_version():
            raise PlanError(f"{path}: plan written for native ABI {self.meta['abi']}, library is "
                            f"{L.hz_abi_version()} (re-export with `hipzap plan`)")
        no_sdma_default()
        tm = (C.c_double * len(PHASES))()
        h = L.hz_plan_open(path.encode(), device, int(read_blob), tm)
        if not h:
            raise PlanError(L.hz_plan_last_error().decode())
        self._h = h
        self.timings = {"meta_ms": 0.0}
        if fill_blob is not None:
            nb = C.c_uint64()
            addr = L.hz_plan_blob(h, C.byref(nb))
            ta = time.perf_counter()
            _fill_tls.stream = L.hz_plan_upload_stream(h) or None
            try:
                fill_blob(addr, nb.value)
            finally:
                _fill_tls.stream = None
            self.timings["broadcast_ms"] = (time.perf_counter() - ta) * 1e3
        self.num_contexts = contexts
        self._capture = bool(capture)
        self._lazy = capture == "lazy"
        # HIPZAP_STREAM_KIND=hiprio: the contexts after the first (which takes the upload stream)
        # on highest-priority streams. Not the default here: with the first context on a
        # normal-priority queue and the rest on high-priority ones, the BERT text plan's 4
        # contexts replay at 16.3k seq/s against 22.5k on plain streams (profiles/r6_queues)
        if os.environ.get("HIPZAP_STREAM_KIND", "auto") == "hiprio":
            L.hz_plan_set_stream_priority(h, 1)
        n0 = contexts if eager_contexts is None else max(1, min(eager_contexts, contexts))
        self._check(L.hz_plan_add_contexts(h, n0, 0 if self._lazy else int(bool(capture))), "add_contexts")
        self._uncaptured = list(range(n0)) if self._lazy else []
        self._locks = [threading.Lock() for _ in range(n0)]
        self._rr, self._rr_lock, self._build_lock = 0, threading.Lock(), threading.Lock()
        self._exec = None
        L.hz_plan_timings(h, tm)
        self.timings.update({k: tm[i] for i, k in enumerate(PHASES)})
        self.timings["total_ms"] = (time.perf_counter() - t0) * 1e3
        inp, out = self.meta["inputs"], self.meta["output"]
        self.in_specs = inp
        self.out_spec = out
        # "vision": a request is one image (batch-B plans batch requests dynamically);
        # "text": a request is a whole padded batch of sequences (ids, types, additive mask)
        self.kind = self.meta.get("kind", "vision")
        self._out_n = out["bytes"] // array.array(_TYPECODE[out["dtype"]]).itemsize

    def _check(self, rc: int, what: str) -> None:
        if rc != 0:
            raise PlanError(f"{what} failed ({rc}): {lib().hz_plan_last_error().decode()}")

    @classmethod
    def from_checkpoint(cls, ckpt: str, device: int = 0, contexts: int = 1, batch: int = 1, template: str | None = None,
                        template_contexts: int = 1, **kw) -> "PlanEngine":
        """Cold start from the reference's checkpoint format (a ``torch.save`` state_dict,
        /root/reference/main.py:99) WITHOUT torch: the archive is scanned by the weights-only
        reader (hipzap/pthreader.py), the architecture's weightless plan template supplies the
        program, and the raw fp32 tensors are copied to the GPU and packed there (BN folding, bf16,
        fragment-major: csrc/pack.hip) straight into the plan's weight blob -- byte for byte what
        ``hipzap plan`` would have written (tests/test_pth_lite_gpu.py)."""
        import base64
        from . import hip
        from .engine.nppack import infer_resnet
        from .pthreader import scan
        t0 = time.perf_counter()
        refs = scan(ckpt)
        model, ncls = infer_resnet(refs)
        tmpl = template or template_path(model, batch, template_contexts, ncls, True)
        if not os.path.exists(tmpl):
            raise PlanError(f"no plan template {tmpl} for {model} ({ncls} classes): build it with "
                            f"python -m hipzap.build --templates")
        meta = read_meta(tmpl)
        if not meta.get("weightless") or meta.get("code_stamp") != code_stamp():
            raise PlanError(f"{tmpl}: stale or not a template (rebuild with python -m hipzap.build --templates)")
        recipe = meta["pack"]
        t_scan = (time.perf_counter() - t0) * 1e3
        # every source tensor: fp32, contiguous, the geometry the template was built for
        jobs = []
        for name, e in recipe.items():
            keys = {"w": e["w"], "b": e["b"]}
            if e["bn"]:
                keys.update({f: f"{e['bn']}.{f2}" for f, f2 in (("gamma", "weight"), ("beta", "bias"),
                                                                 ("mean", "running_mean"), ("var", "running_var"))})
            src = {}
            for f, k in keys.items():
                if k is None:
                    continue
                r = refs.get(k)
                if r is None or r.dtype != "float32" or not r.is_contiguous():
                    raise PlanError(f"{ckpt}: {k} missing, not fp32 or not contiguous")
                src[f] = r
            want = (e["cout"], e["cin"]) if e["kind"] == "linear" else (e["cout"], e["cin"], e["r"], e["s"])
            if tuple(src["w"].shape) != want:
                raise PlanError(f"{ckpt}: {e['w']} is {src['w'].shape}, template expects {want}")
            # the pack kernel reads cout elements of every BN vector and of the bias: a short one
            # would read into the next staged tensor (or past the staging buffer)
            for f, r in src.items():
                if f != "w" and tuple(r.shape) != (e["cout"],):
                    raise PlanError(f"{ckpt}: {keys[f]} is {tuple(r.shape)}, template expects ({e['cout']},)")
            jobs.append((name, e, src))
        stores = {}
        for _, _, src in jobs:
            for r in src.values():
                stores[r.storage.key] = r.storage
        timing = {"scan_ms": t_scan}

        def fill(addr: int, nbytes: int) -> None:
            ta = time.perf_counter()
            offs, total = {}, 0
            for k, st in stores.items():
                offs[k] = total
                total += (st.nbytes + 255) // 256 * 256
            staging = hip.DeviceBuffer(total)
            n = len(stores)
            U64 = C.c_uint64 * n
            keys = list(stores)
            stream = upload_stream() or hip._private_stream()
            rc = lib().hz_upload_file(ckpt.encode(), n, U64(*[stores[k].file_off for k in keys]),
                                      U64(*[stores[k].nbytes for k in keys]),
                                      (C.c_void_p * n)(*[staging.ptr + offs[k] for k in keys]), stream)
            if rc:
                raise PlanError(f"checkpoint upload failed: {lib().hz_plan_last_error().decode()}")
            tb = time.perf_counter()
            from . import _native as NN
            for name, e, src in jobs:
                dev = {f: staging.ptr + offs[r.storage.key] + r.offset * 4 for f, r in src.items()}
                p = NN.PackConvParams()
                p.w, p.gamma, p.beta, p.mean, p.var = (dev.get(f, 0) for f in ("w", "gamma", "beta", "mean", "var"))
                p.bias_in = dev.get("b", 0)
                wf_off, wf_nb = meta["blob_map"][f"{name}/wf"]
                b_off, b_nb = meta["blob_map"][f"{name}/bias"]
                if wf_nb != e["rows"] * e["ksteps"] * 64 or b_nb != 4 * e["cout"]:
                    raise PlanError(f"template slot of {name} does not match its recipe")
                p.wf, p.bias_out = addr + wf_off, addr + b_off
                p.cout, p.cin, p.r, p.s, p.cin_p = e["cout"], e["cin"], e["r"], e["s"], e["cin_p"]
                p.rows, p.ksteps, p.eps = e["rows"], e["ksteps"], 1e-5
                if lib().hz_pack_conv_launch(C.byref(p), stream):
                    raise PlanError(f"pack kernel rejected {name}")
            for off, b64 in meta.get("blob_consts", []):
                data = base64.b64decode(b64)
                buf = C.create_string_buffer(data, len(data))
                hip.memcpy(addr + off, C.addressof(buf), len(data), hip.H2D, stream)
            hip.sync(stream)
            staging.free()
            timing.update({"upload_raw_ms": (tb - ta) * 1e3, "pack_ms": (time.perf_counter() - tb) * 1e3,
                           "raw_MB": round(total / 2**20, 1)})

        eng = cls(tmpl, device=device, contexts=contexts, read_blob=False, fill_blob=fill, **kw)
        eng.timings.update(timing)
        eng.source = ckpt
        return eng

    # ---------------------------------------------------------------- contexts
    def ensure_contexts(self) -> float:
        """Build the contexts deferred by ``eager_contexts`` (thread-safe); returns ms spent."""
        with self._build_lock:
            t0 = time.perf_counter()
            for i in self._uncaptured:  # lazy capture of the eager contexts (no request in flight)
                with self._locks[i]:
                    self._check(lib().hz_plan_capture_ctx(self._h, i), "capture_ctx")
            self._uncaptured = []
            have = lib().hz_plan_num_contexts(self._h)
            n = self.num_contexts - have
            if n <= 0:
                return (time.perf_counter() - t0) * 1e3
            self._check(lib().hz_plan_add_contexts(self._h, n, int(self._capture)), "add_contexts")
            with self._rr_lock:
                self._locks += [threading.Lock() for _ in range(n)]
            return (time.perf_counter() - t0) * 1e3

    @property
    def contexts(self) -> int:
        return len(self._locks)

    @property
    def host_io(self) -> bool:
        return self.meta.get("host_io", True)

    # ---------------------------------------------------------------- device-I/O plans (DP shards)
    def device_io(self, ctx: int = 0) -> tuple[list, int]:
        """(input device addresses, output device address) of a device-I/O plan's context."""
        if self.host_io:
            raise PlanError("host-I/O plan: requests go through infer/infer_raw")
        base = lib().hz_plan_device(self._h, ctx)
        return [base + sp["off"] for sp in self.in_specs], base + self.out_spec["off"]

    def stream(self, ctx: int = 0) -> int:
        return lib().hz_plan_stream(self._h, ctx)

    def replay(self, ctx: int = 0) -> None:
        """Enqueue one replay of context ``ctx`` on its stream (no wait)."""
        self._check(lib().hz_plan_replay(self._h, ctx), "replay")

    def sync(self, ctx: int = 0) -> None:
        self._check(lib().hz_plan_sync(self._h, ctx), "sync")

    def blob(self) -> tuple[int, int]:
        """(device address, bytes) of the shared weight blob."""
        nb = C.c_uint64()
        return lib().hz_plan_blob(self._h, C.byref(nb)), nb.value

    def executor(self):
        """Native request executor over all contexts, once every context exists (else None)."""
        ex = getattr(self, "_exec", None)
        if getattr(self, "_bexec", None) is not None:
            raise PlanError("this plan engine serves through the dynamic-batching executor")
        if ex is not None or not self._capture or not self.host_io or len(self._locks) != self.num_contexts \
                or self._uncaptured:
            return ex
        if self.kind != "text" and int(self.in_specs[0]["shape"][0]) > 1:
            raise PlanError("a batch-B plan serves one-image requests through batched_executor()")
        from .executor import Executor
        with self._build_lock:
            if getattr(self, "_exec", None) is None:
                for lk in self._locks:
                    lk.acquire()
                try:
                    L, n = lib(), len(self._locks)
                    hosts = [L.hz_plan_host(self._h, i) for i in range(n)]
                    self._exec = Executor([L.hz_plan_prog(self._h, i) for i in range(n)],
                                          [L.hz_plan_stream(self._h, i) for i in range(n)],
                                          [[h + sp["off"] for h in hosts] for sp in self.in_specs],
                                          [sp["bytes"] for sp in self.in_specs],
                                          [h + self.out_spec["off"] for h in hosts], self.out_spec["bytes"])
                finally:
                    for lk in self._locks:
                        lk.release()
        return self._exec

    def batched_executor(self, max_wait_us: float = 200.0, min_inflight: int = 1):
        """Dynamic-batching executor (csrc/executor.cpp) over every context of a batch-B plan: each
        request is ONE row (one image); concurrent requests share a replay. Built once the
        contexts exist and are captured (else None)."""
        ex = getattr(self, "_bexec", None)
        if ex is not None or not self._capture or not self.host_io or len(self._locks) != self.num_contexts \
                or self._uncaptured:
            return ex
        from .executor import Executor
        with self._build_lock:
            if getattr(self, "_exec", None) is not None:  # same pinned buffers and streams
                raise PlanError("this plan engine already serves through the per-request executor")
            if getattr(self, "_bexec", None) is None:
                # every context lock: a direct hz_plan_infer still in flight owns its context's
                # pinned buffers and stream until it returns
                for lk in self._locks:
                    lk.acquire()
                try:
                    L, n = lib(), len(self._locks)
                    hosts = [L.hz_plan_host(self._h, i) for i in range(n)]
                    self._bexec = Executor([L.hz_plan_prog(self._h, i) for i in range(n)],
                                           [L.hz_plan_stream(self._h, i) for i in range(n)],
                                           [[h + sp["off"] for h in hosts] for sp in self.in_specs],
                                           [sp["bytes"] for sp in self.in_specs],
                                           [h + self.out_spec["off"] for h in hosts], self.out_spec["bytes"],
                                           rows=int(self.in_specs[0]["shape"][0]), max_wait_us=max_wait_us,
                                           min_inflight=min_inflight)
                finally:
                    for lk in self._locks:
                        lk.release()
        return self._bexec

    def _pick(self) -> int:
        with self._rr_lock:
            i = self._rr % len(self._locks)
            self._rr += 1
        return i

    # ---------------------------------------------------------------- requests
    def infer_raw(self, x, ctx: int | None = None, rows: int | None = None) -> array.array:
        """One request: ``x`` = the input's exact bytes (uint8 HWC image for the ResNet plans), or
        for a multi-input plan (BERT: ids, token types, additive mask) a sequence with one buffer
        per input. Returns the output as a flat ``array.array`` (float32 logits). ``rows``: how
        many leading rows of a batch-B request are real (the rest is padding): on the dynamic-
        batching executor only those are submitted, and the padding rows' outputs stay zero."""
        if not self.host_io:
            raise PlanError("infer_raw needs a host-I/O plan")
        if len(self.in_specs) > 1:
            return self._infer_multi(x, ctx)
        addr, nb, keep = _in_buffer(x)
        spec = self.in_specs[0]
        if nb != spec["bytes"]:
            raise PlanError(f"request is {nb} bytes, plan input {spec['shape']} {spec['dtype']} is {spec['bytes']}")
        out = array.array(_TYPECODE[self.out_spec["dtype"]], bytes(self.out_spec["bytes"]))
        oaddr, _ = out.buffer_info()
        bex = getattr(self, "_bexec", None)
        if bex is None and ctx is None and int(spec["shape"][0]) > 1:
            self.ensure_contexts()
            bex = self.batched_executor()
        if bex is not None:
            # the contexts belong to the dynamic-batching executor (native /predict): the real
            # rows join its open batch from this thread (hz_exec_submit_rows), sharing replays
            # with concurrent one-image requests
            m = bex.rows if rows is None else max(1, min(int(rows), bex.rows))
            try:
                bex.submit_rows([addr], m, oaddr)
            finally:
                del keep
            return out
        ex = self.executor() if ctx is None else None
        if ex is not None:
            ex.submit([addr], oaddr)
            del keep
            return out
        i = self._pick() if ctx is None else ctx
        with self._locks[i]:
            rc = lib().hz_plan_infer(self._h, i, addr, spec["off"], nb, oaddr, self.out_spec["off"],
                                     self.out_spec["bytes"])
        del keep
        self._check(rc, "infer")
        return out

    def _infer_multi(self, xs, ctx: int | None) -> array.array:
        """A multi-input request: every input through the per-request executor, or (before it
        exists / with ``ctx``) packed into one copy when the inputs are adjacent in the pinned
        block (they are: the exporter lays them out in order)."""
        if not isinstance(xs, (list, tuple)) or len(xs) != len(self.in_specs):
            raise PlanError(f"this plan takes {len(self.in_specs)} inputs; pass one buffer per input")
        bufs = [_in_buffer(x) for x in xs]
        for (addr, nb, _), sp in zip(bufs, self.in_specs):
            if nb != sp["bytes"]:
                raise PlanError(f"input {sp['shape']} {sp['dtype']} is {sp['bytes']} bytes, got {nb}")
        out = array.array(_TYPECODE[self.out_spec["dtype"]], bytes(self.out_spec["bytes"]))
        oaddr, _ = out.buffer_info()
        ex = self.executor() if ctx is None else None
        if ex is not None:
            ex.submit([b[0] for b in bufs], oaddr)
            del bufs
            return out
        offs = [sp["off"] for sp in self.in_specs]
        if any(offs[i] + self.in_specs[i]["bytes"] != offs[i + 1] for i in range(len(offs) - 1)):
            raise PlanError("plan inputs are not adjacent in the host block")
        packed = bytearray(sum(b[1] for b in bufs))
        pos = 0
        for addr, nb, _ in bufs:
            C.memmove((C.c_char * nb).from_buffer(packed, pos), addr, nb)
            pos += nb
        paddr, pnb, keep = _in_buffer(packed)
        i = self._pick() if ctx is None else ctx
        with self._locks[i]:
            rc = lib().hz_plan_infer(self._h, i, paddr, offs[0], pnb, oaddr, self.out_spec["off"],
                                     self.out_spec["bytes"])
        del keep, bufs
        self._check(rc, "infer")
        return out

    def infer(self, x, ctx: int | None = None):
        """Like :meth:`infer_raw`, shaped ``[batch, classes]`` as a numpy array when numpy is
        importable (it is not needed on the cold path: import happens on first use)."""
        out = self.infer_raw(x, ctx)
        try:
            import numpy as np
        except ImportError:
            return out
        return np.frombuffer(out, dtype=np.float32 if out.typecode == "f" else None).reshape(
            self.out_spec["shape"][0], -1)

    def bench(self, iters: int) -> float:
        """Replay every context ``iters`` times from C++ (no host I/O); seconds."""
        self.ensure_contexts()
        us = lib().hz_plan_bench(self._h, iters)
        if us < 0:
            raise PlanError(f"bench failed ({us})")
        return us * 1e-6

    def close(self) -> None:
        for name in ("_exec", "_bexec"):
            ex = getattr(self, name, None)
            if ex is not None:
                ex.close()
                setattr(self, name, None)
        h, self._h = getattr(self, "_h", None), None
        if h:
            lib().hz_plan_close(h)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def describe(self) -> dict:
        return {"model": self.meta["model"], "batch": self.meta["batch"], "contexts": self.contexts,
                "ops": self.meta["n_ops"], "blob_MB": round(self.meta["blob_bytes"] / 2**20, 2),
                "timings_ms": {k: round(v, 2) for k, v in self.timings.items()}}
