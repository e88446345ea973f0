"""Serving engine: one model on one GPU with a hipGraph-captured warm path.

Cold start: ``torch.load(weights_only=True)`` of a standard state_dict ->
pack/fold on the GPU -> plan a static activation arena -> bind native Programs -> capture
one hipGraph per execution context -> first inference. Warm request: copy the input into a
context's static input buffer, ``hipGraphLaunch``, copy the logits out. Several contexts per
GPU (``num_contexts``) let independent bs=1 requests run concurrently on separate streams
sharing one packed weight set — the GPU analogue of Lambda's per-request container fan-out.
"""
from __future__ import annotations

import os
import threading
import time

import torch

from .. import _native
from ..models import registry
from .program import ExecContext, bench_contexts, serve_bench_contexts


def load_tuning(model: str, batch: int, contexts: int = 1) -> dict | None:
    """Measured launch-config table written by ``python -m hipzap.engine.tune`` (if any).

    Prefers the table tuned for the same request concurrency (``_c<contexts>``), then the one
    tuned for the highest concurrency below it (a throughput objective is closer to ``contexts``
    streams than the latency objective is), then the single-stream (latency) table.
    """
    import json
    from .tune import table_path
    for c in range(contexts, 0, -1):
        p = table_path(model, batch, c)
        if p.exists():
            with open(p) as f:
                return json.load(f)
    return None


def add_softmax_head(g) -> None:
    """Append a row softmax (csrc/transformer.hip softmax_kernel) over the logical classes of
    the graph's logits so the request returns probabilities (``/predict`` with probs)."""
    out = g.outputs[0]
    shape = g.shape(out)
    rows, cols = shape[0], int(torch.tensor(shape[1:]).prod()) if len(shape) > 1 else 1
    D = (getattr(g, "meta", None) or {}).get("num_labels", cols)
    probs = g.tensor((rows, D), torch.float32, "probs", external=True)
    g.add("softmax", [out], [probs], D=D)
    g.outputs[0] = probs


class Engine:
    def __init__(self, model: str, params: dict, device="cuda:0", batch: int = 1, num_contexts: int = 1,
                 capture: bool = True, tuned: dict | None = None, arch_kw: dict | None = None, timings=None,
                 host_io: bool = True, probs: bool = False, zero_copy: str | None = None,
                 eager_contexts: int | None = None, stream_kind: str | None = None):
        """``eager_contexts``: plan + capture only this many of the ``num_contexts`` request
        contexts before the engine is ready (cold start = time to the first served request); the
        rest are built by :meth:`ensure_contexts` (``bench`` calls it), e.g. after the first
        request, the way a warm container scales up its concurrency. None: all up front.
        ``stream_kind``: the contexts' streams (module ``stream_kind``; None: ``HIPZAP_STREAM_KIND``)."""
        self.model = model
        self.adapter = registry.get(model)
        self.device = torch.device(device)
        self.batch = batch
        self.params = params
        self.arch_kw = arch_kw or {}
        self.timings = dict(timings or {})
        if tuned is None:
            tuned = load_tuning(model, batch, num_contexts)
        self.tuned = tuned
        self.num_contexts = num_contexts
        # device-I/O engines are driven from their callers' streams (infer_device, DPPipeline): a
        # wait between a caller's stream and a high-priority context stream is slow (the DP
        # pipeline at shard 4: 11.1k vs 17.5-23.0k img/s, profiles/r6_queues), so under the
        # default policy they keep torch's pooled streams; host-I/O engines (the request executor,
        # the replay loop) take auto's choice
        if stream_kind is None and not host_io and os.environ.get("HIPZAP_STREAM_KIND", "auto") == "auto":
            stream_kind = "torch"
        self._stream_kind = stream_kind
        self._capture, self._zero_copy = capture, zero_copy
        n0 = num_contexts if eager_contexts is None else max(1, min(eager_contexts, num_contexts))
        t0 = time.perf_counter()
        with torch.cuda.device(self.device):
            self.graph = self.adapter.build_graph(batch=batch, **self.arch_kw)
            if probs:
                add_softmax_head(self.graph)
            self.host_io = host_io
            self.contexts, self.streams = self._new_contexts(n0)
            torch.cuda.synchronize(self.device)
            self.timings["plan_ms"] = (time.perf_counter() - t0) * 1e3
            t0 = time.perf_counter()
            self._capture_all(self.contexts, self.streams)
            torch.cuda.synchronize(self.device)
            self.timings["capture_ms"] = (time.perf_counter() - t0) * 1e3
        self._rr = 0
        self._locks = [threading.Lock() for _ in self.contexts]
        self._rr_lock = threading.Lock()
        self._build_lock = threading.Lock()  # ensure_contexts from concurrent request threads
        self._exec = None

    def _new_contexts(self, n: int):
        ctxs = [ExecContext(self.graph, self.params, self.device, self.tuned, host_io=self.host_io,
                            zero_copy=self._zero_copy) for _ in range(n)]
        # HIPZAP_CTX_STREAMS=k: contexts share k streams round-robin instead of one stream each (0,
        # default). k = 4 replays 11 % faster when the 4 streams land on the 4 hardware queues, but
        # which queue a stream gets is the runtime's choice: after engine rebuilds the same k = 4
        # ran at 6.5k (two queues' worth) vs 11.3k with own streams (profiles/r2_dispatch/)
        k = int(os.environ.get("HIPZAP_CTX_STREAMS", "0"))
        pool = getattr(self, "_stream_pool", [])
        self._stream_pool = pool
        base = len(getattr(self, "contexts", []) or [])
        streams = []
        for i in range(n):
            idx = base + i
            if k > 0 and idx >= k:
                streams.append(pool[idx % k])
            else:
                st = _context_stream(self.device, self.num_contexts, idx, self._stream_kind)
                pool.append(st)
                streams.append(st)
        return ctxs, streams

    def _capture_all(self, ctxs, streams) -> None:
        if self._capture:
            # the dedicated-queue streams are shared by every engine of <= 4 contexts in the process
            shared = int(os.environ.get("HIPZAP_CTX_STREAMS", "0")) > 0 or \
                stream_kind(self.num_contexts, self._stream_kind) == "cumask"
            cap = torch.cuda.Stream(device=self.device) if shared else None
            for c, s in zip(ctxs, streams):
                # a shared stream may carry other contexts' replays (other threads) that a capture
                # on it would swallow: capture on a private stream, replay on the shared one
                c.capture(cap if shared else s)
            if cap is not None:
                cap.synchronize()

    def ensure_contexts(self) -> float:
        """Plan + capture the contexts deferred by ``eager_contexts``; returns the ms spent.
        Safe to call from several request threads: one builds, the others find nothing to do."""
        with self._build_lock:
            n = self.num_contexts - len(self.contexts)
            if n <= 0:
                return 0.0
            t0 = time.perf_counter()
            with torch.cuda.device(self.device):
                ctxs, sts = self._new_contexts(n)
                self._capture_all(ctxs, sts)
                torch.cuda.synchronize(self.device)
            with self._rr_lock:  # lists grow in step; _pick reads len(self.contexts) under this lock
                self._locks += [threading.Lock() for _ in ctxs]
                self.streams += sts
                self.contexts += ctxs
            ms = (time.perf_counter() - t0) * 1e3
            self.timings["deferred_contexts_ms"] = ms
            return ms

    # -------------------------------------------------------------- construction
    @classmethod
    def from_state_dict(cls, model: str, sd: dict, device="cuda:0", **kw) -> "Engine":
        t0 = time.perf_counter()
        adapter = registry.get(model)
        dev = torch.device(device)
        with torch.cuda.device(dev):
            sd_dev = {k: v.to(dev, non_blocking=True) for k, v in sd.items() if torch.is_tensor(v)}
            params, arch_kw = adapter.pack(sd_dev, dev)
            torch.cuda.synchronize(dev)
        timings = dict(kw.pop("timings", {}) or {})
        timings["pack_ms"] = (time.perf_counter() - t0) * 1e3
        eng = cls(model, params, device, arch_kw=dict(arch_kw, **(kw.pop("arch_kw", None) or {})), timings=timings,
                  **kw)
        eng.pack_cfg = dict(arch_kw)
        return eng

    @classmethod
    def from_packed(cls, model: str, path: str, device="cuda:0", **kw) -> "Engine":
        """Cold-start fast path: a ``hipzap pack`` / ``write_packed`` file (BN folded, weights in
        the kernels' layouts) streamed straight into device memory — no fold/pack work."""
        from .packfile import load_packed
        t0 = time.perf_counter()
        params, cfg = load_packed(path, device)
        torch.cuda.synchronize(torch.device(device))
        timings = dict(kw.pop("timings", {}) or {})
        timings["load_packed_ms"] = (time.perf_counter() - t0) * 1e3
        arch_kw = dict(cfg, **(kw.pop("arch_kw", None) or {}))
        return cls(model, params, device, arch_kw=arch_kw, timings=timings, **kw)

    @classmethod
    def from_checkpoint(cls, model: str, path: str, device="cuda:0", use_packed: bool = True,
                        write_packed: bool = False, **kw) -> "Engine":
        """``torch.load`` of a standard state_dict (the reference's format, main.py:99), or, when
        ``use_packed`` and an up-to-date ``<path>.hzpack`` exists next to it, the packed fast
        path. ``write_packed``: after packing from the .pth, save the packed copy for next time."""
        from .packfile import find_packed, packed_path, save_packed, source_stamp
        if use_packed:
            pk = find_packed(path, model)
            if pk is not None:
                return cls.from_packed(model, pk, device, **kw)
        t0 = time.perf_counter()
        sd = torch.load(path, map_location="cpu", weights_only=True, mmap=True)
        if isinstance(sd, dict) and "state_dict" in sd and isinstance(sd["state_dict"], dict):
            sd = sd["state_dict"]
        timings = {"load_ms": (time.perf_counter() - t0) * 1e3}
        eng = cls.from_state_dict(model, sd, device, timings=timings, **kw)
        if write_packed:
            try:
                save_packed(eng.params, eng.pack_cfg, packed_path(path), model=model, stamp=source_stamp(path))
            except OSError as e:  # read-only artifact dir: the cache is an optimisation only
                import logging
                logging.getLogger("hipzap.engine").warning("could not write packed weights: %s", e)
        return eng

    # -------------------------------------------------------------- warm path
    def _pick(self) -> int:
        with self._rr_lock:
            i = self._rr
            self._rr = (self._rr + 1) % len(self.contexts)
        return i

    # -------------------------------------------------------------- request executor
    def executor(self):
        """The native request executor over all contexts (csrc/executor.cpp), built once every
        context exists (host-I/O, captured engines only); None otherwise."""
        ex = self._exec
        if ex is not None or not (self.host_io and self._capture and len(self.contexts) == self.num_contexts):
            return ex
        from ..executor import Executor
        with self._build_lock:
            if getattr(self, "_bexec", None) is not None:
                raise RuntimeError("this engine serves through the dynamic-batching executor")
            if self._exec is None:
                for lk in self._locks:  # no request may be in flight on the legacy path meanwhile
                    lk.acquire()
                try:
                    cs = self.contexts
                    self._exec = Executor(
                        [c.prog for c in cs], [s.cuda_stream for s in self.streams],
                        [[c.host_inputs[k].data_ptr() for c in cs] for k in range(len(cs[0].host_inputs))],
                        [h.numel() * h.element_size() for h in cs[0].host_inputs],
                        [c.host_output.data_ptr() for c in cs],
                        cs[0].host_output.numel() * cs[0].host_output.element_size())
                finally:
                    for lk in self._locks:
                        lk.release()
        return self._exec

    def infer(self, x) -> torch.Tensor:
        """Run one request; ``x`` is the graph input tensor, or a list of tensors for
        multi-input graphs (BERT: ids, token types, additive mask). Returns host output.
        Thread-safe: concurrent callers are served by the native executor (one submission
        thread, callers sleep until their own replay completes)."""
        xs = list(x) if isinstance(x, (list, tuple)) else [x]
        ex = self.executor()
        if ex is not None:
            c0 = self.contexts[0]
            # fast path (the common one-tensor request already in the payload's dtype and layout):
            # no per-request tensor views (~2 us each of the single-request latency)
            hbs = c0.host_inputs
            if all(xi.dtype == hb.dtype and xi.is_contiguous() and xi.numel() == hb.numel() and xi.device.type == "cpu"
                   for hb, xi in zip(hbs, xs)):
                ins = xs
            else:
                ins = [xi.to(hb.dtype).reshape(hb.shape).contiguous() for hb, xi in zip(hbs, xs)]
            out = torch.empty_like(c0.host_output)
            ex.submit([t.data_ptr() for t in ins], out.data_ptr())
            if _native.DEBUG:
                from ..utils import kcheck
                kcheck.check(f"{self.model} infer")
            return self._post(out)
        i = self._pick()
        ctx, s = self.contexts[i], self.streams[i]
        with self._locks[i], torch.cuda.device(self.device), torch.cuda.stream(s):
            if self.host_io:  # transfers are inside the captured graph
                for hb, xi in zip(ctx.host_inputs, xs):
                    hb.copy_(xi.reshape(hb.shape))
                ctx.replay(s)
                s.synchronize()
                out = ctx.host_output.clone()
            else:
                for d, xi in zip(ctx.inputs, xs):
                    d.copy_(xi.reshape(d.shape), non_blocking=True)
                ctx.replay(s)
                out = ctx.output.to("cpu", non_blocking=False)
        if _native.DEBUG:  # debug kernel variant: surface any failed device-side contract check
            from ..utils import kcheck
            kcheck.check(f"{self.model} infer")
        return self._post(out)

    def _post(self, out):
        takes_meta = getattr(self, "_post_meta", None)
        if takes_meta is None:  # decided once (a TypeError per request cost ~1 us)
            import inspect
            try:
                takes_meta = len(inspect.signature(self.adapter.postprocess_output).parameters) >= 2
            except (TypeError, ValueError):
                takes_meta = True
            self._post_meta = takes_meta
        if takes_meta:
            return self.adapter.postprocess_output(out, getattr(self.graph, "meta", None))
        return self.adapter.postprocess_output(out)

    def infer_device(self, x: torch.Tensor, ctx_index: int = 0) -> torch.Tensor:
        """Device-resident variant (no host copies); output aliases the static buffer.

        Stream-ordered with the CALLER's current stream (where ``x`` was produced, e.g. by a DP
        scatter, and where the returned output will be read): the context stream waits for the
        caller before reading ``x``, and the caller waits for the replay before it can touch
        the output. ``x`` is recorded on the context stream so the caching allocator cannot
        reuse its memory while the copy is still in flight."""
        ctx, s = self.contexts[ctx_index], self.streams[ctx_index]
        with torch.cuda.device(self.device):
            caller = torch.cuda.current_stream(self.device)
            s.wait_stream(caller)
            with torch.cuda.stream(s):
                if x is not None:
                    ctx.input.copy_(x.reshape(ctx.input.shape), non_blocking=True)
                ctx.replay(s)
            caller.wait_stream(s)
        if x is not None and x.is_cuda:
            x.record_stream(s)
        return ctx.output

    def pipeline_slots(self) -> list:
        """One ``parallel.dp.DPPipeline`` slot per captured context (its static input / output and
        its own stream): DP steps in flight on this rank, one per context."""
        self.ensure_contexts()
        return [_EngineSlot(self, i) for i in range(len(self.contexts))]

    def bench(self, iters: int) -> float:
        """Replay all contexts concurrently ``iters`` times (C++ loop); returns seconds."""
        self.ensure_contexts()
        return bench_contexts(self.contexts, self.streams, iters)

    def batched_executor(self, max_wait_us: float = 200.0, min_inflight: int = 1):
        """Dynamic-batching request executor over this engine's contexts (captured at
        ``self.batch``): each request is ONE image; concurrent requests share a replay."""
        from ..executor import Executor
        self.ensure_contexts()
        with self._build_lock:
            if self._exec is not None:  # both would drive the same pinned buffers and streams
                raise RuntimeError("this engine already serves through the per-request executor")
            if getattr(self, "_bexec", None) is None:
                cs = self.contexts
                self._bexec = Executor(
                    [c.prog for c in cs], [s.cuda_stream for s in self.streams],
                    [[c.host_inputs[k].data_ptr() for c in cs] for k in range(len(cs[0].host_inputs))],
                    [h.numel() * h.element_size() for h in cs[0].host_inputs],
                    [c.host_output.data_ptr() for c in cs],
                    cs[0].host_output.numel() * cs[0].host_output.element_size(),
                    rows=self.batch, max_wait_us=max_wait_us, min_inflight=min_inflight)
        return self._bexec

    def serve_bench(self, iters: int, payload=None, clients: int | None = None,
                    mode: str = "executor") -> tuple[float, list]:
        """Closed-loop serving benchmark: ``clients`` (default: one per context) native client
        threads each send ``iters`` requests back to back, every request = payload copied into
        a pinned input, one replay, wait, logits copied out. ``mode="executor"``: through the
        request executor (the serving path); ``"threads"``: every client drives its own context
        (launch + hipStreamSynchronize per thread; kept for comparison). Returns (seconds,
        per-request latencies in ms)."""
        self.ensure_contexts()
        c0 = self.contexts[0]
        p = payload if payload is not None else c0.host_input
        p = p.to(c0.host_input.dtype).reshape(c0.host_input.shape).contiguous()
        if mode == "threads":
            return serve_bench_contexts(self.contexts, self.streams, iters, [p.clone() for _ in self.contexts])
        ex = self.executor()
        return ex.bench(clients or len(self.contexts), iters, [p.data_ptr()])

    def describe(self) -> dict:
        c = self.contexts[0]
        return {"model": self.model, "batch": self.batch, "contexts": len(self.contexts),
                "ops": c.num_ops(), "arena_MB": round(c.arena_bytes / 2**20, 2),
                "captured": c.captured, "timings_ms": {k: round(v, 2) for k, v in self.timings.items()}}


DEDICATED_QUEUE_MAX_CONTEXTS = 4


def stream_kind(num_contexts: int, kind: str | None = None) -> str:
    """Which stream a request context gets (``kind``, else ``HIPZAP_STREAM_KIND``, default ``auto``;
    measurements in profiles/r6_queues):

    * ``torch``: torch's stream pool. Its streams share the process's 4 normal-priority hardware
      queues (``GPU_MAX_HW_QUEUES``), and which queue a stream lands on depends on what else the
      process created before it: the same 4-context BERT engine replays at 23.3k or 29.9k seq/s
      from one process to the next, the batch-4 ResNet shard at 19.6k or 25.5k img/s.
    * ``hiprio``: fresh non-blocking streams at the highest priority for every engine. HIP keeps a
      separate set of queues per priority and nothing else here asks for high priority, so an
      engine's 2-4 contexts land on distinct queues every time (BERT 4 contexts 28.1-28.6k seq/s
      in any process history). Never destroyed (a destroyed stream may still be recorded on a
      tensor the caching allocator frees later); an engine is built once per serving process.
    * ``hiprio_torch``: torch's high-priority pool; ``native``: fresh normal-priority streams;
      ``cumask``: a per-process pool of full-CU-mask streams (a queue each, but BLOCKING: a NULL-
      stream command waits for their work). Measured, not defaults.
    * ``auto``: ``hiprio`` for engines of 2-4 contexts (host-I/O engines only: ``Engine`` keeps a
      device-I/O engine on ``torch``, whose callers' stream waits into a high-priority stream are
      slow), ``torch`` otherwise -- 16 ResNet-50 bs=1
      contexts need the shared queues (16 queues of their own: 14.3k -> 7.4k inf/s; alternating
      them over the normal- and high-priority sets, 8 queues: 6.7k), and a
      DPPipeline over big batches does better on them too (``bench.py`` passes ``torch``)."""
    kind = kind or os.environ.get("HIPZAP_STREAM_KIND", "auto")
    if kind == "auto":
        return "hiprio" if 2 <= num_contexts <= DEDICATED_QUEUE_MAX_CONTEXTS else "torch"
    if kind not in ("torch", "hiprio", "hiprio_torch", "native", "cumask"):
        raise ValueError(f"HIPZAP_STREAM_KIND={kind!r}: auto, torch, hiprio, hiprio_torch, native or cumask")
    return kind


_DEDICATED: dict = {}  # device index -> the process's dedicated-queue streams (never destroyed)


def _context_stream(device, num_contexts: int = 1, index: int = 0, kind: str | None = None):
    """Context ``index``'s stream, of the kind ``stream_kind(num_contexts)`` picks. The CU-masked
    streams are a per-process pool of at most ``DEDICATED_QUEUE_MAX_CONTEXTS`` per device, shared by
    every engine that takes them (context i gets stream i) and alive until the process ends: a
    hardware queue per engine rebuild would pile up queues, and a destroyed stream may still be
    recorded on a tensor the caching allocator frees later (``Tensor.record_stream``)."""
    kind = stream_kind(num_contexts, kind)
    if kind == "torch":
        return torch.cuda.Stream(device=device)
    if kind == "hiprio_torch":  # torch's high-priority pool (its 32 streams share the 4 high-priority queues)
        return torch.cuda.Stream(device=device, priority=-1)
    if kind in ("native", "hiprio"):  # fresh streams for every engine (never destroyed: see above)
        return torch.cuda.ExternalStream(_new_hip_stream(device, kind), device=device)
    dev = torch.device(device)
    dev_i = dev.index if dev.index is not None else torch.cuda.current_device()
    pool = _DEDICATED.setdefault((dev_i, kind), [])
    while len(pool) <= index % DEDICATED_QUEUE_MAX_CONTEXTS:
        pool.append(torch.cuda.ExternalStream(_new_hip_stream(dev, kind), device=dev))
    return pool[index % DEDICATED_QUEUE_MAX_CONTEXTS]


def _new_hip_stream(device, kind: str) -> int:
    """A new HIP stream: ``cumask`` -- created with a full CU mask, which HIP backs with a hardware
    queue of its own (a blocking stream: the API takes no flags); ``hiprio`` -- non-blocking at the
    highest priority (HIP keeps a separate set of up to 4 queues per priority, and nothing else in
    this process asks for high priority, so the pool's first four get four queues of their own);
    ``native`` -- plain non-blocking."""
    import ctypes as C
    from .. import hip as H
    h = H.hip()
    p = C.c_void_p()
    with torch.cuda.device(device):
        if kind == "hiprio":
            lo, hi = C.c_int(0), C.c_int(0)
            g = h.hipDeviceGetStreamPriorityRange
            g.restype, g.argtypes = C.c_int, [C.POINTER(C.c_int), C.POINTER(C.c_int)]
            H.check(g(C.byref(lo), C.byref(hi)), "hipDeviceGetStreamPriorityRange")
            f = h.hipStreamCreateWithPriority
            f.restype, f.argtypes = C.c_int, [C.POINTER(C.c_void_p), C.c_uint, C.c_int]
            H.check(f(C.byref(p), 1, hi.value), "hipStreamCreateWithPriority")
        elif kind == "cumask":
            f = h.hipExtStreamCreateWithCUMask
            f.restype, f.argtypes = C.c_int, [C.POINTER(C.c_void_p), C.c_uint32, C.POINTER(C.c_uint32)]
            ncu = torch.cuda.get_device_properties(device).multi_processor_count
            words = (ncu + 31) // 32
            mask = (C.c_uint32 * words)(*([0xFFFFFFFF] * words))
            H.check(f(C.byref(p), words, mask), "hipExtStreamCreateWithCUMask")
        else:
            H.check(h.hipStreamCreateWithFlags(C.byref(p), 1), "hipStreamCreateWithFlags")
    return p.value


class _EngineSlot:
    """``DPPipeline`` slot over one captured context: ``launch`` orders the context's stream after
    the caller's current stream and replays; ``join`` orders the caller after the replay."""

    def __init__(self, eng: Engine, i: int):
        self.eng, self.i = eng, i
        self.input = eng.contexts[i].input
        self.output = eng.contexts[i].output

    def launch(self) -> None:
        ctx, s = self.eng.contexts[self.i], self.eng.streams[self.i]
        with torch.cuda.device(self.eng.device):
            s.wait_stream(torch.cuda.current_stream(self.eng.device))
            with torch.cuda.stream(s):
                ctx.replay(s)

    def join(self) -> torch.Tensor:
        with torch.cuda.device(self.eng.device):
            torch.cuda.current_stream(self.eng.device).wait_stream(self.eng.streams[self.i])
        return self.output
