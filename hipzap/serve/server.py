"""Model server: lazily cold-loads models once per process and keeps them warm.

The reference rebuilt and reloaded the AWD-LSTM on EVERY request (main.py:84-103, measured
8.9 s per GET /inference in SURVEY.md §6). Here a model is loaded on first use (the "cold
start" of a Lambda container) and every later request reuses the packed weights and the
captured hipGraphs (the warm path). Backends:
  * ``gpu``: the native hipzap Engine (HIP kernels, hipGraph replay) — default whenever a GPU
    is visible; the native library is REQUIRED there (no silent eager fallback);
  * ``cpu``: eager PyTorch on the host — the BASELINE config-1 "CPU plumbing" path and the
    development path in GPU-less containers.
Vision models whose checkpoint has an up-to-date plan image next to it (``<ckpt>.hzplan``,
``hipzap plan``) are served by :class:`PlanVisionBackend`: torch-free (hipzap/lite.py), uint8
images straight into the captured graph. torch is imported lazily, only by the paths that
need it, so a plan-backed server process never pays for it.
"""
from __future__ import annotations

import logging
import os
import threading
import time

from .artifacts import ArtifactStore
from .settings import ModelSpec, Settings
from ..utils.tracing import trace_range
from ..utils.watchdog import maybe_fault

log = logging.getLogger("hipzap.server")


def _random_state_dict(name: str, seed: int = 0) -> dict:
    import torch
    from ..models import registry
    from ..models.resnet import randomize_bn
    torch.manual_seed(seed)
    m = registry.get(name).make_model()
    if hasattr(m, "layer1"):
        randomize_bn(m, seed)
    return m.eval().state_dict()


def _gpu_engine(name: str, src, device: str, **kw):
    """``src``: a state_dict, or the local path of a .pth checkpoint (then an up-to-date packed
    copy next to it is used, and written after the first pack: the cold-start fast path)."""
    from ..engine.engine import Engine
    if isinstance(src, str):
        return Engine.from_checkpoint(name, src, device, use_packed=True,
                                      write_packed=os.environ.get("HIPZAP_WRITE_PACKED", "1") != "0", **kw)
    return Engine.from_state_dict(name, src, device, **kw)


def _state_dict(src) -> dict:
    import torch
    if not isinstance(src, str):
        return src
    sd = torch.load(src, map_location="cpu", weights_only=True)
    if isinstance(sd, dict) and isinstance(sd.get("state_dict"), dict):
        sd = sd["state_dict"]
    return sd


class VisionBackend:
    def __init__(self, name: str, sd, backend: str, device: str, spec: ModelSpec, capture: bool):
        from ..models import registry
        self.name, self.backend = name, backend
        t0 = time.perf_counter()
        self.adapter = registry.get(name)
        # "probs": true in the model's settings block -> the softmax runs on device, responses are probabilities
        self.probs = bool(spec.extra.get("probs", False))
        if backend == "gpu":
            self.engine = _gpu_engine(name, sd, device, batch=spec.batch, num_contexts=spec.contexts,
                                      capture=capture, probs=self.probs)
            self.model = None
        else:
            from ..models.resnet import infer_arch
            sd = _state_dict(sd)
            _, ncls = infer_arch(sd)
            self.model = self.adapter.make_model(ncls)
            self.model.load_state_dict(sd)
            self.model.eval()
            self.engine = None
        self.batch = spec.batch
        # "batching": {"max_wait_ms": 2} in the model's settings block -> concurrent small requests
        # are coalesced into one captured-batch replay (serve/batcher.py)
        bcfg = spec.extra.get("batching")
        self.batcher = None
        if bcfg and self.engine is not None and self.batch > 1:
            from .batcher import DynamicBatcher
            self.batcher = DynamicBatcher(self._run_padded, self.batch, float(bcfg.get("max_wait_ms", 2.0)), name)
        self.cold_ms = (time.perf_counter() - t0) * 1e3

    def _run_padded(self, chunk):
        import torch
        n = chunk.shape[0]
        if n < self.batch:  # pad the remainder to the captured batch size
            chunk = torch.cat([chunk, chunk.new_zeros((self.batch - n,) + tuple(chunk.shape[1:]))])
        return self.engine.infer(chunk)[:n]

    def __call__(self, x):
        import torch
        if self.engine is not None:
            if self.batcher is not None and x.shape[0] < self.batch:
                return self.batcher(x)
            return torch.cat([self._run_padded(x[i: i + self.batch]) for i in range(0, x.shape[0], self.batch)])
        with torch.no_grad():
            y = self.model(x.float())
            return torch.softmax(y, 1) if self.probs else y


class TextBackend:
    """BERT-style sequence classifier; requests are padded to the captured (batch, seq_len)."""

    def __init__(self, name: str, sd, backend: str, device: str, spec: ModelSpec, capture: bool):
        from ..models import registry
        self.name, self.backend = name, backend
        t0 = time.perf_counter()
        self.adapter = registry.get(name)
        self.seq_len = int(spec.extra.get("seq_len", 128))
        if backend == "gpu":
            self.engine = _gpu_engine(name, sd, device, batch=spec.batch, num_contexts=spec.contexts, capture=capture)
            self.model = None
        else:
            from ..models.bert import config_from_sd, make_model
            sd = _state_dict(sd)
            cfg = config_from_sd(sd)
            self.model = make_model(cfg["num_labels"], num_hidden_layers=cfg["layers"], hidden_size=cfg["hidden"],
                                    num_attention_heads=cfg["heads"], intermediate_size=cfg["ffn"],
                                    vocab_size=sd["bert.embeddings.word_embeddings.weight"].shape[0],
                                    max_position_embeddings=cfg["max_pos"])
            self.model.load_state_dict(sd)
            self.engine = None
        self.batch = spec.batch
        self.cold_ms = (time.perf_counter() - t0) * 1e3

    def __call__(self, ids, types=None, mask=None):
        import torch
        B, L = ids.shape
        types = types if types is not None else torch.zeros_like(ids)
        mask = mask if mask is not None else torch.ones_like(ids)
        if self.engine is None:
            with torch.no_grad():
                return self.model(input_ids=ids, token_type_ids=types, attention_mask=mask).logits
        from ..models.bert import encode_inputs
        Lc = self.engine.arch_kw.get("seq_len", self.seq_len)
        if L > Lc:
            raise ValueError(f"sequence length {L} exceeds the captured {Lc}")
        pad = Lc - L
        ids, types, mask = (torch.nn.functional.pad(t, (0, pad)) for t in (ids, types, mask))
        outs = []
        for i in range(0, B, self.batch):
            sl = slice(i, i + self.batch)
            ci, ct, cm = ids[sl], types[sl], mask[sl]
            n = ci.shape[0]
            if n < self.batch:
                z = self.batch - n
                ci, ct, cm = (torch.cat([t, t.new_zeros(z, Lc)]) for t in (ci, ct, cm))
            outs.append(self.engine.infer(encode_inputs(ci, ct, cm))[:n])
        return torch.cat(outs)


class RoundRobin:
    """One backend per GPU of the node; requests are dealt round-robin (DP replica serving)."""

    def __init__(self, backends: list, devices: list | None = None, healthy=None):
        self.backends = backends
        self.devices = devices or [None] * len(backends)
        self.healthy = healthy  # callable(device) -> bool (DeviceWatchdog), or None
        self.backend = backends[0].backend
        self.cold_ms = sum(b.cold_ms for b in backends)
        self._i = 0
        self._lock = threading.Lock()

    def __call__(self, *a, **kw):
        with self._lock:
            for _ in range(len(self.backends)):
                i = self._i
                self._i = (self._i + 1) % len(self.backends)
                if self.healthy is None or self.healthy(self.devices[i]):
                    break
            else:
                raise RuntimeError("no healthy device replica")
        return self.backends[i](*a, **kw)


class LMBackend:
    """AWD-LSTM text generation (GET /inference)."""

    def __init__(self, sd: dict, itos: list, backend: str, device: str):
        from ..models.awd_lstm import reference_lm
        from .text import make_stoi
        t0 = time.perf_counter()
        self.itos, self.stoi = itos, make_stoi(itos)
        self.backend = backend
        if backend == "gpu":
            # default: continuous batching -- concurrent requests share every decode step
            # (engine/lmbatch.py); HIPZAP_LM_ENGINE=pool: independent per-request contexts
            kind = os.environ.get("HIPZAP_LM_ENGINE", "batch")
            if kind == "batch":
                from ..engine.lmbatch import LMBatchEngine
                self.engine = LMBatchEngine.for_vocab(sd, self.stoi, device,
                                                      rows=int(os.environ.get("HIPZAP_LM_ROWS", 32)),
                                                      unroll=int(os.environ.get("HIPZAP_LM_UNROLL", 8)))
            else:
                from ..engine.lm import LMPool
                self.engine = LMPool.for_vocab(sd, self.stoi, device,
                                               contexts=int(os.environ.get("HIPZAP_LM_CONTEXTS", 4)))
            self.engine_kind = kind
            self.model = None
        else:
            self.model = reference_lm(len(itos))
            self.model.load_state_dict(sd)
            self.model.eval()
            self.engine = None
            self.engine_kind = "eager-cpu"
        self.cold_ms = (time.perf_counter() - t0) * 1e3
        self._lock = threading.Lock()

    def generate(self, prompt_words, n_words, seed=None) -> str:
        import torch
        from .text import generate_text
        gen = torch.Generator().manual_seed(seed) if seed is not None else None
        if self.engine is not None:  # batched decode / pool of contexts: reentrant
            return self.engine.generate(prompt_words, n_words, self.itos, self.stoi, seed=seed)
        with self._lock:  # the eager CPU model's recurrent state makes it non-reentrant
            with torch.no_grad():
                def step(tok):
                    res, *_ = self.model(torch.tensor([[tok]]))
                    return res[-1]
                return generate_text(step, self.model.reset, self.itos, self.stoi, prompt_words, n_words, gen)


class ModelServer:
    def __init__(self, settings: Settings, backend: str | None = None):
        self.settings = settings
        self.store = ArtifactStore(settings.models_bucket, settings.artifact_root)
        if backend is None:
            backend = os.environ.get("HIPZAP_BACKEND") or ("gpu" if gpu_visible() else "cpu")
        self.backend = backend
        self.device = f"cuda:{settings.devices[0]}" if backend == "gpu" else "cpu"
        self._models: dict = {}
        self._lock = threading.Lock()
        self._watchdog = None
        self.comm = None  # set by a DP cluster worker (serve/cluster.py): plan weights arrive by RCCL broadcast
        self.stats = {"requests": 0, "errors": 0, "cold_loads": 0}
        self.lm_listeners: list = []  # called with the GET /inference backend once it is loaded

    def spec(self, name: str) -> ModelSpec:
        return self.settings.models.get(name) or ModelSpec(name=name)

    def _load_sd(self, spec: ModelSpec):
        """A state_dict (random-init demo weights) or the local path of the fetched checkpoint
        (backends torch.load it, or use its packed copy on the GPU)."""
        if spec.key in (None, "random") or os.environ.get("HIPZAP_RANDOM_WEIGHTS"):
            log.warning("model %s: no checkpoint key configured, using random-init weights", spec.name)
            return _random_state_dict(spec.name)
        return self.store.fetch(spec.key)

    def watchdog(self):
        """Per-GPU liveness watchdog (started on first GPU model load; HIPZAP_WATCHDOG=0 disables)."""
        if self.backend != "gpu" or os.environ.get("HIPZAP_WATCHDOG", "1") == "0":
            return None
        if self._watchdog is None:
            from ..utils.watchdog import DeviceWatchdog
            self._watchdog = DeviceWatchdog(self._devices(), interval_s=float(os.environ.get("HIPZAP_WATCHDOG_S", 5)))
            self._watchdog.start()
        return self._watchdog

    def _devices(self) -> list[str]:
        if self.backend != "gpu":
            return ["cpu"]
        return [f"cuda:{d}" for d in self.settings.devices]

    def _load(self, name: str, cls):
        with self._lock:
            if name not in self._models:
                spec = self.spec(name)
                sd = self._load_sd(spec)
                maybe_fault("load")
                devs = self._devices()
                with trace_range(f"cold_start:{name}"):
                    bes = [cls(spec.name, sd, self.backend, dev, spec, self.settings.capture_graphs) for dev in devs]
                wd = self.watchdog()
                healthy = (lambda d: wd.healthy.get(d, True)) if wd is not None else None
                self._models[name] = bes[0] if len(bes) == 1 else RoundRobin(bes, devs, healthy)
                self.stats["cold_loads"] += 1
            return self._models[name]

    def vision(self, name: str):
        plan = self._plan_for(name)
        if plan is not None:
            with self._lock:
                if name not in self._models:
                    spec = self.spec(name)
                    with trace_range(f"cold_start:{name}"):
                        self._models[name] = PlanVisionBackend(name, plan, self.settings.devices[0], spec,
                                                               comm=self.comm)
                    self.stats["cold_loads"] += 1
                return self._models[name]
        return self._load(name, VisionBackend)

    def _plan_for(self, name: str) -> str | None:
        """The up-to-date plan image of this model's checkpoint, if the GPU backend can use it
        (``extra.plan`` names one explicitly; else ``<ckpt>.hzplan`` next to the fetched
        checkpoint -- fetched from the artifact store too when it was published there,
        ``hipzap plan`` + ``hipzap upload`` -- validated by content; HIPZAP_PLAN=0 disables)."""
        if self.backend != "gpu" or os.environ.get("HIPZAP_PLAN", "1") == "0":
            return None
        spec = self.spec(name)
        if spec.extra.get("plan"):
            return spec.extra["plan"]
        if spec.key in (None, "random") or os.environ.get("HIPZAP_RANDOM_WEIGHTS"):
            return None
        from ..lite import plan_usable, read_meta
        from ..engine.packfile import same_source
        ckpt = self.store.fetch(spec.key)
        path = ckpt + ".hzplan"
        fetched = False
        if not os.path.exists(path):
            try:  # published next to the checkpoint in the store (its cache path is <ckpt>.hzplan)
                path = self.store.fetch(spec.key + ".hzplan")
                fetched = True
            except Exception:  # noqa: BLE001 - no plan in the store: the checkpoint path serves
                return None
        try:
            meta = read_meta(path)
            if plan_usable(path) and meta.get("model") == name and \
                    same_source(meta.get("source"), ckpt, content_only=fetched or self.store.bucket is not None):
                return path
        except OSError:
            pass
        return None

    def text(self, name: str):
        plan = self._plan_for(name)
        if plan is not None:
            from ..lite import read_meta
            if read_meta(plan).get("kind") == "text":
                with self._lock:
                    if name not in self._models:
                        with trace_range(f"cold_start:{name}"):
                            self._models[name] = PlanTextBackend(name, plan, self.settings.devices[0], self.spec(name))
                        self.stats["cold_loads"] += 1
                    return self._models[name]
        return self._load(name, TextBackend)

    def lm(self):
        """The GET /inference backend, loaded once. A GPU server whose checkpoint is a zip ``.pth``
        builds the batched engine WITHOUT torch (hipzap/lmlite.py: weights-only reader, raw upload,
        device packing); anything that path refuses (legacy files, non-fp32 records) and the random
        demo weights go through torch (LMBackend)."""
        from .text import load_itos
        key = "__lm__"
        with self._lock:
            if key not in self._models:
                st = self.settings
                be = None
                if os.environ.get("HIPZAP_RANDOM_WEIGHTS") or st.models_bucket is None:
                    import torch
                    from ..models.awd_lstm import reference_lm
                    itos = synthetic_vocab(int(os.environ.get("HIPZAP_LM_VOCAB", 2000)))
                    torch.manual_seed(0)
                    be = LMBackend(reference_lm(len(itos)).state_dict(), itos, self.backend, self.device)
                else:
                    ckpt, vocab = self.store.fetch(st.lm_model_key), self.store.fetch(st.lm_vocab_key)
                    if self.backend == "gpu" and os.environ.get("HIPZAP_LM_LITE", "1") != "0":
                        import zipfile
                        from ..lmlite import LMLiteBackend, LMLiteError
                        if zipfile.is_zipfile(ckpt):
                            try:
                                be = LMLiteBackend(ckpt, vocab, st.devices[0])
                            except LMLiteError as e:
                                log.warning("torch-free LM path refused %s (%s); loading it with torch", ckpt, e)
                    if be is None:
                        be = LMBackend(load_checkpoint(ckpt), load_itos(vocab), self.backend, self.device)
                self._models[key] = be
                self.stats["cold_loads"] += 1
                for cb in list(self.lm_listeners):  # e.g. the native HTTP front end's GET /inference route
                    try:
                        cb(be)
                    except Exception:  # noqa: BLE001 - the WSGI route keeps serving
                        log.exception("GET /inference listener failed")
            return self._models[key]

    def loaded(self) -> dict:
        return {k: {"backend": getattr(v, "backend", "?"), "cold_ms": round(getattr(v, "cold_ms", 0), 1)}
                for k, v in self._models.items()}


def load_checkpoint(path: str) -> dict:
    """A ``torch.save`` state_dict as torch tensors (main.py:99 ``torch.load(map_location='cpu')``):
    the weights-only zip reader (hipzap/pthreader.py: mmap, zero copy, shared storages stay
    shared), falling back to ``torch.load(weights_only=True)`` for legacy (pre-zip) files."""
    import torch
    from ..pthreader import NotAZipCheckpoint, load_state_dict
    try:
        raw = load_state_dict(path)
    except NotAZipCheckpoint:
        return torch.load(path, map_location="cpu", weights_only=True)
    import warnings
    out = {}
    with warnings.catch_warnings():  # read-only mmap views: the packers only read them
        warnings.simplefilter("ignore", UserWarning)
        for k, a in raw.items():
            if hasattr(a, "to_float32"):
                out[k] = torch.from_numpy(a.view("int16")).view(torch.bfloat16)
            else:
                out[k] = torch.from_numpy(a)
    return out


def gpu_visible() -> bool:
    """A GPU is visible to this process (HIP runtime query; torch is not imported)."""
    try:
        from ..hip import device_count
        return device_count() > 0
    except Exception:
        return False


class PlanVisionBackend:
    """Torch-free vision serving from a plan image (``hipzap plan``; hipzap/lite.py): a request
    is a uint8 HWC image (the decoded-JPEG format) copied into a pinned input and one hipGraph
    replay (device preprocess -> convs -> pool+FC [-> softmax]) through the native request
    executor. ``comm`` (DP cluster worker): rank 0 reads the weights and RCCL-broadcasts them,
    the other ranks never read the blob from disk. Other input formats (fp32 NCHW tensors) go
    to a torch-built :class:`VisionBackend`, constructed on first use."""
    backend = "gpu"

    def __init__(self, name: str, plan: str, device: int, spec: ModelSpec, comm=None):
        from ..lite import PlanEngine
        t0 = time.perf_counter()
        self.name, self.plan, self.spec, self.device = name, plan, spec, device
        fill = None
        if comm is not None and comm.world > 1:
            fill = lambda addr, n: comm.broadcast_ptr(addr, n, 0)  # noqa: E731
        # first request runs the bound program eagerly; the background scale-up below captures it
        self.engine = PlanEngine(plan, device=device, contexts=max(1, spec.contexts), eager_contexts=1,
                                 read_blob=comm is None or comm.rank == 0, fill_blob=fill, capture="lazy")
        self.meta = self.engine.meta
        self.in_shape = tuple(self.meta["inputs"][0]["shape"])  # [B, H, W, 3] uint8
        self.batch = self.in_shape[0]
        self.probs = bool(self.meta.get("probs"))
        self.num_labels = self.meta["output"].get("num_labels") or self.meta["output"]["shape"][-1]
        # batch-B plan behind the native /predict route: dynamic batching, "batching": {"max_wait_ms"}
        self.max_wait_us = float((spec.extra.get("batching") or {}).get("max_wait_ms", 0.2)) * 1e3
        self._torch, self._torch_lock = None, threading.Lock()
        self.cold_ms = (time.perf_counter() - t0) * 1e3
        # the other request contexts are built right after the engine is ready (warm scale-up)
        threading.Thread(target=self.engine.ensure_contexts, daemon=True, name=f"{name}-contexts").start()

    def accepts_u8(self, shape) -> bool:
        return len(shape) == 4 and tuple(shape[1:]) == self.in_shape[1:]

    def infer_u8(self, imgs):
        """``imgs``: uint8 numpy array [N, H, W, 3] -> numpy [N, classes] (logits or probs)."""
        import numpy as np
        n = imgs.shape[0]
        out = np.empty((n, self.num_labels), np.float32)
        B = self.batch
        for i in range(0, n, B):
            chunk = imgs[i: i + B]
            m = chunk.shape[0]
            if m < B:
                chunk = np.concatenate([chunk, np.zeros((B - m,) + chunk.shape[1:], np.uint8)])
            y = np.frombuffer(self.engine.infer_raw(np.ascontiguousarray(chunk), rows=m), np.float32)
            out[i: i + m] = y.reshape(B, -1)[:m, : self.num_labels]
        return out

    def __call__(self, x):
        """torch-tensor entry (fp32 NCHW etc.): served by a torch-built engine of the same
        checkpoint (the plan's source), built on first use."""
        with self._torch_lock:
            if self._torch is None:
                ckpt = self.plan[: -len(".hzplan")]
                if not os.path.exists(ckpt):
                    raise ValueError(f"{self.name} is served from a plan image: send uint8 HWC images "
                                     f"{list(self.in_shape[1:])} (image_b64 or a uint8 .npy)")
                self._torch = VisionBackend(self.name, ckpt, "gpu", f"cuda:{self.device}", self.spec, True)
        return self._torch(x)

class PlanTextBackend:
    """Torch-free BERT-style serving from a text plan image (``hipzap plan --model bert-base
    --batch B``; meta ``kind: text``): a request is up to B sequences of token ids (+ optional
    token types / attention mask), padded on the host to the captured (B, seq_len) -- padding
    tokens are masked out with the additive mask, exactly as :class:`TextBackend` pads -- and one
    hipGraph replay through the native per-request executor. Token ids outside the vocabulary
    are rejected here (the embedding kernel also clamps them)."""
    backend = "gpu"

    def __init__(self, name: str, plan: str, device: int, spec: ModelSpec):
        from ..lite import PlanEngine
        t0 = time.perf_counter()
        self.name, self.plan, self.spec, self.device = name, plan, spec, device
        self.engine = PlanEngine(plan, device=device, contexts=max(1, spec.contexts), eager_contexts=1,
                                 capture="lazy")
        m = self.engine.meta
        if m.get("kind") != "text":
            raise ValueError(f"{plan} is not a text plan")
        self.meta = m
        self.batch, self.seq_len = int(m["batch"]), int(m["seq_len"])
        self.vocab, self.type_vocab = int(m["vocab"]), int(m["type_vocab"])
        self.num_labels = m["output"].get("num_labels") or m["output"]["shape"][-1]
        self.cold_ms = (time.perf_counter() - t0) * 1e3
        threading.Thread(target=self.engine.ensure_contexts, daemon=True, name=f"{name}-contexts").start()

    def infer_np(self, ids, types=None, mask=None):
        """``ids`` (and optional ``types`` / ``mask``): int arrays [n, L] with L <= seq_len ->
        numpy float32 logits [n, num_labels]."""
        import numpy as np
        ids = np.asarray(ids)
        if ids.ndim == 1:
            ids = ids[None]
        n, L = ids.shape
        types = np.zeros_like(ids) if types is None else np.asarray(types).reshape(ids.shape)
        mask = np.ones_like(ids) if mask is None else np.asarray(mask).reshape(ids.shape)
        if L > self.seq_len:
            raise ValueError(f"sequence length {L} exceeds the captured {self.seq_len}")
        if ids.size and (ids.min() < 0 or ids.max() >= self.vocab):
            raise ValueError(f"token ids must lie in [0, {self.vocab})")
        if types.size and (types.min() < 0 or types.max() >= self.type_vocab):
            raise ValueError(f"token type ids must lie in [0, {self.type_vocab})")
        B, Lc = self.batch, self.seq_len
        out = np.empty((n, self.num_labels), np.float32)
        for i in range(0, n, B):
            m = min(B, n - i)
            ci = np.zeros((B, Lc), np.int32)
            ct = np.zeros((B, Lc), np.int32)
            cm = np.zeros((B, Lc), np.float32)  # padding tokens and rows: mask 0 -> additive -1e9
            ci[:m, :L] = ids[i: i + m]
            ct[:m, :L] = types[i: i + m]
            cm[:m, :L] = mask[i: i + m]
            madd = (np.float32(1.0) - cm) * np.float32(-1e9)
            y = np.frombuffer(self.engine.infer_raw([ci, ct, madd]), np.float32).reshape(B, -1)
            out[i: i + m] = y[:m, : self.num_labels]
        return out

    def __call__(self, ids, types=None, mask=None):
        """torch-tensor entry (TextBackend's interface): logits as a torch tensor."""
        import torch
        def arr(t):
            return None if t is None else t.cpu().numpy()
        return torch.from_numpy(self.infer_np(arr(ids), arr(types), arr(mask)))


def synthetic_vocab(n: int) -> list[str]:
    """fastai-style vocabulary for random-weight demos: specials first, then pseudo-words."""
    specials = ["xxunk", "xxpad", "xxbos", "xxfld", "xxmaj", "xxup", "xxrep", "xxwrep", ".", ",", "!", "?", "'s",
                "\n", "the", "a", "and", "to", "of", "i", "you", "it", "is", "that", "what", "why", "did"]
    words = list(specials)
    syll = ["ka", "lo", "mi", "ne", "ru", "ta", "bo", "shi", "en", "po", "di", "ga"]
    i = 0
    while len(words) < n:
        a, b = divmod(i, len(syll))
        words.append(syll[a % len(syll)] + syll[b] + ("" if i % 3 else "s"))
        i += 1
    return words[:n]
