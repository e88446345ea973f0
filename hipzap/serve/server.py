"""Model server: lazily cold-loads models once per process and keeps them warm.

The reference rebuilt and reloaded the AWD-LSTM on EVERY request (main.py:84-103, measured
8.9 s per GET /inference in SURVEY.md §6). Here a model is loaded on first use (the "cold
start" of a Lambda container) and every later request reuses the packed weights and the
captured hipGraphs (the warm path). Backends:
  * ``gpu``: the native hipzap Engine (HIP kernels, hipGraph replay) — default whenever a GPU
    is visible; the native library is REQUIRED there (no silent eager fallback);
  * ``cpu``: eager PyTorch on the host — the BASELINE config-1 "CPU plumbing" path and the
    development path in GPU-less containers.
"""
from __future__ import annotations

import logging
import os
import threading
import time

import torch

from ..models import registry
from .artifacts import ArtifactStore
from .settings import ModelSpec, Settings
from ..utils.tracing import trace_range
from ..utils.watchdog import maybe_fault
from .text import generate_text, load_itos, make_stoi

log = logging.getLogger("hipzap.server")


def _random_state_dict(name: str, seed: int = 0) -> dict:
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
    if not isinstance(src, str):
        return src
    sd = torch.load(src, map_location="cpu", weights_only=True)
    if isinstance(sd, dict) and isinstance(sd.get("state_dict"), dict):
        sd = sd["state_dict"]
    return sd


class VisionBackend:
    def __init__(self, name: str, sd, backend: str, device: str, spec: ModelSpec, capture: bool):
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

    def _run_padded(self, chunk: torch.Tensor) -> torch.Tensor:
        n = chunk.shape[0]
        if n < self.batch:  # pad the remainder to the captured batch size
            chunk = torch.cat([chunk, chunk.new_zeros((self.batch - n,) + tuple(chunk.shape[1:]))])
        return self.engine.infer(chunk)[:n]

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
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

    def __call__(self, ids: torch.Tensor, types=None, mask=None) -> torch.Tensor:
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
        t0 = time.perf_counter()
        self.itos, self.stoi = itos, make_stoi(itos)
        self.backend = backend
        if backend == "gpu":
            from ..engine.lm import LMPool
            self.engine = LMPool.for_vocab(sd, self.stoi, device, contexts=int(os.environ.get("HIPZAP_LM_CONTEXTS", 4)))
            self.model = None
        else:
            self.model = reference_lm(len(itos))
            self.model.load_state_dict(sd)
            self.model.eval()
            self.engine = None
        self.cold_ms = (time.perf_counter() - t0) * 1e3
        self._lock = threading.Lock()

    def generate(self, prompt_words, n_words, seed=None) -> str:
        gen = torch.Generator().manual_seed(seed) if seed is not None else None
        if self.engine is not None:  # pool of independent decode contexts: reentrant
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
            backend = os.environ.get("HIPZAP_BACKEND") or ("gpu" if torch.cuda.is_available() else "cpu")
        self.backend = backend
        self.device = f"cuda:{settings.devices[0]}" if backend == "gpu" else "cpu"
        self._models: dict = {}
        self._lock = threading.Lock()
        self._watchdog = None
        self.stats = {"requests": 0, "errors": 0, "cold_loads": 0}

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
        return self._load(name, VisionBackend)

    def text(self, name: str):
        return self._load(name, TextBackend)

    def lm(self) -> LMBackend:
        key = "__lm__"
        with self._lock:
            if key not in self._models:
                st = self.settings
                if os.environ.get("HIPZAP_RANDOM_WEIGHTS") or st.models_bucket is None:
                    from ..models.awd_lstm import reference_lm
                    itos = synthetic_vocab(int(os.environ.get("HIPZAP_LM_VOCAB", 2000)))
                    torch.manual_seed(0)
                    sd = reference_lm(len(itos)).state_dict()
                else:
                    itos = load_itos(self.store.fetch(st.lm_vocab_key))
                    sd = torch.load(self.store.fetch(st.lm_model_key), map_location="cpu", weights_only=True)
                self._models[key] = LMBackend(sd, itos, self.backend, self.device)
                self.stats["cold_loads"] += 1
            return self._models[key]

    def loaded(self) -> dict:
        return {k: {"backend": getattr(v, "backend", "?"), "cold_ms": round(getattr(v, "cold_ms", 0), 1)}
                for k, v in self._models.items()}


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
