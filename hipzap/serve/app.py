"""Flask WSGI application — the Zappa ``app_function`` (``main.app``).

Routes (reference: /root/reference/main.py:17-18, 105-112):
  GET  /inference   AWD-LSTM text generation -> {"response": {"text": str}}   (parity, P3)
                    optional query: prompt, words, seed
  POST /predict     image / tensor classification -> {"model", "top5", "timing_ms", ...}
                    (north-star API; ``model`` selects resnet50 (default), resnet18, ...)
  GET  /health      liveness + loaded models;  GET /metrics  Prometheus text;  GET /  info
CORS is applied to every route and origin (main.py:18 used flask_cors, which is not
installed here: implemented in-house — ``Access-Control-Allow-Origin: *`` plus preflight).
"""
from __future__ import annotations

import base64
import io
import json
import logging
import time

import numpy as np
import torch
from flask import Flask, Response, g, request

from .. import __version__
from ..utils.metrics import METRICS
from ..utils.tracing import PhaseTimer, trace_range
from .server import ModelServer
from .settings import load_settings

log = logging.getLogger("hipzap.app")

app = Flask("hipzap")
_server: ModelServer | None = None


def serve_threaded() -> bool:
    """Threaded WSGI serving for the GPU backend (engines take concurrent requests on their own
    contexts/streams). The CPU backend serves on the main thread: eager PyTorch CPU inference
    called from a WSGI worker thread ran 3.5x slower than from the main thread here (OpenMP /
    oneDNN thread handling; 72-77 ms vs 20 ms per ResNet-18 forward), and the eager AWD-LSTM is
    not reentrant anyway."""
    return get_server().backend != "cpu"


def get_server() -> ModelServer:
    global _server
    if _server is None:
        _server = ModelServer(load_settings())
    return _server


def set_server(server: ModelServer | None) -> None:
    global _server
    _server = server


def _json(obj, status=200) -> Response:
    return Response(response=json.dumps(obj), status=status, mimetype="application/json")


def phase(name: str):
    """Time a request phase: roctx range + the request's ``X-Timing`` header entry."""
    return trace_range(name, getattr(g, "hz_timer", None))


@app.after_request
def _cors(resp: Response) -> Response:
    resp.headers["Access-Control-Allow-Origin"] = "*"
    timer = getattr(g, "hz_timer", None)
    t0 = getattr(request, "_hz_t0", None)
    if timer is not None and t0 is not None:  # per-request phase timers (SURVEY.md §5 tracing)
        timer.add("total", (time.perf_counter() - t0) * 1e3)
        resp.headers["X-Timing"] = timer.header()
        resp.headers["Access-Control-Expose-Headers"] = "X-Timing"
    if request.method == "OPTIONS":
        resp.headers["Access-Control-Allow-Methods"] = "GET, POST, OPTIONS"
        req_h = request.headers.get("Access-Control-Request-Headers")
        resp.headers["Access-Control-Allow-Headers"] = req_h or "Content-Type"
        resp.headers["Access-Control-Max-Age"] = "600"
    return resp


@app.before_request
def _preflight():
    request._hz_t0 = time.perf_counter()
    g.hz_timer = PhaseTimer()
    if request.method == "OPTIONS":
        return Response(status=200)
    return None


@app.teardown_request
def _count(exc):
    t0 = getattr(request, "_hz_t0", None)
    if t0 is not None:
        METRICS.observe("hipzap_request_seconds", time.perf_counter() - t0, {"path": request.path})
    METRICS.inc("hipzap_requests_total", {"path": request.path})
    if exc is not None:
        METRICS.inc("hipzap_errors_total", {"path": request.path})


@app.errorhandler(Exception)
def _error(e):
    code = getattr(e, "code", 500)
    if not isinstance(code, int):
        code = 500
    if code >= 500:
        log.exception("request failed")
    METRICS.inc("hipzap_errors_total", {"path": request.path})
    return _json({"error": type(e).__name__, "message": str(e)}, status=code)


@app.route("/", methods=["GET"])
def index():
    s = get_server()
    return _json({"service": "hipzap", "version": __version__, "backend": s.backend,
                  "routes": ["GET /inference", "POST /predict", "GET /health", "GET /metrics"]})


@app.route("/inference", methods=["GET"])
def inference():
    """GET: perform inference on the language model (main.py:105-112)."""
    s = get_server()
    prompt = request.args.get("prompt")
    words = [""] if not prompt else prompt.split()
    n = int(request.args.get("words", s.settings.lm_words))
    seed = request.args.get("seed")
    with phase("load"):
        lm = s.lm()
    with phase("generate"):
        text = lm.generate(words, n, seed=int(seed) if seed is not None else None)
    return _json({"response": {"text": text}})


def decode_input(req) -> tuple[str, torch.Tensor]:
    """Accepted request bodies:
    * ``application/octet-stream``: a ``.npy`` array (``np.save``; no pickles);
    * JSON ``{"inputs": nested list, "model": ...}`` (float tensor, NCHW or CHW);
    * JSON ``{"image_b64": base64 uint8 HWC bytes, "shape": [H, W, 3]}`` — normalised with
      ImageNet mean/std on the way in;
    * JSON ``{"tensor_b64": base64 float32 bytes, "shape": [...]}``.
    """
    model = req.args.get("model")
    if req.mimetype == "application/octet-stream":
        arr = np.load(io.BytesIO(req.get_data()), allow_pickle=False)
        x = torch.from_numpy(np.ascontiguousarray(arr))
    else:
        body = req.get_json(force=True, silent=False)
        model = body.get("model", model)
        if "inputs" in body:
            x = torch.tensor(body["inputs"], dtype=torch.float32)
        elif "tensor_b64" in body:
            raw = base64.b64decode(body["tensor_b64"])
            x = torch.from_numpy(np.frombuffer(raw, dtype=np.float32).copy()).reshape(body["shape"])
        elif "image_b64" in body:
            raw = base64.b64decode(body["image_b64"])
            img = torch.from_numpy(np.frombuffer(raw, dtype=np.uint8).copy()).reshape(body["shape"])
            x = img
        else:
            raise ValueError("request needs one of: inputs, tensor_b64, image_b64 (or an .npy body)")
    if x.dtype == torch.uint8:  # HWC / NHWC image bytes -> normalised NCHW float
        # in numpy: torch's multi-threaded elementwise ops on this request thread would start an
        # OpenMP team per WSGI thread, spinning against the model's own thread pool
        from ..ops.vision import IMAGENET_MEAN, IMAGENET_STD
        a = x.numpy()
        if a.ndim == 3:
            a = a[None]
        a = (a.astype(np.float32) * np.float32(1 / 255.0) - np.asarray(IMAGENET_MEAN, np.float32)) \
            / np.asarray(IMAGENET_STD, np.float32)
        x = torch.from_numpy(np.ascontiguousarray(a.transpose(0, 3, 1, 2)))
    x = x.float().contiguous()  # NCHW-contiguous: a permuted view sends CPU convs down a slow path
    if x.dim() == 3:
        x = x[None]
    return model or get_server().settings.default_model, x


def _predict_text(s, body):
    """BERT-style sequence classification: {"model", "input_ids", "token_type_ids"?,
    "attention_mask"?} -> class probabilities."""
    model = body.get("model") or "bert-base"
    ids = torch.tensor(body["input_ids"], dtype=torch.long)
    if ids.dim() == 1:
        ids = ids[None]
    tt = body.get("token_type_ids")
    am = body.get("attention_mask")
    tt = torch.tensor(tt, dtype=torch.long).reshape(ids.shape) if tt is not None else None
    am = torch.tensor(am, dtype=torch.long).reshape(ids.shape) if am is not None else None
    with phase("load"):
        backend = s.text(model)
    t0 = time.perf_counter()
    with phase("infer"):
        logits = backend(ids, tt, am)
    dt = (time.perf_counter() - t0) * 1e3
    probs = torch.softmax(logits.float(), dim=-1)
    return _json({"model": model, "backend": backend.backend, "batch": int(ids.shape[0]),
                  "probs": [[round(float(p), 6) for p in row] for row in probs],
                  "label": [int(i) for i in probs.argmax(-1)], "timing_ms": round(dt, 3)})


@app.route("/predict", methods=["POST"])
def predict():
    s = get_server()
    if request.mimetype != "application/octet-stream":
        body = request.get_json(force=True, silent=True) or {}
        if "input_ids" in body:
            return _predict_text(s, body)
    with phase("decode"):
        model, x = decode_input(request)
    with phase("load"):
        backend = s.vision(model)
    t0 = time.perf_counter()
    with phase("infer"):
        logits = backend(x)
    dt = (time.perf_counter() - t0) * 1e3
    probs = torch.softmax(logits.float(), dim=-1)
    k = min(5, probs.shape[-1])
    top = torch.topk(probs, k, dim=-1)
    out = {"model": model, "backend": backend.backend, "batch": int(x.shape[0]),
           "top5": [[[int(i), round(float(p), 6)] for i, p in zip(ti, tp)] for ti, tp in zip(top.indices, top.values)],
           "timing_ms": round(dt, 3)}
    if request.args.get("logits"):
        out["logits"] = logits.float().tolist()
    return _json(out)


@app.route("/health", methods=["GET"])
def health():
    s = get_server()
    info = {"status": "ok", "backend": s.backend, "models": s.loaded()}
    if s.backend == "gpu":
        info["devices"] = [torch.cuda.get_device_name(d) for d in s.settings.devices]
    return _json(info)


@app.route("/metrics", methods=["GET"])
def metrics():
    return Response(METRICS.render(), mimetype="text/plain; version=0.0.4")
