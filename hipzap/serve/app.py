"""Flask WSGI application — the Zappa ``app_function`` (``main.app``).

Routes (reference: /root/reference/main.py:17-18, 105-112):
  GET  /inference   AWD-LSTM text generation -> {"response": {"text": str}}   (parity, P3)
                    optional query: prompt, words, seed
  POST /predict     image / tensor classification -> {"model", "top5", "timing_ms", ...}
                    (north-star API; ``model`` selects resnet50 (default), resnet18, ...)
  GET  /health      liveness + loaded models;  GET /metrics  Prometheus text;  GET /  info
torch is imported lazily: a plan-backed vision model (server.PlanVisionBackend) serves uint8
images end to end without it (decode -> pinned input -> hipGraph -> top-5 in numpy).
CORS is applied to every route and origin (main.py:18 used flask_cors, which is not
installed here: implemented in-house — ``Access-Control-Allow-Origin: *`` plus preflight).
"""
from __future__ import annotations

import base64
import io
import json
import logging
import sys
import time

import numpy as np
from flask import Flask, Response, g, request

from .. import __version__
from ..utils.metrics import METRICS
from ..utils.tracing import PhaseTimer, trace_range
from .server import ModelServer
from .settings import load_settings

log = logging.getLogger("hipzap.app")

app = Flask("hipzap")
_server: ModelServer | None = None
# DP cluster worker state (serve/cluster.py): batched uint8 requests for the DP model are
# scattered over every GPU of the node through the cluster's control plane
CLUSTER: dict = {}
_DP = {"member": None, "model": None, "item_shape": None}


def set_dp(member, model: str | None, item_shape) -> None:
    _DP.update(member=member, model=model, item_shape=tuple(item_shape) if item_shape else None)


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
    code = getattr(e, "code", 400 if isinstance(e, ValueError) else 500)  # bad input: client error
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


def decode_input(req):
    """-> (model, numpy array). Accepted request bodies:
    * ``application/octet-stream``: a ``.npy`` array (``np.save``; no pickles);
    * JSON ``{"inputs": nested list, "model": ...}`` (float tensor, NCHW or CHW);
    * JSON ``{"image_b64": base64 uint8 HWC bytes, "shape": [H, W, 3]}`` (or [N, H, W, 3]);
    * JSON ``{"tensor_b64": base64 float32 bytes, "shape": [...]}``.
    uint8 arrays are images (HWC / NHWC), served as is by plan-backed models (normalised on
    device) and normalised to NCHW float for the others (:func:`to_model_input`)."""
    model = req.args.get("model")
    if req.mimetype == "application/octet-stream":
        arr = np.load(io.BytesIO(req.get_data()), allow_pickle=False)
    else:
        body = req.get_json(force=True, silent=False)
        model = body.get("model", model)
        if "inputs" in body:
            arr = np.asarray(body["inputs"], dtype=np.float32)
        elif "tensor_b64" in body:
            arr = np.frombuffer(base64.b64decode(body["tensor_b64"]), dtype=np.float32).reshape(body["shape"])
        elif "image_b64" in body:
            arr = np.frombuffer(base64.b64decode(body["image_b64"]), dtype=np.uint8).reshape(body["shape"])
        else:
            raise ValueError("request needs one of: inputs, tensor_b64, image_b64 (or an .npy body)")
    if arr.dtype == np.uint8 and arr.ndim == 3:
        arr = arr[None]
    return model or get_server().settings.default_model, arr


def to_model_input(arr):
    """numpy request array -> float32 NCHW torch tensor for the torch-built backends."""
    import torch
    if arr.dtype == np.uint8:  # NHWC image bytes -> normalised NCHW float
        # in numpy: torch's multi-threaded elementwise ops on this request thread would start an
        # OpenMP team per WSGI thread, spinning against the model's own thread pool
        from ..ops.vision import IMAGENET_MEAN, IMAGENET_STD
        a = (arr.astype(np.float32) * np.float32(1 / 255.0) - np.asarray(IMAGENET_MEAN, np.float32)) \
            / np.asarray(IMAGENET_STD, np.float32)
        arr = a.transpose(0, 3, 1, 2)
    x = torch.from_numpy(np.require(arr, np.float32, ["C", "W"]))  # NCHW-contiguous (CPU convs), writable
    if x.dim() == 3:
        x = x[None]
    return x


def softmax_np(x):
    x = np.asarray(x, np.float32)
    e = np.exp(x - x.max(-1, keepdims=True))
    return e / e.sum(-1, keepdims=True)


def topk_np(p, k: int):
    """[(indices, values)] per row, highest first."""
    idx = np.argpartition(-p, k - 1, axis=-1)[:, :k]
    vals = np.take_along_axis(p, idx, -1)
    order = np.argsort(-vals, axis=-1)
    return np.take_along_axis(idx, order, -1), np.take_along_axis(vals, order, -1)


def _predict_text(s, body):
    """BERT-style sequence classification: {"model", "input_ids", "token_type_ids"?,
    "attention_mask"?} -> class probabilities."""
    model = body.get("model") or "bert-base"
    ids = np.asarray(body["input_ids"], dtype=np.int64)
    if ids.ndim == 1:
        ids = ids[None]
    tt = body.get("token_type_ids")
    am = body.get("attention_mask")
    tt = np.asarray(tt, dtype=np.int64).reshape(ids.shape) if tt is not None else None
    am = np.asarray(am, dtype=np.int64).reshape(ids.shape) if am is not None else None
    with phase("load"):
        backend = s.text(model)
    t0 = time.perf_counter()
    with phase("infer"):
        if hasattr(backend, "infer_np"):  # plan-backed: torch-free
            logits = backend.infer_np(ids, tt, am)
        else:
            import torch
            def tens(a):
                return None if a is None else torch.from_numpy(a)
            logits = backend(tens(ids), tens(tt), tens(am)).float().numpy()
    dt = (time.perf_counter() - t0) * 1e3
    probs = softmax_np(logits)
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
        model, arr = decode_input(request)
    with phase("load"):
        backend = s.vision(model)
    t0 = time.perf_counter()
    dp = _DP["member"]
    if (dp is not None and dp.alive and model == _DP["model"] and arr.dtype == np.uint8 and arr.shape[0] > 1
            and tuple(arr.shape[1:]) == _DP["item_shape"]):
        with phase("dp_scatter_gather"):  # C2 scatter -> every GPU's shard -> C3 gather
            out = dp.submit(arr)
        logits, probs = out, softmax_np(out)
    elif arr.dtype == np.uint8 and hasattr(backend, "infer_u8") and backend.accepts_u8(arr.shape):
        with phase("infer"):  # torch-free: pinned input -> captured graph (preprocess on device)
            out = backend.infer_u8(arr)
        logits = None if backend.probs else out
        probs = out if backend.probs else softmax_np(out)
    else:
        x = to_model_input(arr)
        with phase("infer"):
            lg = backend(x)
        logits = lg.float().numpy()
        probs = softmax_np(logits)
    dt = (time.perf_counter() - t0) * 1e3
    k = min(5, probs.shape[-1])
    ti, tp = topk_np(probs, k)
    out = {"model": model, "backend": backend.backend, "batch": int(arr.shape[0]),
           "top5": [[[int(i), round(float(p), 6)] for i, p in zip(r_i, r_p)] for r_i, r_p in zip(ti, tp)],
           "timing_ms": round(dt, 3)}
    if request.args.get("logits") and logits is not None:
        out["logits"] = logits.tolist()
    return _json(out)


@app.route("/health", methods=["GET"])
def health():
    s = get_server()
    info = {"status": "ok", "backend": s.backend, "models": s.loaded()}
    if CLUSTER:
        m, c = CLUSTER.get("member"), CLUSTER.get("coordinator")
        info["cluster"] = {"rank": CLUSTER["rank"], "world": CLUSTER["world"], "device": CLUSTER["device"],
                           "cold_start_ms": CLUSTER["cold_start_ms"],
                           "members": m.members if m else None, "epoch": m.epoch if m else None,
                           "health": m.health if m else None, "dp": _DP["member"] is not None,
                           "reforms": c.reforms if c else (m.reforms if m else None)}
    if s.backend == "gpu":
        info["devices"] = list(s.settings.devices)
        if "torch" in sys.modules:  # names only when torch is loaded anyway (never imported for this)
            import torch
            info["device_names"] = [torch.cuda.get_device_name(d) for d in s.settings.devices]
    return _json(info)


@app.route("/metrics", methods=["GET"])
def metrics():
    from ..utils.gpu_metrics import render as gpu_render
    return Response(METRICS.render() + gpu_render(), mimetype="text/plain; version=0.0.4")
