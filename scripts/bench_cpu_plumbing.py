#!/usr/bin/env python3
"""BASELINE config 1: ResNet-18 single-image POST /predict through the Flask/WSGI handler on
the CPU backend (the plumbing path; no GPU). Boots the real dev server (``main.py``) as a
subprocess, measures cold start (process start -> first 200 OK) and warm request latency over
HTTP for a uint8 224x224 image and for an fp32 tensor payload, plus the same request through
the Zappa-style Lambda handler in-process. One JSON line.

    python scripts/bench_cpu_plumbing.py [--requests 50]
"""
import argparse
import base64
import json
import os
import socket
import statistics
import subprocess
import sys
import time
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _post(url, payload: bytes):
    req = urllib.request.Request(url, data=payload, headers={"Content-Type": "application/json"})
    return json.loads(urllib.request.urlopen(req, timeout=120).read())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--requests", type=int, default=50)
    ap.add_argument("--backend", default="cpu", help="cpu (config 1) or gpu (the same HTTP path on MI355X)")
    ap.add_argument("--model", default="resnet18")
    args = ap.parse_args()
    import numpy as np
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (224, 224, 3), dtype=np.uint8)
    body_img = json.dumps({"model": args.model, "image_b64": base64.b64encode(img.tobytes()).decode(),
                           "shape": [224, 224, 3]}).encode()
    x = rng.standard_normal((1, 3, 224, 224), dtype=np.float32)
    body_t = json.dumps({"model": args.model, "tensor_b64": base64.b64encode(x.tobytes()).decode(),
                         "shape": [1, 3, 224, 224]}).encode()

    port = _port()
    env = dict(os.environ, HIPZAP_RANDOM_WEIGHTS="1", HIPZAP_PORT=str(port), HIPZAP_BACKEND=args.backend,
               HIPZAP_SETTINGS="/nonexistent", HIPZAP_LM_VOCAB="300")
    t0 = time.perf_counter()
    proc = subprocess.Popen([sys.executable, "main.py"], cwd=ROOT, env=env, stdout=subprocess.DEVNULL,
                            stderr=subprocess.DEVNULL)
    base = f"http://127.0.0.1:{port}"
    try:
        while True:
            try:
                urllib.request.urlopen(base + "/health", timeout=1)
                break
            except Exception:
                if proc.poll() is not None or time.perf_counter() - t0 > 300:
                    raise RuntimeError("server did not come up")
                time.sleep(0.05)
        up_ms = (time.perf_counter() - t0) * 1e3
        ta = time.perf_counter()
        first = _post(base + "/predict", body_img)
        first_ms = (time.perf_counter() - ta) * 1e3  # includes the model's cold load
        cold_ms = (time.perf_counter() - t0) * 1e3
        lat = {"image_b64": [], "tensor_b64": []}
        for _ in range(args.requests):
            for name, body in (("image_b64", body_img), ("tensor_b64", body_t)):
                ta = time.perf_counter()
                r = _post(base + "/predict", body)
                lat[name].append((time.perf_counter() - ta) * 1e3)
                assert r["backend"] == args.backend and len(r["top5"][0]) == 5
    finally:
        proc.terminate()
        proc.wait(timeout=30)

    # the same request through the Lambda (API Gateway v1) adapter, in process
    os.environ.update(HIPZAP_RANDOM_WEIGHTS="1", HIPZAP_BACKEND=args.backend, HIPZAP_SETTINGS="/nonexistent")
    sys.path.insert(0, ROOT)
    from hipzap.serve.lambda_handler import lambda_handler
    ev = {"httpMethod": "POST", "path": "/predict", "headers": {"content-type": "application/json"},
          "body": body_img.decode(), "isBase64Encoded": False}
    assert lambda_handler(ev)["statusCode"] == 200
    lam = []
    for _ in range(args.requests):
        ta = time.perf_counter()
        assert lambda_handler(ev)["statusCode"] == 200
        lam.append((time.perf_counter() - ta) * 1e3)
    print(json.dumps({
        "metric": f"single-image POST /predict through the Flask/WSGI handler: {args.model}, {args.backend} backend"
                  + (" (config 1: plumbing, no GPU)" if args.backend == "cpu" else ""),
        "requests": args.requests, "cpu_threads": os.cpu_count(),
        "server_up_ms": round(up_ms, 1), "first_request_ms": round(first_ms, 1),
        "cold_start_to_first_200_ms": round(cold_ms, 1),
        "http_image_b64_ms_p50": round(statistics.median(lat["image_b64"]), 2),
        "http_tensor_b64_ms_p50": round(statistics.median(lat["tensor_b64"]), 2),
        "lambda_event_ms_p50": round(statistics.median(lam), 2),
        "reference_cpu_resnet18_ms": 16.6,
        "data": f"random-init {args.model} weights, random uint8 image / fp32 tensor",
        "first_top1": first["top5"][0][0]}), flush=True)


if __name__ == "__main__":
    main()
