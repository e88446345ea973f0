#!/usr/bin/env python3
"""Concurrent HTTP load test of POST /predict: req/s, p50 and p99 latency as
seen by clients of a real server process.

    python scripts/http_load.py [--clients 16] [--requests 200] [--gpus 1] [--format json|npy]

Writes (untimed) a random-init ResNet-50 checkpoint and its plan image, starts
``python -m hipzap serve`` (``--gpus N``: the DP cluster, one worker process per GPU sharing
the listening socket) with a settings file pointing at the plan, waits for /health, then runs
``--clients`` client PROCESSES (so the load generator does not share a GIL with anything),
each sending ``--requests`` uint8 224x224x3 images back to back over one keep-alive connection.
Prints one JSON line.
"""
import argparse
import base64
import http.client
import io
import json
import multiprocessing as mp
import os
import statistics
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def client(port, n, fmt, q):
    import numpy as np
    rng = np.random.default_rng(os.getpid())
    img = rng.integers(0, 256, (224, 224, 3), dtype=np.uint8)
    if fmt == "npy":
        buf = io.BytesIO()
        np.save(buf, img[None])
        body, ctype = buf.getvalue(), "application/octet-stream"
    else:
        body = json.dumps({"image_b64": base64.b64encode(img.tobytes()).decode(), "shape": [224, 224, 3]})
        ctype = "application/json"
    conn = http.client.HTTPConnection("127.0.0.1", port, timeout=60)
    lat, errors = [], 0
    for _ in range(n):
        t = time.perf_counter()
        try:
            conn.request("POST", "/predict", body=body, headers={"Content-Type": ctype})
            r = conn.getresponse()
            r.read()
            if r.status != 200:
                errors += 1
        except (ConnectionError, http.client.HTTPException, OSError):
            errors += 1
            conn = http.client.HTTPConnection("127.0.0.1", port, timeout=60)
        lat.append((time.perf_counter() - t) * 1e3)
    q.put((lat, errors))


def x_timing(port, fmt):
    """Server-side phase timings (X-Timing header) of a few sequential requests (last one)."""
    import numpy as np
    img = np.zeros((224, 224, 3), np.uint8)
    if fmt == "npy":
        buf = io.BytesIO()
        np.save(buf, img[None])
        body, ctype = buf.getvalue(), "application/octet-stream"
    else:
        body = json.dumps({"image_b64": base64.b64encode(img.tobytes()).decode(), "shape": [224, 224, 3]})
        ctype = "application/json"
    conn = http.client.HTTPConnection("127.0.0.1", port, timeout=60)
    hdr, lat = None, []
    for _ in range(20):
        t = time.perf_counter()
        conn.request("POST", "/predict", body=body, headers={"Content-Type": ctype})
        r = conn.getresponse()
        r.read()
        lat.append((time.perf_counter() - t) * 1e3)
        hdr = r.getheader("X-Timing")
    return {"x_timing": hdr, "sequential_p50_ms": round(statistics.median(lat), 3)}


def wait_health(port, proc, timeout=300):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if proc.poll() is not None:
            raise RuntimeError(f"server exited with {proc.returncode}")
        try:
            c = http.client.HTTPConnection("127.0.0.1", port, timeout=5)
            c.request("GET", "/health")
            if c.getresponse().status == 200:
                return time.time() - t0
        except OSError:
            pass
        time.sleep(0.05)
    raise RuntimeError("server did not become healthy")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=16)
    ap.add_argument("--requests", type=int, default=200)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--contexts", type=int, default=8)
    ap.add_argument("--format", choices=["json", "npy"], default="json")
    ap.add_argument("--port", type=int, default=18082)
    ap.add_argument("--server-log", default=None, help="copy the server log here")
    ap.add_argument("--native", action="store_true",
                    help="serve with the Python-free hipzap-serve-plan binary instead of python -m hipzap serve")
    ap.add_argument("--plan-batch", type=int, default=1,
                    help="serve a batch-B plan: one-image requests dynamically batched into B-row replays")
    ap.add_argument("--max-wait-ms", type=float, default=0.2)
    a = ap.parse_args()
    from bench import prepare_artifacts
    ckpt, plan = prepare_artifacts("resnet50", "/tmp/hipzap_bench")
    if a.plan_batch > 1:
        from hipzap.engine.plan import export_from_checkpoint
        plan = export_from_checkpoint("resnet50", ckpt, path=f"{ckpt}.b{a.plan_batch}.hzplan", batch=a.plan_batch,
                                      contexts=a.contexts)
    d = tempfile.mkdtemp(prefix="hz_http_")
    settings = os.path.join(d, "zappa_settings.json")
    with open(settings, "w") as f:
        json.dump({"dev": {"hipzap": {"default_model": "resnet50", "models": {
            "resnet50": {"contexts": a.contexts, "extra": {"plan": plan, "batching": {"max_wait_ms": a.max_wait_ms}}}}}}},
                  f)
    cmd = [sys.executable, "-m", "hipzap", "serve", "--settings", settings, "--port", str(a.port)]
    if a.gpus > 1:
        cmd += ["--gpus", str(a.gpus)]
    if a.native:
        cmd = [os.path.join(ROOT, "hipzap", "_lib", "hipzap-serve-plan"), plan, "--port", str(a.port),
               "--contexts", str(a.contexts), "--max-wait-us", str(a.max_wait_ms * 1e3)]
    env = dict(os.environ, HIPZAP_WATCHDOG="0")
    log_path = os.path.join(d, "server.log")
    log_f = open(log_path, "w")  # never a pipe: the access log would fill it and block the server
    srv = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=log_f, stderr=subprocess.STDOUT, text=True)
    print(f"server pid {srv.pid}, log {log_path}", file=sys.stderr, flush=True)
    try:
        ready_s = wait_health(a.port, srv)
        print(f"healthy after {ready_s:.2f} s", file=sys.stderr, flush=True)
        # first request (cold model load happens on first use)
        t = time.time()
        q = mp.Queue()
        client(a.port, 1, a.format, q)
        first_ms = (time.time() - t) * 1e3
        q.get()
        timing = x_timing(a.port, a.format)
        print(f"first request {first_ms:.1f} ms; warm X-Timing {timing}", file=sys.stderr, flush=True)
        for _ in range(2):  # warm every worker / context
            ps = [mp.Process(target=client, args=(a.port, 20, a.format, q)) for _ in range(a.clients)]
            [p.start() for p in ps]
            [q.get() for _ in ps]
            [p.join() for p in ps]
        print("warm", file=sys.stderr, flush=True)
        ps = [mp.Process(target=client, args=(a.port, a.requests, a.format, q)) for _ in range(a.clients)]
        t0 = time.perf_counter()
        [p.start() for p in ps]
        res = [q.get() for _ in ps]
        wall = time.perf_counter() - t0
        [p.join() for p in ps]
    finally:
        srv.terminate()
        try:
            srv.wait(timeout=30)
        except subprocess.TimeoutExpired:
            srv.kill()
            srv.wait()
        log_f.close()
        with open(log_path) as f:
            out = f.read()
        if a.server_log:
            with open(a.server_log, "w") as f:
                f.write(out)
    lat = sorted(x for r in res for x in r[0])
    errors = sum(r[1] for r in res)
    print(json.dumps({
        "server": "hipzap-serve-plan" if a.native else "python -m hipzap serve", "plan_batch": a.plan_batch,
        "gpus": a.gpus, "clients": a.clients, "requests": len(lat), "format": a.format, "errors": errors,
        "req_per_s": round(len(lat) / wall, 1), "p50_ms": round(statistics.median(lat), 3),
        "p99_ms": round(lat[int(0.99 * (len(lat) - 1))], 3), "max_ms": round(lat[-1], 3),
        "server_ready_s": round(ready_s, 3), "spawn_to_ready_s": round(ready_s, 3),
        "first_request_ms": round(first_ms, 2), "contexts_per_gpu": a.contexts, "warm_single": timing,
        "server_log_tail": out[-1500:] if errors else ""}))


if __name__ == "__main__":
    main()
