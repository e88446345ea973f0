"""Concurrent HTTP load test of ``POST /predict`` against a real server process (VERDICT r1 #6,
r2 #1 "cluster figure"): req/s, p50 and p99 latency as seen by clients.

:func:`run_load` starts ``python -m hipzap serve`` (``gpus > 1``: the DP serving cluster,
serve/cluster.py -- one worker process per GPU sharing the listening socket, RCCL between them)
or the Python-free ``hipzap-serve-plan`` binary on a plan image, waits for /health, then runs
``clients`` client PROCESSES (the load generator shares no GIL with anything), each sending
``requests`` uint8 224x224x3 images back to back over one keep-alive connection. Used by
``scripts/http_load.py`` and as ``bench.py``'s ``http_serving`` secondary figure.
"""
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

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# launcher variables of a torchrun / bench rank must not leak into the server's own launcher
_LAUNCH_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK", "ROLE_WORLD_SIZE",
               "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID", "TORCHELASTIC_RESTART_COUNT",
               "TORCHELASTIC_MAX_RESTARTS", "HIPZAP_SELF_LAUNCHED")


def client(port, n, fmt, q, start=None):
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
    conn.connect()
    lat, errors = [], 0
    if start is not None:  # every client set up (interpreter, numpy, body, connection) before the window
        start.wait()
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


def wait_health(port, proc, timeout=300.0):
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


def run_load(plan: str, gpus: int = 1, clients: int = 16, requests: int = 200, contexts: int = 8,
             fmt: str = "json", port: int | None = None, native: bool = False, plan_batch: int = 1,
             max_wait_ms: float = 0.2, server_log: str | None = None, ready_timeout: float = 300.0) -> dict:
    """Serve ``plan`` over HTTP and load it; returns the result dict (``errors`` counts non-200s)."""
    if port is None:
        import socket
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
    d = tempfile.mkdtemp(prefix="hz_http_")
    settings = os.path.join(d, "zappa_settings.json")
    with open(settings, "w") as f:
        json.dump({"dev": {"hipzap": {"default_model": "resnet50", "models": {
            "resnet50": {"contexts": contexts, "extra": {"plan": plan, "batching": {"max_wait_ms": max_wait_ms}}}}}}}, f)
    cmd = [sys.executable, "-m", "hipzap", "serve", "--settings", settings, "--host", "127.0.0.1", "--port", str(port)]
    if gpus > 1:
        cmd += ["--gpus", str(gpus)]
    if native:
        cmd = [os.path.join(ROOT, "hipzap", "_lib", "hipzap-serve-plan"), plan, "--port", str(port),
               "--contexts", str(contexts), "--max-wait-us", str(max_wait_ms * 1e3)]
    env = {k: v for k, v in os.environ.items() if k not in _LAUNCH_ENV}
    env["HIPZAP_WATCHDOG"] = "0"
    if env.get("HIPZAP_SHARE_GPU") == "1":  # several workers on one GPU: RCCL refuses that, rehearse on sockets
        env.setdefault("HIPZAP_COMM", "socket")
    log_path = os.path.join(d, "server.log")
    log_f = open(log_path, "w")  # never a pipe: the access log would fill it and block the server
    t_spawn = time.time()
    srv = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=log_f, stderr=subprocess.STDOUT, text=True,
                           start_new_session=True)
    print(f"server pid {srv.pid}, log {log_path}", file=sys.stderr, flush=True)
    ctx = mp.get_context("spawn")
    try:
        ready_s = wait_health(port, srv, ready_timeout)
        t = time.time()
        q = ctx.Queue()
        client(port, 1, fmt, q)  # first request (cold model load happens on first use)
        first_ms = (time.time() - t) * 1e3
        q.get()
        timing = x_timing(port, fmt)
        for _ in range(2):  # warm every worker / context
            ps = [ctx.Process(target=client, args=(port, 20, fmt, q)) for _ in range(clients)]
            [p.start() for p in ps]
            [q.get() for _ in ps]
            [p.join() for p in ps]
        start = ctx.Barrier(clients + 1)
        ps = [ctx.Process(target=client, args=(port, requests, fmt, q, start)) for _ in range(clients)]
        [p.start() for p in ps]
        start.wait(timeout=120)  # the timed window opens once every client is connected
        t0 = time.perf_counter()
        res = [q.get() for _ in ps]
        wall = time.perf_counter() - t0
        [p.join() for p in ps]
    finally:
        import signal
        try:
            os.killpg(srv.pid, signal.SIGTERM)
        except ProcessLookupError:
            pass
        try:
            srv.wait(timeout=30)
        except subprocess.TimeoutExpired:
            os.killpg(srv.pid, signal.SIGKILL)
            srv.wait()
        log_f.close()
        with open(log_path) as f:
            out = f.read()
        if server_log:
            with open(server_log, "w") as f:
                f.write(out)
    lat = sorted(x for r in res for x in r[0])
    errors = sum(r[1] for r in res)
    return {"server": "hipzap-serve-plan" if native else "python -m hipzap serve", "plan_batch": plan_batch,
            "gpus": gpus, "clients": clients, "requests": len(lat), "format": fmt, "errors": errors,
            "req_per_s": round(len(lat) / wall, 1), "window_s": round(wall, 3),
            "p50_ms": round(statistics.median(lat), 3), "p99_ms": round(lat[int(0.99 * (len(lat) - 1))], 3),
            "max_ms": round(lat[-1], 3), "spawn_to_ready_s": round(ready_s, 3),
            "first_request_ms": round(first_ms, 2), "contexts_per_gpu": contexts, "warm_single": timing,
            "server_log_tail": out[-1500:] if errors else ""}
