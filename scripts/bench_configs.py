#!/usr/bin/env python3
"""BASELINE config 4 and the reference's own route, timed in a fresh process (bench.py runs this
on rank 0's GPU after the headline). One JSON line:

* ``bert_base_bs16`` (config 4): BERT-base seq-cls, bs 16, L 128, random-init weights, bf16;
  hipGraph replays of 1 and of 4 concurrent contexts (``Engine.bench``: the C++ replay loop over
  every context's stream, synchronised) -> seq/s; plus the one-context request latency p50
  (``Engine.infer``: pinned token ids in, logits out).
* ``awd_lstm_get_inference`` (/root/reference/main.py:105-112): ``GET /inference`` through the
  WSGI app (``hipzap.serve.app``, Flask test clients in this process: routing, the batched
  AWD-LSTM engine, 200 sampled words, detokenisation, the JSON body) on the reference's
  dimensions (emb 1000, hidden 1150, 3 layers, tied, V = 60000, random-init); the lone-request
  latency p50 (one request at a time) and the req/s of 32 concurrent clients (wall over all their
  requests).
* ``awd_lstm_get_inference_http``: the same route over HTTP through the native front end (the
  request is answered in C++: scheduler submit + detokenizer table + JSON, no GIL), 32 client
  PROCESSES (scripts/lm_http_client.py; 32 Python client threads in one process were the
  bottleneck: 1.4k req/s against the engine's 2.76k), one keep-alive connection each.

    python scripts/bench_configs.py [--device D] [--steps K]
"""
import json
import os
import statistics
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def bert_figure(device: str, steps: int) -> dict:
    import torch
    from hipzap.engine.engine import Engine
    from hipzap.models import registry
    a = registry.get("bert-base")
    torch.manual_seed(0)
    sd = a.make_model().eval().state_dict()
    res = {"model": "bert-base (seq-cls, 2 labels)", "batch": 16, "seq_len": 128, "dtype": "bf16",
           "data": "synthetic (random-init weights, random token ids)"}
    iters = max(100, steps * 10)
    for ctx in (1, 4):
        eng = Engine.from_state_dict("bert-base", sd, device, batch=16, num_contexts=ctx)
        x = a.example_input(16)
        eng.infer(x)
        if ctx == 1:
            lat = []
            for _ in range(50):
                t = time.perf_counter()
                eng.infer(x)
                lat.append((time.perf_counter() - t) * 1e3)
            res["latency_ms_p50_1ctx"] = round(statistics.median(lat), 4)
        eng.bench(10)
        t = eng.bench(iters)  # seconds for iters replays of every context, synchronised
        res[f"seq_s_{ctx}ctx"] = round(16 * ctx * iters / t, 1)
        res[f"ms_per_replay_{ctx}ctx"] = round(t / iters * 1e3, 4)
        del eng
        torch.cuda.synchronize(device)
    res["timed_region"] = f"{iters} hipGraph replays per context, all contexts concurrently, synchronised"
    return res


def lm_route_figure() -> dict:
    os.environ.setdefault("HIPZAP_SETTINGS", "/nonexistent")
    os.environ.update(HIPZAP_RANDOM_WEIGHTS="1", HIPZAP_LM_VOCAB="60000", HIPZAP_BACKEND="gpu")
    from hipzap.serve.app import app, get_server
    srv = get_server()
    t = time.perf_counter()
    srv.lm()  # the cold load (random-init reference-dims model packed on the GPU), untimed below
    load_ms = (time.perf_counter() - t) * 1e3
    cl = app.test_client()

    def get(c, seed):
        r = c.get(f"/inference?seed={seed}")
        assert r.status_code == 200 and r.get_json()["response"]["text"]

    for i in range(3):
        get(cl, i)
    lat = []
    for i in range(15):
        t = time.perf_counter()
        get(cl, 100 + i)
        lat.append((time.perf_counter() - t) * 1e3)
    clients, per = 32, 8
    errs = []

    def client(c):
        cc = app.test_client()
        for k in range(per):
            try:
                get(cc, 1000 + c * per + k)
            except Exception as e:  # noqa: BLE001
                errs.append(repr(e))

    th = [threading.Thread(target=client, args=(c,)) for c in range(clients)]
    t = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    wall = time.perf_counter() - t
    words, done = srv.settings.lm_words, clients * per - len(errs)
    return {"route": "GET /inference (WSGI app in process: Flask test clients)", "words": words,
            "model": "AWD-LSTM emb 1000 / hidden 1150 / 3 layers / tied, V = 60000 (main.py:96)",
            "data": "random-init weights, synthetic vocabulary", "load_ms": round(load_ms, 1),
            "lone_request_ms_p50": round(statistics.median(lat), 3), "lone_request_ms_min": round(min(lat), 3),
            "concurrent_clients": clients, "concurrent_requests": done,
            "concurrent_req_s": round(done / wall, 1), "concurrent_words_s": round(done * words / wall, 0),
            "errors": len(errs),
            "timed_region": f"lone: one request at a time, 15 requests; concurrent: {clients} threads x {per} "
                            "requests, wall"}


def lm_http_figure() -> dict:
    """The same route over HTTP through the native front end (``hipzap serve``'s server:
    csrc/http.cpp answers GET /inference in C++ once the LM backend exists, no GIL on the request
    path); the lone request from this process, the concurrent load from client processes."""
    import http.client
    from hipzap.serve.app import app, get_server
    from hipzap.serve.native_http import NativeHTTPServer, listening_socket
    srv = get_server()
    srv.lm()
    sock = listening_socket("127.0.0.1", 0)
    port = sock.getsockname()[1]
    hs = NativeHTTPServer(app, sock, server=srv)
    try:
        def conn():
            return http.client.HTTPConnection("127.0.0.1", port, timeout=120)

        def get(c, seed):
            c.request("GET", f"/inference?seed={seed}")
            r = c.getresponse()
            b = r.read()
            assert r.status == 200 and b.startswith(b'{"response": {"text": ')
            return r.getheader("X-Hipzap-Path")

        c = conn()
        paths = {get(c, i) for i in range(3)}
        lat = []
        for i in range(15):
            t = time.perf_counter()
            get(c, 100 + i)
            lat.append((time.perf_counter() - t) * 1e3)
        c.close()
        clients, per = 32, 12
        import subprocess
        import tempfile
        go = os.path.join(tempfile.mkdtemp(prefix="hz_lmgo_"), "go")
        procs = [subprocess.Popen([sys.executable, "-S", os.path.join(ROOT, "scripts", "lm_http_client.py"), str(port),
                                   str(per), str(5000 + k * per), go], stdout=subprocess.PIPE, text=True)
                 for k in range(clients)]
        time.sleep(1.0)  # every client process started and connected
        t_go = time.time()
        open(go, "w").close()
        outs = [json.loads(p.communicate(timeout=300)[0].strip().splitlines()[-1]) for p in procs]
        wall = max(o["t_end"] for o in outs) - t_go  # go signal -> the last client's last response
        errs = [o["errors"] for o in outs if o["errors"]]
        done = clients * per - sum(errs)
        lat_all = sorted(x for o in outs for x in o["lat"])
        paths |= {p for o in outs for p in o["paths"]}
        return {"route": "GET /inference over HTTP/1.1 (native front end, csrc/http.cpp)",
                "native": paths == {"native"}, "lone_request_ms_p50": round(statistics.median(lat), 3),
                "lone_request_ms_min": round(min(lat), 3), "concurrent_clients": clients,
                "concurrent_requests": done, "concurrent_req_s": round(done / wall, 1), "errors": sum(errs),
                "concurrent_latency_ms_p50": round(lat_all[len(lat_all) // 2], 3),
                "concurrent_latency_ms_p99": round(lat_all[int(0.99 * (len(lat_all) - 1))], 3),
                "timed_region": f"lone: 15 sequential keep-alive requests; concurrent: {clients} client processes "
                                f"(scripts/lm_http_client.py), one keep-alive connection x {per} requests each, "
                                "wall from the go signal to the last client's last response"}
    finally:
        hs.stop()


def main():
    dev = int(sys.argv[sys.argv.index("--device") + 1]) if "--device" in sys.argv else 0
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 20
    import torch
    torch.cuda.set_device(dev)
    out = {}
    for name, fn in (("bert_base_bs16", lambda: bert_figure(f"cuda:{dev}", steps)),
                     ("awd_lstm_get_inference", lm_route_figure),
                     ("awd_lstm_get_inference_http", lm_http_figure)):
        try:
            out[name] = fn()
        except Exception as e:  # noqa: BLE001 - each figure on its own
            out[name] = {"error": repr(e)[:500]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
