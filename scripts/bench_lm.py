#!/usr/bin/env python3
"""Reference-parity benchmark: AWD-LSTM GET /inference (200 sampled words) on MI355X.

Config = the reference's serving model (main.py:95-96: emb 1000, hidden 1150, 3 layers,
tied) with V=60000 (SURVEY.md §2d assumption; the real rjokes vocab is not in the repo),
random-init weights. Reports cold start, per-request latency p50 (200 words, prompt ['']),
per-token latency, and the same request through the Flask app. Reference on the sandbox CPU:
8.86 s per request."""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from hipzap.engine.lm import LMEngine  # noqa: E402
from hipzap.models.awd_lstm import reference_lm  # noqa: E402
from hipzap.serve.server import synthetic_vocab  # noqa: E402

REFERENCE_REQUEST_S = 8.86


def main():
    V = int(os.environ.get("HIPZAP_LM_VOCAB", 60000))
    words = int(os.environ.get("HIPZAP_LM_WORDS", 200))
    unroll = int(os.environ.get("HIPZAP_LM_UNROLL", 8))  # decode steps per captured graph
    torch.manual_seed(0)
    itos = synthetic_vocab(V)
    stoi = {w: i for i, w in enumerate(itos)}
    sd = reference_lm(V).state_dict()
    t0 = time.perf_counter()
    eng = LMEngine.for_vocab(sd, stoi, "cuda:0", unroll=unroll)
    cold_ms = (time.perf_counter() - t0) * 1e3
    eng.generate([""], words, itos, stoi, seed=0)  # warm
    lat = []
    for s in range(7):
        t = time.perf_counter()
        text = eng.generate([""], words, itos, stoi, seed=s)
        lat.append(time.perf_counter() - t)
    p50 = statistics.median(lat)
    # Flask end-to-end (GET /inference) on the same engine
    from hipzap.serve import app as app_mod
    from hipzap.serve.server import LMBackend, ModelServer
    from hipzap.serve.settings import Settings
    srv = ModelServer(Settings(lm_words=words), backend="gpu")
    be = LMBackend.__new__(LMBackend)
    be.itos, be.stoi, be.backend, be.engine, be.model, be.cold_ms = itos, stoi, "gpu", eng, None, cold_ms
    import threading
    be._lock = threading.Lock()
    srv._models["__lm__"] = be
    app_mod.set_server(srv)
    c = app_mod.app.test_client()
    c.get("/inference")
    http = []
    for _ in range(5):
        t = time.perf_counter()
        r = c.get("/inference")
        http.append(time.perf_counter() - t)
        assert r.status_code == 200
    # concurrent requests: LMPool of independent decode contexts sharing the packed weights
    from concurrent.futures import ThreadPoolExecutor
    from hipzap.engine.lm import LMPool
    conc = int(os.environ.get("HIPZAP_LM_CONTEXTS", 4))
    pool = LMPool(eng.p, "cuda:0", contexts=conc, exclude_ids=[], unroll=unroll)
    n_req = 4 * conc
    with ThreadPoolExecutor(conc) as ex:
        list(ex.map(lambda s: pool.run_tokens([1], words, s), range(conc)))  # warm
        t = time.perf_counter()
        list(ex.map(lambda s: pool.run_tokens([1], words, s), range(n_req)))
        pool_rps = n_req / (time.perf_counter() - t)
    res = {"metric": "AWD-LSTM GET /inference latency (200 words)", "vocab": V, "words": words, "steps_per_graph": unroll,
           "concurrent_contexts": conc, "requests_per_s_concurrent": round(pool_rps, 2),
           "cold_start_ms": round(cold_ms, 1), "request_s_p50": round(p50, 5),
           "ms_per_token": round(p50 / (words) * 1e3, 4), "http_request_s_p50": round(statistics.median(http), 5),
           "speedup_vs_reference_cpu": round(REFERENCE_REQUEST_S / statistics.median(http), 1),
           "sample_text_head": text[:80]}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
