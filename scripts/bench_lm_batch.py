#!/usr/bin/env python3
"""Concurrent GET /inference throughput of the batched AWD-LSTM engine.

The reference's request (main.py:84-112): the empty prompt, 200 sampled words. ``--clients``
threads submit such requests back to back (random seeds) to one LMBatchEngine for ``--requests``
requests each; prints one JSON line with req/s, latency p50/p99 and row utilisation. The
reference-dims model (emb 1000, hidden 1150, 3 layers, tied) is random-init at ``--vocab``.
``--compare-pool N``: the same load on the single-request engine pool (engine/lm.py LMPool).
"""
import argparse
import json
import os
import statistics
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run_load(fn, clients, requests, words):
    lat, errs = [], []
    lock = threading.Lock()

    def client(c):
        import random
        rnd = random.Random(c)
        for _ in range(requests):
            t = time.perf_counter()
            try:
                toks = fn([0], words, rnd.getrandbits(62))
                assert len(toks) == words
            except Exception as e:  # noqa: BLE001
                with lock:
                    errs.append(repr(e))
                return
            with lock:
                lat.append((time.perf_counter() - t) * 1e3)

    th = [threading.Thread(target=client, args=(c,)) for c in range(clients)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    wall = time.perf_counter() - t0
    lat.sort()
    return {"clients": clients, "requests": len(lat), "errors": len(errs), "first_error": errs[0] if errs else None,
            "req_per_s": round(len(lat) / wall, 1), "tokens_per_s": round(len(lat) * words / wall, 0),
            "p50_ms": round(statistics.median(lat), 3) if lat else None,
            "p99_ms": round(lat[int(0.99 * (len(lat) - 1))], 3) if lat else None, "wall_s": round(wall, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--vocab", type=int, default=60000)
    ap.add_argument("--rows", type=int, default=32)
    ap.add_argument("--unroll", type=int, default=8)
    ap.add_argument("--clients", type=int, nargs="+", default=[1, 8, 32, 64])
    ap.add_argument("--requests", type=int, default=20, help="per client")
    ap.add_argument("--words", type=int, default=200)
    ap.add_argument("--compare-pool", type=int, default=0, help="also the single-request LMPool with N contexts")
    a = ap.parse_args()
    import torch
    from hipzap.engine.lmbatch import LMBatchEngine, pack_lmb
    from hipzap.models.awd_lstm import reference_lm
    torch.manual_seed(0)
    m = reference_lm(a.vocab).eval()
    sd = m.state_dict()
    t = time.perf_counter()
    eng = LMBatchEngine(pack_lmb(sd, "cuda:0"), "cuda:0", rows=a.rows, unroll=a.unroll, exclude_ids=[2, 5, 6])
    build_ms = (time.perf_counter() - t) * 1e3
    eng.run_tokens([0], a.words, 1)  # warm
    res = {"engine": "LMBatchEngine", "vocab": a.vocab, "rows": a.rows, "unroll": a.unroll, "words": a.words,
           "build_ms": round(build_ms, 1), "load": []}
    single = []
    for _ in range(5):
        t = time.perf_counter()
        eng.run_tokens([0], a.words, 3)
        single.append((time.perf_counter() - t) * 1e3)
    res["single_request_ms"] = round(statistics.median(single), 3)
    res["single_us_per_step"] = round(statistics.median(single) * 1e3 / (a.words + 1), 2)
    for c in a.clients:
        s0 = eng.stats()
        r = run_load(lambda p, n, s: eng.run_tokens(p, n, s), c, a.requests, a.words)
        s1 = eng.stats()
        steps = (s1["replays"] - s0["replays"]) * a.unroll
        r["us_per_step"] = round(r["wall_s"] * 1e6 / max(1, steps), 2)
        r["row_utilisation"] = round((s1["row_steps_used"] - s0["row_steps_used"]) /
                                     max(1, s1["row_steps"] - s0["row_steps"]), 3)
        res["load"].append(r)
        print(json.dumps(r), file=sys.stderr, flush=True)
    eng.close()
    if a.compare_pool:
        from hipzap.engine.lm import LMPool, pack_awd_lstm
        pool = LMPool(pack_awd_lstm(sd, "cuda:0"), "cuda:0", contexts=a.compare_pool, exclude_ids=[2, 5, 6])
        pool.run_tokens([0], a.words, 1)
        res["pool"] = run_load(lambda p, n, s: pool.run_tokens(p, n, s), a.compare_pool * 2, max(2, a.requests // 4),
                               a.words)
        res["pool"]["contexts"] = a.compare_pool
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
