#!/usr/bin/env python3
"""Interleaved A/B of the plan cold start's device-code warm-thread order:
``HIPZAP_PLAN_WARM_ORDER=init`` (rounds 3-4: the thread starts right after HIP init, beside the
process's first hipStreamCreate) vs ``stream`` (round 5 default: it starts once the upload stream
exists, beside the blob DMA). Fresh processes (hipzap/coldstart.py), one trial per variant per
round, ``--trials`` rounds; prints one JSON line per trial (wall + child phases) and a summary with
the p50 and the median trial's phases per variant.

    python scripts/cold_order_ab.py [--trials 10] [--dir /tmp/hipzap_bench]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=10)
    ap.add_argument("--dir", default=os.environ.get("HIPZAP_BENCH_DIR", "/tmp/hipzap_bench"))
    ap.add_argument("--model", default="resnet50")
    a = ap.parse_args()
    import bench  # the deploy artifacts exactly as bench.py writes them (CPU, untimed)
    from hipzap.coldstart import measure_fresh
    _, plan = bench.prepare_artifacts(a.model, a.dir)
    runs = {"init": [], "stream": []}
    for t in range(a.trials):
        for v in (("init", "stream") if t % 2 == 0 else ("stream", "init")):
            env = dict(os.environ, HIPZAP_PLAN_WARM_ORDER=v)
            r = measure_fresh("plan", plan, a.model, 1, env=env)
            row = {"trial": t, "order": v, "ms": r["p50_ms"], "phases": r["median_trial_phases_ms"]}
            runs[v].append(row)
            print(json.dumps(row), flush=True)
    summary = {}
    for v, rows in runs.items():
        rows = sorted(rows, key=lambda r: r["ms"])
        med = rows[len(rows) // 2]
        keys = ("hip_init_ms", "stream_ms", "upload_dma_ms", "warm_wait_ms", "warm_thread_ms", "first_request")
        summary[v] = {"p50_ms": round(statistics.median(r["ms"] for r in rows), 2),
                      "min_ms": rows[0]["ms"], "max_ms": rows[-1]["ms"],
                      "median_trial": {k: med["phases"].get(k) for k in keys},
                      "stream_ms_p50": round(statistics.median(r["phases"].get("stream_ms", 0) for r in rows), 2),
                      "warm_wait_ms_p50": round(statistics.median(r["phases"].get("warm_wait_ms", 0) for r in rows), 2)}
    print(json.dumps({"summary": summary}), flush=True)


if __name__ == "__main__":
    main()
