#!/bin/bash
# Python-free serving binary: fresh-process cold start (interleaved with the Python plan path)
# and concurrent HTTP load against hipzap-serve-plan.
set -e
o=gpurun_out/native
mkdir -p $o
timeout -k 10 300 python -u - > $o/coldstart.jsonl 2> $o/coldstart.err <<'PY'
import json, sys
sys.path.insert(0, ".")
from bench import prepare_artifacts
from hipzap.coldstart import measure_fresh
_, plan = prepare_artifacts("resnet50", "/tmp/hipzap_bench")
res = {"native": [], "plan": []}
for _ in range(11):
    for m in ("native", "plan"):
        res[m].append(measure_fresh(m, plan, trials=1))
for m, rs in res.items():
    w = sorted(r["p50_ms"] for r in rs)
    med = sorted(rs, key=lambda r: r["p50_ms"])[len(rs) // 2]
    print(json.dumps({"mode": m, "p50_ms": w[len(w) // 2], "min_ms": w[0], "max_ms": w[-1],
                      "median_trial_phases_ms": med["median_trial_phases_ms"]}), flush=True)
PY
timeout -k 10 300 python -u scripts/http_load.py --native --contexts 24 --clients 16 --requests 300 --format json > $o/http_json.json 2> $o/http_json.err
timeout -k 10 300 python -u scripts/http_load.py --native --contexts 24 --clients 32 --requests 300 --format npy > $o/http_npy.json 2> $o/http_npy.err
