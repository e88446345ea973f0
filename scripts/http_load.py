#!/usr/bin/env python3
"""Concurrent HTTP load test of POST /predict (hipzap/serve/loadtest.py): req/s, p50 and p99.

    python scripts/http_load.py [--clients 16] [--requests 200] [--gpus 1] [--format json|npy]

Writes (untimed) a random-init ResNet-50 checkpoint and its plan image, then serves and loads it.
Prints one JSON line.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


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
    from hipzap.serve.loadtest import run_load
    ckpt, plan = prepare_artifacts("resnet50", "/tmp/hipzap_bench")
    if a.plan_batch > 1:
        from hipzap.engine.plan import export_from_checkpoint
        plan = export_from_checkpoint("resnet50", ckpt, path=f"{ckpt}.b{a.plan_batch}.hzplan", batch=a.plan_batch,
                                      contexts=a.contexts)
    print(json.dumps(run_load(plan, a.gpus, a.clients, a.requests, a.contexts, a.format, a.port, a.native,
                              a.plan_batch, a.max_wait_ms, a.server_log)))


if __name__ == "__main__":
    main()
