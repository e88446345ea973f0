#!/usr/bin/env python3
"""A/B of the torch-free plan cold start (spawn -> first logits, fresh processes, interleaved):
weight upload strategy (HIPZAP_PLAN_UPLOAD = staged | register | pageable | kernel) x lazy graph
capture (HIPZAP_PLAN_LAZY_CAPTURE), optionally with the first-DMA probe (HIPZAP_PLAN_PROBE=1: a
4 KiB copy timed on its own before the upload). One JSON line per variant with p50 and the
median trial's phases.

    python scripts/cold_start_variants.py [trials] [upload,upload,...] [lazy values e.g. 0,1] [probe 0|1]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    from bench import prepare_artifacts
    from hipzap.coldstart import measure_fresh
    _, plan = prepare_artifacts("resnet50", "/tmp/hipzap_bench")
    uploads = sys.argv[2].split(",") if len(sys.argv) > 2 else ["staged", "register", "pageable", "kernel"]
    lazies = sys.argv[3].split(",") if len(sys.argv) > 3 else ["0", "1"]
    probe = sys.argv[4] if len(sys.argv) > 4 else "0"
    variants = [(u, lz) for lz in lazies for u in uploads]
    res = {v: [] for v in variants}
    for _ in range(trials):  # interleave the variants: box noise hits them alike
        for u, lz in variants:
            env = dict(os.environ, HIPZAP_PLAN_UPLOAD=u, HIPZAP_PLAN_LAZY_CAPTURE=lz, HIPZAP_PLAN_PROBE=probe)
            res[(u, lz)].append(measure_fresh("plan", plan, trials=1, env=env))
    for (u, lz), rs in res.items():
        walls = sorted(r["p50_ms"] for r in rs)
        med = sorted(rs, key=lambda r: r["p50_ms"])[len(rs) // 2]
        print(json.dumps({"upload": u, "lazy_capture": lz == "1", "trials": trials, "probe": probe == "1",
                          "p50_ms": walls[len(walls) // 2], "min_ms": walls[0], "max_ms": walls[-1],
                          "median_trial_phases_ms": med["median_trial_phases_ms"]}), flush=True)


if __name__ == "__main__":
    main()
