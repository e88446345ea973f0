#!/usr/bin/env python3
"""Plan-image cold start against the idle time before each fresh child (hipzap/coldstart.py
``_fresh_trial`` gap): which gap lets the previous child's GPU process teardown finish before the
next child's HIP init. Gaps interleaved trial by trial; per gap: p50 spawn -> first logits and the
p50 of the child's own HIP-init phase. Run before this process touches a GPU.

    python scripts/cold_gap_sweep.py [--gaps 0,25,50,100,200,400,800] [--trials 8]
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _arg(name, default):
    return sys.argv[sys.argv.index(name) + 1] if name in sys.argv else default


def main():
    import bench
    from hipzap.coldstart import _fresh_cmd, _fresh_trial, isolated_env
    gaps = [float(g) for g in _arg("--gaps", "0,25,50,100,200,400,800").split(",")]
    trials = int(_arg("--trials", "8"))
    bench._import_torch()
    _, plan = bench.prepare_artifacts("resnet50", "/tmp/hipzap_bench")
    env, dev = isolated_env(None, 0)
    cmd = _fresh_cmd("plan", plan, "resnet50", dev, None)
    walls = {g: [] for g in gaps}
    hips = {g: [] for g in gaps}
    for _ in range(trials):
        for g in gaps:
            w, out = _fresh_trial(cmd, "plan", env, 120.0, g / 1e3)
            walls[g].append(w)
            ph = out.get("phases_ms", {})
            h = ph.get("hip_init_ms", ph.get("hip_init"))
            if isinstance(h, (int, float)):
                hips[g].append(h)
    for g in gaps:
        print(json.dumps({"gap_ms": g, "trials": trials, "p50_ms": round(statistics.median(walls[g]), 1),
                          "hip_init_ms_p50": round(statistics.median(hips[g]), 1) if hips[g] else None,
                          "min_ms": round(min(walls[g]), 1), "max_ms": round(max(walls[g]), 1)}), flush=True)


if __name__ == "__main__":
    main()
