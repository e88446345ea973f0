#!/usr/bin/env python3
"""A/B of the torch-free cold start with and without the interpreter's site-packages scan
(``python -S``, hipzap/coldstart.py ``python_cmd``): fresh ``plan`` processes in alternation, one
JSON line per trial, then a summary line.  python scripts/cold_site_ab.py PLAN [--trials 10]"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hipzap import coldstart as cs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("plan")
    ap.add_argument("--trials", type=int, default=10)
    a = ap.parse_args()
    env, device = cs.isolated_env(None, 0)
    variants = {"no_site": [sys.executable, "-S"], "site": [sys.executable]}
    walls = {k: [] for k in variants}
    for t in range(a.trials):
        for name, py in variants.items():
            cmd = [*py, "-m", "hipzap.coldstart", "plan", a.plan, "--device", str(device)]
            w, out = cs._fresh_trial(cmd, "plan", env, 300.0)
            walls[name].append(w)
            print(json.dumps({"trial": t, "variant": name, "ms": round(w, 2), "no_site": out.get("no_site"),
                              "phases": {k: round(v, 2) for k, v in out["phases_ms"].items()}}), flush=True)
    print(json.dumps({"summary": {k: {"p50_ms": round(statistics.median(v), 2), "min_ms": round(min(v), 2)}
                                  for k, v in walls.items()}}), flush=True)


if __name__ == "__main__":
    main()
