#!/usr/bin/env python3
"""The torch-free BERT text plan (bs16) with 4 request contexts: seq/s of ``PlanEngine.bench``
with the contexts after the first on highest-priority streams (``HIPZAP_STREAM_KIND=auto``) vs
plain streams (``torch``), each in a fresh child process, interleaved. Prints one JSON line per
run. The plan is exported once (random-init weights) under /tmp/hipzap_bench.

    python scripts/diag_plan_kinds.py [--reps 2]
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(plan: str) -> None:
    from hipzap.lite import PlanEngine
    eng = PlanEngine(plan, device=0, contexts=4)
    eng.ensure_contexts()
    eng.bench(10)
    rates = [round(16 * 4 * 200 / eng.bench(200), 1) for _ in range(3)]
    print(json.dumps({"kind": os.environ.get("HIPZAP_STREAM_KIND", "auto"), "seq_s": rates}), flush=True)


def main():
    if "--child" in sys.argv:
        return child(sys.argv[sys.argv.index("--child") + 1])
    import bench
    bench._import_torch()
    plan = bench.prepare_bert_plan("/tmp/hipzap_bench")
    reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 2
    for _ in range(reps):
        for kind in ("auto", "torch"):
            env = dict(os.environ, HIPZAP_STREAM_KIND=kind)
            r = subprocess.run([sys.executable, __file__, "--child", plan], env=env, capture_output=True, text=True,
                               timeout=300)
            line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            print(line[-1] if line else json.dumps({"kind": kind, "error": r.stderr[-500:]}), flush=True)


if __name__ == "__main__":
    main()
