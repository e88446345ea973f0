#!/usr/bin/env python3
"""Cold-start p50 over fresh processes (what a new Lambda container / replica pays).

Each trial spawns a NEW python process that imports hipzap, torch.load()s a ResNet-50
state_dict, packs it on the GPU, plans, captures the hipGraph and returns the first result;
we time process spawn -> first logits on stdout. Reported alongside the in-process phases."""
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import time, json, sys
t0 = time.time()
sys.path.insert(0, %r)
import torch
from hipzap.engine.engine import Engine
t1 = time.time()
eng = Engine.from_checkpoint(%r, %r, "cuda:0", batch=1, num_contexts=1)
y = eng.infer(torch.randn(1, 3, 224, 224))
t2 = time.time()
print(json.dumps({"import_s": t1 - t0, "engine_s": t2 - t1, "timings_ms": eng.timings, "ok": bool(torch.isfinite(y).all())}))
"""


def main():
    model = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
    trials = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    ckpt = f"/tmp/hipzap_bench/{model}_seed0.pth"
    if not os.path.exists(ckpt):
        sys.path.insert(0, ROOT)
        from bench import write_checkpoint
        write_checkpoint(ckpt, model)
    walls, inner = [], []
    for _ in range(trials):
        t = time.time()
        out = subprocess.run([sys.executable, "-c", CHILD % (ROOT, model, ckpt)], capture_output=True, text=True,
                             timeout=300)
        walls.append((time.time() - t) * 1e3)
        line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
        if out.returncode != 0 or not line:
            print(out.stderr[-2000:], file=sys.stderr)
            sys.exit(1)
        inner.append(json.loads(line[-1]))
    print(json.dumps({"model": model, "trials": trials, "process_cold_start_ms_p50": round(statistics.median(walls), 1),
                      "process_cold_start_ms_all": [round(w, 1) for w in walls],
                      "engine_cold_start_ms_p50": round(statistics.median(i["engine_s"] for i in inner) * 1e3, 1),
                      "import_ms_p50": round(statistics.median(i["import_s"] for i in inner) * 1e3, 1),
                      "phases_ms_last": {k: round(v, 2) for k, v in inner[-1]["timings_ms"].items()}}))


if __name__ == "__main__":
    main()
