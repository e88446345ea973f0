#!/usr/bin/env python3
"""Batched ResNet-50 programs with several captured contexts in flight (config 3's per-rank
program, the question behind a pipelined DP step): img/s of ``Engine.bench`` (every context
replayed ``iters`` times on its own stream, synchronised) at batch B and C contexts.

One context is the DP step as bench.py times it today (scatter -> replay -> gather, back to
back); C > 1 is what a step pipeline with C steps in flight would give the rank's compute.
Random-init ResNet-50, uint8 input, bf16. Prints one JSON line per (B, C).

    python scripts/diag_batch_ctx.py [--batches 4,32] [--contexts 1,2,3,4] [--iters 200]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _arg(name, default):
    return sys.argv[sys.argv.index(name) + 1] if name in sys.argv else default


def main():
    import torch
    from hipzap.engine.engine import Engine
    from hipzap.models import registry
    batches = [int(b) for b in _arg("--batches", "4,32").split(",")]
    ctxs = [int(c) for c in _arg("--contexts", "1,2,3,4").split(",")]
    iters = int(_arg("--iters", "200"))
    dev = "cuda:0"
    a = registry.get("resnet50")
    torch.manual_seed(0)
    params, arch_kw = a.pack(a.make_model().eval().state_dict(), dev)
    for b in batches:
        for c in ctxs:
            eng = Engine("resnet50", params, dev, batch=b, num_contexts=c, arch_kw=arch_kw, host_io=False)
            eng.bench(10)
            n = max(20, iters * 4 // b) if b < 16 else iters // 4
            reps = []
            for _ in range(2):
                t = eng.bench(n)
                reps.append(round(b * c * n / t, 1))
            print(json.dumps({"batch": b, "contexts": c, "iters": n, "img_s": reps,
                              "ms_per_replay_each": round(t / n * 1e3, 4)}), flush=True)
            del eng
            torch.cuda.synchronize()


if __name__ == "__main__":
    main()
