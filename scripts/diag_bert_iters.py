#!/usr/bin/env python3
"""BERT-base bs16 L128 (config 4): seq/s of C concurrent contexts against the length of the timed
window (``Engine.bench(iters)``: iters replays of every context, synchronised). A rate that falls
as the window grows is the chip slowing under sustained load (power / clocks), not a code path:
round 5 quoted 4 contexts over 100 replays, bench_configs.py times 200.

    python scripts/diag_bert_iters.py [--contexts 1,4] [--iters 25,50,100,200,400,800]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _arg(name, default):
    return sys.argv[sys.argv.index(name) + 1] if name in sys.argv else default


def main():
    import torch
    from hipzap.engine.engine import Engine
    from hipzap.models import registry
    ctxs = [int(c) for c in _arg("--contexts", "1,4").split(",")]
    iters = [int(i) for i in _arg("--iters", "25,50,100,200,400,800").split(",")]
    a = registry.get("bert-base")
    torch.manual_seed(0)
    sd = a.make_model().eval().state_dict()
    mode = _arg("--mode", "")
    if mode:  # process-state probe: one 4-context figure after a given history (run each in a fresh process)
        if mode.startswith("after1"):
            e1 = Engine.from_state_dict("bert-base", sd, "cuda:0", batch=16, num_contexts=1)
            e1.bench(20)
            del e1
            torch.cuda.synchronize()
        eng = Engine.from_state_dict("bert-base", sd, "cuda:0", batch=16, num_contexts=4)
        if mode.endswith("infer"):
            x = a.example_input(16)
            for _ in range(21):
                eng.infer(x)
        eng.bench(10)
        rates = []
        for _ in range(3):
            t = eng.bench(200)
            rates.append(round(16 * 4 * 200 / t, 1))
        print(json.dumps({"mode": mode, "contexts": 4, "seq_s": rates}), flush=True)
        return
    for c in ctxs:
        eng = Engine.from_state_dict("bert-base", sd, "cuda:0", batch=16, num_contexts=c)
        eng.bench(10)
        for rep in range(2):
            for n in iters:
                time.sleep(1.0)  # an idle second before each window
                t = eng.bench(n)
                print(json.dumps({"contexts": c, "iters": n, "rep": rep, "window_ms": round(t * 1e3, 1),
                                  "seq_s": round(16 * c * n / t, 1)}), flush=True)
        del eng
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
