#!/usr/bin/env python3
"""BERT-base bs16 seq/s against the number of request contexts and their stream kind
(``Engine(..., stream_kind=...)``: torch's pool vs fresh high-priority streams), each engine
built fresh in this process in turn. One JSON line per (contexts, kind).

    python scripts/diag_ctx_kinds.py [--contexts 2,3,4,6,8] [--kinds torch,hiprio]
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
    ctxs = [int(c) for c in _arg("--contexts", "2,3,4,6,8").split(",")]
    kinds = _arg("--kinds", "torch,hiprio").split(",")
    a = registry.get("bert-base")
    torch.manual_seed(0)
    params, arch_kw = a.pack(a.make_model().eval().state_dict(), "cuda:0")
    for c in ctxs:
        for k in kinds:
            eng = Engine("bert-base", params, "cuda:0", batch=16, num_contexts=c, arch_kw=arch_kw, stream_kind=k)
            eng.bench(10)
            rates = [round(16 * c * 200 / eng.bench(200), 1) for _ in range(2)]
            print(json.dumps({"contexts": c, "kind": k, "seq_s": rates}), flush=True)
            del eng
            torch.cuda.synchronize()


if __name__ == "__main__":
    main()
