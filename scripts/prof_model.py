#!/usr/bin/env python3
"""Run one model's captured forward N times (for `rocprofv3 --kernel-trace --stats`).

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert -o run --output-format csv -- \
        python3 scripts/prof_model.py --model bert-base --batch 16 --iters 20
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hipzap.engine.engine import Engine  # noqa: E402
from hipzap.models import registry  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="bert-base")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    a = registry.get(args.model)
    torch.manual_seed(0)
    m = a.make_model()
    eng = Engine.from_state_dict(args.model, m.state_dict(), "cuda:0", batch=args.batch)
    x = a.example_input(args.batch)
    for _ in range(args.iters):
        eng.infer(x)
    torch.cuda.synchronize()
    print(f"{args.model} bs{args.batch}: {args.iters} forwards, {len(eng.contexts[0].configs)} GEMM/conv launches")


if __name__ == "__main__":
    main()
