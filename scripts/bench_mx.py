#!/usr/bin/env python3
"""MX-fp8 GEMM microbenchmark on one MI355X: every MX tile config (csrc/fp8.hip) on the ViT-B/16
fp8 projection shapes at batch 64 (M = 12,608 tokens), timed like the tuner (20 launches per
hipGraph replay, best of 3; random e4m3 operands). One JSON line per shape with us and TF/s per
config.

    python scripts/bench_mx.py [--M 12608] [--cfgs 24,40,43]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hipzap import _native as N  # noqa: E402
from hipzap.engine import tune  # noqa: E402
from hipzap.ops import conv as C  # noqa: E402
from hipzap.ops import fp8 as F8  # noqa: E402

# (name, N, K, mode): mode as the tuner keys it -- ":xs" MX8 input, ":o8" MX8 output
SHAPES = [("qkv", 2304, 768, "fp8"), ("o", 768, 768, "fp8:xs"), ("fc1", 3072, 768, "fp8:o8"),
          ("fc2", 768, 3072, "fp8:xs")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=12608)
    ap.add_argument("--cfgs", default="")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = N.lib()
    g = torch.Generator(device=dev).manual_seed(0)
    want = [int(c) for c in a.cfgs.split(",") if c] or sorted(F8.MX_TILES)
    for name, Nn, K, mode in SHAPES:
        M = a.M
        w = (torch.rand(Nn, K, device=dev, generator=g) - 0.5) * 0.1
        pc = F8.quantize_linear(C.pack_linear(w.float().cpu(), torch.zeros(Nn)))
        pw = F8.PackedFp8(pc.w8.to(dev), pc.sw.to(dev), pc.bias.to(dev), pc.cin, pc.cout, pc.w8mx.to(dev))
        x = torch.randint(0, 120, (M * K,), dtype=torch.uint8, device=dev, generator=g)
        o = torch.empty(M * Nn, dtype=torch.bfloat16, device=dev)
        bufs = [(x, o, o)]
        streams = [torch.cuda.Stream(dev)]
        shape = (pw, (M, 1, 1), M, False, "gelu" if name == "fc1" else "none", False, mode)
        fl = 2.0 * M * Nn * K
        res = {}
        for cfg in want:
            if cfg not in F8.MX_TILES or not F8.mx_fits(cfg, Nn):
                continue
            t = tune._time_candidate(lib, shape, (cfg, 1), bufs, streams, 1)
            res[cfg] = (round(t, 2), round(fl / t / 1e6, 1))
        best = min(res, key=lambda c: res[c][0])
        print(json.dumps({"shape": name, "M": M, "N": Nn, "K": K, "mode": mode, "best_cfg": best,
                          "best_us": res[best][0], "best_tflops": res[best][1],
                          "cfgs": {str(c): {"us": v[0], "tflops": v[1]} for c, v in sorted(res.items())}}), flush=True)


if __name__ == "__main__":
    main()
