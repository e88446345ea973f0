#!/usr/bin/env python3
"""GEMM microbenchmark on one MI355X: hipzap's GEMM kernels (every legal launch config, timed
inside hipGraphs like the tuner does) vs torch.matmul (hipBLASLt) on the BERT-base / ViT-B/16
projection shapes. Prints one JSON line per shape with µs and TFLOP/s (random bf16 operands)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hipzap.engine import tune  # noqa: E402
from hipzap import _native as N  # noqa: E402
from hipzap.ops import conv as C  # noqa: E402

SHAPES = [  # (M, N, K): BERT bs16 L128 and ViT-B/16 bs8
    (2048, 2304, 768), (2048, 768, 768), (2048, 3072, 768), (2048, 768, 3072),
    (1576, 2304, 768), (1576, 768, 768), (1576, 3072, 768), (1576, 768, 3072),
    (4096, 4096, 4096),
]


def time_torch(x, w, reps=20):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            torch.matmul(x, w.t())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                torch.matmul(x, w.t())
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(5):
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) * 1e6 / reps)
    return best


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default=None, help="M,N,K;M,N,K;... (default: the BERT / ViT projections)")
    a = ap.parse_args()
    shapes = [tuple(int(v) for v in t.split(",")) for t in a.shapes.split(";")] if a.shapes else SHAPES
    dev = torch.device("cuda:0")
    lib = N.lib()
    gen = torch.Generator(device=dev).manual_seed(0)
    for M, Nn, K in shapes:
        w = (torch.rand(Nn, K, device=dev, generator=gen) - 0.5).to(torch.bfloat16)
        x = (torch.rand(M, K, device=dev, generator=gen) - 0.5).to(torch.bfloat16)
        t_torch = time_torch(x, w)
        pc = C.pack_linear(w.float(), torch.zeros(Nn, device=dev))
        shape = (pc, (M, 1, 1), M, False, "none", False, True)
        o = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
        bufs = [(x.reshape(-1), o.reshape(-1), o.reshape(-1))]
        streams = [torch.cuda.Stream(dev)]
        res = []
        for cand in C.candidates(M, Nn, K, True, pc):
            t = tune._time_candidate(lib, shape, cand, bufs, streams, 1)
            res.append((t, list(cand)))
        res.sort()
        fl = 2.0 * M * Nn * K
        print(json.dumps({"M": M, "N": Nn, "K": K, "hipblaslt_us": round(t_torch, 2),
                          "hipblaslt_tflops": round(fl / t_torch / 1e6, 1), "hipzap_us": round(res[0][0], 2),
                          "hipzap_tflops": round(fl / res[0][0] / 1e6, 1), "hipzap_cfg": res[0][1],
                          "lds_cfgs": {str(c[0]): round(t, 2) for t, c in res if c[0] >= 16}}), flush=True)


if __name__ == "__main__":
    main()
