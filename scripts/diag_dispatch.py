#!/usr/bin/env python3
"""Is ResNet-50 bs=1 serving bound by the GPU's kernel-dispatch rate? Replays S concurrent
hipGraphs of 57 kernels each (no-op kernels, then 1-MB copies with 64 workgroups) and reports the
whole-device dispatch rate next to the ResNet-50 figure (57 dispatches per inference). If no-op
graphs saturate near 57 x 11k = 630k dispatches/s, fusion / fewer launches is the only lever.
Prints one JSON document."""
import ctypes as C
import json
import sys

import torch

sys.path.insert(0, ".")
from hipzap import _native as N  # noqa: E402


def bench2(progs, streams, iters):
    n = len(progs)
    P = (C.c_void_p * n)(*progs)
    S = (C.c_void_p * n)(*[s.cuda_stream for s in streams])
    out = (C.c_double * 2)()
    N.check(N.lib().hz_prog_bench2(P, S, n, iters, 0, out), "bench2")
    return out[0], out[1]


def graphs(kind, S, nk, blocks, nbytes):
    lib = N.lib()
    progs, streams, keep = [], [], []
    for _ in range(S):
        a = torch.zeros(max(nbytes, 16) // 4, dtype=torch.int32, device="cuda")
        b = torch.zeros_like(a)
        keep += [a, b]
        p = lib.hz_prog_create()
        for i in range(nk):
            src, dst = (a, b) if i % 2 == 0 else (b, a)
            N.check(lib.hz_prog_add_diag(p, kind, blocks, 256, src.data_ptr(), dst.data_ptr(), nbytes, 0), "diag")
        s = torch.cuda.Stream()
        N.check(lib.hz_prog_capture(p, s.cuda_stream), "cap")
        progs.append(p)
        streams.append(s)
    bench2(progs, streams, 5)
    iters = 200
    _, tot = bench2(progs, streams, iters)  # tot: us for `iters` rounds of all S graphs
    for p in progs:
        lib.hz_prog_destroy(p)
    rate = S * iters * nk / (tot * 1e-6)
    return {"kind": ["noop", "copy"][kind], "streams": S, "kernels_per_graph": nk, "blocks": blocks,
            "bytes": nbytes, "graphs_per_s": round(S * iters / (tot * 1e-6)), "dispatches_per_s": round(rate)}


def main():
    rows = []
    for S in (1, 2, 4, 8, 16):
        rows.append(graphs(0, S, 57, 64, 0))
        print(json.dumps(rows[-1]), flush=True)
    for S in (1, 4, 16):
        rows.append(graphs(0, S, 57, 512, 0))
        print(json.dumps(rows[-1]), flush=True)
    for S in (1, 4, 16):
        rows.append(graphs(1, S, 57, 64, 1 << 20))
        print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
