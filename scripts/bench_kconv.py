#!/usr/bin/env python3
"""Microbenchmark of the layer3 / layer4 3x3 convs of ResNet-50 at bs=1 (VERDICT r4 #1b): the tuned
register-ring conv (bf16 input), the same kernel on a seam's fp32 accumulator (x_f32), and the
K-split LDS kernel (block.hip kconv_kernel) at each slice width. Each variant: REPS dependent
launches captured in one hipGraph (kernel boundaries included), replayed on 1 stream (latency) and
on 4 concurrent streams (throughput, the served regime); us per launch, best of 5.

    python scripts/bench_kconv.py
"""
import ctypes as C
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from hipzap import _native as N  # noqa: E402
from hipzap.ops import conv as CV  # noqa: E402

REPS = 64
from hipzap.engine.fusion import HZ_K_KCONV, KconvParams  # noqa: E402  (the struct the launcher reads)


def prog_of(add, reps=REPS):
    lib = N.lib()
    p = lib.hz_prog_create()
    for _ in range(reps):
        add(lib, p)
    return p


def timed(progs, streams):
    lib = N.lib()
    for p, s in zip(progs, streams):
        N.check(lib.hz_prog_capture(p, s.cuda_stream), "capture")
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(5):
        t0 = time.perf_counter()
        for p, s in zip(progs, streams):
            lib.hz_prog_replay(p, s.cuda_stream)
        for s in streams:
            s.synchronize()
        best = min(best, (time.perf_counter() - t0) * 1e6 / (REPS * len(progs)))
    return best


def main():
    dev = torch.device("cuda:0")
    for c, h, cks in ((256, 14, (64, 32)), (512, 7, (128, 64))):
        pc = CV.pack_conv(torch.randn(c, c, 3, 3) * (2.0 / (9 * c)) ** 0.5, torch.zeros(c), None, 1, 1).to(dev)
        res = {}
        for conc in (1, 4):
            streams = [torch.cuda.Stream(dev) for _ in range(conc)]
            bufs = [(torch.randn(c // 32, h, h, 32, device=dev), torch.zeros(c // 32, h, h, 32, device=dev),
                     torch.zeros(c * h * h, dtype=torch.bfloat16, device=dev)) for _ in range(conc)]
            variants = {}
            for xf in (0, 1):
                def add_conv(lib, p, i, xf=xf):
                    xb = bufs[i][0] if xf else bufs[i][0].to(torch.bfloat16)
                    bufs[i] = bufs[i] + (xb,)
                    prm, _, _ = CV.make_params(xb.data_ptr(), pc, 1, h, h, bufs[i][2].data_ptr(), 0, "relu", False, 3, 16)
                    prm.x_f32 = xf
                    N.check(lib.hz_prog_add_conv(p, C.byref(prm), 3, 0), "add_conv")
                variants[f"conv_cfg3_kw16{'_f32in' if xf else ''}"] = add_conv
            for ck in cks:
                def add_k(lib, p, i, ck=ck):
                    prm = KconvParams()
                    prm.x, prm.w, prm.out = bufs[i][0].data_ptr(), pc.wf.data_ptr(), bufs[i][1].data_ptr()
                    prm.N, prm.H, prm.W, prm.C, prm.Cout, prm.x_f32, prm.ck = 1, h, h, c, c, 1, ck
                    N.check(lib.hz_prog_add_kernel(p, HZ_K_KCONV, C.byref(prm), C.sizeof(prm), 0), "add_kconv")
                variants[f"kconv_ck{ck}"] = add_k
            for name, add in variants.items():
                progs = [prog_of(lambda lib, p, i=i: add(lib, p, i)) for i in range(conc)]
                res.setdefault(name, {})[f"us_{conc}stream"] = round(timed(progs, streams), 3)
                for p in progs:
                    N.lib().hz_prog_destroy(p)
        print(json.dumps({"shape": f"{h}x{h}x{c}", "variants": res}), flush=True)


if __name__ == "__main__":
    main()
