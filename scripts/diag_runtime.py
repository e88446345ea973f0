#!/usr/bin/env python3
"""Measure the runtime floor on MI355X: per-kernel cost inside hipGraphs (no-op and 1 MB copy
chains), host submission cost of graph replays, and ResNet-50 bs=1 throughput vs the number
of concurrent contexts / side streams / submitting threads. Prints one JSON document."""
import ctypes as C
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from hipzap import _native as N  # noqa: E402
from hipzap.engine.engine import Engine  # noqa: E402
from hipzap.models import registry  # noqa: E402
from hipzap.models.resnet import randomize_bn  # noqa: E402


def bench2(progs, streams, iters, threads=0):
    n = len(progs)
    P = (C.c_void_p * n)(*progs)
    S = (C.c_void_p * n)(*[s.cuda_stream for s in streams])
    out = (C.c_double * 2)()
    N.check(N.lib().hz_prog_bench2(P, S, n, iters, threads, out), "bench2")
    return out[0], out[1]


def chain(kind, nk, blocks, nbytes):
    lib = N.lib()
    a = torch.zeros(max(nbytes, 16) // 4, dtype=torch.int32, device="cuda")
    b = torch.zeros_like(a)
    prog = lib.hz_prog_create()
    for i in range(nk):
        src, dst = (a, b) if i % 2 == 0 else (b, a)
        N.check(lib.hz_prog_add_diag(prog, kind, blocks, 256, src.data_ptr(), dst.data_ptr(), nbytes, 0), "diag")
    s = torch.cuda.Stream()
    N.check(lib.hz_prog_capture(prog, s.cuda_stream), "cap")
    bench2([prog], [s], 5)
    host, tot = bench2([prog], [s], 50)
    res = {"kernels": nk, "blocks": blocks, "bytes": nbytes, "us_per_kernel": tot / 50 / nk,
           "host_us_per_replay": host / 50}
    lib.hz_prog_destroy(prog)
    return res


def main():
    out = {"device": torch.cuda.get_device_name(0)}
    out["noop_256wg"] = chain(0, 50, 256, 0)
    out["noop_1wg"] = chain(0, 50, 1, 0)
    out["copy_1MB_512wg"] = chain(1, 50, 512, 1 << 20)
    out["copy_4MB_1024wg"] = chain(1, 50, 1024, 4 << 20)
    torch.manual_seed(0)
    a = registry.get("resnet50")
    sd = randomize_bn(a.make_model()).eval().state_dict()
    params, kw = a.pack({k: v.cuda() for k, v in sd.items()}, torch.device("cuda:0"))
    rows = []
    for side in (True, False):
        for S in (1, 2, 4, 8):
            eng = Engine("resnet50", params, "cuda:0", batch=1, num_contexts=S,
                         arch_kw=dict(kw, side_stream=side), host_io=True)
            progs = [c.prog for c in eng.contexts]
            for threads in (0, 1) if S > 1 else (0,):
                bench2(progs, eng.streams, 10, threads)
                iters = 200
                host, tot = bench2(progs, eng.streams, iters, threads)
                rows.append({"side_stream": side, "contexts": S, "threads": threads,
                             "inf_per_s": round(S * iters / tot * 1e6, 1),
                             "host_us_per_replay": round(host / (S * iters), 2),
                             "us_per_inf": round(tot / (S * iters), 2)})
                print(rows[-1], flush=True)
            del eng
    out["resnet50"] = rows
    print(json.dumps(out))


if __name__ == "__main__":
    main()
