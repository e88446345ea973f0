#!/usr/bin/env python3
"""Concurrent ResNet-50 bs=1 request graphs on CU-masked streams (hipExtStreamCreateWithCUMask):
does partitioning the 256 CUs between the ~4 concurrently running request chains (one partition
per hardware queue, optionally XCD-aligned) beat letting every kernel spread over the whole chip?
Replays the captured per-context graphs back to back (device-bound, hz_prog_bench2) on each
stream layout; prints one JSON line per layout."""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hipzap import _native as N  # noqa: E402
from hipzap.engine.engine import Engine  # noqa: E402
from hipzap.models import registry  # noqa: E402
from hipzap.models.resnet import randomize_bn  # noqa: E402

NCU = 256


def masked_stream(cus):
    hip = C.CDLL("libamdhip64.so")
    words = (C.c_uint32 * (NCU // 32))()
    for c in cus:
        words[c // 32] |= 1 << (c % 32)
    s = C.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(C.byref(s), C.c_uint32(NCU // 32), words)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask rc={rc}")
    return s.value


def bench(progs, streams, iters=200):
    n = len(progs)
    P = (C.c_void_p * n)(*progs)
    S = (C.c_void_p * n)(*streams)
    out = (C.c_double * 2)()
    N.check(N.lib().hz_prog_bench2(P, S, n, 10, 0, out), "warm")
    N.check(N.lib().hz_prog_bench2(P, S, n, iters, 0, out), "bench")
    return n * iters / (out[1] * 1e-6)


def main():
    torch.manual_seed(0)
    a = registry.get("resnet50")
    sd = randomize_bn(a.make_model()).eval().state_dict()
    nctx = 16
    eng = Engine.from_state_dict("resnet50", sd, "cuda:0", batch=1, num_contexts=nctx)
    eng.ensure_contexts()
    progs = [c.prog for c in eng.contexts]
    own = [s.cuda_stream for s in eng.streams]
    layouts = {"own_streams_16": own}
    plain4 = [torch.cuda.Stream().cuda_stream for _ in range(4)]
    layouts["plain_4_streams"] = [plain4[i % 4] for i in range(nctx)]
    for name, parts in (("contig_4x64", [range(64 * p, 64 * p + 64) for p in range(4)]),
                        ("stride4", [range(p, NCU, 4) for p in range(4)]),
                        ("stride8_pairs", [[c for c in range(NCU) if (c % 8) // 2 == p] for p in range(4)]),
                        ("contig_2x128", [range(128 * p, 128 * p + 128) for p in range(2)])):
        ss = [masked_stream(list(cus)) for cus in parts]
        layouts[name] = [ss[i % len(ss)] for i in range(nctx)]
    for name, streams in layouts.items():
        r = bench(progs, streams)
        print(json.dumps({"layout": name, "contexts": nctx, "inf_s": round(r, 1)}), flush=True)


if __name__ == "__main__":
    main()
