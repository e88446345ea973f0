#!/usr/bin/env python3
"""Is the multi-stream ResNet-50 bs=1 bench host-submission-bound? Replays every context
``iters`` times from one C++ thread and reports the time until the last hipGraphLaunch returned
(submit) vs until every stream drained (total). submit ~= total means the host is the limit."""
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


def main():
    iters = int(os.environ.get("ITERS", 300))
    a = registry.get("resnet50")
    torch.manual_seed(0)
    sd = randomize_bn(a.make_model()).eval().state_dict()
    for streams in (1, 4, 8):
        eng = Engine.from_state_dict("resnet50", sd, "cuda:0", batch=1, num_contexts=streams,
                                     arch_kw={"input_uint8": True, "num_classes": 1000}, host_io=True, zero_copy="all")
        eng.bench(20)
        n = len(eng.contexts)
        progs = (C.c_void_p * n)(*[c.prog for c in eng.contexts])
        strs = (C.c_void_p * n)(*[s.cuda_stream for s in eng.streams])
        for threads in (0, 1):
            out = (C.c_double * 2)()
            rc = N.lib().hz_prog_bench2(progs, strs, n, iters, threads, out)
            assert rc == 0, rc
            print(json.dumps({"streams": streams, "threads": threads, "submit_us_per_replay": round(out[0] / iters / n, 2),
                              "total_us_per_replay": round(out[1] / iters / n, 2),
                              "inf_s": round(n * iters / (out[1] * 1e-6), 1)}), flush=True)
        del eng
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
