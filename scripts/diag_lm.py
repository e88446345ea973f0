#!/usr/bin/env python3
"""AWD-LSTM decode step, kernel by kernel (V=60000, reference dims): each op of the step
captured alone 50x into one graph and replayed back to back, then the whole step, so the
per-kernel time is measured without the profiler (and with the weights of only that op cycling
through the caches vs the whole step's 181 MB). Prints one JSON document."""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hipzap import _native as N  # noqa: E402
from hipzap.engine.lm import LMEngine  # noqa: E402
from hipzap.models.awd_lstm import reference_lm  # noqa: E402


def timed(build, reps=50, iters=20):
    lib = N.lib()
    s = torch.cuda.Stream()
    prog = lib.hz_prog_create()
    for _ in range(reps):
        build(prog)
    N.check(lib.hz_prog_capture(prog, s.cuda_stream), "capture")
    P = (C.c_void_p * 1)(prog)
    S = (C.c_void_p * 1)(s.cuda_stream)
    out = (C.c_double * 2)()
    N.check(lib.hz_prog_bench2(P, S, 1, 3, 0, out), "warm")
    N.check(lib.hz_prog_bench2(P, S, 1, iters, 0, out), "bench")
    lib.hz_prog_destroy(prog)
    return round(out[1] / iters / reps, 3)


def main():
    V = int(os.environ.get("HIPZAP_LM_VOCAB", 60000))
    torch.manual_seed(0)
    eng = LMEngine.from_state_dict(reference_lm(V).state_dict(), "cuda:0", unroll=1)
    eng.run_tokens([1, 2], 4, 0)
    lib = N.lib()
    ops = eng._ops  # (kind, params) in step order; the sampler is fused into layer 0
    res_final = None if eng._final is None else \
        timed(lambda p: N.check(lib.hz_prog_add_sampler(p, C.byref(eng._final), 0), "final"))
    res = {"V": V, "standalone_argmax_sampler_us": res_final}
    for k, (kind, prm) in enumerate(ops):
        add = {"lstm": lib.hz_prog_add_lstm, "decoder": lib.hz_prog_add_decoder,
               "sampler": lib.hz_prog_add_sampler}[kind]
        res[f"{k}_{kind}_us"] = timed(lambda p, add=add, prm=prm: N.check(add(p, C.byref(prm), 0), kind))

    def step(p):
        for kind, prm in ops:
            add = {"lstm": lib.hz_prog_add_lstm, "decoder": lib.hz_prog_add_decoder,
                   "sampler": lib.hz_prog_add_sampler}[kind]
            N.check(add(p, C.byref(prm), 0), kind)
        N.check(lib.hz_prog_add_step_bump(p, eng.step.data_ptr(), 1, 0), "bump")
    res["step_us"] = timed(step, reps=8)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
