#!/usr/bin/env python3
"""Where the batched AWD-LSTM engine's build time goes (reference dims, V=60000): state_dict ->
device copies, pack_lmb, LMBatchEngine construction (program + capture + scheduler), cold (first
in the process) and warm (second build). One JSON line."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hipzap.engine.lmbatch import LMBatchEngine, pack_lmb  # noqa: E402
from hipzap.models.awd_lstm import reference_lm  # noqa: E402


def build(sd, dev):
    t = {}
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    sdd = {k: v.to(dev, non_blocking=False) for k, v in sd.items()}
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    p = pack_lmb(sdd, dev)
    torch.cuda.synchronize(dev)
    t2 = time.perf_counter()
    eng = LMBatchEngine(p, dev, rows=32, unroll=8)
    torch.cuda.synchronize(dev)
    t3 = time.perf_counter()
    ids = eng.run_tokens([1], 4, seed=0)
    t4 = time.perf_counter()
    t.update(h2d_ms=(t1 - t0) * 1e3, pack_ms=(t2 - t1) * 1e3, engine_ms=(t3 - t2) * 1e3, first_request_4w_ms=(t4 - t3) * 1e3,
             total_ms=(t4 - t0) * 1e3)
    return eng, {k: round(v, 2) for k, v in t.items()}


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    sd = reference_lm(60000).state_dict()
    t_init = time.perf_counter()
    torch.zeros(1, device=dev)
    init_ms = (time.perf_counter() - t_init) * 1e3
    e1, cold = build(sd, dev)
    del e1
    e2, warm = build(sd, dev)
    sd_pin = {k: v.pin_memory() for k, v in sd.items()}
    del e2
    e3, pinned = build(sd_pin, dev)
    print(json.dumps({"torch_cuda_init_ms": round(init_ms, 1), "cold": cold, "warm": warm, "warm_pinned_src": pinned}))


if __name__ == "__main__":
    main()
