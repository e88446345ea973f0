"""Sweep the dynamic-batching executor (replay batch B x contexts K x closed-loop clients C x
max wait) on ResNet-50 with random weights; one JSON line per point (profiles/r2_dyn_batch)."""
import argparse
import json
import time

import torch

from hipzap.engine.engine import Engine
from hipzap.models import registry
from hipzap.models.resnet import randomize_bn


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", nargs="+", default=["8,4,32,200", "8,6,48,200", "8,8,64,200", "16,4,64,200",
                                                      "16,6,96,200", "8,6,48,50", "8,6,48,1000"])
    ap.add_argument("--iters", type=int, default=150)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    a = registry.get("resnet50")
    sd = randomize_bn(a.make_model()).eval().state_dict()
    params, kw = a.pack({k: v.to(dev) for k, v in sd.items()}, dev)
    kw = dict(kw, input_uint8=True)
    engines = {}
    for pt in args.points:
        B, K, Cc, wait = (float(v) for v in pt.split(","))
        B, K, Cc = int(B), int(K), int(Cc)
        if (B, K) not in engines:
            engines.clear()
            engines[(B, K)] = Engine("resnet50", params, dev, batch=B, num_contexts=K, arch_kw=kw, zero_copy="all")
        eng = engines[(B, K)]
        eng._bexec = None
        ex = eng.batched_executor(max_wait_us=wait)
        row = (torch.rand(ex.in_bytes[0]) * 255).to(torch.uint8)
        ex.bench(Cc, 20, [row.data_ptr()])
        s0 = ex.stats()
        t = time.perf_counter()
        wall, lat = ex.bench(Cc, args.iters, [row.data_ptr()])
        s1 = ex.stats()
        lat = sorted(lat)
        print(json.dumps({"replay_batch": B, "contexts": K, "clients": Cc, "max_wait_us": wait,
                          "inf_s": round(Cc * args.iters / wall, 1),
                          "mean_rows": round((s1["served"] - s0["served"]) / max(1, s1["batches"] - s0["batches"]), 2),
                          "p50_ms": round(lat[len(lat) // 2], 3), "p99_ms": round(lat[int(0.99 * (len(lat) - 1))], 3),
                          "wall_s": round(time.perf_counter() - t, 2)}), flush=True)
        ex.close()


if __name__ == "__main__":
    main()
