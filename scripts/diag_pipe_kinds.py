#!/usr/bin/env python3
"""The DP pipeline's per-rank work at small shards (the DP = 8 shards of configs 3 / 5) with its
contexts on torch's pooled streams vs fresh high-priority streams: ``DPPipeline`` at world 1 with
shard B and depth D, issued from a non-default stream as bench.py does. One JSON line per case.

    python scripts/diag_pipe_kinds.py [--steps 400]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from hipzap.engine.engine import Engine
    from hipzap.models import registry
    from hipzap.parallel.dp import DPPipeline
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 400
    dev = torch.device("cuda:0")
    for model, shard in (("resnet50", 4), ("vit-b16-fp8", 8), ("resnet50", 32)):
        a = registry.get(model)
        torch.manual_seed(0)
        params, arch_kw = a.pack(a.make_model().eval().state_dict(), dev)
        for kind in ("torch", "hiprio", "torch", "hiprio"):
            eng = Engine(model, params, dev, batch=shard, num_contexts=4, arch_kw=arch_kw, host_io=False,
                         stream_kind=kind)
            cin, cout = eng.contexts[0].input, eng.contexts[0].output
            x = (torch.randint(0, 256, (shard,) + tuple(cin.shape[1:]), dtype=torch.uint8, device=dev)
                 if cin.dtype == torch.uint8 else torch.randn((shard,) + tuple(cin.shape[1:]), device=dev).to(cin.dtype))
            pipe = DPPipeline(eng.pipeline_slots(), shard, tuple(cout.shape[1:]), dev, out_dtype=cout.dtype)
            issue = torch.cuda.Stream(dev)
            torch.cuda.synchronize()
            with torch.cuda.stream(issue):
                for _ in range(20):
                    pipe.submit(x)
                pipe.flush()
            torch.cuda.synchronize()
            t = time.perf_counter()
            with torch.cuda.stream(issue):
                for _ in range(steps):
                    pipe.submit(x)
                pipe.flush()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            print(json.dumps({"model": model, "shard": shard, "depth": 4, "kind": kind,
                              "img_s": round(shard * steps / dt, 1)}), flush=True)
            del pipe, eng
            torch.cuda.synchronize()


if __name__ == "__main__":
    main()
