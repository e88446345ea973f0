#!/usr/bin/env python3
"""A minimal ResNet-50 bs=1 workload for counter passes: one captured context replayed back to
back on one stream (no request executor, no other queues) -- the TCC (L2) counter passes crashed
rocprofv3 on the bench process (profiles/r6_chain). ``python scripts/pmc_resnet_single.py [iters]``"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from hipzap.engine.engine import Engine
    from hipzap.models import registry
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    a = registry.get("resnet50")
    torch.manual_seed(0)
    params, arch_kw = a.pack(a.make_model().eval().state_dict(), "cuda:0")
    eng = Engine("resnet50", params, "cuda:0", batch=1, num_contexts=1, arch_kw=arch_kw, host_io=False)
    eng.bench(20)
    t = eng.bench(iters)
    print(f"{iters} replays, {t / iters * 1e6:.1f} us each", flush=True)


if __name__ == "__main__":
    main()
