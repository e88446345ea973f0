#!/usr/bin/env python3
"""Throughput/latency of the non-headline BASELINE configs on one MI355X (random-init weights,
synthetic inputs): BERT-base seq-cls bs=16 L=128, ViT-B/16 (bf16 / fp8) per-GPU batch 8,
ResNet-50 per-GPU batch 4 (the bs=32 DP=8 config's per-GPU share). One JSON line per config."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hipzap.engine.engine import Engine  # noqa: E402
from hipzap.models import registry  # noqa: E402

CONFIGS = {
    "bert-base": dict(batch=16, unit="seq/s", ref_cpu=24.3),
    "bert-base-fp8": dict(batch=16, unit="seq/s", ref_cpu=24.3),
    "vit-b16": dict(batch=8, unit="img/s", ref_cpu=21.9),
    "vit-b16-fp8": dict(batch=8, unit="img/s", ref_cpu=21.9),
    "resnet50": dict(batch=4, unit="img/s", ref_cpu=27.2),
}


def run(name, batch, contexts, iters=100):
    a = registry.get(name)
    torch.manual_seed(0)
    m = a.make_model()
    if hasattr(m, "layer1"):
        from hipzap.models.resnet import randomize_bn
        randomize_bn(m)
    sd = m.state_dict()
    t0 = time.perf_counter()
    eng = Engine.from_state_dict(name, sd, "cuda:0", batch=batch, num_contexts=contexts)
    x = a.example_input(batch)
    eng.infer(x)
    cold = (time.perf_counter() - t0) * 1e3
    lat = []
    for _ in range(20):
        t = time.perf_counter()
        eng.infer(x)
        lat.append((time.perf_counter() - t) * 1e3)
    lat.sort()
    eng.bench(10)
    secs = eng.bench(iters)
    return {"model": name, "batch": batch, "contexts": contexts, "items_per_s": round(batch * contexts * iters / secs, 1),
            "latency_ms_p50": round(lat[len(lat) // 2], 3), "cold_start_ms": round(cold, 1),
            "ms_per_batch_concurrent": round(secs / iters / contexts * 1e3, 4)}


def torch_reference(name, batch, iters=100):
    """Stock PyTorch on the same GPU: the HF / eager model in bf16 (channels_last for CNNs),
    captured in a CUDA(HIP) graph -> hipBLASLt/MIOpen kernels. Same batch, same inputs."""
    a = registry.get(name)
    torch.manual_seed(0)
    dev = torch.device("cuda:0")
    m = a.make_model().eval().to(device=dev, dtype=torch.bfloat16)
    if name.startswith("bert"):
        ids = torch.randint(1000, 30000, (batch, 128), device=dev)
        fwd = lambda: m(input_ids=ids, attention_mask=torch.ones_like(ids)).logits  # noqa: E731
    elif name.startswith("vit"):
        x = torch.randn(batch, 3, 224, 224, device=dev, dtype=torch.bfloat16)
        fwd = lambda: m(pixel_values=x).logits  # noqa: E731
    else:
        m = m.to(memory_format=torch.channels_last)
        x = torch.randn(batch, 3, 224, 224, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        fwd = lambda: m(x)  # noqa: E731
    s = torch.cuda.Stream(dev)
    with torch.no_grad(), torch.cuda.stream(s):
        for _ in range(3):
            fwd()
    torch.cuda.synchronize(dev)
    g = torch.cuda.CUDAGraph()
    with torch.no_grad(), torch.cuda.graph(g):
        fwd()
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    for _ in range(iters):
        g.replay()
    torch.cuda.synchronize(dev)
    return batch * iters / (time.perf_counter() - t)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    names = args or list(CONFIGS)
    for name in names:
        c = CONFIGS[name]
        if "--torch" in sys.argv and not name.endswith("fp8"):
            try:
                v = torch_reference(name, c["batch"])
                print(json.dumps({"model": name, "batch": c["batch"], "impl": "pytorch-bf16-hipgraph",
                                  "items_per_s": round(v, 1), "unit": c["unit"]}), flush=True)
            except Exception as e:
                print(json.dumps({"model": name, "impl": "pytorch", "error": repr(e)[:300]}), flush=True)
        for ctx in (1, 4):
            try:
                r = run(name, c["batch"], ctx)
                r["unit"] = c["unit"]
                r["vs_sandbox_cpu"] = round(r["items_per_s"] / c["ref_cpu"], 1)
                print(json.dumps(r), flush=True)
            except Exception as e:
                print(json.dumps({"model": name, "contexts": ctx, "error": repr(e)[:300]}), flush=True)


if __name__ == "__main__":
    main()
