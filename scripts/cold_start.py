#!/usr/bin/env python3
"""Cold-start p50 over fresh processes (what a new Lambda container / replica pays).

    python scripts/cold_start.py [model] [trials]

Writes the checkpoint (random-init weights of the real architecture), its packed copy and its
plan image once, untimed (deploy time), then spawns ``trials`` fresh processes per path and
times process spawn -> first logits (hipzap/coldstart.py):
  plan    torch-free: mmap the .hzplan, one DMA of the weights, bind + capture, first request
  hzpack  import torch, packed safetensors straight to the GPU, plan + capture, first request
  pth     import torch, torch.load the state_dict, fold/pack on the GPU, plan + capture, first request
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    model = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
    trials = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    from bench import prepare_artifacts
    ckpt, plan = prepare_artifacts(model, "/tmp/hipzap_bench")
    from hipzap.coldstart import measure_fresh
    out = {"model": model}
    for mode, path in (("plan", plan), ("hzpack", ckpt), ("pth", ckpt)):
        out[mode] = measure_fresh(mode, path, model, trials)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
