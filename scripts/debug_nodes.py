#!/usr/bin/env python3
"""Per-node numerics check of a native program against the fp32 oracle interpreter.

Runs one eager (uncaptured) pass with ``HIPZAP_ARENA_NOREUSE=1`` so every intermediate stays
in its own arena slot, then prints, node by node, the relative error of the device output
against ``engine/reference.run_graph_reference`` on the same input. The first node whose error
jumps is the broken kernel/lowering. fp8 tensors are dequantised first (per-row scales or MX8
E8M0 block scales).

    python scripts/debug_nodes.py --model vit-b16-fp8 --batch 4
"""
import argparse
import os
import sys

os.environ["HIPZAP_ARENA_NOREUSE"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def dequant(g, n, ctx):
    """Device value of node ``n``'s primary output as fp32 (dequantising fp8 outputs)."""
    t0 = n.outputs[0]
    v = ctx.view(t0).cpu()
    if v.dtype != torch.uint8:
        return v.float()
    f = v.view(torch.float8_e4m3fn).float()
    s = ctx.view(n.outputs[1]).cpu()
    if s.dtype == torch.float32:  # per-row scales
        return f * s.reshape(-1, 1)
    e = s.to(torch.int32) - 127  # MX8: E8M0 per 32 columns
    sc = torch.ldexp(torch.ones_like(e, dtype=torch.float32), e)
    return (f.reshape(f.shape[0], -1, 32) * sc.unsqueeze(-1)).reshape(f.shape)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="vit-b16-fp8")
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--device", default="cuda:0")
    args = ap.parse_args()
    from hipzap.engine.engine import Engine
    from hipzap.engine.reference import run_graph_reference
    from hipzap.models import registry
    torch.manual_seed(0)
    ad = registry.get(args.model)
    m = ad.make_model()
    sd = m.state_dict()
    eng = Engine.from_state_dict(args.model, sd, args.device, batch=args.batch, capture=False)
    g = eng.graph
    ctx = eng.contexts[0]
    x0 = ad.example_input(args.batch)
    xs = list(x0) if isinstance(x0, (tuple, list)) else [x0]
    for i, (t, x) in enumerate(zip(g.inputs, xs)):
        dst = ctx.host_inputs[i] if ctx.host_io else ctx.ext[t]  # host_io: the program H2D-copies first
        dst.copy_(x.reshape(dst.shape))
    ctx.run()
    torch.cuda.synchronize()
    params_cpu = ad.pack(sd, "cpu")[0]
    ref = run_graph_reference(g, params_cpu, [x.cpu() for x in xs])
    for i, n in enumerate(g.nodes):
        if n.kind in ("fork", "join"):
            continue
        dev = dequant(g, n, ctx).reshape(-1)
        r = ref[n.outputs[0]].float().reshape(-1)
        if dev.numel() != r.numel():
            print(f"{i:4d} {n.kind:10s} {n.attrs.get('name', '')!s:14s} size mismatch {dev.numel()} vs {r.numel()}")
            continue
        rel = ((dev - r).abs().max() / r.abs().max().clamp_min(1e-12)).item()
        cos = torch.nn.functional.cosine_similarity(dev, r, dim=0).item()
        flag = "  <-- " if rel > 0.1 else ""
        print(f"{i:4d} {n.kind:10s} {str(n.attrs.get('name', n.attrs.get('w', ''))):14s} rel {rel:.3e} cos {cos:.5f}{flag}",
              flush=True)


if __name__ == "__main__":
    main()
