"""Where the persistent conv chain (csrc/conv.hip conv_chain_kernel) spends its time.

Builds ResNet-50 bs=1 contexts with HIPZAP_CONV_CHAIN=<prefix> for each (prefix, grid, cfg)
configuration given, times single-stream graph replays with events against the per-conv
program, and decodes one traced replay (HIPZAP_CHAIN_TRACE=1: s_memrealtime stamps per workgroup
and stage) into per-stage hand-off latency (last producer done -> first consumer released) and
tile time. Prints one JSON line per configuration.

  python scripts/diag_chain.py layer3:128 layer3:256 layer3:128:3 layer4:64
"""
import json
import os
import sys

import torch

from hipzap.engine.program import ExecContext
from hipzap.models import registry
from hipzap.models.resnet import randomize_bn

DEV = torch.device("cuda:0")


def build(a, params, kw, prefix, grid, cfg, trace):
    for k in ("HIPZAP_CONV_CHAIN", "HIPZAP_CHAIN_GRID", "HIPZAP_CHAIN_CFG", "HIPZAP_CHAIN_TRACE"):
        os.environ.pop(k, None)
    if prefix:
        os.environ["HIPZAP_CONV_CHAIN"] = prefix
        os.environ["HIPZAP_CHAIN_GRID"] = str(grid)
        if cfg is not None:
            os.environ["HIPZAP_CHAIN_CFG"] = str(cfg)
        if trace:
            os.environ["HIPZAP_CHAIN_TRACE"] = "1"
    ctx = ExecContext(a.build_graph(batch=1, **kw), params, DEV)
    s = torch.cuda.Stream()
    ctx.capture(s)
    return ctx, s


def time_replays(ctx, s, n=300):
    for _ in range(30):
        ctx.replay(s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(s)
    for _ in range(n):
        ctx.replay(s)
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n  # us per replay


def decode(ctx):
    tr = ctx.chain_trace.cpu().numpy().astype("float64") / 100.0  # 100 MHz -> us
    info = ctx.chain_info
    G, S = tr.shape[0], tr.shape[1]
    rows, prev_end = [], None
    t0 = None
    for s in range(S):
        act = [b for b in range(min(G, info["stage_tiles"][s])) if tr[b, s, 2] > 0]
        t_in = [tr[b, s, 0] for b in act]
        t_rel = [tr[b, s, 1] for b in act]
        t_done = [tr[b, s, 2] for b in act]
        if t0 is None:
            t0 = min(t_in)
        end = max(t_done)
        tile = sorted(t_done[i] - t_rel[i] for i in range(len(act)))
        rows.append({"stage": s, "tiles": info["stage_tiles"][s], "wgs": len(act),
                     "handoff_us": round(min(t_rel) - prev_end, 2) if prev_end is not None else None,
                     "release_skew_us": round(max(t_rel) - min(t_rel), 2),
                     "tile_med_us": round(tile[len(tile) // 2], 2), "tile_max_us": round(tile[-1], 2),
                     "stage_us": round(end - (prev_end if prev_end is not None else min(t_rel)), 2)})
        prev_end = end
    return rows, round(prev_end - t0, 2)


def main():
    torch.manual_seed(0)
    a = registry.get("resnet50")
    sd = randomize_bn(a.make_model()).eval().state_dict()
    params, kw = a.pack({k: v.to(DEV) for k, v in sd.items()}, DEV)
    base, sb = build(a, params, kw, None, 0, None, False)
    t_base = time_replays(base, sb)
    print(json.dumps({"config": "per-conv launches", "us_per_replay": round(t_base, 1)}), flush=True)
    for spec in sys.argv[1:]:
        parts = spec.split(":")
        prefix, grid = parts[0], int(parts[1]) if len(parts) > 1 else 128
        cfg = int(parts[2]) if len(parts) > 2 else None
        ctx, s = build(a, params, kw, prefix, grid, cfg, False)
        t = time_replays(ctx, s)
        tctx, ts = build(a, params, kw, prefix, grid, cfg, True)
        time_replays(tctx, ts, 5)
        rows, chain_us = decode(tctx)
        print(json.dumps({"config": spec, "us_per_replay": round(t, 1), "delta_us": round(t - t_base, 1),
                          "chain_us_traced": chain_us, "err": ctx.chain_error(), "info": ctx.chain_info,
                          "stages": rows}), flush=True)
        del ctx, tctx


if __name__ == "__main__":
    main()
