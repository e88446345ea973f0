"""On-device autotuner for the conv/GEMM launch configuration of a lowered graph.

For every distinct conv shape in a :class:`Graph`, each legal launch choice
``(cfg, splitk, kw)`` (``ops.conv.candidates``) is timed the way it will run in
production: ``REPS`` dependent launches captured in a hipGraph and replayed, so the number
includes kernel-boundary cost and excludes host launch overhead. The winner per shape is
written to a JSON table (``hipzap/tuning/<model>_bs<N>.json``) that ``ExecContext`` /
``choose_config`` consult at cold start, so tuning is paid once per (model, batch), never
on the serving path.

    python -m hipzap.engine.tune --model resnet50 --batch 1
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import time
from pathlib import Path

import torch

from .. import _native as N
from ..ops import conv as conv_ops

TUNING_DIR = Path(__file__).resolve().parent.parent / "tuning"
REPS = 16


def conv_shapes(graph, params) -> dict:
    """key -> (node, PackedConv, (n,h,w), M) for each distinct conv shape."""
    out = {}
    for n in graph.nodes:
        if n.kind != "conv":
            continue
        pc = params[n.attrs["w"]]
        nb, h, w, _ = graph.shape(n.inputs[0])
        p = (h + 2 * pc.pad - pc.r) // pc.stride + 1
        q = (w + 2 * pc.pad - pc.s) // pc.stride + 1
        M = nb * p * q
        key = f"{M}x{pc.cout}x{pc.K}x{pc.r}{pc.s}s{pc.stride}"
        res = len(n.inputs) > 1
        out.setdefault(key, (n, pc, (nb, h, w), M, res, n.attrs.get("act", "relu"), n.attrs.get("out_f32", False)))
    return out


def _time_candidate(lib, pc, nhw, M, res, act, out_f32, cand, bufs, stream) -> float:
    cfg, splitk, kw = cand
    nb, h, w = nhw
    x, r, o = bufs
    wsb, ncnt = conv_ops.workspace_bytes(M, pc.cout, cfg, splitk)
    ws = torch.empty(max(wsb, 256), dtype=torch.uint8, device=x.device)
    cnt = torch.zeros(max(ncnt, 64), dtype=torch.int32, device=x.device)
    prm, _, _ = conv_ops.make_params(x.data_ptr(), pc, nb, h, w, o.data_ptr(), r.data_ptr() if res else 0, act,
                                     out_f32, cfg, splitk, ws.data_ptr(), cnt.data_ptr(), kw=kw)
    rc = lib.hz_conv_launch(C.byref(prm), cfg, stream.cuda_stream)
    if rc != 0:
        return float("inf")
    prog = lib.hz_prog_create()
    try:
        for _ in range(REPS):
            N.check(lib.hz_prog_add_conv(prog, C.byref(prm), cfg, 0), "add_conv")
        N.check(lib.hz_prog_capture(prog, stream.cuda_stream), "capture")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(stream):
            lib.hz_prog_replay(prog, stream.cuda_stream)
            best = float("inf")
            for _ in range(3):
                e0.record(stream)
                lib.hz_prog_replay(prog, stream.cuda_stream)
                e1.record(stream)
                e1.synchronize()
                best = min(best, e0.elapsed_time(e1) * 1e3 / REPS)
        return best
    finally:
        lib.hz_prog_destroy(prog)
        del ws, cnt


def tune_graph(graph, params, device, verbose=False, max_candidates=None) -> tuple[dict, dict]:
    lib = N.lib()
    dev = torch.device(device)
    stream = torch.cuda.Stream(dev)
    table, report = {}, {}
    g = torch.Generator(device=dev).manual_seed(0)
    with torch.cuda.device(dev):
        for key, (node, pc, nhw, M, res, act, out_f32) in conv_shapes(graph, params).items():
            nb, h, w = nhw
            x = (torch.randn(nb, h, w, pc.cin, device=dev, generator=g) * 0.5).to(torch.bfloat16)
            r = (torch.randn(M, pc.cout, device=dev, generator=g) * 0.5).to(torch.bfloat16)
            o = torch.empty(M, pc.cout, device=dev, dtype=torch.float32 if out_f32 else torch.bfloat16)
            cands = conv_ops.candidates(M, pc.cout, pc.K)
            if max_candidates:
                cands = cands[:max_candidates]
            times = []
            for cand in cands:
                t = _time_candidate(lib, pc, nhw, M, res, act, out_f32, cand, (x, r, o), stream)
                times.append((t, cand))
            times.sort()
            best_t, best = times[0]
            heur = conv_ops.choose_config(M, pc.cout, pc.K)
            heur_t = next((t for t, c in times if tuple(c) == tuple(heur)), None)
            table[key] = list(best)
            report[key] = {"best_us": round(best_t, 2), "best": list(best), "heuristic": list(heur),
                           "heuristic_us": None if heur_t is None else round(heur_t, 2),
                           "top5": [[round(t, 2), list(c)] for t, c in times[:5]]}
            if verbose:
                print(f"{key:28s} best {best_t:7.2f}us {best}  heuristic {heur} {heur_t}", flush=True)
    return table, report


def table_path(model: str, batch: int) -> Path:
    return TUNING_DIR / f"{model}_bs{batch}.json"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, nargs="+", default=[1])
    ap.add_argument("--report", default=None)
    args = ap.parse_args()
    from ..models import registry
    a = registry.get(args.model)
    dev = torch.device("cuda:0")
    meta, kw = a.meta_params()
    # random weights of the real shapes are enough for timing
    params = {}
    for k, v in meta.items():
        params[k] = conv_ops.PackedConv((torch.randn(v.w.shape, device=dev) * 0.02).to(torch.bfloat16),
                                        torch.zeros(v.bias.shape, device=dev), v.cin, v.cout, v.r, v.s, v.stride,
                                        v.pad)
    full_report = {}
    for b in args.batch:
        t0 = time.time()
        graph = a.build_graph(batch=b, **kw)
        table, report = tune_graph(graph, params, dev, verbose=True)
        TUNING_DIR.mkdir(exist_ok=True)
        with open(table_path(args.model, b), "w") as f:
            json.dump(table, f, indent=1, sort_keys=True)
        full_report[f"bs{b}"] = report
        print(f"tuned {args.model} bs{b}: {len(table)} shapes in {time.time() - t0:.1f}s -> {table_path(args.model, b)}")
    if args.report:
        os.makedirs(os.path.dirname(args.report) or ".", exist_ok=True)
        with open(args.report, "w") as f:
            json.dump(full_report, f, indent=1)


if __name__ == "__main__":
    main()
