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
from ..ops import fp8 as fp8_ops

TUNING_DIR = Path(__file__).resolve().parent.parent / "tuning"
REPS = 16


def conv_shapes(graph, params) -> dict:
    """key -> (PackedConv, (n,h,w), M, has_residual, act, out_f32, rowmajor) per distinct conv /
    bf16 GEMM shape (GEMM keys carry the ``r`` prefix ExecContext looks up)."""
    out = {}
    for n in graph.nodes:
        if n.kind == "gemm_fp8":
            pw = params[n.attrs["w"]]
            M = n.attrs["rows"]
            mode = "fp8" + (":xs" if graph.tensors[n.inputs[1]].dtype == torch.uint8 else "") + \
                (":o8" if len(n.outputs) == 2 else "")
            out.setdefault(f"f8r{M}x{pw.cout}x{pw.K}", (pw, (M, 1, 1), M, len(n.inputs) > 2,
                                                        n.attrs.get("act", "none"), n.attrs.get("out_f32", False),
                                                        mode))
            continue
        if n.kind == "gemm":
            pc = params[n.attrs["w"]]
            M = n.attrs["rows"]
            out.setdefault("r" + conv_ops.conv_key(M, pc), (pc, (M, 1, 1), M, len(n.inputs) > 1,
                                                            n.attrs.get("act", "none"), n.attrs.get("out_f32", False),
                                                            True))
            continue
        if n.kind != "conv":
            continue
        pc = params[n.attrs["w"]]
        nb, h, w, _ = graph.shape(n.inputs[0])
        p = (h + 2 * pc.pad - pc.r) // pc.stride + 1
        q = (w + 2 * pc.pad - pc.s) // pc.stride + 1
        M = nb * p * q
        out.setdefault(conv_ops.conv_key(M, pc), (pc, (nb, h, w), M, len(n.inputs) > 1, n.attrs.get("act", "relu"),
                                                  n.attrs.get("out_f32", False), False))
    return out


def _capture(lib, prm, cfg, stream):
    prog = lib.hz_prog_create()
    for _ in range(REPS):
        if isinstance(prm, fp8_ops.GemmFp8Params):
            N.check(lib.hz_prog_add_kernel(prog, fp8_ops.K_GEMM_FP8, C.byref(prm), C.sizeof(prm), 0), "add_fp8")
        else:
            N.check(lib.hz_prog_add_conv(prog, C.byref(prm), cfg, 0), "add_conv")
    N.check(lib.hz_prog_capture(prog, stream.cuda_stream), "capture")
    return prog


def _time_candidate(lib, shape, cand, bufs, streams, concurrent: int) -> float:
    """Median-of-3 us per launch; with ``concurrent`` > 1, that many independent copies run
    on separate streams (throughput under request concurrency)."""
    pc, (nb, h, w), M, res, act, out_f32, rowmajor = shape
    cfg, kw = cand
    progs = []
    try:
        for c in range(concurrent):
            x, r, o = bufs[c][:3]
            if str(rowmajor).startswith("fp8"):
                sx = torch.full((M,), 1e-2, device=x.device)
                xs = torch.full((M * pc.K // 32,), 120, dtype=torch.uint8, device=x.device)
                o8 = torch.empty(M * pc.cout, dtype=torch.uint8, device=x.device)
                os8 = torch.empty(M * pc.cout // 32, dtype=torch.uint8, device=x.device)
                bufs[c] = (x, r, o, sx, xs, o8, os8)
                use_xs, use_o8 = ":xs" in rowmajor, ":o8" in rowmajor
                prm = fp8_ops.gemm_params(x.data_ptr(), 0 if use_xs else sx.data_ptr(), pc, M,
                                          0 if use_o8 else o.data_ptr(), r.data_ptr() if res else 0, act, out_f32,
                                          cfg, kw, xs_ptr=xs.data_ptr() if use_xs else 0,
                                          out8_ptr=o8.data_ptr() if use_o8 else 0,
                                          os8_ptr=os8.data_ptr() if use_o8 else 0)
                rc = lib.hz_launch_kernel(fp8_ops.K_GEMM_FP8, C.byref(prm), streams[c].cuda_stream)
            else:
                prm, _, _ = conv_ops.make_params(x.data_ptr(), pc, nb, h, w, o.data_ptr(), r.data_ptr() if res else 0,
                                                 act, out_f32, cfg, kw, out_rowmajor=rowmajor, x_rowmajor=rowmajor)
                rc = lib.hz_conv_launch(C.byref(prm), cfg, streams[c].cuda_stream)
            if rc != 0:
                return float("inf")
            progs.append(_capture(lib, prm, cfg, streams[c]))
        torch.cuda.synchronize()
        best = float("inf")
        for _ in range(3):
            t0 = time.perf_counter()
            for c in range(concurrent):
                lib.hz_prog_replay(progs[c], streams[c].cuda_stream)
            for c in range(concurrent):
                streams[c].synchronize()
            best = min(best, (time.perf_counter() - t0) * 1e6 / (REPS * concurrent))
        return best
    finally:
        for pg in progs:
            lib.hz_prog_destroy(pg)


def tune_graph(graph, params, device, verbose=False, concurrent: int = 1) -> tuple[dict, dict]:
    lib = N.lib()
    dev = torch.device(device)
    table, report = {}, {}
    g = torch.Generator(device=dev).manual_seed(0)
    with torch.cuda.device(dev):
        streams = [torch.cuda.Stream(dev) for _ in range(concurrent)]
        for key, shape in conv_shapes(graph, params).items():
            pc, (nb, h, w), M, res, act, out_f32, rowmajor = shape
            bufs = []
            for _ in range(concurrent):
                if str(rowmajor).startswith("fp8"):
                    x = torch.randint(0, 120, (M * pc.K,), device=dev, dtype=torch.uint8, generator=g)
                else:
                    x = (torch.randn(nb * h * w * pc.cin, device=dev, generator=g) * 0.5).to(torch.bfloat16)
                r = (torch.randn(M * pc.cout, device=dev, generator=g) * 0.5).to(torch.bfloat16)
                o = torch.empty(M * pc.cout, device=dev, dtype=torch.float32 if out_f32 else torch.bfloat16)
                bufs.append((x, r, o))
            times = []
            fp8_mode = str(rowmajor).startswith("fp8")
            cands = (fp8_ops.candidates_fp8(M, pc, mx_io=rowmajor != "fp8") if fp8_mode
                     else conv_ops.candidates(M, pc.cout, pc.K, rowmajor, pc))
            for cand in cands:
                times.append((_time_candidate(lib, shape, cand, bufs, streams, concurrent), cand))
            times.sort()
            best_t, best = times[0]
            heur = (fp8_ops.choose_config_fp8(M, pc, mx_io=rowmajor != "fp8") if fp8_mode
                    else conv_ops.choose_config(M, pc.cout, pc.K, rowmajor=rowmajor, pc=pc))
            heur_t = next((t for t, c in times if tuple(c) == tuple(heur)), None)
            table[key] = list(best)
            report[key] = {"best_us": round(best_t, 2), "best": list(best), "heuristic": list(heur),
                           "heuristic_us": None if heur_t is None else round(heur_t, 2),
                           "top5": [[round(t, 2), list(c)] for t, c in times[:5]]}
            if verbose:
                print(f"{key:28s} best {best_t:7.2f}us {best}  heuristic {heur} {heur_t}", flush=True)
    return table, report


def _time_pair(lib, sa, sb, cand, bufs, stream) -> float:
    """us per grouped launch (conv2_kernel) of two convs sharing (cfg, kw)."""
    cfg, kw = cand
    prms = []
    for (pc, (nb, h, w), M, res, act, out_f32, _), (x, r, o) in zip((sa, sb), bufs):
        prm, _, _ = conv_ops.make_params(x.data_ptr(), pc, nb, h, w, o.data_ptr(), 0, act, out_f32, cfg, kw)
        prms.append(prm)
    if lib.hz_conv2_launch(C.byref(prms[0]), C.byref(prms[1]), cfg, stream.cuda_stream) != 0:
        return float("inf")
    prog = lib.hz_prog_create()
    try:
        for _ in range(REPS):
            N.check(lib.hz_prog_add_conv2(prog, C.byref(prms[0]), C.byref(prms[1]), cfg, 0), "add_conv2")
        N.check(lib.hz_prog_capture(prog, stream.cuda_stream), "capture")
        torch.cuda.synchronize()
        best = float("inf")
        for _ in range(3):
            t0 = time.perf_counter()
            lib.hz_prog_replay(prog, stream.cuda_stream)
            stream.synchronize()
            best = min(best, (time.perf_counter() - t0) * 1e6 / REPS)
        return best
    finally:
        lib.hz_prog_destroy(prog)


def tune_pairs(graph, params, device, verbose=False) -> tuple[dict, dict]:
    """Shared (cfg, kw) for every grouped conv pair ExecContext will launch (program.conv_pairs)."""
    from .program import conv_pairs, pair_key
    lib = N.lib()
    dev = torch.device(device)
    shapes = conv_shapes(graph, params)
    table, report = {}, {}
    g = torch.Generator(device=dev).manual_seed(1)
    stream = torch.cuda.Stream(dev)
    for i, j in conv_pairs(graph).items():
        keys = []
        for n in (graph.nodes[i], graph.nodes[j]):
            pc = params[n.attrs["w"]]
            nb, h, w, _ = graph.shape(n.inputs[0])
            _, p, q, _ = graph.shape(n.outputs[0])
            keys.append(conv_ops.conv_key(nb * p * q, pc))
        key = pair_key(*keys)
        if key in table:
            continue
        sa, sb = shapes[keys[0]], shapes[keys[1]]
        bufs = []
        for (pc, (nb, h, w), M, *_rest) in (sa, sb):
            x = (torch.randn(nb * h * w * pc.cin, device=dev, generator=g) * 0.5).to(torch.bfloat16)
            bufs.append((x, None, torch.empty(M * pc.cout, device=dev, dtype=torch.bfloat16)))
        ca = set(map(tuple, conv_ops.candidates(sa[2], sa[0].cout, sa[0].K)))
        cands = [c for c in conv_ops.candidates(sb[2], sb[0].cout, sb[0].K) if tuple(c) in ca]
        times = sorted((_time_pair(lib, sa, sb, c, bufs, stream), list(c)) for c in cands)
        if not times:
            continue
        table[key] = times[0][1]
        report[key] = {"best_us": round(times[0][0], 2), "best": times[0][1],
                       "top5": [[round(t, 2), c] for t, c in times[:5]]}
        if verbose:
            print(f"{key:60s} best {times[0][0]:7.2f}us {times[0][1]}", flush=True)
    return table, report


def table_path(model: str, batch: int, concurrent: int = 1) -> Path:
    suffix = "" if concurrent <= 1 else f"_c{concurrent}"
    return TUNING_DIR / f"{model}_bs{batch}{suffix}.json"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, nargs="+", default=[1])
    ap.add_argument("--report", default=None)
    ap.add_argument("--concurrent", type=int, nargs="+", default=[1],
                    help="tune for throughput with this many concurrent request streams")
    args = ap.parse_args()
    from ..models import registry
    a = registry.get(args.model)
    dev = torch.device("cuda:0")
    meta, kw = a.meta_params()
    # random weights of the real shapes are enough for timing
    params = {}
    for k, v in meta.items():
        if isinstance(v, fp8_ops.PackedFp8):
            params[k] = fp8_ops.PackedFp8(
                torch.randint(0, 120, v.w8.shape, device=dev, dtype=torch.uint8),
                torch.full(v.sw.shape, 1e-2, device=dev), torch.zeros(v.bias.shape, device=dev), v.cin, v.cout,
                None if v.w8mx is None else torch.randint(0, 120, v.w8mx.shape, device=dev, dtype=torch.uint8))
            continue
        if not isinstance(v, conv_ops.PackedConv):
            continue
        params[k] = conv_ops.PackedConv((torch.randn(v.wf.shape, device=dev) * 0.02).to(torch.bfloat16),
                                        torch.zeros(v.bias.shape, device=dev), v.cin, v.cout, v.r, v.s, v.stride,
                                        v.pad)
    full_report = {}
    for b in args.batch:
        for conc in args.concurrent:
            t0 = time.time()
            graph = a.build_graph(batch=b, **kw)
            table, report = tune_graph(graph, params, dev, verbose=True, concurrent=conc)
            ptable, preport = tune_pairs(graph, params, dev, verbose=True)
            table.update(ptable)
            report.update(preport)
            TUNING_DIR.mkdir(exist_ok=True)
            path = table_path(args.model, b, conc)
            with open(path, "w") as f:
                json.dump(table, f, indent=1, sort_keys=True)
            full_report[f"bs{b}_c{conc}"] = report
            print(f"tuned {args.model} bs{b} concurrent={conc}: {len(table)} shapes in {time.time() - t0:.1f}s -> {path}")
    if args.report:
        os.makedirs(os.path.dirname(args.report) or ".", exist_ok=True)
        with open(args.report, "w") as f:
            json.dump(full_report, f, indent=1)


if __name__ == "__main__":
    main()
