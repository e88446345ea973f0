#!/usr/bin/env python3
"""hipzap headline benchmark: ResNet-50 bs=1 serving throughput (whole node) + cold start.

Metric (BASELINE.json): inferences/sec (whole node) + p50 cold-start ms, ResNet-50 bs=1 at
1/2/4/8 GPU. One process per GPU (torchrun); every rank is a serving replica:
  cold start  rank 0 torch.load()s a standard state_dict checkpoint (random-init weights of
              the real ResNet-50 architecture, written untimed beforehand) -> packs/folds BN
              on its GPU -> RCCL-broadcasts the packed blob to the other ranks -> every rank
              plans its arena, binds native programs, captures hipGraphs -> first inference.
              Also reported: the same from the pre-packed copy (<ckpt>.hzpack, safetensors
              streamed to the GPU: no fold/pack), `cold_start_packed_ms_p50`.
              Only the first request context is built before that first inference; the other
              streams-1 are planned + captured right after it (``deferred_contexts_ms``).
  warm step   every rank serves ``--streams`` (default 32: the peak of the measured
              concurrency sweep, profiles/r1_session5/streams_sweep.md) independent bs=1 requests
              concurrently: each is
              one hipGraph replay that includes the pinned H2D of the fp32 image, preprocess,
              53 fused conv kernels, pools, FC and the D2H of the logits.
Timed region: K steps bracketed by barrier + cuda.synchronize on both sides; the slowest
rank's time is used. value = world * streams * K / t  (weak scaling: fixed work per GPU).
"""
import time

T_PROC0 = time.time()

import argparse  # noqa: E402
import json  # noqa: E402
import os  # noqa: E402
import statistics  # noqa: E402
import sys  # noqa: E402

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "inferences/sec (whole node) + p50 cold-start ms, ResNet-50 bs=1 at 1/2/4/8 GPU"
BASELINE_INF_S = 27.2  # reference execution model (CPU PyTorch in a WSGI handler), ResNet-50 bs=1


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=1, help="per-request batch (headline: 1)")
    ap.add_argument("--streams", type=int, default=int(os.environ.get("HIPZAP_STREAMS", 32)),
                    help="concurrent bs=1 request contexts per GPU")
    ap.add_argument("--ckpt-dir", default=os.environ.get("HIPZAP_BENCH_DIR", "/tmp/hipzap_bench"))
    ap.add_argument("--cold-runs", type=int, default=3, help="extra in-process engine rebuilds for p50")
    ap.add_argument("--compare-torch", action="store_true", help="also time PyTorch/MIOpen bf16 + CUDA graph")
    ap.add_argument("--no-capture", action="store_true")
    ap.add_argument("--tuned", default=None, help="conv tuning table JSON")
    ap.add_argument("--mode", choices=["replica", "scatter"], default="replica",
                    help="replica: independent bs=1 request streams per GPU (headline); scatter: rank 0 scatters "
                         "a global batch over ranks and gathers the logits (configs 3/5)")
    ap.add_argument("--global-batch", type=int, default=32, help="scatter mode: global batch over all ranks")
    ap.add_argument("--input", choices=["uint8", "fp32"], default=os.environ.get("HIPZAP_BENCH_INPUT", "uint8"),
                    help="request payload: uint8 HWC images (decoded-JPEG format, ImageNet mean/std applied on "
                         "device by the preprocess kernel) or pre-normalised fp32 NCHW tensors")
    return ap.parse_args()


def run_scatter(args, rank, world, device, adapter, ckpt):
    """BASELINE configs 3/5: global batch scattered over ranks (RCCL), per-rank hipGraph, logits
    gathered to rank 0. Step = scatter + per-rank forward + gather."""
    from hipzap.engine.engine import Engine
    from hipzap.parallel.comm import broadcast_params, is_dist, max_over_ranks
    from hipzap.parallel.dp import DPExecutor
    shard = args.global_batch // world
    assert shard * world == args.global_batch, "global batch must divide over ranks"
    t0 = time.perf_counter()
    params, arch_kw = (None, None)
    if rank == 0:
        sd = torch.load(ckpt, map_location="cpu", weights_only=True)
        params, arch_kw = adapter.pack({k: v.to(device) for k, v in sd.items()}, device)
    meta, meta_kw = adapter.meta_params()
    params = broadcast_params(params, meta, device)
    eng = Engine(args.model, params, device, batch=shard, num_contexts=1, arch_kw=arch_kw or meta_kw,
                 host_io=False)
    x_in = adapter.example_input(shard)
    in_shape = tuple(eng.contexts[0].input.shape[1:])
    out_shape = tuple(eng.contexts[0].output.shape[1:])
    ex = DPExecutor(lambda xs: eng.infer_device(xs), shard, in_shape, out_shape, device)
    xg = adapter.example_input(args.global_batch).to(device) if rank == 0 else None
    ex.step(xg)
    torch.cuda.synchronize(device)
    cold = (time.perf_counter() - t0) * 1e3
    for _ in range(args.warmup):
        ex.step(xg)
    if is_dist():
        dist.barrier()
    torch.cuda.synchronize(device)
    t1 = time.perf_counter()
    for _ in range(args.steps):
        ex.step(xg)
    torch.cuda.synchronize(device)
    dt = time.perf_counter() - t1
    if is_dist():
        dist.barrier()
    dt = max_over_ranks(dt, device)
    del x_in
    if rank == 0:
        value = args.global_batch * args.steps / dt
        print(json.dumps({
            "metric": f"{args.model} images/s, global batch {args.global_batch} scattered over {world} GPU(s)",
            "value": round(value, 2), "unit": "inferences/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "fp8" if "fp8" in args.model else "bf16",
            "data": "synthetic (random-init weights, random inputs)",
            "config": {"model": args.model, "global_batch": args.global_batch, "seq_len": None,
                       "parallelism": f"dp{world}-scatter-gather"},
            "cold_start_ms": round(cold, 2)}), flush=True)


def write_checkpoint(path, model):
    from hipzap.models import registry
    from hipzap.models.resnet import randomize_bn
    torch.manual_seed(0)
    m = randomize_bn(registry.get(model).make_model()).eval()
    os.makedirs(os.path.dirname(path), exist_ok=True)
    tmp = path + f".tmp{os.getpid()}"
    torch.save(m.state_dict(), tmp)
    os.replace(tmp, path)


def torch_reference_throughput(model, device, iters=200):
    """Stock PyTorch path on the same GPU: bf16 channels_last + CUDA(HIP) graph, bs=1."""
    from hipzap.models import registry
    m = registry.get(model).make_model().eval().to(device=device, dtype=torch.bfloat16)
    m = m.to(memory_format=torch.channels_last)
    x = torch.randn(1, 3, 224, 224, device=device, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    s = torch.cuda.Stream(device)
    with torch.no_grad(), torch.cuda.stream(s):
        for _ in range(5):
            m(x)
    torch.cuda.synchronize(device)
    g = torch.cuda.CUDAGraph()
    with torch.no_grad(), torch.cuda.graph(g):
        y = m(x)
    torch.cuda.synchronize(device)
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize(device)
    t = time.perf_counter()
    for _ in range(iters):
        g.replay()
    torch.cuda.synchronize(device)
    dt = time.perf_counter() - t
    del y
    return iters / dt


def request_input(args, adapter):
    """One request's payload: a decoded uint8 HWC image (default) or an fp32 NCHW tensor."""
    if args.input == "uint8" and args.model.startswith("resnet"):
        return torch.randint(0, 256, (args.batch, 224, 224, 3), dtype=torch.uint8)
    return adapter.example_input(args.batch)


def main():
    args = parse()
    from hipzap.engine.engine import Engine
    from hipzap.models import registry
    from hipzap.parallel.comm import (broadcast_params, env_rank, init_distributed, is_dist, local_device,
                                      max_over_ranks)

    rank, world, local = env_rank()
    device = local_device(local)
    torch.cuda.set_device(device)
    init_distributed(device=device)
    adapter = registry.get(args.model)
    ckpt = os.path.join(args.ckpt_dir, f"{args.model}_seed0.pth")
    if rank == 0 and not os.path.exists(ckpt):
        write_checkpoint(ckpt, args.model)
    tuned = None  # Engine picks hipzap/tuning/<model>_bs<B>[_c<streams>].json
    if args.tuned:
        with open(args.tuned) as f:
            tuned = json.load(f)
    if is_dist():
        dist.barrier()
    if args.mode == "scatter":
        run_scatter(args, rank, world, device, adapter, ckpt)
        if is_dist():
            dist.barrier()
            dist.destroy_process_group()
        return

    def cold_start(packed: str | None = None):
        """``packed``: start from the pre-packed copy of the checkpoint (``<ckpt>.hzpack``, the
        deploy-time artifact of ``hipzap pack``) instead of torch.load + fold/pack."""
        t0 = time.perf_counter()
        timings = {}
        if rank == 0 and packed:
            from hipzap.engine.packfile import load_packed
            ta = time.perf_counter()
            params, arch_kw = load_packed(packed, device)
            torch.cuda.synchronize(device)
            timings["load_packed_ms"] = (time.perf_counter() - ta) * 1e3
        elif rank == 0:
            ta = time.perf_counter()
            sd = torch.load(ckpt, map_location="cpu", weights_only=True, mmap=True)
            timings["load_ms"] = (time.perf_counter() - ta) * 1e3
            ta = time.perf_counter()
            sd = {k: v.to(device, non_blocking=True) for k, v in sd.items()}
            params, arch_kw = adapter.pack(sd, device)
            torch.cuda.synchronize(device)
            timings["pack_ms"] = (time.perf_counter() - ta) * 1e3
        else:
            params, arch_kw = None, None
        if arch_kw is None:  # receiving rank: shapes from a meta-device construction
            meta, arch_kw = adapter.meta_params()
        else:
            meta = None
        arch_kw = dict(arch_kw)
        if args.input == "uint8" and args.model.startswith("resnet"):
            arch_kw["input_uint8"] = True
        ta = time.perf_counter()
        params = broadcast_params(params, meta, device)
        torch.cuda.synchronize(device)
        timings["broadcast_ms"] = (time.perf_counter() - ta) * 1e3
        # zero-copy request IO: the preprocess kernel reads the pinned request bytes and pool_fc writes
        # the pinned logits directly (no copy nodes): +1.7 % single stream, +0.5-1 % at 8 streams
        # (profiles/r1_ab/zero_copy.txt, interleaved on one box)
        eng = Engine(args.model, params, device, batch=args.batch, num_contexts=args.streams,
                     capture=not args.no_capture, tuned=tuned, arch_kw=arch_kw, timings=timings, host_io=True,
                     zero_copy=os.environ.get("HIPZAP_ZERO_COPY", "all"), eager_contexts=1)
        x = request_input(args, adapter)
        out = eng.infer(x)
        cold_ms = (time.perf_counter() - t0) * 1e3
        eng.timings["first_infer_total_ms"] = cold_ms
        return eng, out, cold_ms

    eng, out, cold_first = cold_start()
    cold_process_ms = (time.time() - T_PROC0) * 1e3
    colds = [cold_first]
    for _ in range(args.cold_runs):
        del eng
        torch.cuda.synchronize(device)
        eng, out, c = cold_start()
        colds.append(c)
    assert torch.isfinite(out).all(), "non-finite logits"
    breakdown_pth = dict(eng.timings)
    # packed fast path: rank 0 writes <ckpt>.hzpack once (untimed, as `hipzap pack` would at deploy
    # time), then every rank cold-starts from it
    colds_packed, breakdown_packed = [], {}
    if args.cold_runs:
        from hipzap.engine.packfile import packed_path, save_packed, source_stamp
        pk = packed_path(ckpt)
        if rank == 0:
            params0, kw0 = adapter.pack(torch.load(ckpt, map_location="cpu", weights_only=True), "cpu")
            save_packed(params0, kw0, pk, model=args.model, stamp=source_stamp(ckpt))
        for _ in range(args.cold_runs):
            del eng
            torch.cuda.synchronize(device)
            eng, out, c = cold_start(packed=pk)
            colds_packed.append(c)
        breakdown_packed = dict(eng.timings)
        assert torch.isfinite(out).all(), "non-finite logits (packed path)"

    # the other streams-1 request contexts are planned + captured after the first request was served
    # (a warm container scaling up its concurrency), outside the cold-start figure; reported below
    deferred_ms = eng.ensure_contexts()
    # single-request latency (one context, full round trip incl. host copies), p50
    x = request_input(args, adapter)
    lat = []
    for i in range(210):
        t = time.perf_counter()
        eng.infer(x)
        lat.append((time.perf_counter() - t) * 1e3)
    lat = sorted(lat[10:])
    lat_p50, lat_p99 = statistics.median(lat), lat[min(len(lat) - 1, int(0.99 * len(lat)))]

    # throughput: warmup then K timed steps, each step = `streams` concurrent bs=1 requests
    if args.warmup:
        eng.bench(args.warmup)
    if is_dist():
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    eng.bench(args.steps)
    torch.cuda.synchronize(device)
    dt = time.perf_counter() - t0
    if is_dist():
        dist.barrier()
    dt = max_over_ranks(dt, device)
    inf = world * args.streams * args.batch * args.steps
    value = inf / dt
    torch_ref = None
    if args.compare_torch and rank == 0:
        try:
            torch_ref = torch_reference_throughput(args.model, device)
        except Exception as e:  # comparison only
            print(f"torch reference failed: {e}", file=sys.stderr)
    if rank == 0:
        res = {
            "metric": METRIC, "value": round(value, 2), "unit": "inferences/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": round(value / BASELINE_INF_S, 2), "dtype": "bf16",
            "data": "synthetic (random-init ResNet-50 weights via torch.save/torch.load; "
                    + ("random uint8 224x224x3 images, normalised on device)" if args.input == "uint8"
                       else "random fp32 NCHW images)"),
            "config": {"model": "ResNet-50", "global_batch": args.batch * world, "seq_len": None,
                       "parallelism": f"dp{world}", "request_batch": args.batch,
                       "streams_per_gpu": args.streams, "hipgraph": not args.no_capture},
            "cold_start_ms_p50": round(statistics.median(colds), 2),
            "cold_start_ms_first": round(cold_first, 2),
            "cold_start_process_ms": round(cold_process_ms, 2),
            "cold_start_breakdown_ms": {k: round(v, 2) for k, v in breakdown_pth.items()},
            "cold_start_packed_ms_p50": round(statistics.median(colds_packed), 2) if colds_packed else None,
            "cold_start_packed_breakdown_ms": {k: round(v, 2) for k, v in breakdown_packed.items()},
            "deferred_contexts_ms": round(deferred_ms, 2),
            "latency_ms_p50_single": round(lat_p50, 4),
            "latency_ms_under_load": round(dt / args.steps * 1e3, 4),
            "latency_ms_p99_single": round(lat_p99, 4),
            "baseline_note": "vs_baseline against BASELINE.md sandbox-CPU ResNet-50 bs=1 (27.2 inf/s); "
                             "no published numbers exist",
        }
        if torch_ref is not None:
            res["torch_miopen_graph_inf_s_1gpu_1stream"] = round(torch_ref, 2)
        print(json.dumps(res), flush=True)
    if is_dist():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
