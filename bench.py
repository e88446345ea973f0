#!/usr/bin/env python3
"""hipzap headline benchmark: ResNet-50 bs=1 serving throughput (whole node) + cold start.

Metric (BASELINE.json): inferences/sec (whole node) + p50 cold-start ms, ResNet-50 bs=1 at
1/2/4/8 GPU. One process per GPU (torchrun); every rank is a serving replica.

cold start (headline ``cold_start_ms_p50``): measured FIRST, before this process touches a GPU,
  as the p50 over ``--cold-trials`` FRESH child processes of spawn -> first logits
  (hipzap/coldstart.py) from the deploy artifact a serverless replica starts from: the
  ``.hzplan`` plan image (torch-free: mmap, one DMA of the packed weights, bind, hipGraph
  capture, one bs=1 request). ``cold_start_pth_ms_p50``: the same from the ``.pth``
  state_dict (import torch, torch.load, fold/pack on the GPU). Artifacts (random-init weights
  of the real ResNet-50 architecture, their plan image) are written untimed beforehand, on the
  CPU, as ``hipzap plan`` does at deploy time. In-process rebuilds inside this warm process are
  reported separately (``cold_start_inprocess_*``).
warm path: every rank serves ``--streams`` (default 12: the rate of 16-24 streams at three quarters of the 16-stream latency under load, profiles/r6_final/streams_dyn_sweep_s20.txt)
  concurrent bs=1 request streams; each request is one hipGraph replay (zero-copy pinned uint8
  image -> preprocess -> 37 kernels: conv+maxpool, fused layer1/layer2 bottlenecks, layer3/layer4 convs -> pool+FC -> logits in pinned memory).
  ``--serve executor`` (default): one native client thread per stream sends requests back to
  back through the request executor (csrc/executor.cpp, the serving path of Engine.infer):
  payload copied into a pinned input, one replay, the client sleeps until ITS result is done,
  logits copied out — throughput and p50/p99 latency are what concurrent clients see.
  ``--serve pipelined``: replays queued back to back without host work (device-bound ceiling,
  always reported too).
Timed region: K steps bracketed by barrier + cuda.synchronize on both sides; one step = ``--step-requests``
(default 32) back-to-back requests on EVERY stream, so the driver's ``--steps 20`` covers ~0.75 s of
serving rather than ~25 ms; the slowest rank's time is used.
value = world * streams * step_requests * K / t (weak scaling).
"""
import time

T_PROC0 = time.time()

import argparse  # noqa: E402
import json  # noqa: E402
import os  # noqa: E402
import statistics  # noqa: E402
import sys  # noqa: E402

# torch (which maps libamdhip64) is imported by the rank processes only, after the launch decision:
# the N-rank launcher counts GPUs from the KFD topology and spawns the ranks without ever mapping or
# initialising HIP
torch = dist = None


def _import_torch():
    global torch, dist
    import torch as _torch
    import torch.distributed as _dist
    torch, dist = _torch, _dist

METRIC = "inferences/sec (whole node) + p50 cold-start ms, ResNet-50 bs=1 at 1/2/4/8 GPU"
BASELINE_INF_S = 27.2  # reference execution model (CPU PyTorch in a WSGI handler), ResNet-50 bs=1


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--step-requests", type=int, default=int(os.environ.get("HIPZAP_STEP_REQUESTS", 32)),
                    help="requests per stream in one timed step (replica mode)")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=1, help="per-request batch (headline: 1)")
    ap.add_argument("--streams", type=int, default=int(os.environ.get("HIPZAP_STREAMS", 12)),
                    help="concurrent bs=1 request contexts per GPU (12: the 16-24 rate, 14.24-14.35k, at p50 0.83 ms under "
                         "load vs 1.11 at 16, profiles/r6_final/streams_dyn_sweep_s20.txt)")
    ap.add_argument("--ckpt-dir", default=os.environ.get("HIPZAP_BENCH_DIR", "/tmp/hipzap_bench"))
    ap.add_argument("--cold-trials", type=int, default=int(os.environ.get("HIPZAP_COLD_TRIALS", 15)),
                    help="fresh processes per cold-start path (0: skip)")
    ap.add_argument("--cold-runs", type=int, default=3, help="extra in-process engine rebuilds (secondary figure)")
    ap.add_argument("--serve", choices=["executor", "threads", "pipelined"], default="executor",
                    help="executor: closed-loop clients through the native request executor (headline); "
                         "threads: every client thread launches + synchronises its own context; "
                         "pipelined: replays queued back to back, no host work (device ceiling)")
    ap.add_argument("--compare-torch", action="store_true", help="also time PyTorch/MIOpen bf16 + CUDA graph")
    ap.add_argument("--no-capture", action="store_true")
    ap.add_argument("--dyn-batch", type=int, default=16,
                    help="secondary figure: the same bs=1 requests served with dynamic batching into replays "
                         "of this batch (0: skip)")
    ap.add_argument("--dyn-contexts", type=int, default=6)
    ap.add_argument("--dyn-clients", type=int, default=96)
    ap.add_argument("--dyn-wait-us", type=float, default=200.0)
    ap.add_argument("--tuned", default=None, help="conv tuning table JSON")
    ap.add_argument("--http-clients", type=int, default=int(os.environ.get("HIPZAP_BENCH_HTTP_CLIENTS", 16)),
                    help="secondary figure: HTTP client processes PER GPU against `hipzap serve --gpus N` "
                         "(0 disables)")
    ap.add_argument("--http-requests", type=int, default=800, help="requests per HTTP client process")
    ap.add_argument("--bert-cold", type=int, default=1, help="also report the BERT-base text-plan cold start")
    ap.add_argument("--lm-cold", type=int, default=1,
                    help="also report the GET /inference (AWD-LSTM V=60000, 200 words) torch-free cold start")
    ap.add_argument("--dp-figures", type=int, default=int(os.environ.get("HIPZAP_BENCH_DP", 1)),
                    help="also measure BASELINE configs 3 / 5 (scatter-gather DP) in the same launch")
    ap.add_argument("--config-figures", type=int, default=int(os.environ.get("HIPZAP_BENCH_CONFIGS", 1)),
                    help="also time BASELINE configs 1 / 4 and the reference's GET /inference route (rank 0)")
    ap.add_argument("--sustained-s", type=float, default=2.0,
                    help="secondary figure: served throughput over a self-timed window of at least this long")
    ap.add_argument("--mode", choices=["replica", "scatter"], default="replica",
                    help="replica: independent bs=1 request streams per GPU (headline); scatter: rank 0 scatters "
                         "a global batch over ranks and gathers the logits (configs 3/5)")
    ap.add_argument("--global-batch", type=int, default=32, help="scatter mode: global batch over all ranks")
    ap.add_argument("--launch-check", action="store_true",
                    help="rehearse the N-rank launch only (rendezvous + one all-reduce, no GPU work); rank 0 "
                         "prints {n_gpus, ranks_seen}")
    ap.add_argument("--input", choices=["uint8", "fp32"], default=os.environ.get("HIPZAP_BENCH_INPUT", "uint8"),
                    help="request payload: uint8 HWC images (decoded-JPEG format, ImageNet mean/std applied on "
                         "device by the preprocess kernel) or pre-normalised fp32 NCHW tensors")
    return ap.parse_args()


def run_scatter(args, rank, world, device, adapter, ckpt, tuned=None):
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
    params, arch_kw = broadcast_params(params, lambda kw: adapter.meta_params(**kw), device, arch_kw=arch_kw)
    eng = Engine(args.model, params, device, batch=shard, num_contexts=1, arch_kw=arch_kw, host_io=False,
                 tuned=tuned)
    x_in = adapter.example_input(shard)
    in_shape = tuple(eng.contexts[0].input.shape[1:])
    out_shape = tuple(eng.contexts[0].output.shape[1:])
    ex = DPExecutor(lambda xs: eng.infer_device(xs), shard, in_shape, out_shape, device,
                    in_dtype=eng.contexts[0].input.dtype, out_dtype=eng.contexts[0].output.dtype,
                    in_buf=eng.contexts[0].input, copy_out=False)
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


def prepare_artifacts(model: str, ckpt_dir: str, plan_contexts: int = 1) -> tuple[str, str]:
    """Deploy-time artifacts, written untimed on the CPU (no GPU call): the random-init
    checkpoint, its packed safetensors copy and its plan image; reused while up to date."""
    from hipzap.engine.packfile import find_packed, packed_path, save_packed, source_stamp
    from hipzap.engine.plan import export_from_checkpoint, plan_path
    from hipzap.lite import plan_usable, read_meta
    from hipzap.models import registry
    ckpt = os.path.join(ckpt_dir, f"{model}_seed0.pth")
    if not os.path.exists(ckpt):
        write_checkpoint(ckpt, model)
    stamp = source_stamp(ckpt)
    if find_packed(ckpt, model) is None:
        params, kw = registry.get(model).pack(torch.load(ckpt, map_location="cpu", weights_only=True), "cpu")
        save_packed(params, kw, packed_path(ckpt), model=model, stamp=stamp)
    plan = plan_path(ckpt)
    if not (plan_usable(plan) and read_meta(plan).get("source") == stamp):
        export_from_checkpoint(model, ckpt, plan, batch=1, contexts=plan_contexts)
    return ckpt, plan


def prepare_lm_artifacts(ckpt_dir: str, vocab: int = 60000) -> tuple[str, str]:
    """Deploy-time AWD-LSTM artifacts of the reference's route (untimed, CPU): a random-init
    checkpoint of the reference's dimensions (main.py:96: emb 1000, hidden 1150, 3 layers, tied,
    V = 60000 as SURVEY §2d assumes; ~357 MB fp32, torch.save) and its pickled itos list."""
    import pickle
    from hipzap.models.awd_lstm import reference_lm
    ckpt = os.path.join(ckpt_dir, f"awd_lstm_v{vocab}_seed0.pth")
    itos = os.path.join(ckpt_dir, f"awd_lstm_v{vocab}.itos.pkl")
    if not os.path.exists(ckpt):
        torch.manual_seed(0)
        os.makedirs(ckpt_dir, exist_ok=True)
        tmp = ckpt + f".tmp{os.getpid()}"
        torch.save(reference_lm(vocab).eval().state_dict(), tmp)
        os.replace(tmp, ckpt)
    if not os.path.exists(itos):
        words = ["xxunk", "xxpad", "xxbos", "xxfld", "xxmaj", "xxup", "xxrep", ".", ",", "!", "\n", "'s"]
        with open(itos, "wb") as f:
            pickle.dump(words + [f"w{i}" for i in range(vocab - len(words))], f)
    return ckpt, itos


def fresh_cold_start(args, device_index: int, world: int = 1) -> dict:
    """Cold start over fresh processes (hipzap/coldstart.py), before this process uses a GPU."""
    from hipzap.coldstart import measure_fresh, measure_fresh_interleaved, measure_node
    ckpt, plan = prepare_artifacts(args.model, args.ckpt_dir)
    # the three torch-free routes share HIP init (120-230 ms, box- and trial-dependent): measured in
    # alternation so their p50s compare like for like
    il = measure_fresh_interleaved({"plan": ("plan", plan, args.model, None),
                                    "pth_lite": ("pth-lite", ckpt, args.model, None),
                                    "native": ("native", plan, args.model, None)},
                                   args.cold_trials, device=device_index)
    if "error" in il["plan"]:
        raise RuntimeError(f"plan cold start failed: {il['plan']['error']}")
    res = {"plan": il["plan"]}
    # the same plan trials back to back (no idle gap): each child's HIP init then overlaps the driver's
    # teardown of the previous child (hipzap/coldstart.py trial_gap_s, profiles/r6_cold)
    try:
        res["plan_back_to_back"] = measure_fresh("plan", plan, args.model, args.cold_trials, device=device_index,
                                                 gap_s=0.0)
    except Exception as e:  # noqa: BLE001 - secondary figure
        print(f"back-to-back plan cold start skipped: {e}", file=sys.stderr)
    from hipzap.coldstart import isolated_env, narrow_env
    res["narrowing"] = narrow_env(os.environ, device_index)[2] if isolated_env(None, device_index)[0] is not None \
        else "unchanged"
    try:  # the node: N torch-free workers, RCCL rendezvous, C1 weight broadcast, first logits on every rank
        if world > torch.cuda.device_count():  # (a shared-GPU rehearsal: one RCCL rank per GPU only)
            raise RuntimeError(f"{world} workers need {world} visible GPUs, {torch.cuda.device_count()} visible")
        res["node"] = measure_node(plan, world, trials=max(3, min(5, args.cold_trials)), timeout=120)
    except Exception as e:  # noqa: BLE001 - secondary to the one-GPU figure
        print(f"node cold start skipped: {e}", file=sys.stderr)
    if args.lm_cold:
        try:  # the reference's own route: GET /inference (AWD-LSTM, 200 words) from its .pth, no torch
            lm_ckpt, itos = prepare_lm_artifacts(args.ckpt_dir)
            res["lm"] = measure_fresh("lm", lm_ckpt, "awd-lstm", args.cold_trials, device=device_index,
                                      extra_args=["--vocab", itos])
        except Exception as e:  # noqa: BLE001 - secondary figure
            print(f"LM cold start skipped: {e}", file=sys.stderr)
    # the .pth itself without torch (weights-only reader + plan template + device-side packing) and
    # the Python-free server binary (csrc/tools/serve_plan.cpp) on the plan image: interleaved above
    for name, what in (("pth_lite", "torch-free .pth"), ("native", "native")):
        if "error" in il[name]:  # template / binary not built: the torch path stays the .pth figure
            print(f"{what} cold start skipped: {il[name]['error']}", file=sys.stderr)
        else:
            res[name] = il[name]
    # import torch + torch.load + pack: ~1.9 s a trial, so at most 5
    res["pth"] = measure_fresh("pth", ckpt, args.model, min(5, args.cold_trials), device=device_index)
    if args.bert_cold:
        try:  # BERT-base seq-cls (BASELINE config 4) from its text plan image: torch-free too
            res["bert_plan"] = measure_fresh("plan", prepare_bert_plan(args.ckpt_dir), "bert-base",
                                             min(3, args.cold_trials), device=device_index)
        except Exception as e:  # noqa: BLE001 - secondary figure
            print(f"BERT plan cold start skipped: {e}", file=sys.stderr)
    return res


def prepare_bert_plan(ckpt_dir: str) -> str:
    """Deploy-time BERT-base artifacts (untimed, CPU): a random-init checkpoint and its bs16 text
    plan image (``hipzap plan --model bert-base --batch 16``); reused while up to date."""
    from hipzap.engine.packfile import source_stamp
    from hipzap.engine.plan import export_from_checkpoint, plan_path
    from hipzap.lite import plan_usable, read_meta
    from hipzap.models import registry
    ckpt = os.path.join(ckpt_dir, "bert-base_seed0.pth")
    if not os.path.exists(ckpt):
        torch.manual_seed(0)
        os.makedirs(ckpt_dir, exist_ok=True)
        tmp = ckpt + f".tmp{os.getpid()}"
        torch.save(registry.get("bert-base").make_model().eval().state_dict(), tmp)
        os.replace(tmp, ckpt)
    plan = plan_path(ckpt)
    if not (plan_usable(plan) and read_meta(plan).get("source") == source_stamp(ckpt)):
        export_from_checkpoint("bert-base", ckpt, plan, batch=16, contexts=1)
    return plan


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


def dynamic_batching(args, eng, device, world):
    """Secondary serving figure (not the headline): the SAME bs=1 requests -- one uint8 image
    each, ``--dyn-clients`` closed-loop native client threads -- served by the dynamic-batching
    executor (csrc/executor.cpp) over ``--dyn-contexts`` contexts captured at ``--dyn-batch``
    (batched convs on the LDS implicit GEMM). Whole-job inf/s = max wall over ranks."""
    from hipzap.engine.engine import Engine
    from hipzap.parallel.comm import is_dist, max_over_ranks
    ok = 1.0
    try:
        deng = Engine(args.model, eng.params, device, batch=args.dyn_batch, num_contexts=args.dyn_contexts,
                      capture=not args.no_capture, arch_kw=eng.arch_kw, host_io=True,
                      zero_copy=os.environ.get("HIPZAP_ZERO_COPY", "all"))
        ex = deng.batched_executor(max_wait_us=args.dyn_wait_us)
        h = eng.contexts[0].host_input
        row = h.reshape(-1)[: ex.in_bytes[0] // h.element_size()].clone()
        row.copy_((torch.rand(row.shape) * 255).to(row.dtype))
        ex.bench(args.dyn_clients, max(1, args.warmup), [row.data_ptr()])
    except Exception as e:  # noqa: BLE001 - a secondary figure must not take the headline down
        print(f"dynamic batching figure skipped: {e!r}", file=sys.stderr)
        ok = 0.0
    # every rank agrees before the timed collective section (a rank that failed would never reach it)
    if -max_over_ranks(-ok, device) < 1.0:
        return None
    s0 = ex.stats()
    if is_dist():
        dist.barrier()
    wall, lat = ex.bench(args.dyn_clients, args.steps, [row.data_ptr()])
    wall = max_over_ranks(wall, device)
    s1 = ex.stats()
    lat = sorted(lat)
    n = args.dyn_clients * args.steps
    batches = s1["batches"] - s0["batches"]
    out = {"inf_s": round(world * n / wall, 2), "request_batch": 1, "replay_batch": args.dyn_batch,
           "contexts": args.dyn_contexts, "clients": args.dyn_clients, "max_wait_us": args.dyn_wait_us,
           "mean_rows_per_replay": round((s1["served"] - s0["served"]) / max(1, batches), 2),
           "latency_ms_p50": round(lat[len(lat) // 2], 4), "latency_ms_p99": round(lat[int(0.99 * (len(lat) - 1))], 4)}
    ex.close()
    del deng
    return out


def dp_figures(args, eng, device, world: int, rank: int, native_comm):
    """Secondary figures: BASELINE configs 3 and 5 measured in the same N-rank launch. A global
    batch is scattered from rank 0 over the N ranks (C2), every rank runs its captured shard
    program, the logits are gathered back to rank 0 (C3); one step = scatter + forward + gather
    (``parallel/dp.py`` DPExecutor), images/s over the whole job = global batch x K / the slowest
    rank's wall. ResNet-50 at global batch 32 (uint8 images, the headline's broadcast weights)
    and ViT-B/16 fp8 at global batch 64 (random-init weights packed on every rank from the same
    seed). ``img_s``: ``dp_depth(model, shard)`` steps in flight (``parallel/dp.py`` DPPipeline: one captured
    context and stream per in-flight step, collectives in pipelined order on the caller's
    stream; every step's gather issued and completed inside the timed region);
    ``img_s_one_in_flight``: each step alone, back to back. Collectives run on the native RCCL communicator when the headline uses it (bounded
    waits: a stuck collective raises instead of hanging the launch), else torch.distributed.
    Every rank builds first and all agree before the first collective; a failure skips the
    figure (None), never the headline."""
    from hipzap.engine.engine import Engine
    from hipzap.models import registry
    from hipzap.parallel.comm import is_dist, max_over_ranks
    from hipzap.parallel.dp import DPPipeline
    out = {}
    for name, model, gb in (("resnet50_gb32", args.model, 32), ("vit_b16_fp8_gb64", "vit-b16-fp8", 64)):
        ok, seng, xg = 1.0, None, None
        depth = dp_depth(model, gb // world)
        try:
            shard = gb // world
            if shard * world != gb:
                raise ValueError(f"global batch {gb} does not divide over {world} ranks")
            if model == args.model:
                params, arch_kw = eng.params, eng.arch_kw
            else:
                a = registry.get(model)
                torch.manual_seed(0)
                params, arch_kw = a.pack(a.make_model().eval().state_dict(), device)
            # torch's pooled streams: over global batches of 32 / 64 the pipeline's steps run better sharing
            # the 4 queues than on queues of their own (gb32 43.7k vs 36.5k img/s, profiles/r6_queues)
            seng = Engine(model, params, device, batch=shard, num_contexts=depth, arch_kw=arch_kw, host_io=False,
                          stream_kind="torch")
            cin, cout = seng.contexts[0].input, seng.contexts[0].output
            if rank == 0:
                xg = (torch.randint(0, 256, (gb,) + tuple(cin.shape[1:]), dtype=torch.uint8, device=device)
                      if cin.dtype == torch.uint8 else torch.randn((gb,) + tuple(cin.shape[1:]), device=device).to(cin.dtype))
        except Exception as e:  # noqa: BLE001 - a secondary figure must not take the headline down
            print(f"dp figure {name} skipped: {e!r}", file=sys.stderr)
            ok = 0.0
        if -max_over_ranks(-ok, device) < 1.0:
            out[name] = None
            continue
        res = {"global_batch": gb, "per_rank_batch": gb // world, "steps": args.steps, "model": model,
               "comm": "native-rccl" if native_comm is not None else ("torch.distributed" if world > 1 else None),
               "dtype": "fp8" if "fp8" in model else "bf16"}
        # the scatter writes each shard straight into a captured context's input, the gather reads its output
        # in place; D steps in flight (DPPipeline): the rank keeps D batches moving, one per context / stream
        for d in sorted({1, depth}):
            pipe = DPPipeline(seng.pipeline_slots()[:d], gb // world, tuple(cout.shape[1:]), device,
                              out_dtype=cout.dtype, comm=native_comm)
            # the steps are issued from a non-default stream: the dedicated-queue context streams
            # (engine.py stream_kind) are blocking streams, which any NULL-stream command would
            # serialise against
            issue = torch.cuda.Stream(device)
            try:
                with torch.cuda.stream(issue):
                    for _ in range(max(1, args.warmup)):
                        pipe.submit(xg)
                    pipe.flush()
                    pipe.sync()
                torch.cuda.synchronize(device)
                if is_dist():
                    dist.barrier()
                t0 = time.perf_counter()
                with torch.cuda.stream(issue):
                    for i in range(args.steps):  # one bounded host sync per 8 steps
                        pipe.submit(xg)
                        if i % 8 == 7:
                            pipe.sync()
                    pipe.flush()  # every step's gather issued: all K steps complete inside the timed region
                    pipe.sync()
                torch.cuda.synchronize(device)
                dt = time.perf_counter() - t0
            except Exception as e:  # noqa: BLE001
                print(f"dp figure {name} (in flight {d}) failed: {e!r}", file=sys.stderr)
                dt = float("inf")
            dt = max_over_ranks(dt, device)
            if dt == float("inf"):
                continue
            key = "" if d == depth else "_one_in_flight"
            res[f"img_s{key}"] = round(gb * args.steps / dt, 2)
            res[f"ms_per_step{key}"] = round(dt / args.steps * 1e3, 4)
            del pipe
        res["in_flight"] = depth
        out[name] = res if "img_s" in res else None
        del seng
    out["dp_shard_w8"] = dp_shard_figures(args, eng, device)
    return out


def dp_depth(model: str, shard: int) -> int:
    """DP steps in flight per rank for the config 3 / 5 figures: ``HIPZAP_DP_DEPTH`` (1-8), else
    by the measured optimum (profiles/r6_dp_pipeline): 4 for ResNet-50 at any shard and for small
    ViT shards; 3 for ViT-B/16 fp8 shards of >= 32 images, whose per-step GEMMs already fill the
    chip (gb64 on one GPU over six runs: 22.5-23.3k img/s at 3, 20.0-23.8k at 2, 21.8-22.3k at 4)."""
    env = os.environ.get("HIPZAP_DP_DEPTH", "")
    if env:
        return max(1, min(8, int(env)))
    return 3 if "vit" in model and shard >= 32 else 4


def dp_shard_figures(args, eng, device) -> dict:
    """The per-rank compute of configs 3 / 5 at N = 8, timed on this GPU (VERDICT r4 #5a): at DP = 8
    a rank runs ResNet-50 on 32 / 8 = 4 images and ViT-B/16 fp8 on 64 / 8 = 8, one captured context
    each, replays back to back (no collectives: ``node_upper_img_s`` = 8 x the per-rank rate is what
    the node reaches if the scatter / gather cost nothing)."""
    from hipzap.engine.engine import Engine
    from hipzap.models import registry
    res = {}
    for name, model, shard in (("resnet50_bs4", args.model, 4), ("vit_b16_fp8_bs8", "vit-b16-fp8", 8)):
        try:
            if model == args.model:
                params, arch_kw = eng.params, eng.arch_kw
            else:
                a = registry.get(model)
                torch.manual_seed(0)
                params, arch_kw = a.pack(a.make_model().eval().state_dict(), device)
            seng = Engine(model, params, device, batch=shard, num_contexts=1, arch_kw=arch_kw, host_io=False)
            seng.bench(max(5, args.warmup))
            iters = max(50, args.steps * 10)
            t = seng.bench(iters)
            res[name] = {"img_s": round(shard * iters / t, 2), "ms_per_batch": round(t / iters * 1e3, 4),
                         "batch": shard, "node_upper_img_s": round(8 * shard * iters / t, 2), "model": model}
            del seng
            depth = dp_depth(model, shard)
            if depth > 1:  # the same shard program with D batches in flight (DPPipeline's compute side)
                seng = Engine(model, params, device, batch=shard, num_contexts=depth, arch_kw=arch_kw, host_io=False)
                seng.bench(max(5, args.warmup))
                t = seng.bench(iters)  # iters replays of every context, concurrently, synchronised
                res[name].update(in_flight=depth, img_s_in_flight=round(shard * depth * iters / t, 2),
                                 node_upper_img_s_in_flight=round(8 * shard * depth * iters / t, 2))
                del seng
        except Exception as e:  # noqa: BLE001 - a secondary figure must not take the headline down
            print(f"dp shard figure {name} skipped: {e!r}", file=sys.stderr)
            res[name] = None
    return res


def http_figure(args, world: int, rank: int):
    """Secondary figure: the serving SYSTEM over HTTP on the whole node -- ``python -m hipzap
    serve --gpus N`` (serve/cluster.py: one worker process per GPU sharing the listening socket,
    RCCL between the workers; N = 1: one server) from the plan image, loaded by
    ``--http-clients`` x N client processes sending bs=1 uint8 images (npy bodies) over
    keep-alive connections (hipzap/serve/loadtest.py). Run by rank 0 after the headline; the other
    ranks wait on the process group's TCP store (a CPU wait: no collective kernel spins on the
    GPUs the servers use). Returns the load result, or None if it could not run."""
    from datetime import timedelta
    from hipzap.parallel.comm import is_dist
    res = None
    if rank == 0:
        try:
            from hipzap.serve.loadtest import run_load
            _, plan = prepare_artifacts(args.model, args.ckpt_dir)
            res = run_load(plan, gpus=world, clients=args.http_clients * world, requests=args.http_requests,
                           contexts=16, fmt="npy", ready_timeout=150.0)  # 16 x 16: +5 % over 12 x 8 (r4_final/http_contexts)
            if not res.get("errors"):
                res.pop("server_log_tail", None)
        except Exception as e:  # noqa: BLE001 - a secondary figure must not take the headline down
            print(f"http serving figure skipped: {e!r}", file=sys.stderr)
            res = None
    if is_dist():
        store = dist.distributed_c10d._get_default_store()
        if rank == 0:
            store.set("hipzap_http_done", "1")
        else:
            store.wait(["hipzap_http_done"], timedelta(seconds=1200))
    return res


def config_figures(args, device, world: int, rank: int) -> dict | None:
    """The other BASELINE configs and the reference's own route, on the driver's clock in the same
    launch. Run by rank 0 after the headline (the other ranks wait on the
    process group's store, a CPU wait), each in a FRESH child process on rank 0's GPU: this process
    already holds dozens of streams over HIP's 4 hardware queues, which would fold a figure's
    concurrent contexts onto shared queues (BERT 4 contexts measured 24.4k seq/s in-process vs
    29.2k fresh). Figures and their timed regions: ``scripts/bench_configs.py`` (config 4: BERT-base
    bs16 at 1 and 4 contexts; the reference's ``GET /inference`` route through the WSGI app) and
    ``scripts/bench_cpu_plumbing.py`` (config 1: ResNet-18 POST through the CPU Flask handler).
    Returns the dict (rank 0) or None; a figure that fails is recorded as its error."""
    from datetime import timedelta
    from hipzap.parallel.comm import is_dist
    out = None
    if rank == 0:
        out = {}
        try:
            out.update(_child_json(["scripts/bench_configs.py", "--device", str(device.index or 0),
                                    "--steps", str(args.steps)], timeout=600))
        except Exception as e:  # noqa: BLE001 - a secondary figure must not take the headline down
            out["bert_base_bs16"] = out["awd_lstm_get_inference"] = {"error": repr(e)[:500]}
        try:
            out["resnet18_cpu_plumbing"] = _plumbing_figure()
        except Exception as e:  # noqa: BLE001
            out["resnet18_cpu_plumbing"] = {"error": repr(e)[:500]}
    if is_dist():
        store = dist.distributed_c10d._get_default_store()
        if rank == 0:
            store.set("hipzap_configs_done", "1")
        else:
            store.wait(["hipzap_configs_done"], timedelta(seconds=1200))
    return out


def _child_json(argv: list, timeout: float, env: dict | None = None) -> dict:
    import subprocess
    root = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(root, argv[0]), *argv[1:]], capture_output=True, text=True,
                       timeout=timeout, cwd=root, env=env)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        raise RuntimeError(f"{argv[0]} rc={r.returncode}: {r.stderr[-800:]}")
    return json.loads(lines[-1])


def _plumbing_figure() -> dict:
    res = _child_json(["scripts/bench_cpu_plumbing.py", "--requests", "30"], timeout=300,
                      env=dict(os.environ, HIPZAP_RANDOM_WEIGHTS="1"))
    res["req_s_sequential"] = round(1e3 / res["http_image_b64_ms_p50"], 1)
    res["timed_region"] = "30 sequential HTTP POST /predict per payload kind, per-request wall"
    return res


def request_input(args, adapter):
    """One request's payload: a decoded uint8 HWC image (default) or an fp32 NCHW tensor."""
    if args.input == "uint8" and args.model.startswith("resnet"):
        return torch.randint(0, 256, (args.batch, 224, 224, 3), dtype=torch.uint8)
    return adapter.example_input(args.batch)


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def check_gpus(n: int, share: bool) -> None:
    """Fail loudly unless this node has ``n`` GPUs for ``n`` ranks, counted from the KFD topology
    in sysfs narrowed by the visibility variables (hipzap/utils/gpucount.py): no HIP call, no
    fallback to ``hipGetDeviceCount``."""
    from hipzap.utils.gpucount import visible_gpu_count
    have = visible_gpu_count()
    if share:  # multi-rank rehearsal folded onto the visible GPU(s): HIPZAP_SHARE_GPU=1
        if have < 1:
            raise SystemExit(f"bench: --gpus {n} with HIPZAP_SHARE_GPU=1 needs at least one GPU, found none")
        return
    if have < n:
        raise SystemExit(f"bench: --gpus {n} needs {n} GPUs on this node, found {have} "
                         "(HIPZAP_SHARE_GPU=1 rehearses several ranks on one GPU)")


def self_launch(args) -> int:
    """``python bench.py --gpus N`` without torchrun: spawn N rank processes of this script
    (one per GPU, fresh interpreters started before this process makes any GPU call) with
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, exactly as torchrun would. Rank 0 prints the
    JSON line (stdout is inherited); the launcher exits with the worst rank's code. When one
    rank fails, the others are stopped after a grace period instead of waiting on its
    collectives until the process-group timeout."""
    import signal
    import subprocess
    from hipzap.utils.gpucount import hip_mapped
    if not args.launch_check:
        check_gpus(args.gpus, os.environ.get("HIPZAP_SHARE_GPU") == "1")
    if hip_mapped():  # the ranks must be the only processes on the GPUs
        raise SystemExit("bench: the launcher mapped the HIP runtime before spawning its ranks")
    port = int(os.environ.get("MASTER_PORT") or _free_port())
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HIPZAP_SELF_LAUNCHED="1", HIPZAP_LAUNCHER_HIP_MAPPED="0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env,
                                      start_new_session=True))
    codes: dict[int, int] = {}
    fail_at = None
    while len(codes) < len(procs):
        for r, p in enumerate(procs):
            if r not in codes and p.poll() is not None:
                codes[r] = p.returncode
                if p.returncode != 0 and fail_at is None:
                    print(f"bench: rank {r} exited with {p.returncode}", file=sys.stderr, flush=True)
                    fail_at = time.time()
        if fail_at is not None and time.time() - fail_at > 30:
            for r, p in enumerate(procs):
                if r not in codes:
                    try:
                        os.killpg(p.pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
            for r, p in enumerate(procs):
                if r not in codes:
                    try:
                        codes[r] = p.wait(timeout=15)
                    except subprocess.TimeoutExpired:
                        os.killpg(p.pid, signal.SIGKILL)
                        codes[r] = p.wait()
        time.sleep(0.05)
    # a rank killed by signal s reports -s: map it to the shell's 128 + s
    bad = [c if c > 0 else 128 - c for c in codes.values() if c != 0]
    return max(bad) if bad else 0


def launch_check(rank: int, world: int) -> None:
    """--launch-check: every rank joins the process group (gloo: no GPU call) and all-reduces 1."""
    from hipzap.parallel.comm import init_distributed, is_dist
    init_distributed(backend="gloo", timeout_s=60)
    t = torch.ones(1)
    if is_dist():
        dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "ranks_seen": int(t.item()),
                          "self_launched": os.environ.get("HIPZAP_SELF_LAUNCHED") == "1",
                          "launcher_hip_mapped": os.environ.get("HIPZAP_LAUNCHER_HIP_MAPPED")}), flush=True)
    if is_dist():
        dist.barrier()
        dist.destroy_process_group()


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(self_launch(args))
    _import_torch()
    from hipzap.parallel.comm import env_rank
    rank, world, local = env_rank()
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but the launcher started {world} rank(s) (WORLD_SIZE)")
    if args.launch_check:
        return launch_check(rank, world)
    if rank == 0 and world > 1 and os.environ.get("HIPZAP_SELF_LAUNCHED") != "1":
        check_gpus(world, os.environ.get("HIPZAP_SHARE_GPU") == "1")
    # 1. cold start over fresh processes, before this process makes any GPU call (the other
    #    ranks wait in the process-group rendezvous meanwhile)
    fresh = None
    if rank == 0:
        if args.mode == "replica" and args.cold_trials > 0 and args.model.startswith("resnet"):
            dev_index = local % max(1, torch.cuda.device_count()) if os.environ.get("HIPZAP_SHARE_GPU") == "1" \
                else local
            fresh = fresh_cold_start(args, dev_index, world)
        else:
            prepare_artifacts(args.model, args.ckpt_dir)

    from hipzap.engine.engine import Engine
    from hipzap.models import registry
    from hipzap.parallel.comm import broadcast_params, init_distributed, is_dist, local_device, max_over_ranks

    device = local_device(local)
    torch.cuda.set_device(device)
    init_distributed(device=device)
    adapter = registry.get(args.model)
    ckpt = os.path.join(args.ckpt_dir, f"{args.model}_seed0.pth")
    tuned = None  # Engine picks hipzap/tuning/<model>_bs<B>[_c<streams>].json
    if args.tuned:
        with open(args.tuned) as f:
            tuned = json.load(f)
    # C1 weight broadcast over the native RCCL communicator (csrc/comm, the serving cluster's
    # transport); every rank agrees on it or all fall back to torch.distributed
    native_comm = None
    if is_dist() and dist.get_backend() == "nccl" and os.environ.get("HIPZAP_NATIVE_COMM", "1") != "0":
        ok = 1
        try:
            from hipzap.parallel.rccl import RcclComm
            native_comm = RcclComm.from_torch(device.index, timeout_s=120)
        except Exception as e:  # noqa: BLE001
            print(f"rank {rank}: native RCCL communicator unavailable ({e}); using torch.distributed", file=sys.stderr)
            ok = 0
        flag = torch.tensor([ok], dtype=torch.int32, device=device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if not int(flag.item()):
            native_comm = None
    # which RCCL build each rank mapped (libhipzap_comm.so's librccl.so.1 resolves to torch's bundled
    # copy in a torch-imported process) and its version; every rank reports
    from hipzap.parallel.rccl import mapped_rccl
    # per rank: the RCCL build it mapped, and the rank / size its communicator reports
    # (ncclCommUserRank / ncclCommCount) -- a world the driver launched must be one communicator
    mine = dict(mapped_rccl(), rank=rank, device=device.index)
    if native_comm is not None:
        mine.update(comm_rank=native_comm.comm_rank(), comm_count=native_comm.comm_size())
    rccl_map = [mine]
    if is_dist():
        rccl_map = [None] * world
        dist.all_gather_object(rccl_map, mine)
    if is_dist():
        dist.barrier()
    if args.mode == "scatter":
        run_scatter(args, rank, world, device, adapter, ckpt, tuned)
        if is_dist():
            dist.barrier()
            dist.destroy_process_group()
        return

    def cold_start(packed: str | None = None):
        """In-process cold start: rank 0 loads (``packed``: the pre-packed copy ``<ckpt>.hzpack``)
        and RCCL-broadcasts the packed blob + its architecture metadata; every rank plans and
        captures its first request context and serves one request."""
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
        ta = time.perf_counter()
        params, arch_kw = broadcast_params(params, lambda kw: adapter.meta_params(**kw), device, arch_kw=arch_kw,
                                           comm=native_comm)
        torch.cuda.synchronize(device)
        timings["broadcast_ms"] = (time.perf_counter() - ta) * 1e3
        arch_kw = dict(arch_kw)
        if args.input == "uint8" and args.model.startswith("resnet"):
            arch_kw["input_uint8"] = True
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

    # 2. in-process cold starts (secondary figures: warm torch, warm HIP runtime)
    eng, out, cold_first = cold_start()
    colds = [cold_first]
    for _ in range(args.cold_runs):
        del eng
        torch.cuda.synchronize(device)
        eng, out, c = cold_start()
        colds.append(c)
    assert torch.isfinite(out).all(), "non-finite logits"
    breakdown_pth = dict(eng.timings)
    colds_packed, breakdown_packed = [], {}
    if args.cold_runs:
        from hipzap.engine.packfile import packed_path
        for _ in range(args.cold_runs):
            del eng
            torch.cuda.synchronize(device)
            eng, out, c = cold_start(packed=packed_path(ckpt))
            colds_packed.append(c)
        breakdown_packed = dict(eng.timings)
        assert torch.isfinite(out).all(), "non-finite logits (packed path)"

    # the other streams-1 request contexts are planned + captured after the first request was served
    # (a warm container scaling up its concurrency), outside the cold-start figure; reported below
    deferred_ms = eng.ensure_contexts()
    # single-request latency, one request at a time (round-robin over the contexts), p50/p99
    x = request_input(args, adapter)
    lat = []
    for i in range(210):
        t = time.perf_counter()
        eng.infer(x)
        lat.append((time.perf_counter() - t) * 1e3)
    lat = sorted(lat[10:])
    lat_p50, lat_p99 = statistics.median(lat), lat[min(len(lat) - 1, int(0.99 * len(lat)))]

    def pct(v, q):
        v = sorted(v)
        return v[min(len(v) - 1, int(q * len(v)))]

    # 3. throughput: W warmup steps, then K timed steps; a step = one request on every stream
    payload = x.reshape(eng.contexts[0].host_input.shape)

    def run(steps, mode):
        if mode == "pipelined":
            return eng.bench(steps), None
        return eng.serve_bench(steps, payload, mode=mode)

    other = "pipelined" if args.serve != "pipelined" else "executor"
    rps = max(1, args.step_requests)  # requests per stream in one step
    if args.warmup:
        run(args.warmup * rps, args.serve)
    if is_dist():
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    _, lat_load = run(args.steps * rps, args.serve)
    torch.cuda.synchronize(device)
    dt = time.perf_counter() - t0
    if is_dist():
        dist.barrier()
    dt = max_over_ranks(dt, device)
    # a longer self-timed window of the same serving loop (>= --sustained-s), so box noise over the
    # driver's short K-step region is not mistaken for kernel wins (same on every rank: dt is the max)
    sustained = None
    if args.sustained_s > 0:
        n_long = int(min(50000, max(args.steps * rps, -(-args.sustained_s * args.steps * rps // dt))))
        if is_dist():
            dist.barrier()
        torch.cuda.synchronize(device)
        t_l = time.perf_counter()
        run(n_long, args.serve)
        torch.cuda.synchronize(device)
        dt_l = max_over_ranks(time.perf_counter() - t_l, device)
        sustained = {"inf_s": round(world * args.streams * args.batch * n_long / dt_l, 2), "steps": n_long,
                     "window_s": round(dt_l, 3)}
    # the other serving mode, untimed for the headline (same K), for reference
    dt_other, lat_other = run(args.steps * rps, other)
    dt_other = max_over_ranks(dt_other, device)
    lat_closed = lat_load if args.serve != "pipelined" else lat_other
    inf = world * args.streams * args.batch * args.steps * rps
    value = inf / dt
    # strict single-stream throughput (one context, replays back to back)
    single = eng.contexts[0]
    from hipzap.engine.program import bench_contexts
    t_single = bench_contexts([single], [eng.streams[0]], 200)
    dyn = dynamic_batching(args, eng, device, world) if args.dyn_batch > 1 and args.batch == 1 else None
    http = http_figure(args, world, rank) if args.http_clients > 0 and args.batch == 1 else None
    dpf = dp_figures(args, eng, device, world, rank, native_comm) \
        if args.dp_figures and args.batch == 1 and args.model == "resnet50" else None
    cfgs = config_figures(args, device, world, rank) if args.config_figures and args.batch == 1 else None
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
                       "streams_per_gpu": args.streams, "requests_per_stream_per_step": rps,
                       "hipgraph": not args.no_capture,
                       "serving": args.serve,
                       "weight_broadcast": "native-rccl" if native_comm is not None else
                       ("torch.distributed" if world > 1 else None)},
            "rccl_mapped": rccl_map,
            "cold_start_ms_p50": fresh["plan"]["p50_ms"] if fresh else None,
            # the same trials back to back (no idle gap before each child)
            "cold_start_back_to_back_ms_p50": ((fresh or {}).get("plan_back_to_back") or {}).get("p50_ms"),
            "cold_start_gap_ms": (fresh or {}).get("plan", {}).get("gap_ms"),
            "cold_start_note": "p50 over fresh processes, spawn -> first logits, from the .hzplan deploy artifact "
                               "(torch-free runtime), each child started on an idle GPU (cold_start_gap_ms after "
                               "the previous child exited: back to back, the driver's teardown of the previous "
                               "process delays the next one's HIP init by ~130 ms, profiles/r6_cold; that set is "
                               "cold_start_back_to_back_ms_p50); cold_start_pth_ms_p50 = same from the .pth state_dict "
                               "without torch (weights-only zip reader + plan template + device-side packing; "
                               "cold_start_pth_torch_ms_p50: import torch + torch.load + pack); "
                               "each child sees only its own GPU (ROCR_VISIBLE_DEVICES, a one-GPU worker) unless "
                               "the launcher already restricts visibility",
            # how each cold-start child was narrowed to its one GPU (hipzap/coldstart.py narrow_env):
            # "rocr" (nothing set by the launcher), "rocr_from_<var>" (the launcher set a HIP-level
            # list), "unchanged" (ROCR_VISIBLE_DEVICES already set / isolation off); the child's
            # environment (visibility variables, KFD nodes, render nodes) is in cold_start_fresh_process
            "cold_start_isolated": (fresh or {}).get("narrowing", "unchanged") != "unchanged",
            "cold_start_narrowing": (fresh or {}).get("narrowing"),
            # the reference's checkpoint format (main.py:99): torch-free when the template exists
            "cold_start_pth_ms_p50": ((fresh.get("pth_lite") or fresh["pth"])["p50_ms"]) if fresh else None,
            "cold_start_pth_torch_ms_p50": fresh["pth"]["p50_ms"] if fresh else None,
            # the Python-free server binary (hipzap-serve-plan --once) on the same plan image
            "cold_start_native_ms_p50": (fresh.get("native") or {}).get("p50_ms") if fresh else None,
            # BERT-base bs16 seq-cls from its text plan image (torch-free)
            "cold_start_bert_plan_ms_p50": (fresh.get("bert_plan") or {}).get("p50_ms") if fresh else None,
            # the node: spawn N torch-free workers -> RCCL init -> C1 broadcast -> first logits on EVERY rank
            "cold_start_node_ms_p50": (fresh.get("node") or {}).get("p50_ms") if fresh else None,
            # the reference's route: fresh process -> first 200-word GET /inference response, torch-free
            "cold_start_lm_ms_p50": (fresh.get("lm") or {}).get("p50_ms") if fresh else None,
            "cold_start_fresh_process": fresh,
            "cold_start_inprocess_ms_first": round(cold_first, 2),
            "cold_start_inprocess_ms_p50": round(statistics.median(colds), 2),
            "cold_start_inprocess_breakdown_ms": {k: round(v, 2) for k, v in breakdown_pth.items()},
            "cold_start_inprocess_packed_ms_p50": round(statistics.median(colds_packed), 2) if colds_packed else None,
            "cold_start_inprocess_packed_breakdown_ms": {k: round(v, 2) for k, v in breakdown_packed.items()},
            "deferred_contexts_ms": round(deferred_ms, 2),
            "served_closed_loop_inf_s": round(inf / (dt if args.serve != "pipelined" else dt_other), 2),
            "device_pipelined_inf_s": round(inf / (dt if args.serve == "pipelined" else dt_other), 2),
            "latency_ms_under_load_p50": round(pct(lat_closed, 0.5), 4),
            "latency_ms_under_load_p99": round(pct(lat_closed, 0.99), 4),
            "latency_ms_p50_single": round(lat_p50, 4),
            "latency_ms_p99_single": round(lat_p99, 4),
            "single_stream_inf_s": round(200 / t_single, 2),
            "baseline_note": "vs_baseline against BASELINE.md sandbox-CPU ResNet-50 bs=1 (27.2 inf/s); "
                             "no published numbers exist",
        }
        if dyn is not None:
            res["dynamic_batching"] = dyn
        if sustained is not None:
            res["served_sustained"] = sustained
        if http is not None:
            res["http_serving"] = http
        if dpf is not None:  # BASELINE configs 3 and 5 (scatter / gather DP) in the same launch
            res["dp_scatter"] = dpf
        if cfgs is not None:  # BASELINE configs 1 and 4 and the reference's GET /inference route
            res["configs"] = cfgs
        if torch_ref is not None:
            res["torch_miopen_graph_inf_s_1gpu_1stream"] = round(torch_ref, 2)
        print(json.dumps(res), flush=True)
    if is_dist():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
