"""Multi-GPU RCCL self-test worker (tests/test_rccl_multi_gpu.py; VERDICT r3 "next round" 3b).

One process per GPU, started fresh by the test. Every rank joins the native communicator
(``parallel/rccl.py`` over ``libhipzap_comm.so``) through a file rendezvous and checks the serving
collectives of SURVEY.md §2f BITWISE:

* C1 broadcast of a byte pattern from rank 0 (the cold-start weight broadcast);
* C2 scatter of per-rank patterns from rank 0 and C3 gather back to rank 0;
* C4 the 1-int health all-reduce, which must return the world size;
* (``--mode torch``: after ``import torch``, i.e. the library mix bench.py runs with: torch's
  bundled librccl may be the one mapped) the same through the tensor interface, plus
  ``DPExecutor`` on the RCCL communicator -- a ResNet-18 global batch scattered, run per shard and
  gathered -- against rank 0 running every shard alone, bitwise; and the asynchronous step
  (``sync=False`` then one ``sync``) equal to the synchronous one.

Prints one JSON line per rank: ``{"rank", "world", "ok", "checks": {...}}``.

    python -m hipzap.parallel.selftest --mode lite|torch --rank R --world W --rdzv DIR
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import sys


def _pattern(n: int, salt: int) -> bytes:
    return bytes(((i * 131 + salt * 17 + (i >> 8)) & 0xFF) for i in range(n))


def run_lite(rank: int, world: int, rdzv_dir: str) -> dict:
    from .. import hip
    from .rccl import FileRendezvous, RcclComm
    hip.set_device(rank)
    comm = RcclComm.from_rendezvous(FileRendezvous(rdzv_dir), world, rank, rank, timeout_s=60)
    checks = {}
    nb = 1 << 20
    buf = hip.DeviceBuffer(nb * world)
    host = (C.c_char * (nb * world))()

    def put(data: bytes, off: int = 0):
        C.memmove(C.addressof(host) + off, data, len(data))
        hip.memcpy(buf.ptr + off, C.addressof(host) + off, len(data), hip.H2D)

    def get(n: int, off: int = 0) -> bytes:
        hip.memcpy(C.addressof(host) + off, buf.ptr + off, n, hip.D2H)
        return bytes(host)[off: off + n]

    # C1 broadcast
    put(_pattern(nb, 1) if rank == 0 else bytes(nb))
    comm.broadcast_ptr(buf.ptr, nb, 0)
    checks["broadcast"] = get(nb) == _pattern(nb, 1)
    # C2 scatter: rank 0 holds world chunks, rank r receives chunk r into a separate buffer
    chunk = 1 << 16
    recv = hip.DeviceBuffer(chunk)
    if rank == 0:
        put(b"".join(_pattern(chunk, 10 + r) for r in range(world)))
    comm.scatter_ptr(buf.ptr if rank == 0 else 0, recv.ptr, chunk, 0)
    out = (C.c_char * chunk)()
    hip.memcpy(C.addressof(out), recv.ptr, chunk, hip.D2H)
    checks["scatter"] = bytes(out) == _pattern(chunk, 10 + rank)
    # C3 gather: every rank sends its own pattern, rank 0 collects world chunks
    C.memmove(C.addressof(out), _pattern(chunk, 50 + rank), chunk)
    hip.memcpy(recv.ptr, C.addressof(out), chunk, hip.H2D)
    comm.gather_ptr(recv.ptr, buf.ptr if rank == 0 else 0, chunk, 0)
    if rank == 0:
        checks["gather"] = get(chunk * world) == b"".join(_pattern(chunk, 50 + r) for r in range(world))
    # C4 health all-reduce
    one = C.c_int(1)
    hb = hip.DeviceBuffer(4)
    hip.memcpy(hb.ptr, C.addressof(one), 4, hip.H2D)
    comm.allreduce_ptr(hb.ptr, 1, "int32", "sum")
    hip.memcpy(C.addressof(one), hb.ptr, 4, hip.D2H)
    checks["health"] = one.value == world
    comm.close()
    return {"rank": rank, "world": world, "mode": "lite", "ok": all(checks.values()), "checks": checks,
            "torch_imported": "torch" in sys.modules}


def run_torch(rank: int, world: int, rdzv_dir: str) -> dict:
    import torch
    from ..engine.engine import Engine
    from ..models import registry
    from ..models.resnet import randomize_bn
    from .dp import DPExecutor
    from .rccl import FileRendezvous, RcclComm
    dev = torch.device(f"cuda:{rank}")
    torch.cuda.set_device(dev)
    comm = RcclComm.from_rendezvous(FileRendezvous(rdzv_dir), world, rank, rank, timeout_s=60)
    checks = {}
    g = torch.Generator().manual_seed(7)
    ref = torch.randint(-2**31, 2**31 - 1, (world, 4096), dtype=torch.int32, generator=g)
    t = ref[0].to(dev) if rank == 0 else torch.zeros(4096, dtype=torch.int32, device=dev)
    comm.broadcast(t, 0)
    checks["broadcast"] = torch.equal(t.cpu(), ref[0])
    out = torch.zeros(4096, dtype=torch.int32, device=dev)
    allx = ref.to(dev)
    comm.scatter(out, list(allx.unbind(0)) if rank == 0 else None, 0)
    checks["scatter"] = torch.equal(out.cpu(), ref[rank])
    mine = ref[rank].to(dev)
    got = torch.zeros(world, 4096, dtype=torch.int32, device=dev)
    comm.gather(mine, list(got.unbind(0)) if rank == 0 else None, 0)
    if rank == 0:
        checks["gather"] = torch.equal(got.cpu(), ref)
    h = torch.ones(1, dtype=torch.int32, device=dev)
    comm.all_reduce(h)
    checks["health"] = int(h.item()) == world
    # DPExecutor over RCCL: ResNet-18, shard 2 per rank, same random-init weights on every rank
    torch.manual_seed(0)
    a = registry.get("resnet18")
    sd = randomize_bn(a.make_model()).eval().state_dict()
    params, kw = a.pack({k: v.to(dev) for k, v in sd.items()}, dev)
    shard = 2
    eng = Engine("resnet18", params, dev, batch=shard, num_contexts=1, arch_kw=kw, host_io=False)
    cin, cout = eng.contexts[0].input, eng.contexts[0].output
    ex = DPExecutor(lambda xs: eng.infer_device(xs), shard, tuple(cin.shape[1:]), tuple(cout.shape[1:]), dev,
                    in_dtype=cin.dtype, out_dtype=cout.dtype, comm=comm)
    xg = torch.randn((shard * world,) + tuple(cin.shape[1:]), generator=torch.Generator().manual_seed(3)).to(dev) \
        if rank == 0 else None
    y_sync = ex.step(xg)
    y_async = ex.step(xg, sync=False)
    ex.sync()
    if rank == 0:
        alone = torch.cat([eng.infer_device(xg[r * shard:(r + 1) * shard]).clone() for r in range(world)])
        torch.cuda.synchronize(dev)
        checks["dp_vs_shards_alone"] = torch.equal(y_sync.reshape(alone.shape), alone)
        checks["dp_async_equals_sync"] = torch.equal(y_sync, y_async)
    # DPPipeline over RCCL: three steps in flight (three contexts), five different global batches;
    # every step's gathered logits == its shards run alone
    from .dp import DPPipeline
    eng3 = Engine("resnet18", params, dev, batch=shard, num_contexts=3, arch_kw=kw, host_io=False)
    pipe = DPPipeline(eng3.pipeline_slots(), shard, tuple(cout.shape[1:]), dev, out_dtype=cout.dtype, comm=comm)
    xs = [xg * (0.5 + i) if rank == 0 else None for i in range(5)]
    got = []
    for x in xs:
        y = pipe.submit(x)
        if y is not None:
            got.append(y.clone())
    got += [y.clone() for y in pipe.flush() if y is not None]
    pipe.sync()
    if rank == 0:
        ok = len(got) == len(xs)
        for x, y in zip(xs, got):
            alone = torch.cat([eng.infer_device(x[r * shard:(r + 1) * shard]).clone() for r in range(world)])
            torch.cuda.synchronize(dev)
            ok = ok and torch.equal(y.reshape(alone.shape), alone)
        checks["dp_pipeline_vs_shards_alone"] = ok
    comm.close()
    return {"rank": rank, "world": world, "mode": "torch", "ok": all(checks.values()), "checks": checks}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["lite", "torch"], default="lite")
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--rdzv", required=True)
    a = ap.parse_args(argv)
    res = (run_lite if a.mode == "lite" else run_torch)(a.rank, a.world, a.rdzv)
    print(json.dumps(res), flush=True)
    return 0 if res["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
