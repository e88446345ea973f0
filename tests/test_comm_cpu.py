"""Weight-blob broadcast (C1) and DP helpers over gloo with world_size 2 (CPU)."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hipzap.parallel.comm import broadcast_params, flat_layout, pack_blob, unpack_blob


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hipzap.models import registry
    a = registry.get("resnet18")
    meta, _ = a.meta_params()
    params = None
    if rank == 0:
        torch.manual_seed(0)
        params = a.pack(a.make_model().state_dict(), "cpu")[0]
    got = broadcast_params(params, meta, "cpu")
    digest = sum(float(p.wf.float().sum() + p.bias.sum()) for p in got.values())
    q.put((rank, digest, got["fc"].cout))
    dist.destroy_process_group()


def test_blob_roundtrip():
    from hipzap.models import registry
    a = registry.get("resnet18")
    params = a.pack(a.make_model().state_dict(), "cpu")[0]
    blob = pack_blob(params, "cpu")
    _, total = flat_layout(params)
    assert blob.numel() == total
    back = unpack_blob(blob, params)
    for k in params:
        assert torch.equal(back[k].wf, params[k].wf) and torch.equal(back[k].bias, params[k].bias)


def test_broadcast_world2_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res[0][1] == res[1][1] and res[0][2] == res[1][2] == 1000


def _dp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hipzap.parallel.dp import DPExecutor
    seen = []

    def runner(x):  # per-rank "model": tag rows with the rank that computed them
        seen.append(x.clone())
        return x.sum(dim=(1, 2)) + 1000 * rank

    ex = DPExecutor(runner, shard_batch=3, in_shape=(2, 4), out_shape=(), device="cpu")
    x = torch.arange(5 * 8, dtype=torch.float32).reshape(5, 2, 4) if rank == 0 else None  # uneven: 5 of 6
    y = ex.step(x)
    if rank == 0:
        q.put(("y", y.tolist()))
    q.put(("shard", rank, seen[0].shape[0]))
    dist.destroy_process_group()


def test_dp_scatter_gather_world2_uneven():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    msgs = [q.get(timeout=300) for _ in range(3)]
    for p in procs:
        p.join(timeout=60)
    y = next(m[1] for m in msgs if m[0] == "y")
    x = torch.arange(5 * 8, dtype=torch.float32).reshape(5, 2, 4)
    expect = (x.sum(dim=(1, 2)) + torch.tensor([0, 0, 0, 1000, 1000])).tolist()
    assert y == expect
    assert sorted(m[2] for m in msgs if m[0] == "shard") == [3, 3]


def test_mapped_rccl_report_parses_maps():
    """The bench's per-rank RCCL report: the librccl paths a process mapped (torch's bundled copy
    flagged), read from /proc/self/maps."""
    from hipzap.parallel.rccl import mapped_rccl
    maps = "\n".join([
        "7f00-7f10 r-xp 00000000 08:01 1 /usr/lib/libc.so.6",
        "7f10-7f20 r-xp 00000000 08:01 2 /usr/local/lib/python3.10/dist-packages/torch/lib/librccl.so",
        "7f20-7f30 r--p 00100000 08:01 2 /usr/local/lib/python3.10/dist-packages/torch/lib/librccl.so",
        "7f30-7f40 rw-p 00000000 00:00 0 ",
    ])
    r = mapped_rccl(maps)
    assert r["paths"] == ["/usr/local/lib/python3.10/dist-packages/torch/lib/librccl.so"]
    assert r["torch_bundled"] is True
    assert mapped_rccl("7f00-7f10 r-xp 00000000 08:01 1 /opt/rocm/lib/librccl.so.1")["torch_bundled"] is False
    live = mapped_rccl()  # this process: whatever is mapped, a well-formed report
    assert set(live) == {"paths", "version", "torch_bundled", "has_comm_shrink"}


def _pipe_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hipzap.parallel.dp import DPPipeline, FnSlot
    runner = lambda x: x.sum(dim=1) + 1000 * rank  # noqa: E731
    pipe = DPPipeline([FnSlot(runner, 2, (4,)) for _ in range(3)], 2, (), "cpu")
    outs = []
    for i in range(5):
        x = torch.arange(4 * 4, dtype=torch.float32).reshape(4, 4) * (i + 1) if rank == 0 else None
        y = pipe.submit(x)
        if y is not None:
            outs.append(y.tolist())
    outs += [y.tolist() for y in pipe.flush() if y is not None]
    if rank == 0:
        q.put(outs)
    dist.destroy_process_group()


def test_dp_pipeline_world2_gloo():
    """Three DP steps in flight over torch.distributed (gloo, two processes): the five steps'
    logits come back in order, each row tagged by the rank that computed it."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipe_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
    assert len(outs) == 5
    for i, y in enumerate(outs):
        x = torch.arange(16, dtype=torch.float32).reshape(4, 4) * (i + 1)
        assert y == (x.sum(dim=1) + torch.tensor([0, 0, 1000, 1000])).tolist()
