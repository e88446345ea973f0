"""DP logic on the in-process loopback communicator (SURVEY.md §4.2 T-comm-fake): world sizes
1-8 in one process — weight-blob broadcast (C1), scatter/gather executor (C2/C3) incl. uneven
batches, health all-reduce (C4), and the failure path (a failing rank aborts its peers)."""
import pytest
import torch

from hipzap.parallel.comm import broadcast_params, health_check
from hipzap.parallel.dp import DPExecutor
from hipzap.parallel.loopback import CommError, run_ranks


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_collectives(world):
    def fn(c):
        t = torch.full((4,), float(c.rank))
        c.broadcast(t, src=world - 1)
        s = torch.tensor([c.rank + 1.0])
        c.all_reduce(s)
        m = torch.tensor([float(c.rank)])
        c.all_reduce(m, op="max")
        out = torch.zeros(2)
        chunks = [torch.full((2,), 10.0 * r) for r in range(world)] if c.rank == 0 else None
        c.scatter(out, chunks, src=0) if world > 1 else out.copy_(torch.zeros(2))
        return t.tolist(), s.item(), m.item(), out.tolist()
    res = run_ranks(world, fn)
    for r, (t, s, m, out) in enumerate(res):
        assert t == [float(world - 1)] * 4
        assert s == world * (world + 1) / 2 and m == world - 1
        assert out == [10.0 * r] * 2


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_dp_executor_uneven_batches(world):
    shard = 3

    def fn(c):
        def runner(x):  # per-rank "model": row sums + 1000 * rank (which rank computed a row)
            return x.sum(dim=(1, 2)) + 1000 * c.rank
        ex = DPExecutor(runner, shard, (2, 4), (), "cpu", comm=c)
        outs = []
        for n in (world * shard, world * shard - 1, 1):
            x = torch.arange(n * 8, dtype=torch.float32).reshape(n, 2, 4) if c.rank == 0 else None
            outs.append(ex.step(x))
        return outs
    res = run_ranks(world, fn)
    for r in range(1, world):
        assert res[r] == [None, None, None]
    for n, y in zip((world * shard, world * shard - 1, 1), res[0]):
        x = torch.arange(n * 8, dtype=torch.float32).reshape(n, 2, 4)
        expect = x.sum(dim=(1, 2)) + 1000 * (torch.arange(n) // shard)
        assert y.shape == (n,) and torch.equal(y, expect)
    with pytest.raises(ValueError):
        DPExecutor(lambda x: x, 2, (1,), (1,), "cpu").step(torch.zeros(3, 1))


@pytest.mark.parametrize("world", [2, 5])
def test_weight_blob_broadcast_resnet18(world):
    from hipzap.models import registry
    a = registry.get("resnet18")
    torch.manual_seed(0)
    src = a.pack(a.make_model().state_dict(), "cpu")[0]
    meta, _ = a.meta_params()

    def fn(c):
        got = broadcast_params(src if c.rank == 0 else None, meta, "cpu", comm=c)
        return sum(float(p.wf.float().sum() + p.bias.sum()) for p in got.values()), health_check(comm=c)
    res = run_ranks(world, fn)
    assert len({d for d, _ in res}) == 1 and all(h == world for _, h in res)


def test_failing_rank_aborts_peers_instead_of_hanging():
    def fn(c):
        if c.rank == 2:
            c.fail_at = "gather"
        ex = DPExecutor(lambda x: x * 2, 1, (1,), (1,), "cpu", comm=c)
        return ex.step(torch.ones(4, 1) if c.rank == 0 else None)
    res = run_ranks(4, fn, timeout_s=10)
    assert all(isinstance(e, CommError) for e in res), res


class _CountingAsyncComm:
    """A loopback rank that advertises asynchronous collectives and counts host waits: a
    collective called with wait=True (or without ``wait``) is a host sync, and so is sync()."""
    supports_async = True

    def __init__(self, inner):
        self.inner, self.rank, self.world = inner, inner.rank, inner.world
        self.host_syncs, self.async_calls = 0, 0

    def scatter(self, out, chunks, src=0, wait=True):
        self.host_syncs += int(wait)
        self.async_calls += int(not wait)
        self.inner.scatter(out, chunks, src)

    def gather(self, t, outs, dst=0, wait=True):
        self.host_syncs += int(wait)
        self.async_calls += int(not wait)
        self.inner.gather(t, outs, dst)

    def sync(self, stream=None):
        self.host_syncs += 1


def test_dp_step_one_host_sync_per_step():
    """VERDICT r3 "next round" 7: on an asynchronous communicator a DP step enqueues scatter and
    gather without waiting and synchronises the host exactly once (sync=False: not at all), and the
    results are the blocking step's, bitwise."""
    from hipzap.parallel.loopback import run_ranks

    def runner(xs):
        return xs.sum(dim=1) * 2.0

    x = torch.arange(4 * 3 * 5, dtype=torch.float32).reshape(12, 5)

    def body(comm):
        c = _CountingAsyncComm(comm)
        ex = DPExecutor(runner, shard_batch=3, in_shape=(5,), out_shape=(), device="cpu", comm=c)
        outs = [ex.step(x if c.rank == 0 else None) for _ in range(3)]
        syncs_after_3 = c.host_syncs
        ex.step(x if c.rank == 0 else None, sync=False)
        return outs, syncs_after_3, c.host_syncs, c.async_calls

    res = run_ranks(4, body)
    for r, (outs, s3, s4, a) in enumerate(res):
        assert s3 == 3 and s4 == 3 and a == 8, (r, s3, s4, a)  # 1 sync per step; 2 async collectives per step
    for y in res[0][0]:
        assert torch.equal(y, runner(x))


@pytest.mark.parametrize("world,depth", [(1, 1), (1, 3), (2, 2), (4, 3)])
def test_dp_pipeline_results_and_collective_order(world, depth):
    """DPPipeline with ``depth`` steps in flight returns every step's logits in order, equal to the
    blocking one-step executor's (uneven batches included), and issues the collectives in the
    pipelined order sc0 .. sc(D-1), g0, scD, g1, ... on every rank."""
    from hipzap.parallel.dp import DPPipeline, FnSlot
    shard, steps = 3, 7
    sizes = [world * shard - (i % 2) for i in range(steps)]

    def body(c):
        log = []

        class Logged:
            rank, world = c.rank, c.world

            def scatter(self, out, chunks, src=0):
                log.append("s")
                c.scatter(out, chunks, src)

            def gather(self, t, outs, dst=0):
                log.append("g")
                c.gather(t, outs, dst)

        def runner(x):  # row sums + 1000 * rank
            return x.sum(dim=1) + 1000 * c.rank
        slots = [FnSlot(runner, shard, (4,)) for _ in range(depth)]
        pipe = DPPipeline(slots, shard, (), "cpu", comm=Logged() if world > 1 else c)
        outs = []
        for i, n in enumerate(sizes):
            x = torch.arange(n * 4, dtype=torch.float32).reshape(n, 4) + i if c.rank == 0 else None
            y = pipe.submit(x)
            if y is not None:
                outs.append(y.clone() if c.rank == 0 else None)
            elif c.rank != 0 and len(log) and log[-1] == "g":
                outs.append(None)
        tail = pipe.flush()
        outs += [t.clone() if t is not None else None for t in tail]
        return outs, "".join(log)

    res = run_ranks(world, body)
    outs0, log0 = res[0]
    assert len(outs0) == steps
    for i, (n, y) in enumerate(zip(sizes, outs0)):
        x = torch.arange(n * 4, dtype=torch.float32).reshape(n, 4) + i
        assert torch.equal(y, x.sum(dim=1) + 1000 * (torch.arange(n) // shard)), i
    if world > 1:
        expect = "s" * depth + "gs" * (steps - depth) + "g" * depth
        assert all(lg == expect for _, lg in res), [lg for _, lg in res]


def test_dp_pipeline_depth1_is_the_executor():
    from hipzap.parallel.dp import DPPipeline, FnSlot

    def fn(c):
        runner = lambda x: x * 2 + c.rank  # noqa: E731
        ex = DPExecutor(runner, 2, (3,), (3,), "cpu", comm=c)
        pipe = DPPipeline([FnSlot(runner, 2, (3,))], 2, (3,), "cpu", comm=c)
        a, b = [], []
        for i in range(3):
            x = torch.randn(4, 3, generator=torch.Generator().manual_seed(i)) if c.rank == 0 else None
            a.append(ex.step(x))
            y = pipe.submit(x)  # a view of the gather buffer, valid until the next submit at depth 1
            b.append(y.clone() if y is not None else None)
        return a, b, pipe.flush()
    for r, (a, b, rest) in enumerate(run_ranks(2, fn)):
        assert rest == []
        if r == 0:
            assert all(torch.equal(p, q) for p, q in zip(a, b))
        else:
            assert a == b == [None] * 3


def test_dp_pipeline_rejects_bad_slots():
    from hipzap.parallel.dp import DPPipeline, FnSlot
    with pytest.raises(ValueError):
        DPPipeline([], 2, (1,), "cpu")
    with pytest.raises(ValueError):
        DPPipeline([FnSlot(lambda x: x, 3, (1,))], 2, (1,), "cpu")
