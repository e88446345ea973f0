"""Elastic DP (parallel/elastic.py): a rank dies mid-step, the survivors re-form the group
without it and the step (and later ones) completes over the smaller world — on the in-process
loopback communicator (world 4) and on real gloo process groups (world 3, one process killed)."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hipzap.parallel.elastic import ElasticDPExecutor, ElasticGroup, LoopbackEpochs, torch_comm_factory

SHARD = 2


def _expected(x):
    return x.sum(dim=1)


class Crash(BaseException):
    """A rank dying (not a collective error: the elastic retry must not catch it)."""


def test_loopback_rank_failure_is_survived():
    import threading
    world = 4
    epochs = LoopbackEpochs(timeout_s=10)
    store = dist.HashStore()
    results = {}

    def body(r):
        grp = ElasticGroup(store, r, world, epochs.make)
        calls = {"n": 0}

        def runner(xs):
            calls["n"] += 1
            if r == 2 and calls["n"] == 2:  # rank 2 dies inside its second shard
                grp.stop()  # its heartbeat stops with it
                epochs.abort_all()
                raise Crash()
            return xs.sum(dim=1)
        ex = ElasticDPExecutor(grp, runner, SHARD, (3,), (), "cpu")
        outs = []
        try:
            if grp.rank == 0:
                for step in range(3):
                    outs.append(ex.step(torch.arange(8 * 3, dtype=torch.float32).reshape(8, 3) + step))
                ex.close()
            else:
                ex.serve()
        except Crash:
            results[r] = "crashed"
            return
        results[r] = (outs, grp.world, ex.reforms)
        grp.stop()
    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(60)
    assert results[2] == "crashed"
    outs, w, reforms = results[0]
    assert w == 3 and reforms == 1
    for step, y in enumerate(outs):
        x = torch.arange(8 * 3, dtype=torch.float32).reshape(8, 3) + step
        assert torch.equal(y, _expected(x))  # the 8-row batch is served by 3 ranks in 2 rounds
    assert results[1][1] == 3 and results[3][1] == 3 and results[1][0] == []


def _worker(rank, world, path, q):
    os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
    store = dist.FileStore(path, world)
    make, teardown = torch_comm_factory(store, "gloo", timeout_s=15)
    grp = ElasticGroup(store, rank, world, make)
    calls = {"n": 0}

    def runner(xs):
        calls["n"] += 1
        if rank == 2 and calls["n"] == 2:
            os._exit(1)  # a real crash: the process disappears mid-collective
        return xs.sum(dim=1)
    ex = ElasticDPExecutor(grp, runner, SHARD, (3,), (), "cpu", teardown=teardown)
    outs = []
    if grp.rank == 0:
        for step in range(3):
            outs.append(ex.step(torch.arange(6 * 3, dtype=torch.float32).reshape(6, 3) + step).tolist())
        ex.close()
    else:
        ex.serve()
    q.put((rank, outs, grp.world, ex.reforms))
    grp.stop()
    teardown()


def test_gloo_rank_killed_is_survived(tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    path = str(tmp_path / "store")
    procs = [ctx.Process(target=_worker, args=(r, 3, path, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, outs, w, reforms = q.get(timeout=120)
        res[r] = (outs, w, reforms)
    for p in procs:
        p.join(timeout=60)
    assert procs[2].exitcode == 1
    outs, w, reforms = res[0]
    assert w == 2 and reforms == 1
    for step, y in enumerate(outs):
        x = torch.arange(6 * 3, dtype=torch.float32).reshape(6, 3) + step
        assert y == _expected(x).tolist()
    assert res[1][1] == 2
