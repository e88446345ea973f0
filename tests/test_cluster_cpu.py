"""DP serving cluster control plane (serve/cluster.py) across real worker PROCESSES on the CPU:
SocketComm (host staging) + HostShardRunner stand in for RCCL + the GPU shard plan. Batched jobs
are scattered/gathered through the sequencer from any rank, health all-reduces run, and when a
worker dies the survivors reform and keep serving batches (SURVEY.md §4.2 T-comm-fake, §5)."""
import multiprocessing as mp
import os
import time

import numpy as np
import pytest

ITEM, CLASSES, SHARD = 6, 3, 2


def model_fn(x):
    x = x.astype(np.float32)
    return np.stack([x.sum(1), x.max(1), x[:, 0] * 2 + 1], 1)


def _worker(rank, world, rdzv, conn, join=False):
    from hipzap.parallel.sockcomm import SocketComm, host_memcpy
    from hipzap.serve.cluster import Coordinator, HostShardRunner, Member

    def factory(epoch, members):
        return SocketComm(rdzv, f"c{epoch}", len(members), members.index(rank), memcpy=host_memcpy, timeout_s=5.0)

    coord = Coordinator(os.path.join(rdzv, "ctl.sock"), health_s=0.3, world=world) if rank == 0 else None
    comm = None if join else factory(0, list(range(world)))
    runner = HostShardRunner(SHARD, ITEM, CLASSES, world, model_fn)
    m = Member(os.path.join(rdzv, "ctl.sock"), rank, world, comm, factory, runner, timeout_s=20.0, join=join)
    conn.send("ready")
    while True:
        cmd, arg = conn.recv()
        if cmd == "submit":
            try:
                conn.send(("ok", m.submit(arg)))
            except Exception as e:  # noqa: BLE001
                conn.send(("err", repr(e)))
        elif cmd == "submit_timeout":  # the caller gives up before the sequenced run arrives
            try:
                m.submit(arg, timeout=1e-9)
                conn.send(("ok", None))
            except Exception as e:  # noqa: BLE001
                conn.send(("err", type(e).__name__))
        elif cmd == "state":
            conn.send({"members": m.members, "epoch": m.epoch, "health": dict(m.health), "alive": m.alive,
                       "abandoned": m.abandoned, "reforms": coord.reforms if coord else None,
                       "member_reforms": list(m.reforms)})
        elif cmd == "crash":
            os._exit(3)


@pytest.fixture()
def cluster(tmp_path):
    ctx = mp.get_context("spawn")
    world = 3
    pipes, procs = [], []
    for r in range(world):
        a, b = ctx.Pipe()
        p = ctx.Process(target=_worker, args=(r, world, str(tmp_path), b), daemon=True)
        p.start()
        pipes.append(a)
        procs.append(p)
    for a in pipes:
        assert a.poll(60), "worker did not start"
        assert a.recv() == "ready"
    yield pipes, procs
    for p in procs:
        p.kill()
        p.join(5)


def _call(pipe, cmd, arg=None, timeout=60):
    pipe.send((cmd, arg))
    assert pipe.poll(timeout), f"no answer to {cmd}"
    return pipe.recv()


@pytest.mark.timeout(240)
def test_batched_jobs_from_any_rank_and_reform_after_a_worker_dies(cluster):
    pipes, procs = cluster
    rng = np.random.default_rng(0)
    for root, n in ((1, 7), (0, 6), (2, 1), (1, 13)):  # uneven, smaller than and larger than world*shard
        x = rng.integers(0, 256, (n, ITEM), dtype=np.uint8)
        status, y = _call(pipes[root], "submit", x)
        assert status == "ok", y
        np.testing.assert_array_equal(y, model_fn(x))
    time.sleep(1.0)
    st = _call(pipes[1], "state")
    assert st["health"]["ok"] >= 1 and st["health"]["last_world"] == 3
    # a worker dies: the coordinator sees its control connection drop and reforms over the survivors
    pipes[2].send(("crash", None))
    procs[2].join(10)
    t0 = time.time()
    while time.time() - t0 < 30:
        st = _call(pipes[1], "state")
        if st["members"] == [0, 1]:
            break
        time.sleep(0.1)
    assert st["members"] == [0, 1], st
    x = rng.integers(0, 256, (9, ITEM), dtype=np.uint8)
    status, y = _call(pipes[1], "submit", x)
    assert status == "ok", y
    np.testing.assert_array_equal(y, model_fn(x))
    coord = _call(pipes[0], "state")["reforms"]
    assert coord and coord[-1]["members"] == [0, 1] and "lost" in coord[-1]["reason"]
    # a lost member only: the survivors shrank their communicator (no new rendezvous id)
    assert coord[-1]["shrink"] is True
    for r in (0, 1):
        mr = _call(pipes[r], "state")["member_reforms"]
        assert mr and mr[-1]["how"] == "shrink" and mr[-1]["members"] == [0, 1], mr


@pytest.mark.timeout(240)
def test_abandoned_submit_still_joins_the_collectives(cluster):
    """a root whose caller timed out must still run its sequenced scatter/gather
    (with zeros), or the other ranks block until the comm timeout and the cluster reforms."""
    pipes, procs = cluster
    rng = np.random.default_rng(1)
    x = rng.integers(0, 256, (5, ITEM), dtype=np.uint8)
    status, err = _call(pipes[1], "submit_timeout", x)
    assert status == "err" and "Timeout" in err
    for root in (2, 0, 1):  # later jobs from every rank go straight through, no reform
        y_in = rng.integers(0, 256, (4, ITEM), dtype=np.uint8)
        status, y = _call(pipes[root], "submit", y_in, timeout=30)
        assert status == "ok", y
        np.testing.assert_array_equal(y, model_fn(y_in))
    st = _call(pipes[1], "state")
    assert st["abandoned"] == 1 and st["epoch"] == 0 and st["members"] == [0, 1, 2], st
    assert not _call(pipes[0], "state")["reforms"]


@pytest.mark.timeout(240)
def test_members_rejoin_a_restarted_sequencer(cluster, tmp_path):
    """rank 0 (the sequencer's host) dies and is restarted with join: the other
    members reconnect to the new coordinator and batched DP works again over all three."""
    pipes, procs = cluster
    pipes[0].send(("crash", None))
    procs[0].join(10)
    ctx = mp.get_context("spawn")
    a, b = ctx.Pipe()
    p = ctx.Process(target=_worker, args=(0, 3, str(tmp_path), b, True), daemon=True)
    p.start()
    procs.append(p)
    assert a.poll(60) and a.recv() == "ready"
    pipes[0] = a
    t0 = time.time()
    while time.time() - t0 < 60:
        sts = [_call(pp, "state") for pp in pipes]
        if all(s["alive"] and s["members"] == [0, 1, 2] for s in sts) and len({s["epoch"] for s in sts}) == 1:
            break
        time.sleep(0.2)
    assert all(s["members"] == [0, 1, 2] for s in sts), sts
    assert sts[0]["epoch"] >= 1
    rng = np.random.default_rng(2)
    for root in (1, 0, 2):
        x = rng.integers(0, 256, (7, ITEM), dtype=np.uint8)
        status, y = _call(pipes[root], "submit", x, timeout=30)
        assert status == "ok", y
        np.testing.assert_array_equal(y, model_fn(x))
