"""Communicator interface + an in-process loopback backend (SURVEY.md §4.2 T-comm-fake).

The DP code (``comm.broadcast_params``, ``comm.health_check``, ``dp.DPExecutor``) talks to a
small ``Comm`` interface instead of ``torch.distributed`` directly:

* ``TorchComm`` — the real thing: ``torch.distributed`` (RCCL over xGMI on ROCm, gloo on CPU),
  one process per GPU;
* ``LoopbackComm`` — N "ranks" that are threads of ONE process; collectives are copies through a
  shared rendezvous slot guarded by a barrier. It runs anywhere (no sockets, no devices), so
  the DP executor's ordering, root logic, uneven-batch padding and failure paths are tested at
  world sizes 1-8 in a single pytest process. A rank can be made to fail (``fail_rank``) to
  exercise the error path: every peer then raises ``CommError`` instead of hanging.

Both implement exactly the collectives the serving path uses:
broadcast, scatter, gather, all_reduce(sum/max), barrier.
"""
from __future__ import annotations

import threading

import torch

from .base import Comm, CommError  # noqa: F401  (re-exported: callers import them from here)


class SingleComm(Comm):
    """World size 1: every collective is a local copy (or nothing)."""

    def broadcast(self, t, src=0):
        return None

    def scatter(self, out, chunks, src=0):
        out.copy_(chunks[0])

    def gather(self, t, outs, dst=0):
        outs[0].copy_(t)

    def all_reduce(self, t, op="sum"):
        return None

    def barrier(self):
        return None


class TorchComm(Comm):
    """``torch.distributed`` default group (or ``group``): RCCL on GPUs, gloo on CPU."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist, self.group = dist, group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        # gloo (CPU tests, or a multi-rank rehearsal sharing one GPU) has no device scatter/gather:
        # stage device tensors through host memory. RCCL never takes this path.
        self.host_stage = dist.get_backend(group) == "gloo"

    def _h(self, t):
        return t.cpu() if (t is not None and self.host_stage and t.is_cuda) else t

    @staticmethod
    def _back(dst, src):
        if dst is not None and src is not dst:
            dst.copy_(src)

    def broadcast(self, t, src=0):
        h = self._h(t)
        self.dist.broadcast(h, src=src, group=self.group)
        self._back(t, h)

    def scatter(self, out, chunks, src=0):
        h = self._h(out)
        hc = [self._h(c) for c in chunks] if self.rank == src else None
        self.dist.scatter(h, hc, src=src, group=self.group)
        self._back(out, h)

    def gather(self, t, outs, dst=0):
        ho = [self._h(o) for o in outs] if self.rank == dst else None
        self.dist.gather(self._h(t), ho, dst=dst, group=self.group)
        if ho is not None:
            for o, h in zip(outs, ho):
                self._back(o, h)

    def all_reduce(self, t, op="sum"):
        rop = {"sum": self.dist.ReduceOp.SUM, "max": self.dist.ReduceOp.MAX}[op]
        h = self._h(t)
        self.dist.all_reduce(h, op=rop, group=self.group)
        self._back(t, h)

    def barrier(self):
        self.dist.barrier(group=self.group)


class LoopbackHub:
    """Shared state of one simulated process group (``world`` ranks = threads)."""

    def __init__(self, world: int, timeout_s: float = 30.0):
        self.world = world
        self.timeout = timeout_s
        self._barrier = threading.Barrier(world)
        self.slots: list = [None] * world
        self.failed: set = set()

    def comm(self, rank: int) -> "LoopbackComm":
        return LoopbackComm(self, rank)

    def sync(self):
        try:
            self._barrier.wait(self.timeout)
        except threading.BrokenBarrierError as e:
            raise CommError(f"loopback collective aborted (failed ranks: {sorted(self.failed)})") from e

    def abort(self, rank: int):
        self.failed.add(rank)
        self._barrier.abort()


class LoopbackComm(Comm):
    def __init__(self, hub: LoopbackHub, rank: int):
        self.hub, self.rank, self.world = hub, rank, hub.world
        self.fail_at: str | None = None  # fault injection: "broadcast", "scatter", ... on this rank

    def _enter(self, op: str):
        if self.fail_at == op:
            self.hub.abort(self.rank)
            raise CommError(f"rank {self.rank}: injected failure in {op}")

    def _exchange(self, op: str, value):
        """Publish ``value`` in this rank's slot; return every rank's slot (consistent snapshot)."""
        self._enter(op)
        h = self.hub
        h.slots[self.rank] = value
        h.sync()
        snap = list(h.slots)
        h.sync()  # nobody overwrites a slot before every rank has read the snapshot
        return snap

    def broadcast(self, t, src=0):
        snap = self._exchange("broadcast", t if self.rank == src else None)
        if self.rank != src:
            t.copy_(snap[src])

    def scatter(self, out, chunks, src=0):
        snap = self._exchange("scatter", list(chunks) if self.rank == src else None)
        out.copy_(snap[src][self.rank])

    def gather(self, t, outs, dst=0):
        snap = self._exchange("gather", t.clone())
        if self.rank == dst:
            for o, v in zip(outs, snap):
                o.copy_(v)

    def all_reduce(self, t, op="sum"):
        snap = self._exchange("all_reduce", t.clone())
        acc = snap[0].clone()
        for v in snap[1:]:
            acc = acc + v if op == "sum" else torch.maximum(acc, v)
        t.copy_(acc)

    def barrier(self):
        self._exchange("barrier", None)


def run_ranks(world: int, fn, timeout_s: float = 60.0) -> list:
    """Run ``fn(comm)`` on ``world`` loopback ranks (threads); returns per-rank results, or
    the exception a rank raised in its slot."""
    hub = LoopbackHub(world, timeout_s)
    out: list = [None] * world

    def body(r):
        try:
            out[r] = fn(hub.comm(r))
        except BaseException as e:  # noqa: BLE001 — reported per rank
            out[r] = e
            hub.abort(r)
    th = [threading.Thread(target=body, args=(r,), name=f"loopback-rank{r}") for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout_s + 5)
    return out


def default_comm(group=None) -> Comm:
    """TorchComm when a multi-rank process group is up, else the world-1 SingleComm."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        return TorchComm(group)
    return SingleComm()
