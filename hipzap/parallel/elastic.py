"""Elastic data parallelism: keep serving when a rank dies (SURVEY.md §5 'Failure detection /
elastic recovery': "on a device fault, drop that rank from the DP set (re-init the communicator
with the survivors) and keep serving").

Protocol (all state lives in a rendezvous store that outlives any single rank — a
``FileStore`` on the node, or an in-process ``HashStore`` for the loopback communicator):

* every rank heartbeats ``hb/<rank>`` (wall-clock time) from a daemon thread, including while
  its main thread is blocked inside a collective;
* after a collective fails, a survivor tears down the broken communicator, and the first one to
  get there publishes the live set — the ranks whose heartbeat is fresher than ``stale_s`` —
  with ``compare_set(decided/<epoch>)``; everybody adopts that one published set (no split
  brain), even ranks that notice the failure much later (a peer still blocked until its
  collective timeout); a rank left out of the set stops;
* survivors meet at ``arrive/<epoch+1>`` (store wait with a long timeout) and build the next
  communicator over the survivors, ranks renumbered in order.

``ElasticDPExecutor`` wraps the scatter/gather executor: rank 0 of the current group (the
request front-end) calls ``step(batch)`` per global batch and ``close()`` at the end, the other
ranks call ``serve()``. The front-end owns the global batch, which is processed in rounds of ``world * shard`` so a
smaller group still serves the whole batch. A failure of the front-end itself loses its in-flight
requests (they live only there); any other rank may fail and the step is retried on the
survivors.
"""
from __future__ import annotations

import datetime
import json
import threading
import time
from typing import Callable

import torch

from .dp import DPExecutor
from .loopback import Comm, CommError, LoopbackHub, TorchComm


class ElasticGroup:
    def __init__(self, store, orig_rank: int, world: int, make_comm: Callable[[int, int, int], Comm],
                 stale_s: float = 1.0, heartbeat_s: float = 0.1, arrive_timeout_s: float = 120.0):
        """``make_comm(epoch, rank, world) -> Comm`` builds the communicator of one epoch."""
        self.store = store
        self.orig_rank = orig_rank
        self.live = list(range(world))
        self.epoch = 0
        self.stale_s, self.heartbeat_s = stale_s, heartbeat_s
        self.arrive_timeout = datetime.timedelta(seconds=arrive_timeout_s)
        self.make_comm = make_comm
        self._stop = threading.Event()
        self._beat()
        self._hb = threading.Thread(target=self._heartbeat, name=f"hipzap-hb{orig_rank}", daemon=True)
        self._hb.start()
        self.comm = make_comm(0, orig_rank, world)

    def _beat(self):
        self.store.set(f"hz/hb/{self.orig_rank}", repr(time.time()))

    def _heartbeat(self):
        while not self._stop.wait(self.heartbeat_s):
            try:
                self._beat()
            except Exception:  # noqa: BLE001 — store gone: the process is shutting down
                return

    def stop(self):
        self._stop.set()

    @property
    def rank(self) -> int:
        return self.live.index(self.orig_rank)

    @property
    def world(self) -> int:
        return len(self.live)

    def alive(self) -> list[int]:
        """Members of the current group whose heartbeat is fresh."""
        now, out = time.time(), []
        for r in self.live:
            key = f"hz/hb/{r}"
            if self.store.check([key]) and now - float(self.store.get(key)) < self.stale_s:
                out.append(r)
        return out

    def reform(self, teardown: Callable[[], None] | None = None) -> None:
        ep = self.epoch
        if teardown is not None:
            try:
                teardown()
            except Exception:  # noqa: BLE001 — the old group is broken anyway
                pass
        # a peer that crashed just now still has a fresh beat: let it go stale first
        time.sleep(self.stale_s + self.heartbeat_s)
        decided = self.store.compare_set(f"hz/decided/{ep}", "", json.dumps(self.alive()))
        live = json.loads(decided.decode() if isinstance(decided, bytes) else decided)
        if self.orig_rank not in live:
            self.stop()
            raise CommError(f"rank {self.orig_rank} was left out of the re-formed group {live}")
        self.store.set(f"hz/arrive/{ep + 1}/{self.orig_rank}", "1")
        self.store.wait([f"hz/arrive/{ep + 1}/{r}" for r in live], self.arrive_timeout)
        self.epoch, self.live = ep + 1, live
        self.comm = self.make_comm(self.epoch, self.rank, self.world)


class ElasticDPExecutor:
    """Scatter/gather DP over an :class:`ElasticGroup` that retries a step on the survivors."""

    def __init__(self, group: ElasticGroup, runner: Callable[[torch.Tensor], torch.Tensor], shard_batch: int,
                 in_shape: tuple, out_shape: tuple, device, teardown: Callable[[], None] | None = None,
                 max_reforms: int = 4):
        self.group = group
        self.args = (runner, shard_batch, tuple(in_shape), tuple(out_shape), device)
        self.teardown = teardown
        self.max_reforms = max_reforms
        self.reforms = 0
        self._ex_epoch = -1
        self._ex = None

    def _executor(self) -> DPExecutor:
        if self._ex_epoch != self.group.epoch:
            runner, shard, ins, outs, dev = self.args
            self._ex = DPExecutor(runner, shard, ins, outs, dev, comm=self.group.comm)
            self._ex_epoch = self.group.epoch
        return self._ex

    def _run(self, x, stop: bool = False):
        ex = self._executor()
        comm = self.group.comm
        n0 = -1 if stop else (x.shape[0] if ex.rank == 0 else 0)
        n = torch.tensor([n0], dtype=torch.int64, device=ex.device)
        comm.broadcast(n, src=0)  # the whole group learns how many rounds this batch takes (-1: stop)
        n = int(n.item())
        if n < 0:
            return _STOP
        per = ex.global_batch
        outs = []
        for r0 in range(0, n, per):
            y = ex.step(x[r0: r0 + per] if ex.rank == 0 else None)
            if ex.rank == 0:
                outs.append(y)
        return torch.cat(outs) if ex.rank == 0 else None

    def _retrying(self, fn):
        while True:
            try:
                return fn()
            except (CommError, RuntimeError) as e:  # a collective failed: re-form without the dead
                if self.reforms >= self.max_reforms:
                    raise
                self.reforms += 1
                was_root = self.group.rank == 0
                self.group.reform(self.teardown)
                if self.group.rank == 0 and not was_root:
                    raise CommError("the request front-end (rank 0) failed: its in-flight batch is lost") from e

    def step(self, x: torch.Tensor) -> torch.Tensor:
        """Front-end (group rank 0): serve one global batch over the live group."""
        return self._retrying(lambda: self._run(x))

    def serve(self) -> None:
        """Worker ranks: take part in every step the front-end issues until it calls ``close``.
        (Workers do not count steps: after a failure the front-end retries the step it was in,
        and the workers simply serve whatever comes next.)"""
        while self._retrying(lambda: self._run(None)) is not _STOP:
            pass

    def close(self) -> None:
        """Front-end: release the workers from ``serve``."""
        self._retrying(lambda: self._run(None, stop=True))


_STOP = object()


# ----------------------------------------------------------------------------- factories
def torch_comm_factory(store, backend: str = "gloo", timeout_s: float = 30.0, device=None):
    """Each epoch is a fresh default process group on a ``PrefixStore`` of the shared store."""
    import torch.distributed as dist

    def make(epoch: int, rank: int, world: int) -> Comm:
        if dist.is_initialized():
            dist.destroy_process_group()
        kw = dict(backend=backend, store=dist.PrefixStore(f"hz/pg/{epoch}", store), rank=rank, world_size=world,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl" and device is not None:
            kw["device_id"] = torch.device(device)
        dist.init_process_group(**kw)
        return TorchComm()

    def teardown():
        if dist.is_initialized():
            dist.destroy_process_group()
    return make, teardown


class LoopbackEpochs:
    """Loopback communicators per epoch for threads of one process (tests): every survivor of an
    epoch asks for the same hub, created on first request with the epoch's world size."""

    def __init__(self, timeout_s: float = 10.0):
        self._hubs: dict = {}
        self._lock = threading.Lock()
        self.timeout = timeout_s

    def make(self, epoch: int, rank: int, world: int) -> Comm:
        with self._lock:
            hub = self._hubs.get(epoch)
            if hub is None:
                hub = self._hubs[epoch] = LoopbackHub(world, self.timeout)
        return hub.comm(rank)

    def abort_all(self):
        with self._lock:
            for r, hub in self._hubs.items():
                hub.abort(-1)
