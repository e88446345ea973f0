"""Data-parallel serving cluster: one worker process per GPU of the node (VERDICT r1 #3;
SURVEY.md §2f C1-C4, §5 failure detection).

    hipzap serve --gpus 8            # launcher: binds the port, spawns + supervises 8 workers

Shape (reference scale-out = Lambda's per-request container fan-out,
/root/reference/zappa_settings.rename.json:1-30; here the containers are GPU worker processes):

* **launcher** (never touches a GPU): binds the listening socket once and spawns the workers
  with it inherited (pre-fork: the kernel hands each new connection to one worker's accept),
  plus a node-local rendezvous directory; restarts a worker that dies.
* **worker** (rank r, GPU r): torch-free on the vision path. Cold start = RCCL communicator
  (``parallel/rccl.py``, unique id through the rendezvous dir) -> the model's plan image with
  rank 0 reading the weights and broadcasting them (C1; the others never read the blob) ->
  its own threaded WSGI server on the shared socket. A bs=1 request is served entirely by the
  worker that accepted it: no cross-process hop, no GIL shared between GPUs.
* **batched POSTs** (configs 3/5): scattered over all ranks (C2), each rank runs its captured
  shard program, logits gathered to the rank that received the request (C3). Collectives must
  be issued in the same order everywhere, so the accepting worker only SUBMITs the job to a
  sequencer (the :class:`Coordinator`, a thread of rank 0) which fans ``run`` commands out in
  one global order to every worker's collective thread (:class:`Member`).
* **health** (C4): the coordinator sequences a 1-int all-reduce every ``health_s``; every wait
  polls ``ncclCommGetAsyncError`` with a deadline. A worker whose control connection drops, or
  that reports a collective failure, triggers a ``reform``: every live member drops its old
  communicator and joins a new one over the survivors (fresh unique id per epoch). Weights are
  already resident, so bs=1 serving never stops. When the only change is a lost member (its
  control connection dropped) the survivors SHRINK their communicator instead
  (``ncclCommShrink`` with abort of the parent: no new unique id, no rendezvous, no bootstrap
  of the survivors' connections); a reform after a failed collective, or a rejoin,
  re-initialises. A restarted worker cold-starts from the plan on disk and rejoins through the
  same path. Rank 0 hosts the sequencer: if it dies, batched
  requests fall back to the receiving worker's GPU alone until it is restarted; the other
  members then reconnect to the restarted sequencer and rejoin (one reform).
"""
from __future__ import annotations

import itertools
import json
import logging
import os
import signal
import socket
import subprocess
import sys
import tempfile
import threading
import time
from concurrent.futures import Future
from concurrent.futures import TimeoutError as FutureTimeout

from ..parallel.base import CommError

log = logging.getLogger("hipzap.cluster")


# --------------------------------------------------------------------------- control messages
def _send(f, lock, obj) -> None:
    with lock:
        f.write(json.dumps(obj).encode() + b"\n")
        f.flush()


def _recv(f):
    line = f.readline()
    return json.loads(line) if line else None


class Coordinator:
    """The sequencer (rank 0): one global order for every collective job, membership epochs."""

    def __init__(self, path: str, health_s: float = 5.0, world: int = 1):
        self.path = path
        self.health_s = health_s
        self.world = world
        self.ready = threading.Event()  # every initial member connected: jobs and health may flow
        self.lock = threading.Lock()
        self.members: dict[int, tuple] = {}  # original rank -> (conn, wfile, send lock)
        self.seq = 0
        # epochs name the rendezvous keys of every communicator generation (uid<epoch>): a
        # RESTARTED sequencer continues after the last epoch it published instead of reusing
        # keys whose stale files are still in the rendezvous directory
        self._epoch_file = path + ".epoch"
        try:
            with open(self._epoch_file) as f:
                self.epoch = int(f.read().strip() or 0)
        except (FileNotFoundError, ValueError):
            self.epoch = 0
        self.reforms: list = []
        self.formed: list = list(range(world))  # members of the current communicator generation
        self._stop = threading.Event()
        try:
            os.unlink(path)
        except FileNotFoundError:
            pass
        self.srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.srv.bind(path)
        self.srv.listen(64)
        threading.Thread(target=self._accept, daemon=True, name="hz-coord-accept").start()
        if health_s > 0:
            threading.Thread(target=self._health, daemon=True, name="hz-coord-health").start()

    def _accept(self):
        while not self._stop.is_set():
            try:
                conn, _ = self.srv.accept()
            except OSError:
                return
            threading.Thread(target=self._serve, args=(conn,), daemon=True, name="hz-coord-conn").start()

    def _serve(self, conn):
        f = conn.makefile("rwb")
        hello = _recv(f)
        if not hello or hello.get("op") != "hello":
            conn.close()
            return
        r = int(hello["rank"])
        with self.lock:
            self.members[r] = (conn, f, threading.Lock())
            if len(self.members) >= self.world:
                self.ready.set()
        if hello.get("join"):
            self.reform(f"rank {r} joined")
        try:
            while True:
                msg = _recv(f)
                if msg is None:
                    break
                op = msg.get("op")
                if op == "submit":
                    self.fanout({"op": "run", "root": r, "token": msg["token"], "n": msg["n"]})
                elif op == "fail":
                    with self.lock:
                        stale = msg.get("epoch", -1) < self.epoch
                    if not stale:
                        self.reform(f"rank {r}: {msg.get('reason', 'collective failed')}")
        except (OSError, ValueError):
            pass
        with self.lock:
            cur = self.members.get(r)
            if cur is not None and cur[0] is conn:
                del self.members[r]
            else:
                return
        if not self._stop.is_set():
            self.reform(f"rank {r} lost", shrink_ok=True)

    def fanout(self, msg: dict) -> None:
        """Send ``msg`` to every live member, stamped with one global sequence number. Waits
        until the initial membership is complete (a collective needs every rank)."""
        self.ready.wait(60.0)
        with self.lock:
            self.seq += 1
            msg = dict(msg, seq=self.seq, epoch=self.epoch)
            dead = []
            for r, (conn, f, lk) in self.members.items():
                try:
                    _send(f, lk, msg)
                except OSError:
                    dead.append(r)
            for r in dead:
                self.members.pop(r, None)

    def reform(self, reason: str, shrink_ok: bool = False) -> None:
        """New communicator generation over the live members. ``shrink`` is offered only when the
        members are a strict subset of the current generation (nobody joins), the trigger is a
        lost control connection (the survivors' communicators were not aborted by a timed-out
        collective). A member that cannot shrink re-initialises; the mismatch ends in a bounded
        timeout -> ``fail`` -> a reform that always re-initialises."""
        with self.lock:
            self.epoch += 1
            tmp = f"{self._epoch_file}.{os.getpid()}"
            with open(tmp, "w") as f:
                f.write(str(self.epoch))
            os.replace(tmp, self._epoch_file)
            members = sorted(self.members)
            prev = list(self.formed)
            shrink = bool(shrink_ok and members and set(members) < set(prev))
            self.formed = members
            self.reforms.append({"epoch": self.epoch, "members": members, "reason": reason, "shrink": shrink})
            log.warning("cluster reform epoch %d: members %s (%s%s)", self.epoch, members, reason,
                        ", shrink" if shrink else "")
            msg = {"op": "reform", "epoch": self.epoch, "members": members, "reason": reason,
                   "shrink": shrink, "prev": prev}
            self.seq += 1
            msg["seq"] = self.seq
            for r, (conn, f, lk) in list(self.members.items()):
                try:
                    _send(f, lk, msg)
                except OSError:
                    self.members.pop(r, None)

    def _health(self):
        self.ready.wait()
        while not self._stop.wait(self.health_s):
            self.fanout({"op": "health"})

    def close(self):
        self._stop.set()
        try:
            self.srv.close()
        except OSError:
            pass


class Member:
    """A worker's end of the control plane: submits batched jobs to the sequencer and runs every
    sequenced collective (DP step, health all-reduce, reform) on ONE thread, in order.

    ``comm_factory(epoch, members) -> comm`` builds the communicator over ``members`` (original
    ranks; this worker's rank in it is its index); ``runner`` executes one shard on this rank's
    GPU (:class:`PlanShardRunner`) or a test double."""

    def __init__(self, ctl_path: str, rank: int, world: int, comm, comm_factory, runner, join: bool = False,
                 timeout_s: float = 60.0):
        self.rank, self.comm, self.comm_factory, self.runner = rank, comm, comm_factory, runner
        self.members = list(range(world)) if comm is not None else [rank]
        self.epoch = 0
        self.timeout_s = timeout_s
        self.pending: dict[str, list] = {}  # token -> [array or None (abandoned), future]
        self.abandoned = 0
        self.ctl_path = ctl_path
        self.reconnect_s = float(os.environ.get("HIPZAP_CTL_RECONNECT_S", 120.0))
        self._closed = False
        self.health = {"ok": 0, "failed": 0, "last_world": None}
        self.reforms: list = []
        self._ids = itertools.count()
        self._lock = threading.Lock()
        self._wlock = threading.Lock()
        self._connect(join=join, timeout_s=timeout_s)
        self.alive = True
        self.thread = threading.Thread(target=self._loop, daemon=True, name=f"hz-member-{rank}")
        self.thread.start()

    # ---------------------------------------------------------------- requests
    def submit(self, arr, timeout: float | None = None):
        """Run a batch over the whole cluster (blocking); ``arr``: numpy [n, ...] of the
        runner's item shape. Returns numpy [n, classes].

        The job stays registered until its sequenced ``run`` reaches this rank, even when the
        caller gives up first: the ``run`` is already on its way to every other rank, which will
        enter the scatter/gather, so this (root) rank must join them (``_run`` stages zeros for
        an abandoned job and drops the output) instead of leaving them blocked until the
        communicator times out and the whole cluster reforms."""
        if not self.alive:
            raise CommError("control plane is down")
        token = f"{self.rank}-{next(self._ids)}"
        fut: Future = Future()
        with self._lock:
            self.pending[token] = [arr, fut]
        try:
            _send(self.f, self._wlock, {"op": "submit", "token": token, "n": int(arr.shape[0])})
        except OSError as e:
            with self._lock:
                self.pending.pop(token, None)
            raise CommError(f"control plane send failed: {e}") from e
        try:
            return fut.result(timeout or self.timeout_s)
        except FutureTimeout:
            with self._lock:
                job = self.pending.get(token)
                if job is not None:
                    job[0] = None  # abandoned: the sequenced run still joins the collectives with zeros
            self.abandoned += 1
            raise

    # ---------------------------------------------------------------- sequenced work
    def _connect(self, join: bool, timeout_s: float) -> None:
        t0 = time.time()
        while True:
            sock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
            try:
                sock.connect(self.ctl_path)
                break
            except (FileNotFoundError, ConnectionRefusedError):
                sock.close()
                if time.time() - t0 > timeout_s or self._closed:
                    raise CommError(f"coordinator {self.ctl_path} not reachable")
                time.sleep(0.01 if not join else 0.2)
        self.sock = sock
        self.f = sock.makefile("rwb")
        _send(self.f, self._wlock, {"op": "hello", "rank": self.rank, "join": join})

    def _loop(self):
        """Sequenced work from the coordinator. When the control connection drops (rank 0, the
        sequencer's host, died), fail the pending jobs, drop the communicator and keep trying to
        reach the RESTARTED coordinator at the same path for ``HIPZAP_CTL_RECONNECT_S``: the
        rejoin (hello with ``join``) makes it reform a communicator over everyone who is back,
        so batched DP resumes after a rank-0 restart instead of staying off."""
        while True:
            try:
                while True:
                    msg = _recv(self.f)
                    if msg is None:
                        break
                    op = msg["op"]
                    if op == "run":
                        self._run(msg)
                    elif op == "health":
                        self._health()
                    elif op == "reform":
                        self._reform(msg)
            except (OSError, ValueError) as e:
                log.warning("rank %d: control connection lost: %s", self.rank, e)
            self.alive = False
            with self._lock:
                for arr, fut in self.pending.values():
                    if not fut.done():
                        fut.set_exception(CommError("control plane lost"))
                self.pending.clear()
            old, self.comm = self.comm, None
            if old is not None:
                try:
                    old.abort()
                    old.close()
                except Exception:  # noqa: BLE001
                    pass
            if self._closed or self.reconnect_s <= 0:
                return
            try:
                self._connect(join=True, timeout_s=self.reconnect_s)
            except (CommError, OSError) as e:
                log.error("rank %d: coordinator did not come back: %s", self.rank, e)
                return
            log.warning("rank %d: reconnected to the coordinator; waiting for the reform", self.rank)
            self.alive = True

    def _fail(self, reason: str) -> None:
        try:
            _send(self.f, self._wlock, {"op": "fail", "epoch": self.epoch, "reason": reason})
        except OSError:
            pass

    def _run(self, msg):
        root_orig = msg["root"]
        mine = root_orig == self.rank
        with self._lock:
            job = self.pending.pop(msg["token"], None) if mine else None
        try:
            if self.comm is None or root_orig not in self.members:
                raise CommError("no communicator for this job")
            # mine but abandoned (caller timed out) or unknown: still the root of this collective
            out = self.dp_step(self.members.index(root_orig), msg["n"], job[0] if job else None)
            if job and not job[1].done():
                job[1].set_result(out)
        except Exception as e:  # noqa: BLE001 - a failed collective must not kill the loop
            if job and not job[1].done():
                job[1].set_exception(e)
            if isinstance(e, CommError):
                self._fail(str(e))

    def dp_step(self, root: int, n: int, arr):
        """C2 scatter -> shard program -> C3 gather, in chunks of world * shard items; the root
        pads the last chunk with zeros and drops the padded rows."""
        import numpy as np
        comm, rn = self.comm, self.runner
        W, S = comm.world, rn.shard
        G = W * S
        out = np.empty((n, rn.classes), np.float32) if comm.rank == root else None
        for off in range(0, n, G):
            m = min(G, n - off)
            if comm.rank == root:
                rn.stage(arr[off: off + m] if arr is not None else np.zeros((m, rn.in_item), np.uint8), G)
            comm.scatter_ptr(rn.staging if comm.rank == root else 0, rn.shard_in, S * rn.in_item, root,
                             stream=rn.stream, wait=False)
            rn.run()
            comm.gather_ptr(rn.shard_out, rn.gather if comm.rank == root else 0, S * rn.out_item, root,
                            stream=rn.stream, wait=True)
            if comm.rank == root:
                y = rn.read_gather(m)
                if arr is not None:
                    out[off: off + m] = y
        return out

    def _health(self):
        if self.comm is None:
            return
        try:
            if self.comm.poll() not in (0,):
                raise CommError(f"asynchronous communicator error {self.comm.poll()}")
            n = self.runner.allreduce_one(self.comm)
            self.health["last_world"] = n
            if n != self.comm.world:
                raise CommError(f"health all-reduce saw {n} of {self.comm.world} ranks")
            self.health["ok"] += 1
        except CommError as e:
            self.health["failed"] += 1
            self._fail(str(e))

    def _reform(self, msg):
        members = msg["members"]
        old, self.comm = self.comm, None
        self.epoch = msg["epoch"]
        t0 = time.perf_counter()
        how = "init"
        if self.rank in members and msg.get("shrink") and old is not None and hasattr(old, "shrink") \
                and list(self.members) == list(msg.get("prev", ())):
            excl = [i for i, r in enumerate(self.members) if r not in members]
            try:
                self.comm = old.shrink(excl, abort_parent=True)
                self.members = members
                how = "shrink"
            except CommError as e:  # the others shrank: this rank's init cannot match them; the
                log.error("rank %d: shrink in epoch %d failed: %s", self.rank, self.epoch, e)  # timeout re-forms
        if old is not None:
            try:
                old.abort()
                old.close()
            except Exception:  # noqa: BLE001
                pass
        if self.rank not in members:
            return
        if self.comm is None:
            try:
                self.comm = self.comm_factory(self.epoch, members) if len(members) > 0 else None
                self.members = members
            except CommError as e:
                log.error("rank %d: reform epoch %d failed: %s", self.rank, self.epoch, e)
                self._fail(str(e))
                return
        self.reforms.append({"epoch": self.epoch, "members": members, "how": how,
                             "ms": (time.perf_counter() - t0) * 1e3})

    def close(self):
        self.alive = False
        self._closed = True
        try:
            self.sock.shutdown(socket.SHUT_RDWR)
            self.sock.close()
        except OSError:
            pass


# --------------------------------------------------------------------------- shard runners
class PlanShardRunner:
    """One rank's shard of a batched request on its GPU: a device-I/O plan image (batch = shard,
    ``hipzap plan --dp-shard``) whose weight blob is a device copy of the serving plan's blob
    (same checkpoint, same packing -> byte-identical; checked by digest), plus the root's
    staging/gather buffers sized for ``max_world`` ranks."""

    def __init__(self, shard_plan: str, device: int, serving_engine, max_world: int):
        import numpy as np
        from .. import hip
        from ..lite import PlanEngine, read_meta
        meta = read_meta(shard_plan)
        same = serving_engine is not None and meta.get("blob_sha256") and \
            meta.get("blob_sha256") == serving_engine.meta.get("blob_sha256")
        fill = None
        if same:
            src, nb = serving_engine.blob()
            fill = lambda addr, n: hip.memcpy(addr, src, n, hip.D2D)  # noqa: E731
        self.engine = PlanEngine(shard_plan, device=device, contexts=1, read_blob=not same, fill_blob=fill)
        (self.shard_in,), self.shard_out = self.engine.device_io(0)
        self.stream = self.engine.stream(0)
        ins, out = meta["inputs"][0], meta["output"]
        self.shard = ins["shape"][0]
        self.in_item = ins["bytes"] // self.shard
        self.out_item = out["bytes"] // self.shard
        self.classes = out.get("num_labels") or out["shape"][-1]
        self.out_cols = out["bytes"] // self.shard // 4
        self.in_shape = tuple(ins["shape"][1:])
        self.max_world = max_world
        G = self.shard * max_world
        self._staging = hip.DeviceBuffer(G * self.in_item)
        self._gather = hip.DeviceBuffer(G * self.out_item)
        self._h_in = hip.PinnedBuffer(G * self.in_item)
        self._h_out = hip.PinnedBuffer(G * self.out_item)
        self._one = hip.DeviceBuffer(64)
        self._one_h = hip.PinnedBuffer(64)
        self._np = np

    @property
    def staging(self) -> int:
        return self._staging.ptr

    @property
    def gather(self) -> int:
        return self._gather.ptr

    def stage(self, arr, G: int) -> None:
        from .. import hip
        np = self._np
        a = np.ascontiguousarray(arr, dtype=np.uint8)
        nb = a.nbytes
        dst = np.frombuffer(self._h_in.view, np.uint8, G * self.in_item)
        dst[:nb] = a.reshape(-1)
        dst[nb:] = 0
        hip.memcpy(self._staging.ptr, self._h_in.ptr, G * self.in_item, hip.H2D, self.stream)

    def run(self) -> None:
        self.engine.replay(0)

    def read_gather(self, m: int):
        from .. import hip
        np = self._np
        hip.memcpy(self._h_out.ptr, self._gather.ptr, m * self.out_item, hip.D2H, self.stream)
        hip.sync(self.stream)
        y = np.frombuffer(self._h_out.view, np.float32, m * self.out_cols).reshape(m, self.out_cols)
        return y[:, : self.classes].copy()

    def allreduce_one(self, comm) -> int:
        import ctypes as C
        from .. import hip
        C.c_int.from_address(self._one_h.ptr).value = 1
        hip.memcpy(self._one.ptr, self._one_h.ptr, 4, hip.H2D)
        comm.allreduce_ptr(self._one.ptr, 1, "int32", "sum")
        hip.memcpy(self._one_h.ptr, self._one.ptr, 4, hip.D2H)
        return C.c_int.from_address(self._one_h.ptr).value


class HostShardRunner:
    """CPU stand-in for :class:`PlanShardRunner` (control-plane tests and rehearsals without a
    GPU): "device" buffers are host memory, the shard program is ``fn(uint8 [shard, item]) ->
    float32 [shard, classes]``. Pair it with a SocketComm using ``host_memcpy``."""

    def __init__(self, shard: int, item_bytes: int, classes: int, max_world: int, fn):
        import ctypes as C
        import numpy as np
        self._np, self._C = np, C
        self.shard, self.in_item, self.classes, self.out_item = shard, item_bytes, classes, classes * 4
        self.fn, self.stream = fn, None
        self._bufs = [(C.c_char * n)() for n in (shard * item_bytes, shard * self.out_item,
                                                 shard * max_world * item_bytes, shard * max_world * self.out_item)]
        self.shard_in, self.shard_out, self.staging, self.gather = (C.addressof(b) for b in self._bufs)

    def stage(self, arr, G: int) -> None:
        np = self._np
        dst = np.frombuffer(self._bufs[2], np.uint8)
        a = np.ascontiguousarray(arr, np.uint8).reshape(-1)
        dst[: a.size] = a
        dst[a.size: G * self.in_item] = 0

    def run(self) -> None:
        np = self._np
        x = np.frombuffer(self._bufs[0], np.uint8).reshape(self.shard, self.in_item)
        np.frombuffer(self._bufs[1], np.float32)[:] = np.asarray(self.fn(x), np.float32).reshape(-1)

    def read_gather(self, m: int):
        np = self._np
        return np.frombuffer(self._bufs[3], np.float32)[: m * self.classes].reshape(m, self.classes).copy()

    def allreduce_one(self, comm) -> int:
        import array
        a = array.array("i", [1])
        comm.allreduce_ptr(a.buffer_info()[0], 1, "int32", "sum")
        return a[0]


# --------------------------------------------------------------------------- worker process
def make_comm_factory(kind: str, rdzv_dir: str, rank: int, device: int, timeout_s: float):
    """epoch, members (original ranks) -> communicator; this worker's rank = its index."""
    def factory(epoch: int, members: list):
        idx = members.index(rank)
        if kind == "socket":
            from ..parallel.sockcomm import SocketComm
            from .. import hip
            return SocketComm(rdzv_dir, f"c{epoch}", len(members), idx, timeout_s=timeout_s, stream_sync=hip.sync)
        from ..parallel.rccl import FileRendezvous, RcclComm, unique_id
        rdzv = FileRendezvous(rdzv_dir)
        key = f"uid{epoch}"
        if idx == 0:
            rdzv.publish(key, unique_id())
        return RcclComm(rdzv.wait(key, timeout=timeout_s), len(members), idx, device, timeout_s)
    return factory


def worker_main() -> int:
    """Entry of one worker process (spawned by :func:`launch`)."""
    import numpy as np
    from werkzeug.serving import WSGIRequestHandler, make_server
    from . import app as app_mod
    from .server import ModelServer
    from .settings import load_settings

    logging.basicConfig(level=os.environ.get("HIPZAP_LOG", "INFO"),
                        format=f"%(asctime)s rank{os.environ.get('RANK', '?')} %(name)s %(message)s")
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    from ..hip import device_count
    ndev = device_count()
    device = local % ndev if ndev and os.environ.get("HIPZAP_SHARE_GPU") == "1" else local
    rdzv = os.environ["HIPZAP_RDZV"]
    join = os.environ.get("HIPZAP_REJOIN") == "1"
    kind = os.environ.get("HIPZAP_COMM", "rccl")
    timeout_s = float(os.environ.get("HIPZAP_COMM_TIMEOUT", 20))
    st = load_settings(os.environ.get("HIPZAP_SETTINGS") or None, os.environ.get("HIPZAP_STAGE") or None)
    st.devices = [device]
    t0 = time.perf_counter()
    factory = make_comm_factory(kind, rdzv, rank, device, timeout_s)
    comm = None if join or world <= 1 else factory(0, list(range(world)))
    srv = ModelServer(st, backend="gpu")
    srv.comm = comm  # plan weights: rank 0 reads + broadcasts (C1), the others receive
    model = st.default_model
    backend = srv.vision(model)  # collective on every rank at the same point: the cold start
    cold_ms = (time.perf_counter() - t0) * 1e3
    srv.comm = None  # a restarted worker or a later reform never re-broadcasts weights
    spec = srv.spec(model)
    member = coord = None
    dp_plan = spec.extra.get("dp_plan")
    if world > 1:
        if rank == 0:
            coord = Coordinator(os.path.join(rdzv, "ctl.sock"), float(os.environ.get("HIPZAP_HEALTH_S", 5)), world)
        runner = None
        if dp_plan and hasattr(backend, "engine"):
            runner = PlanShardRunner(dp_plan, device, backend.engine, world)
        member = Member(os.path.join(rdzv, "ctl.sock"), rank, world, comm, factory, runner, join=join,
                        timeout_s=timeout_s * 3)
        app_mod.set_dp(member if runner is not None else None, model, runner.in_shape if runner else None)
    app_mod.set_server(srv)
    app_mod.CLUSTER.update({"rank": rank, "world": world, "device": device, "cold_start_ms": round(cold_ms, 2),
                            "member": member, "coordinator": coord})
    fd = int(os.environ["HIPZAP_LISTEN_FD"])
    log.info("worker %d/%d on GPU %d ready in %.1f ms (%s)", rank, world, device, cold_ms, backend.__class__.__name__)
    del np
    if os.environ.get("HIPZAP_NATIVE_HTTP", "1") != "0":
        from .native_http import NativeHTTPServer
        from .server import PlanVisionBackend
        fast = backend if isinstance(backend, PlanVisionBackend) else None
        if os.environ.get("HIPZAP_LM_PRELOAD", "0") == "1":
            srv.lm()  # GET /inference backend before the port opens (else on its first request)
        srv_http = NativeHTTPServer(app_mod.app, socket.socket(fileno=fd), fast=fast, server=srv)
        app_mod.CLUSTER["http"] = srv_http
        srv_http.serve_forever()
        return 0
    WSGIRequestHandler.protocol_version = "HTTP/1.1"
    httpd = make_server(st.host, st.port, app_mod.app, threaded=True, fd=fd)
    try:
        httpd.serve_forever()
    except KeyboardInterrupt:
        pass
    return 0


def launch(gpus: int, host: str, port: int, settings: str | None = None, stage: str | None = None,
           restart: bool = True, comm: str | None = None) -> int:
    """Bind ``host:port``, spawn one worker per GPU with the socket inherited, supervise."""
    lsock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    lsock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    lsock.bind((host, port))
    lsock.listen(1024)
    lsock.set_inheritable(True)
    rdzv = tempfile.mkdtemp(prefix="hipzap_rdzv_")
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    base_env = dict(os.environ, WORLD_SIZE=str(gpus), HIPZAP_RDZV=rdzv, HIPZAP_LISTEN_FD=str(lsock.fileno()),
                    HIPZAP_COMM=comm or os.environ.get("HIPZAP_COMM", "rccl"),
                    HIPZAP_WATCHDOG=os.environ.get("HIPZAP_WATCHDOG", "0"))
    if settings:
        base_env["HIPZAP_SETTINGS"] = os.path.abspath(settings)
    if stage:
        base_env["HIPZAP_STAGE"] = stage
    base_env.setdefault("MASTER_ADDR", "127.0.0.1")

    def spawn(r: int, rejoin: bool = False):
        env = dict(base_env, RANK=str(r), LOCAL_RANK=str(r), HIPZAP_REJOIN="1" if rejoin else "0")
        return subprocess.Popen([sys.executable, "-c", "from hipzap.serve.cluster import worker_main; "
                                                       "raise SystemExit(worker_main())"],
                                cwd=root, env=env, pass_fds=(lsock.fileno(),))

    procs = {r: spawn(r) for r in range(gpus)}
    print(f"hipzap cluster: {gpus} workers on {host}:{port} (rendezvous {rdzv})", flush=True)
    stopping = threading.Event()

    def stop(*_):
        stopping.set()

    signal.signal(signal.SIGTERM, stop)
    signal.signal(signal.SIGINT, stop)
    restarts = 0
    while not stopping.is_set():
        time.sleep(0.2)
        for r, p in list(procs.items()):
            rc = p.poll()
            if rc is None:
                continue
            log.warning("worker %d exited with %s", r, rc)
            if restart and restarts < 16 and not stopping.is_set():
                restarts += 1
                procs[r] = spawn(r, rejoin=True)
            else:
                procs.pop(r)
        if not procs:
            break
    for p in procs.values():
        p.terminate()
    for p in procs.values():
        try:
            p.wait(timeout=20)
        except subprocess.TimeoutExpired:
            p.kill()
    lsock.close()
    return 0
