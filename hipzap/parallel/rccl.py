"""Native RCCL communicator (csrc/comm/comm.cpp -> libhipzap_comm.so), torch-free.

One process per GPU. Rendezvous of the 128-byte ncclUniqueId goes through a node-local
directory (``FileRendezvous``: rank 0 writes it atomically, the others poll) or any object
broadcast the caller already has (torch.distributed in ``bench.py``). Collectives take raw
device addresses or anything with ``data_ptr()`` (torch tensors), run on the communicator's
stream (or a given one) and, by default, return only after completion — with
``ncclCommGetAsyncError`` polled and a deadline, so a dead peer surfaces as :class:`CommError`
in bounded time (SURVEY.md §5 failure detection) instead of a hang.

:class:`RcclComm` also implements the ``loopback.Comm`` interface (broadcast, scatter, gather,
all_reduce, barrier on torch tensors), so ``DPExecutor`` and ``broadcast_params`` run on it
unchanged.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
import time
from pathlib import Path

from .. import _native
from .base import Comm, CommError

_LIB_PATH = Path(_native.__file__).resolve().parent / "_lib" / "libhipzap_comm.so"
_lock = threading.Lock()
_lib = None
ID_BYTES = 128
TIMEOUT, ABORTED = -2, -3


def lib():
    global _lib
    with _lock:
        if _lib is None:
            if not _LIB_PATH.exists():
                from .. import build as _b
                _b.build_comm(verbose=False)
            _native.lib()  # the HIP runtime + hipzap core first (shared process state)
            L = C.CDLL(str(_LIB_PATH), mode=C.RTLD_GLOBAL)
            P, I, U64, D = C.c_void_p, C.c_int, C.c_uint64, C.c_double
            sig = _native._sig
            sig(L, "hz_comm_last_error", C.c_char_p)
            sig(L, "hz_comm_unique_id", I, C.c_char_p)
            sig(L, "hz_comm_init", P, C.c_char_p, I, I, I, D)
            sig(L, "hz_comm_rank", I, P)
            sig(L, "hz_comm_size", I, P)
            sig(L, "hz_comm_stream", P, P)
            sig(L, "hz_comm_set_timeout", None, P, D)
            sig(L, "hz_comm_poll", I, P)
            sig(L, "hz_comm_abort", I, P)
            sig(L, "hz_comm_broadcast", I, P, P, U64, I, P, I)
            sig(L, "hz_comm_scatter", I, P, P, P, U64, I, P, I)
            sig(L, "hz_comm_gather", I, P, P, P, U64, I, P, I)
            sig(L, "hz_comm_allreduce", I, P, P, U64, I, I, P, I)
            sig(L, "hz_comm_sync", I, P, P)
            sig(L, "hz_comm_shrink", P, P, C.POINTER(I), I, I)
            sig(L, "hz_comm_destroy", None, P)
            _lib = L
    return _lib


def mapped_rccl(maps_text: str | None = None) -> dict:
    """Which librccl this process has mapped and its ``ncclGetVersion`` (VERDICT r4 missing 1b).

    ``libhipzap_comm.so`` is linked against ``librccl.so.1``; in a process that imported torch the
    dynamic linker resolves that soname to the copy torch already loaded (``torch/lib/librccl.so``,
    same soname), so the native communicator and torch.distributed share ONE RCCL build -- intended:
    two RCCL copies in one process would keep two sets of proxies / IPC handles. That build may lack
    ``ncclCommShrink`` (resolved at run time; the cluster falls back to re-initialising). Reported by
    every bench rank. ``maps_text``: a /proc/self/maps text to parse instead (tests)."""
    if maps_text is None:
        try:
            with open("/proc/self/maps") as f:
                maps_text = f.read()
        except OSError:
            maps_text = ""
    paths = sorted({ln.split()[-1] for ln in maps_text.splitlines()
                    if "librccl" in ln and len(ln.split()) >= 6 and ln.split()[-1].startswith("/")})
    version, shrink = None, None
    if paths and maps_text is not None:
        try:  # RTLD_NOLOAD: a handle to the copy already mapped, never a new load
            L = C.CDLL(paths[0], mode=os.RTLD_NOLOAD | C.RTLD_GLOBAL)
            v = C.c_int(0)
            if L.ncclGetVersion(C.byref(v)) == 0:
                version = v.value
            shrink = hasattr(L, "ncclCommShrink")
        except (OSError, AttributeError):
            pass
    return {"paths": paths, "version": version, "torch_bundled": any("/torch/lib/" in p for p in paths),
            "has_comm_shrink": shrink}


def available() -> bool:
    return _LIB_PATH.exists() or _native.available()


def unique_id() -> bytes:
    buf = C.create_string_buffer(ID_BYTES)
    rc = lib().hz_comm_unique_id(buf)
    if rc:
        raise CommError(f"ncclGetUniqueId failed: {lib().hz_comm_last_error().decode()}")
    return buf.raw


class FileRendezvous:
    """Exchange small blobs through a node-local directory (one node: the 8 GPUs of a box).
    ``publish`` is atomic (write + rename); ``wait`` polls until the file exists."""

    def __init__(self, root: str):
        self.root = Path(root)
        self.root.mkdir(parents=True, exist_ok=True)

    def publish(self, key: str, data: bytes) -> None:
        tmp = self.root / f".{key}.tmp{os.getpid()}"
        tmp.write_bytes(data)
        os.replace(tmp, self.root / key)

    def wait(self, key: str, timeout: float = 120.0) -> bytes:
        p, t0 = self.root / key, time.time()
        while not p.exists():
            if time.time() - t0 > timeout:
                raise CommError(f"rendezvous: {p} did not appear within {timeout:.0f} s")
            time.sleep(0.002)
        return p.read_bytes()


def _ptr(x) -> int:
    if x is None:
        return 0
    if isinstance(x, int):
        return x
    return x.data_ptr()


def _nbytes(t) -> int:
    return t.numel() * t.element_size()


def _stream_of(t):
    """The torch current stream for a tensor's device (the collective is ordered after the
    producer), or None for raw pointers."""
    if hasattr(t, "is_cuda") and t.is_cuda:
        import torch
        return torch.cuda.current_stream(t.device).cuda_stream
    return None


class RcclComm(Comm):
    """A non-blocking RCCL communicator with bounded waits. ``timeout_s`` bounds init and every
    collective; on timeout or an asynchronous error the communicator is aborted and the call
    raises :class:`CommError`."""

    def __init__(self, uid: bytes, world: int, rank: int, device: int, timeout_s: float = 60.0, _handle=None):
        self.world, self.rank, self.device = world, rank, device
        if _handle is None:
            _handle = lib().hz_comm_init(uid, world, rank, device, timeout_s)
            if not _handle:
                raise CommError(f"RCCL init failed (rank {rank}/{world}): {lib().hz_comm_last_error().decode()}")
        self._h = _handle
        self.timeout_s = timeout_s

    @classmethod
    def from_rendezvous(cls, rdzv: FileRendezvous, world: int, rank: int, device: int, key: str = "nccl_uid",
                        timeout_s: float = 60.0) -> "RcclComm":
        if rank == 0:
            rdzv.publish(key, unique_id())
        uid = rdzv.wait(key, timeout=timeout_s)
        return cls(uid, world, rank, device, timeout_s)

    @classmethod
    def from_torch(cls, device: int, timeout_s: float = 60.0) -> "RcclComm":
        """Unique id broadcast over an initialised torch.distributed group (bench.py)."""
        import torch.distributed as dist
        obj = [unique_id() if dist.get_rank() == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        return cls(obj[0], dist.get_world_size(), dist.get_rank(), device, timeout_s)

    # ------------------------------------------------------------------ plumbing
    def _check(self, rc: int, what: str) -> None:
        if rc:
            kind = "timeout" if rc == TIMEOUT else "aborted" if rc == ABORTED else f"error {rc}"
            raise CommError(f"rank {self.rank}: {what} {kind}: {lib().hz_comm_last_error().decode()}")

    def comm_rank(self) -> int:
        """This member's rank as RCCL reports it (ncclCommUserRank)."""
        return int(lib().hz_comm_rank(self._h))

    def comm_size(self) -> int:
        """The communicator's size as RCCL reports it (ncclCommCount)."""
        return int(lib().hz_comm_size(self._h))

    @property
    def stream(self) -> int:
        return lib().hz_comm_stream(self._h)

    def poll(self) -> int:
        """0 healthy; otherwise the asynchronous error (ncclResult_t) or -3 after an abort."""
        return lib().hz_comm_poll(self._h)

    def abort(self) -> None:
        lib().hz_comm_abort(self._h)

    def shrink(self, exclude: list[int], abort_parent: bool = True) -> "RcclComm":
        """Elastic DP: every survivor calls this with the same dead ranks; returns the new
        communicator (ranks renumbered densely)."""
        arr = (C.c_int * len(exclude))(*exclude)
        h = lib().hz_comm_shrink(self._h, arr, len(exclude), int(abort_parent))
        if not h:
            raise CommError(f"ncclCommShrink failed: {lib().hz_comm_last_error().decode()}")
        L = lib()
        return RcclComm(b"", L.hz_comm_size(h), L.hz_comm_rank(h), self.device, self.timeout_s, _handle=h)

    def close(self) -> None:
        h, self._h = getattr(self, "_h", None), None
        if h:
            lib().hz_comm_destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ raw collectives
    def broadcast_ptr(self, ptr: int, nbytes: int, src: int = 0, stream=None, wait: bool = True) -> None:
        self._check(lib().hz_comm_broadcast(self._h, ptr, nbytes, src, stream, int(wait)), "broadcast")

    def scatter_ptr(self, send: int, recv: int, bytes_per_rank: int, src: int = 0, stream=None,
                    wait: bool = True) -> None:
        self._check(lib().hz_comm_scatter(self._h, send, recv, bytes_per_rank, src, stream, int(wait)), "scatter")

    def gather_ptr(self, send: int, recv: int, bytes_per_rank: int, dst: int = 0, stream=None,
                   wait: bool = True) -> None:
        self._check(lib().hz_comm_gather(self._h, send, recv, bytes_per_rank, dst, stream, int(wait)), "gather")

    def allreduce_ptr(self, ptr: int, count: int, dtype: str = "int32", op: str = "sum", stream=None,
                      wait: bool = True) -> None:
        dt = {"int32": 0, "float32": 1, "float64": 2, "int64": 3}[dtype]
        o = {"sum": 0, "max": 2, "min": 3}[op]
        self._check(lib().hz_comm_allreduce(self._h, ptr, count, dt, o, stream, int(wait)), "allreduce")

    # ------------------------------------------------------------------ loopback.Comm (torch tensors)
    supports_async = True  # scatter / gather(wait=False) + sync(stream): DPExecutor's one-sync step

    def broadcast(self, t, src: int = 0) -> None:
        self.broadcast_ptr(_ptr(t), _nbytes(t), src, _stream_of(t))

    def scatter(self, out, chunks, src: int = 0, wait: bool = True) -> None:
        send = 0
        if self.rank == src:
            nb = _nbytes(out)
            send = chunks[0].data_ptr()
            if any(c.data_ptr() != send + i * nb or _nbytes(c) != nb for i, c in enumerate(chunks)):
                raise ValueError("scatter chunks must be equal, contiguous slices of one buffer")
        self.scatter_ptr(send, out.data_ptr(), _nbytes(out), src, _stream_of(out), wait=wait)

    def gather(self, t, outs, dst: int = 0, wait: bool = True) -> None:
        recv = 0
        if self.rank == dst:
            nb = _nbytes(t)
            recv = outs[0].data_ptr()
            if any(o.data_ptr() != recv + i * nb or _nbytes(o) != nb for i, o in enumerate(outs)):
                raise ValueError("gather outputs must be equal, contiguous slices of one buffer")
        self.gather_ptr(t.data_ptr(), recv, _nbytes(t), dst, _stream_of(t), wait=wait)

    def sync(self, stream=None) -> None:
        """Bounded wait for ``stream`` (default: the communicator's): polls the asynchronous
        error state against the deadline; raises CommError on timeout or a transport error."""
        self._check(lib().hz_comm_sync(self._h, stream), "sync")

    def all_reduce(self, t, op: str = "sum") -> None:
        dt = str(t.dtype).replace("torch.", "")
        self.allreduce_ptr(t.data_ptr(), t.numel(), dt, op, _stream_of(t))

    def barrier(self) -> None:
        """1-int all-reduce on a small device scratch buffer owned by the communicator."""
        if not hasattr(self, "_scratch"):
            hip = C.CDLL("libamdhip64.so")
            hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
            p = C.c_void_p()
            if hip.hipMalloc(C.byref(p), 64) != 0:
                raise CommError("hipMalloc failed")
            self._scratch = p.value
        self.allreduce_ptr(self._scratch, 1, "int32", "sum")
