"""The communicator interface shared by every backend, torch-free (so the native RCCL
communicator in ``rccl.py`` can be used by processes that never import torch)."""
from __future__ import annotations


class CommError(RuntimeError):
    pass


class Comm:
    """Collectives of the serving path over tensors of one rank."""
    rank: int = 0
    world: int = 1

    def broadcast(self, t, src: int = 0) -> None: ...
    def scatter(self, out, chunks: list | None, src: int = 0) -> None: ...
    def gather(self, t, outs: list | None, dst: int = 0) -> None: ...
    def all_reduce(self, t, op: str = "sum") -> None: ...
    def barrier(self) -> None: ...

    # asynchronous communicators (RcclComm) set this and accept scatter/gather(..., wait=False)
    # plus sync(stream): the collective is stream-ordered and the host waits once, in sync()
    supports_async: bool = False

    def sync(self, stream=None) -> None: ...
