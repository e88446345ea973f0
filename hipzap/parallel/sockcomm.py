"""Host-staged communicator over Unix sockets (torch-free): the rehearsal / test backend of the
DP serving cluster (serve/cluster.py).

RCCL refuses two ranks on one GPU, so a multi-rank run on the 1-GPU development box, and the
CPU tests of the cluster's control plane (ordering, membership changes, a rank dying mid-run),
use this instead of :class:`~hipzap.parallel.rccl.RcclComm`. Same raw-pointer interface
(``broadcast_ptr``, ``scatter_ptr``, ``gather_ptr``, ``allreduce_ptr``); data moves through
rank 0 (a star), staged in host memory with ``memcpy`` (HIP's UVA copy when a GPU is visible,
``ctypes.memmove`` otherwise). Every socket operation has a deadline, so a dead peer raises
:class:`CommError` instead of hanging.
"""
from __future__ import annotations

import array
import ctypes as C
import os
import socket
import struct
import time

from .base import Comm, CommError

_LEN = struct.Struct("<Q")


def host_memcpy(dst: int, src: int, n: int) -> None:
    C.memmove(dst, src, n)


def uva_memcpy(dst: int, src: int, n: int) -> None:
    from .. import hip
    hip.memcpy(dst, src, n, hip.DEFAULT)


def default_memcpy():
    from ..hip import device_count
    return uva_memcpy if device_count() > 0 else host_memcpy


class SocketComm(Comm):
    def __init__(self, rdzv_dir: str, key: str, world: int, rank: int, memcpy=None, timeout_s: float = 30.0,
                 stream_sync=None):
        self.world, self.rank, self.timeout_s = world, rank, timeout_s
        self.memcpy = memcpy or default_memcpy()
        self.stream_sync = stream_sync  # callable(stream) before reading device memory a stream writes
        self.peers: dict[int, socket.socket] = {}
        self._hub = None
        self._closed = False
        self._rdzv, self._key = rdzv_dir, key
        path = os.path.join(rdzv_dir, f"{key}.sock")
        if world <= 1:
            return
        if rank == 0:
            srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
            try:
                os.unlink(path)
            except FileNotFoundError:
                pass
            srv.bind(path)
            srv.listen(world)
            srv.settimeout(timeout_s)
            try:
                while len(self.peers) < world - 1:
                    c, _ = srv.accept()
                    c.settimeout(timeout_s)
                    r = struct.unpack("<i", self._recvn(c, 4))[0]
                    self.peers[r] = c
            except socket.timeout:
                raise CommError(f"socket comm {key}: only {len(self.peers) + 1}/{world} ranks joined")
            finally:
                srv.close()
        else:
            t0 = time.time()
            while True:
                try:
                    s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
                    s.settimeout(timeout_s)
                    s.connect(path)
                    break
                except (FileNotFoundError, ConnectionRefusedError):
                    s.close()
                    if time.time() - t0 > timeout_s:
                        raise CommError(f"socket comm {key}: rank 0 not reachable")
                    time.sleep(0.005)
            s.sendall(struct.pack("<i", rank))
            self._hub = s

    # ---------------------------------------------------------------- framing
    @staticmethod
    def _recvn(s, n: int) -> bytes:
        buf = bytearray(n)
        view, got = memoryview(buf), 0
        while got < n:
            k = s.recv_into(view[got:], n - got)
            if k == 0:
                raise CommError("peer closed the connection")
            got += k
        return bytes(buf)

    def _send(self, s, data: bytes) -> None:
        try:
            s.sendall(_LEN.pack(len(data)) + data)
        except (OSError, socket.timeout) as e:
            raise CommError(f"rank {self.rank}: send failed: {e}") from e

    def _recv(self, s) -> bytes:
        try:
            n = _LEN.unpack(self._recvn(s, 8))[0]
            return self._recvn(s, n)
        except (OSError, socket.timeout) as e:
            raise CommError(f"rank {self.rank}: receive failed: {e}") from e

    def _read(self, ptr: int, n: int, stream=None) -> bytes:
        if stream is not None and self.stream_sync is not None:
            self.stream_sync(stream)
        buf = (C.c_char * max(1, n))()
        self.memcpy(C.addressof(buf), ptr, n)
        return bytes(buf)[:n]

    def _write(self, ptr: int, data: bytes) -> None:
        buf = C.create_string_buffer(data, len(data))
        self.memcpy(ptr, C.addressof(buf), len(data))

    def _check(self):
        if self._closed:
            raise CommError("communicator closed")

    # ---------------------------------------------------------------- raw collectives
    def broadcast_ptr(self, ptr: int, nbytes: int, src: int = 0, stream=None, wait: bool = True) -> None:
        self._check()
        if self.world <= 1:
            return
        if self.rank == 0:
            data = self._read(ptr, nbytes, stream) if src == 0 else self._recv(self.peers[src])
            if src != 0:
                self._write(ptr, data)
            for r, s in self.peers.items():
                if r != src:
                    self._send(s, data)
        elif self.rank == src:
            self._send(self._hub, self._read(ptr, nbytes, stream))
        else:
            self._write(ptr, self._recv(self._hub))

    def scatter_ptr(self, send: int, recv: int, bytes_per_rank: int, src: int = 0, stream=None,
                    wait: bool = True) -> None:
        self._check()
        nb = bytes_per_rank
        if self.world <= 1:
            self._write(recv, self._read(send, nb, stream))
            return
        if self.rank == 0:
            data = self._read(send, nb * self.world, stream) if src == 0 else self._recv(self.peers[src])
            for r, s in self.peers.items():
                self._send(s, data[r * nb: (r + 1) * nb])
            self._write(recv, data[:nb])
        else:
            if self.rank == src:
                self._send(self._hub, self._read(send, nb * self.world, stream))
            self._write(recv, self._recv(self._hub))

    def gather_ptr(self, send: int, recv: int, bytes_per_rank: int, dst: int = 0, stream=None,
                   wait: bool = True) -> None:
        self._check()
        nb = bytes_per_rank
        mine = self._read(send, nb, stream)
        if self.world <= 1:
            self._write(recv, mine)
            return
        if self.rank == 0:
            parts = [mine] + [b""] * (self.world - 1)
            for r, s in self.peers.items():
                parts[r] = self._recv(s)
            data = b"".join(parts)
            if dst == 0:
                self._write(recv, data)
            else:
                self._send(self.peers[dst], data)
        else:
            self._send(self._hub, mine)
            if self.rank == dst:
                self._write(recv, self._recv(self._hub))

    def allreduce_ptr(self, ptr: int, count: int, dtype: str = "int32", op: str = "sum", stream=None,
                      wait: bool = True) -> None:
        self._check()
        code = {"int32": "i", "float32": "f", "float64": "d", "int64": "q"}[dtype]
        nb = count * array.array(code).itemsize
        mine = self._read(ptr, nb, stream)
        if self.world <= 1:
            return
        if self.rank == 0:
            acc = array.array(code, mine)
            for s in self.peers.values():
                other = array.array(code, self._recv(s))
                for i in range(count):
                    a, b = acc[i], other[i]
                    acc[i] = a + b if op == "sum" else max(a, b) if op == "max" else min(a, b)
            data = acc.tobytes()
            for s in self.peers.values():
                self._send(s, data)
            self._write(ptr, data)
        else:
            self._send(self._hub, mine)
            self._write(ptr, self._recv(self._hub))

    def poll(self) -> int:
        return -3 if self._closed else 0

    def abort(self) -> None:
        self.close()

    def shrink(self, exclude: list[int], abort_parent: bool = True) -> "SocketComm":
        """The survivors' communicator (same contract as ``RcclComm.shrink``: every survivor
        calls it with the same excluded ranks; ranks are renumbered densely). The new star is
        keyed by the parent's key and the excluded set, so no new rendezvous id is needed."""
        if self._closed:
            raise CommError("parent communicator already closed; re-initialise instead")
        excl = sorted(set(int(r) for r in exclude))
        if self.rank in excl:
            raise CommError(f"rank {self.rank} cannot shrink itself out")
        new_rank = self.rank - sum(1 for r in excl if r < self.rank)
        key = f"{self._key}.x{'_'.join(map(str, excl))}"
        if abort_parent:
            self.close()
        return SocketComm(self._rdzv, key, self.world - len(excl), new_rank, memcpy=self.memcpy,
                          timeout_s=self.timeout_s, stream_sync=self.stream_sync)

    def close(self) -> None:
        self._closed = True
        for s in list(self.peers.values()) + ([self._hub] if self._hub else []):
            try:
                s.close()
            except OSError:
                pass
        self.peers, self._hub = {}, None

    # ---------------------------------------------------------------- loopback.Comm (tensors)
    def broadcast(self, t, src: int = 0) -> None:
        self.broadcast_ptr(t.data_ptr(), t.numel() * t.element_size(), src)

    def all_reduce(self, t, op: str = "sum") -> None:
        self.allreduce_ptr(t.data_ptr(), t.numel(), str(t.dtype).replace("torch.", ""), op)

    def barrier(self) -> None:
        one = array.array("i", [1])
        self.allreduce_ptr(one.buffer_info()[0], 1, "int32", "sum")
