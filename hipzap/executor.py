"""Python face of the native request executor (csrc/executor.cpp); torch-free.

Request threads call :meth:`Executor.submit` (the GIL is released inside the native call):
the payload is copied into a free context's pinned input, ONE worker thread launches the
context's hipGraph and polls its completion event, and the caller wakes with the result
copied out. Used by :class:`hipzap.engine.engine.Engine` and :class:`hipzap.lite.PlanEngine`
for every host-I/O request, and by ``bench.py`` (``hz_exec_bench``: native client threads).
"""
from __future__ import annotations

import ctypes as C

from . import _native as N


class Executor:
    def __init__(self, progs: list, streams: list, host_in: list, in_bytes: list, host_out: list, out_bytes: int,
                 rows: int = 1, max_wait_us: float = 200.0, min_inflight: int = 1):
        """``host_in[k][i]``: address of context i's pinned input k; ``host_out[i]``: its output.

        ``rows > 1``: dynamic batching -- the contexts are captured at batch ``rows`` and every
        request is ONE row (``in_bytes[k] / rows`` in, ``out_bytes / rows`` out); a filling batch
        is launched when full, when fewer than ``min_inflight`` batches are on the GPU, or after
        ``max_wait_us`` (csrc/executor.cpp)."""
        n, n_in = len(progs), len(in_bytes)
        assert n > 0 and all(len(h) == n for h in host_in) and len(host_out) == n and 0 < n_in <= 4
        V = C.c_void_p
        flat_in = [a for k in range(n_in) for a in host_in[k]]
        self._keep = ((V * n)(*progs), (V * n)(*streams), (V * (n * n_in))(*flat_in),
                      (C.c_uint64 * n_in)(*in_bytes), (V * n)(*host_out))
        self.n, self.n_in, self.rows = n, n_in, rows
        self.out_bytes, self.in_bytes = out_bytes // rows, [b // rows for b in in_bytes]  # per request
        if rows > 1:
            h = N.lib().hz_exec_create_batched(self._keep[0], self._keep[1], self._keep[2], self._keep[3], n_in,
                                               self._keep[4], out_bytes, n, rows, float(max_wait_us), min_inflight)
        else:
            h = N.lib().hz_exec_create(self._keep[0], self._keep[1], self._keep[2], self._keep[3], n_in,
                                       self._keep[4], out_bytes, n)
        if not h:
            raise RuntimeError("hz_exec_create failed")
        self._h = h

    def submit(self, in_ptrs: list, out_ptr: int) -> float:
        """Blocking request: ``in_ptrs[k]`` = host address of input k's payload (exactly
        ``in_bytes[k]`` bytes), ``out_ptr`` = where the output goes. Returns latency in ms."""
        arr = (C.c_void_p * self.n_in)(*in_ptrs)
        lat = C.c_double()
        rc = N.lib().hz_exec_submit(self._h, arr, out_ptr, C.byref(lat))
        if rc:
            raise RuntimeError(f"executor request failed ({rc})")
        return lat.value * 1e-3

    def submit_rows(self, in_ptrs: list, m: int, out_ptr: int) -> float:
        """Dynamic batching only: one request of ``m`` (1..rows) consecutive rows from this one
        thread (``in_ptrs[k]`` holds m rows of input k, ``out_ptr`` receives m output rows); the
        rows join the open batch like single-row requests. Returns latency in ms."""
        if self.rows <= 1 or not 1 <= m <= self.rows:
            raise ValueError(f"submit_rows: m={m} needs a dynamic-batching executor with rows >= m ({self.rows})")
        arr = (C.c_void_p * self.n_in)(*in_ptrs)
        lat = C.c_double()
        rc = N.lib().hz_exec_submit_rows(self._h, arr, int(m), out_ptr, C.byref(lat))
        if rc:
            raise RuntimeError(f"executor request failed ({rc})")
        return lat.value * 1e-3

    def bench(self, clients: int, iters: int, in_ptrs: list) -> tuple[float, list]:
        """``clients`` native client threads x ``iters`` back-to-back requests each.
        Returns (wall seconds, per-request latencies in ms)."""
        arr = (C.c_void_p * self.n_in)(*in_ptrs)
        lat = (C.c_double * (clients * iters))()
        wall = C.c_double()
        rc = N.lib().hz_exec_bench(self._h, clients, iters, arr, lat, C.byref(wall))
        if rc:
            raise RuntimeError(f"hz_exec_bench failed ({rc})")
        return wall.value * 1e-6, [v * 1e-3 for v in lat]

    def stats(self) -> dict:
        s, p = C.c_uint64(), C.c_uint64()
        N.lib().hz_exec_stats(self._h, C.byref(s), C.byref(p))
        b = C.c_uint64()
        N.lib().hz_exec_batches(self._h, C.byref(b))
        return {"served": s.value, "polls": p.value, "batches": b.value,
                "mean_batch": round(s.value / b.value, 3) if b.value else None}

    def close(self) -> None:
        h, self._h = getattr(self, "_h", None), None
        if h:
            N.lib().hz_exec_destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
