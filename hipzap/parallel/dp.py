"""Data-parallel batched serving across the GPUs of one node (RCCL over xGMI).

Two DP modes:
* **replica** (headline, bs=1): every rank is an independent serving replica with its own
  request stream — the only collective is the cold-start weight broadcast (C1). This is how
  Lambda scales the reference (one container per request), done with GPUs.
* **scatter/gather** (north-star configs 3 and 5: ResNet-50 bs=32 DP=8, ViT-B/16 bs=64 DP=8):
  rank 0 owns the global batch; ``dist.scatter`` (C2) hands each rank its shard, each rank runs
  its captured per-shard program, ``dist.gather`` (C3) returns the logits to rank 0. Shards
  are small (1.2-2.4 MB) and latency-bound, so each step is exactly one scatter and one
  gather of contiguous device buffers — no per-sample messages. The remainder of an uneven
  batch is zero-padded to the captured shard size and sliced off after the gather.
"""
from __future__ import annotations

from collections import deque
from typing import Callable

import torch

from .loopback import Comm, default_comm


class DPExecutor:
    def __init__(self, runner: Callable[[torch.Tensor], torch.Tensor], shard_batch: int, in_shape: tuple,
                 out_shape: tuple, device, in_dtype=torch.float32, out_dtype=torch.float32, group=None,
                 comm: Comm | None = None, in_buf: torch.Tensor | None = None, copy_out: bool = True):
        """``runner(x_shard) -> y_shard`` runs one rank's shard (e.g. ``Engine.infer_device``);
        ``comm``: torch.distributed (default) or a loopback communicator (tests).

        ``in_buf``: the runner's own static input (e.g. the captured context's ``input``): the scatter
        (or, at world 1, the one copy of the request) writes the shard straight into it and the
        runner is called with ``None`` (``Engine.infer_device(None)`` replays in place). The runner's
        output is gathered from where it lies. ``copy_out=False``: ``step`` returns a VIEW of the
        gather buffer (world 1: of the runner's output), valid until the next step. With both, a
        world-1 step is one request copy + the replay; world N adds the scatter and the gather only
        (the five device copies per step before)."""
        self.runner = runner
        self.shard = shard_batch
        self.device = torch.device(device)
        self.comm = comm or default_comm(group)
        self.world = self.comm.world
        self.rank = self.comm.rank
        self.copy_out = copy_out
        self.in_place = in_buf is not None
        shp = (shard_batch,) + tuple(in_shape)
        if in_buf is not None:
            assert in_buf.is_contiguous() and in_buf.numel() == shard_batch * int(torch.tensor(in_shape).prod()) \
                and in_buf.dtype == in_dtype, "in_buf must be the runner's contiguous [shard, *in_shape] input"
            self.x_shard = in_buf.view(shp)
        else:
            self.x_shard = torch.zeros(shp, dtype=in_dtype, device=self.device)
        self.out_shape = (shard_batch,) + tuple(out_shape)
        self.global_batch = shard_batch * self.world
        self.x_all = self.y_all = None
        if self.rank == 0:
            self._pad = None  # rank 0's padded global batch, allocated on the first uneven step
            if self.world > 1:
                self.y_all = torch.zeros((self.global_batch,) + tuple(out_shape), dtype=out_dtype, device=self.device)

    def _send_buffer(self, x: torch.Tensor) -> torch.Tensor:
        """Rank 0's global batch as a contiguous [world * shard, ...] tensor: ``x`` itself when it is
        exactly that, else padded into a persistent buffer (zeros past the last sample)."""
        n = x.shape[0]
        if n == self.global_batch and x.is_contiguous() and x.dtype == self.x_shard.dtype and x.device == self.device:
            return x
        if self._pad is None:
            self._pad = torch.zeros((self.global_batch,) + tuple(self.x_shard.shape[1:]), dtype=self.x_shard.dtype,
                                    device=self.device)
        self._pad[:n].copy_(x, non_blocking=True)
        if n < self.global_batch:
            self._pad[n:].zero_()
        return self._pad

    def step(self, x: torch.Tensor | None = None, sync: bool = True) -> torch.Tensor | None:
        """Collective: every rank calls it; rank 0 passes the global batch (<= world*shard).

        On a communicator that can enqueue without waiting (``supports_async``: the native RCCL
        one), scatter -> shard replay -> gather are all stream-ordered on the caller's current
        stream and the host synchronises at most ONCE per step (``sync``: a bounded wait on that
        stream that also polls the communicator's asynchronous errors); ``sync=False`` leaves the
        step in flight (a bench loop syncs every K steps). Blocking communicators (torch.distributed,
        loopback) keep their own semantics."""
        n = 0
        send = None
        if self.rank == 0:
            n = x.shape[0]
            if n > self.global_batch:
                raise ValueError(f"batch {n} exceeds world*shard = {self.global_batch}")
            if self.world == 1 and n == self.shard and x.data_ptr() == self.x_shard.data_ptr():
                send = None  # already in place
            elif self.world == 1:
                self.x_shard[:n].copy_(x, non_blocking=True)
                if n < self.shard:
                    self.x_shard[n:].zero_()
            else:
                send = self._send_buffer(x)
        aio = bool(getattr(self.comm, "supports_async", False)) and self.world > 1
        kw = {"wait": False} if aio else {}
        if self.world > 1:
            chunks = list(send.chunk(self.world)) if self.rank == 0 else None
            self.comm.scatter(self.x_shard, chunks, src=0, **kw)
        y = self.runner(None if self.in_place else self.x_shard).reshape(self.out_shape)
        if self.world > 1:
            outs = list(self.y_all.chunk(self.world)) if self.rank == 0 else None
            self.comm.gather(y if y.is_contiguous() else y.contiguous(), outs, dst=0, **kw)
            out = self.y_all[:n] if self.rank == 0 else None
        else:
            out = y[:n]
        if out is not None and self.copy_out:  # the buffers are reused by the next step
            out = out.clone()
        if aio and sync:
            self.comm.sync(torch.cuda.current_stream(self.device).cuda_stream if self.device.type == "cuda" else None)
        return out

    def sync(self) -> None:
        """Wait for the steps left in flight by ``step(sync=False)`` (bounded on RCCL)."""
        if getattr(self.comm, "supports_async", False) and self.world > 1:
            self.comm.sync(torch.cuda.current_stream(self.device).cuda_stream if self.device.type == "cuda" else None)
        elif self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()


class FnSlot:
    """A pipeline slot over a plain function (CPU ranks, tests): ``launch`` computes at once."""

    def __init__(self, fn: Callable[[torch.Tensor], torch.Tensor], shard_batch: int, in_shape: tuple,
                 dtype=torch.float32, device="cpu"):
        self.fn = fn
        self.input = torch.zeros((shard_batch,) + tuple(in_shape), dtype=dtype, device=device)
        self.output = None

    def launch(self) -> None:
        self.output = self.fn(self.input)

    def join(self) -> torch.Tensor:
        return self.output


class DPPipeline:
    """The scatter -> shard replay -> gather step with ``len(slots)`` steps in flight.

    Each slot is one captured context of the rank's shard program (``Engine.pipeline_slots``: its
    own static input / output and its own stream; ``FnSlot`` on the CPU): ``slot.input`` is where
    the scatter lands, ``slot.launch()`` enqueues the shard's compute after the caller's current
    stream, ``slot.join()`` makes the caller's current stream wait for it and returns the output.

    Every collective stays on the caller's current stream, in the same order on every rank:
    ``submit`` of step i issues scatter(i), launches i on its slot, and -- once ``depth`` steps are
    pending -- gather(i - depth + 1). So with depth D the issue order is sc0 .. sc(D-1), g0, scD,
    g1, ...: the scatters of the next D - 1 steps are queued before the oldest step's gather
    waits for its compute, and D shard programs run concurrently on their own streams. A slot is
    reused only after its previous step's gather (which waited for that step's compute) was
    issued on the same stream, so no buffer is overwritten while in use. Depth 1 is exactly
    ``DPExecutor.step``.

    ``submit`` returns the oldest pending step's logits once D are pending (else None); ``flush``
    retires every pending step (in order). Rank 0's results are views of per-slot gather buffers,
    valid for the next D - 1 submits. Config 3 as a serving load: one rank keeps D batches moving
    instead of running each one's latency chain alone (``bench.py`` dp figures, ``in_flight``).
    Issue from a non-default stream: engines of 2-4 contexts replay on dedicated-queue streams,
    which HIP creates blocking, so a step issued on the NULL stream would wait for every slot's
    replay in flight (measured: 44k -> 20k img/s at global batch 32)."""

    def __init__(self, slots: list, shard_batch: int, out_shape: tuple, device, out_dtype=torch.float32,
                 group=None, comm: Comm | None = None):
        if not slots:
            raise ValueError("a pipeline needs at least one slot")
        self.slots = list(slots)
        self.depth = len(self.slots)
        self.shard = shard_batch
        self.device = torch.device(device)
        self.comm = comm or default_comm(group)
        self.world, self.rank = self.comm.world, self.comm.rank
        self.global_batch = shard_batch * self.world
        for s in self.slots:
            if tuple(s.input.shape[:1]) != (shard_batch,) or not s.input.is_contiguous():
                raise ValueError("every slot's input must be a contiguous [shard, ...] tensor")
        self.out_shape = (shard_batch,) + tuple(out_shape)
        self._pad = None
        self.y_all = None
        if self.rank == 0 and self.world > 1:
            self.y_all = [torch.zeros((self.global_batch,) + tuple(out_shape), dtype=out_dtype, device=self.device)
                          for _ in self.slots]
        self._aio = bool(getattr(self.comm, "supports_async", False)) and self.world > 1
        self._kw = {"wait": False} if self._aio else {}
        self._pending: deque = deque()
        self._i = 0

    def _send_buffer(self, x: torch.Tensor) -> torch.Tensor:
        n = x.shape[0]
        if n == self.global_batch and x.is_contiguous() and x.dtype == self.slots[0].input.dtype \
                and x.device == self.device:
            return x
        if self._pad is None:
            self._pad = torch.zeros((self.global_batch,) + tuple(self.slots[0].input.shape[1:]),
                                    dtype=self.slots[0].input.dtype, device=self.device)
        self._pad[:n].copy_(x, non_blocking=True)
        if n < self.global_batch:
            self._pad[n:].zero_()
        return self._pad

    def submit(self, x: torch.Tensor | None = None) -> torch.Tensor | None:
        """Collective: every rank calls it once per step; rank 0 passes the global batch."""
        k = self._i % self.depth
        slot = self.slots[k]
        n = 0
        if self.rank == 0:
            n = x.shape[0]
            if n > self.global_batch:
                raise ValueError(f"batch {n} exceeds world*shard = {self.global_batch}")
            if self.world == 1:
                if x.data_ptr() != slot.input.data_ptr():
                    slot.input[:n].copy_(x, non_blocking=True)
                if n < self.shard:
                    slot.input[n:].zero_()
            else:
                send = self._send_buffer(x)
                self.comm.scatter(slot.input, list(send.chunk(self.world)), src=0, **self._kw)
        elif self.world > 1:
            self.comm.scatter(slot.input, None, src=0, **self._kw)
        slot.launch()
        self._pending.append((k, n))
        self._i += 1
        return self._retire() if len(self._pending) == self.depth else None

    def _retire(self) -> torch.Tensor | None:
        k, n = self._pending.popleft()
        y = self.slots[k].join().reshape(self.out_shape)
        if self.world == 1:
            return y[:n]
        outs = list(self.y_all[k].chunk(self.world)) if self.rank == 0 else None
        self.comm.gather(y if y.is_contiguous() else y.contiguous(), outs, dst=0, **self._kw)
        return self.y_all[k][:n] if self.rank == 0 else None

    def flush(self) -> list:
        """Retire every pending step, oldest first (their gathers are issued now)."""
        out = []
        while self._pending:
            out.append(self._retire())
        return out

    def sync(self) -> None:
        """Host wait for everything issued so far (bounded on the native RCCL communicator)."""
        if self._aio:
            self.comm.sync(torch.cuda.current_stream(self.device).cuda_stream if self.device.type == "cuda" else None)
        elif self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()
