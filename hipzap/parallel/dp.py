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
