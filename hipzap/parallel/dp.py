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
                 comm: Comm | None = None):
        """``runner(x_shard) -> y_shard`` runs one rank's shard (e.g. ``Engine.infer_device``);
        ``comm``: torch.distributed (default) or a loopback communicator (tests)."""
        self.runner = runner
        self.shard = shard_batch
        self.device = torch.device(device)
        self.comm = comm or default_comm(group)
        self.world = self.comm.world
        self.rank = self.comm.rank
        self.x_shard = torch.zeros((shard_batch,) + tuple(in_shape), dtype=in_dtype, device=self.device)
        self.y_shard = torch.zeros((shard_batch,) + tuple(out_shape), dtype=out_dtype, device=self.device)
        self.global_batch = shard_batch * self.world
        if self.rank == 0:
            self.x_all = torch.zeros((self.global_batch,) + tuple(in_shape), dtype=in_dtype, device=self.device)
            self.y_all = torch.zeros((self.global_batch,) + tuple(out_shape), dtype=out_dtype, device=self.device)

    def step(self, x: torch.Tensor | None = None, sync: bool = True) -> torch.Tensor | None:
        """Collective: every rank calls it; rank 0 passes the global batch (<= world*shard).

        On a communicator that can enqueue without waiting (``supports_async``: the native RCCL
        one), scatter -> shard replay -> gather are all stream-ordered on the caller's current
        stream and the host synchronises at most ONCE per step (``sync``: a bounded wait on that
        stream that also polls the communicator's asynchronous errors); ``sync=False`` leaves the
        step in flight (a bench loop syncs every K steps). Blocking communicators (torch.distributed,
        loopback) keep their own semantics."""
        n = 0
        if self.rank == 0:
            n = x.shape[0]
            if n > self.global_batch:
                raise ValueError(f"batch {n} exceeds world*shard = {self.global_batch}")
            self.x_all[:n].copy_(x, non_blocking=True)
            if n < self.global_batch:
                self.x_all[n:].zero_()
        aio = bool(getattr(self.comm, "supports_async", False)) and self.world > 1
        kw = {"wait": False} if aio else {}
        if self.world > 1:
            chunks = list(self.x_all.chunk(self.world)) if self.rank == 0 else None
            self.comm.scatter(self.x_shard, chunks, src=0, **kw)
        else:
            self.x_shard.copy_(self.x_all)
        y = self.runner(self.x_shard)
        self.y_shard.copy_(y.reshape(self.y_shard.shape))
        if self.world > 1:
            outs = list(self.y_all.chunk(self.world)) if self.rank == 0 else None
            self.comm.gather(self.y_shard, outs, dst=0, **kw)
        else:
            self.y_all.copy_(self.y_shard)
        # a copy: the gather buffer is reused by the next step
        out = self.y_all[:n].clone() if self.rank == 0 else None
        if aio and sync:
            self.comm.sync(torch.cuda.current_stream(self.device).cuda_stream if self.device.type == "cuda" else None)
        return out

    def sync(self) -> None:
        """Wait for the steps left in flight by ``step(sync=False)`` (bounded on RCCL)."""
        if getattr(self.comm, "supports_async", False) and self.world > 1:
            self.comm.sync(torch.cuda.current_stream(self.device).cuda_stream if self.device.type == "cuda" else None)
        elif self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()
