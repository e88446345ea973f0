"""Dynamic request batching (SURVEY.md §7.1 ``engine/ ... Batcher``).

The reference serves one request per Lambda container (main.py:105-112). A GPU replica can
do better under concurrent load: requests that arrive within ``max_wait_ms`` of the first
queued one are coalesced (up to the engine's captured batch) into ONE hipGraph replay, so N
concurrent bs=1 requests cost one batch-N forward instead of N batch-1 forwards. The
first request of an idle batcher never waits longer than ``max_wait_ms``; a full batch
dispatches immediately.

Threading model: callers (WSGI worker threads) block on a per-request future; one worker
thread per batcher owns the engine (so no lock is needed around the replay). Results are
sliced back per request in arrival order; an exception fails every request of that batch.
"""
from __future__ import annotations

import threading
import time
from concurrent.futures import Future
from typing import Callable

import torch

from ..utils.metrics import METRICS


class DynamicBatcher:
    def __init__(self, run_batch: Callable[[torch.Tensor], torch.Tensor], max_batch: int, max_wait_ms: float = 2.0,
                 name: str = "model"):
        """``run_batch(x[n, ...]) -> y[n, ...]`` for any ``n <= max_batch`` (the caller pads to
        its captured batch)."""
        if max_batch < 1:
            raise ValueError("max_batch must be >= 1")
        self.run_batch = run_batch
        self.max_batch = max_batch
        self.max_wait = max_wait_ms / 1e3
        self.name = name
        self._cv = threading.Condition()
        self._pending: list[tuple[torch.Tensor, Future, float]] = []
        self._rows = 0
        self._stop = False
        self.batches = 0
        self.requests = 0
        self._thread = threading.Thread(target=self._loop, name=f"hipzap-batcher-{name}", daemon=True)
        self._thread.start()

    def submit(self, x: torch.Tensor) -> Future:
        n = x.shape[0]
        if n > self.max_batch:
            raise ValueError(f"request batch {n} exceeds the batcher's max_batch {self.max_batch}")
        fut: Future = Future()
        with self._cv:
            if self._stop:
                raise RuntimeError("batcher is closed")
            self._pending.append((x, fut, time.perf_counter()))
            self._rows += n
            self._cv.notify()
        return fut

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        return self.submit(x).result()

    def _take(self) -> list:
        """Wait for work, then for the batch to fill or the oldest request's deadline."""
        with self._cv:
            while not self._pending and not self._stop:
                self._cv.wait()
            if not self._pending:
                return []
            deadline = self._pending[0][2] + self.max_wait
            while self._rows < self.max_batch and not self._stop:
                left = deadline - time.perf_counter()
                if left <= 0:
                    break
                self._cv.wait(left)
            batch, rows = [], 0
            while self._pending and rows + self._pending[0][0].shape[0] <= self.max_batch:
                item = self._pending.pop(0)
                rows += item[0].shape[0]
                batch.append(item)
            self._rows -= rows
            return batch

    def _loop(self):
        while True:
            batch = self._take()
            if not batch:
                return
            xs = [x for x, _, _ in batch]
            try:
                y = self.run_batch(torch.cat(xs) if len(xs) > 1 else xs[0])
                off = 0
                for x, fut, _ in batch:
                    n = x.shape[0]
                    fut.set_result(y[off: off + n])
                    off += n
            except Exception as e:  # every request of the failed batch sees the error
                for _, fut, _ in batch:
                    if not fut.done():
                        fut.set_exception(e)
            self.batches += 1
            self.requests += len(batch)
            METRICS.observe("hipzap_batch_rows", float(sum(x.shape[0] for x in xs)), {"model": self.name})

    def close(self):
        with self._cv:
            self._stop = True
            self._cv.notify_all()
        self._thread.join(timeout=5)
        with self._cv:
            for _, fut, _ in self._pending:
                if not fut.done():
                    fut.set_exception(RuntimeError("batcher closed"))
            self._pending.clear()
