"""Failure detection and fault injection (SURVEY.md §5 'Failure detection').

* ``DeviceWatchdog``: a background thread that, every ``interval_s``, enqueues a tiny device
  op + event on each watched GPU and checks that it completes within ``timeout_s``
  (``hipEventQuery`` polling, never a blocking sync, so a wedged GPU cannot hang the thread).
  A device that misses its deadline is marked unhealthy; ``/health`` reports it and the
  server stops routing requests to it (RoundRobin skips unhealthy replicas).
* Fault injection for tests: ``HIPZAP_FAULT=<point>[,<point>...]`` makes ``maybe_fault(point)``
  raise ``InjectedFault`` (points used: ``load``, ``pack``, ``infer``, ``rank<N>``).
"""
from __future__ import annotations

import os
import threading
import time


class InjectedFault(RuntimeError):
    pass


def maybe_fault(point: str) -> None:
    spec = os.environ.get("HIPZAP_FAULT", "")
    if spec and point in [p.strip() for p in spec.split(",")]:
        raise InjectedFault(f"injected fault at {point}")


class DeviceWatchdog:
    def __init__(self, devices, interval_s: float = 5.0, timeout_s: float = 2.0, probe=None):
        """``probe(device) -> handle`` enqueues work; ``done(handle) -> bool`` polls it.
        Defaults use torch.cuda events; tests inject fakes."""
        self.devices = list(devices)
        self.interval_s, self.timeout_s = interval_s, timeout_s
        self.healthy = {d: True for d in self.devices}
        self.last_ok = {d: None for d in self.devices}
        self._probe = probe or self._torch_probe
        self._stop = threading.Event()
        self._thread = None

    @staticmethod
    def _torch_probe(device):
        import torch
        with torch.cuda.device(device):
            s = torch.cuda.Stream(device)
            with torch.cuda.stream(s):
                torch.empty(1, device=device).fill_(1.0)
                ev = torch.cuda.Event()
                ev.record(s)
        return ev.query

    def check_once(self) -> dict:
        for d in self.devices:
            try:
                done = self._probe(d)
                t0 = time.monotonic()
                ok = False
                while time.monotonic() - t0 < self.timeout_s:
                    if done():
                        ok = True
                        break
                    time.sleep(0.001)
            except Exception:
                ok = False
            self.healthy[d] = ok
            if ok:
                self.last_ok[d] = time.time()
        return dict(self.healthy)

    def _run(self):
        while not self._stop.wait(self.interval_s):
            self.check_once()

    def start(self):
        if self._thread is None:
            self._thread = threading.Thread(target=self._run, name="hipzap-watchdog", daemon=True)
            self._thread.start()
        return self

    def stop(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=self.interval_s + 1)
            self._thread = None

    def healthy_devices(self) -> list:
        return [d for d, ok in self.healthy.items() if ok]
