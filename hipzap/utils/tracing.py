"""Tracing: roctx ranges (visible in rocprofv3 --marker-trace timelines) + phase timers.

The reference has no tracing at all. Here every cold-start phase and request
phase can be bracketed with ``trace_range(name)``: it pushes a roctx range when the ROCm
profiler SDK's roctx library is loadable (``librocprofiler-sdk-roctx.so``) and always records a
wall-clock duration into an optional ``PhaseTimer`` (surfaced in bench JSON / X-Timing).
Disabled entirely with ``HIPZAP_TRACE=0``.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import threading
import time

_roctx = None
_tried = False
_lock = threading.Lock()


def _load_roctx():
    global _roctx, _tried
    with _lock:
        if _tried:
            return _roctx
        _tried = True
        if os.environ.get("HIPZAP_TRACE", "1") == "0":
            return None
        for name in ("librocprofiler-sdk-roctx.so", "/opt/rocm/lib/librocprofiler-sdk-roctx.so", "libroctx64.so",
                     "/opt/rocm/lib/libroctx64.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                _roctx = lib
                break
            except OSError:
                continue
        return _roctx


def roctx_available() -> bool:
    return _load_roctx() is not None


class PhaseTimer:
    def __init__(self):
        self.phases: dict[str, float] = {}

    def add(self, name: str, ms: float):
        self.phases[name] = self.phases.get(name, 0.0) + ms

    def header(self) -> str:
        """``X-Timing``-style header value: ``phase=ms;phase=ms``."""
        return ";".join(f"{k}={v:.3f}" for k, v in self.phases.items())


@contextlib.contextmanager
def trace_range(name: str, timer: PhaseTimer | None = None):
    lib = _load_roctx()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    t0 = time.perf_counter()
    try:
        yield
    finally:
        if timer is not None:
            timer.add(name, (time.perf_counter() - t0) * 1e3)
        if lib is not None:
            lib.roctxRangePop()
