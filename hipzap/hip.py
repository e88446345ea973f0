"""Minimal torch-free HIP runtime bindings (ctypes over libamdhip64, which libhipzap.so already
links): device count, device/pinned allocation and copies for processes that never import
torch (plan-backed serving workers, hipzap/serve/cluster.py)."""
from __future__ import annotations

import ctypes as C
import threading

from . import _native

_lock = threading.Lock()
_hip = None
H2D, D2H, D2D, DEFAULT = 1, 2, 3, 4


def hip():
    global _hip
    with _lock:
        if _hip is None:
            _native.lib()  # loads libamdhip64 as its dependency
            h = C.CDLL("libamdhip64.so")
            P, I, S = C.c_void_p, C.c_int, C.c_size_t
            for name, res, args in (
                    ("hipGetDeviceCount", I, [C.POINTER(I)]), ("hipSetDevice", I, [I]),
                    ("hipMalloc", I, [C.POINTER(P), S]), ("hipFree", I, [P]),
                    ("hipHostMalloc", I, [C.POINTER(P), S, C.c_uint]), ("hipHostFree", I, [P]),
                    ("hipMemcpy", I, [P, P, S, I]), ("hipMemcpyAsync", I, [P, P, S, I, P]),
                    ("hipMemsetAsync", I, [P, I, S, P]), ("hipStreamSynchronize", I, [P]),
                    ("hipDeviceSynchronize", I, []), ("hipGetErrorString", C.c_char_p, [I]),
                    ("hipStreamCreateWithFlags", I, [C.POINTER(P), C.c_uint]), ("hipGetDevice", I, [C.POINTER(I)])):
                f = getattr(h, name)
                f.restype, f.argtypes = res, args
            _hip = h
    return _hip


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed: {hip().hipGetErrorString(rc).decode()}")


def device_count() -> int:
    """Visible GPUs (0 when the runtime reports none or cannot initialise)."""
    try:
        n = C.c_int(0)
        return n.value if hip().hipGetDeviceCount(C.byref(n)) == 0 else 0
    except OSError:
        return 0


def set_device(d: int) -> None:
    check(hip().hipSetDevice(d), "hipSetDevice")


class DeviceBuffer:
    """Owned device allocation (``.ptr``)."""

    def __init__(self, nbytes: int):
        p = C.c_void_p()
        check(hip().hipMalloc(C.byref(p), max(1, nbytes)), "hipMalloc")
        self.ptr, self.nbytes = p.value, nbytes

    def free(self):
        if getattr(self, "ptr", None):
            hip().hipFree(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class PinnedBuffer:
    """Owned page-locked host allocation, viewable as a ctypes byte array (``.view``)."""

    def __init__(self, nbytes: int):
        p = C.c_void_p()
        check(hip().hipHostMalloc(C.byref(p), max(1, nbytes), 0), "hipHostMalloc")
        self.ptr, self.nbytes = p.value, nbytes
        self.view = (C.c_char * max(1, nbytes)).from_address(self.ptr)

    def free(self):
        if getattr(self, "ptr", None):
            hip().hipHostFree(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


_tls = threading.local()


def _private_stream() -> int:
    """This thread's non-blocking stream on the current device. Synchronous copies go through it
    instead of the legacy NULL stream: a NULL-stream copy while another thread captures a hipGraph
    fails with 'operation would make the legacy stream depend on a capturing blocking stream' (the
    lazy capture of PlanEngine contexts runs in a background thread of the serving workers)."""
    d = C.c_int(0)
    check(hip().hipGetDevice(C.byref(d)), "hipGetDevice")
    streams = getattr(_tls, "streams", None)
    if streams is None:
        streams = _tls.streams = {}
    s = streams.get(d.value)
    if s is None:
        p = C.c_void_p()
        check(hip().hipStreamCreateWithFlags(C.byref(p), 1), "hipStreamCreateWithFlags")  # hipStreamNonBlocking
        s = streams[d.value] = p.value
    return s


def memcpy(dst: int, src: int, nbytes: int, kind: int = DEFAULT, stream=None) -> None:
    """Copy; with ``stream=None`` synchronous (on this thread's private non-blocking stream)."""
    if stream is None:
        s = _private_stream()
        check(hip().hipMemcpyAsync(dst, src, nbytes, kind, s), "hipMemcpyAsync")
        check(hip().hipStreamSynchronize(s), "hipStreamSynchronize")
    else:
        check(hip().hipMemcpyAsync(dst, src, nbytes, kind, stream), "hipMemcpyAsync")


def sync(stream) -> None:
    check(hip().hipStreamSynchronize(stream), "hipStreamSynchronize")
