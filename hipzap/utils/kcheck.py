"""Device-side contract checks of the DEBUG kernel variant (SURVEY.md §5 "Race detection /
sanitizers": bounds-check asserts in a DEBUG kernel variant).

GPU AddressSanitizer and XNACK are not available on the MI355X pool, and a faulting kernel can
reset every GPU of the host, so the debug variant never traps: each ``HZ_DCHECK`` in
``csrc/*.hip`` that fails records the first (line, block, thread) of its source file in a device
word, counts every failure, and skips the guarded access. ``poll()`` reads and clears those
records after a device sync; ``check()`` raises :class:`KernelCheckError` if any fired.

    python -m hipzap.build --debug            # hipzap/_lib/libhipzap_debug.so
    HIPZAP_DEBUG=1 python ...                 # every hipzap op runs the checked kernels;
                                              # Engine.infer() calls check() after each request
"""
from __future__ import annotations

import ctypes as C

from .. import _native


class KernelCheckError(RuntimeError):
    pass


def enabled() -> bool:
    return _native.DEBUG


def poll(sync: bool = True) -> list[dict]:
    """[{unit, line, block, thread, count}] for every source file whose checks fired (cleared)."""
    if not _native.DEBUG:
        return []
    import torch
    if sync:
        torch.cuda.synchronize()
    lib = _native.lib()
    out = []
    for unit in _native.DEBUG_UNITS:
        rec = (C.c_uint * 4)()
        _native.check(getattr(lib, f"hz_debug_poll_{unit}")(rec), f"hz_debug_poll_{unit}")
        if rec[3]:
            out.append({"unit": unit, "line": int(rec[0]), "block": int(rec[1] & 0xFFFFF),
                        "block_y": int(rec[1] >> 20), "thread": int(rec[2]), "count": int(rec[3])})
    return out


def check(what: str = "") -> None:
    fails = poll()
    if fails:
        desc = "; ".join(f"csrc/{f['unit']}.hip:{f['line']} (block {f['block']},{f['block_y']} thread "
                         f"{f['thread']}, {f['count']} failures)" for f in fails)
        raise KernelCheckError(f"hipzap kernel contract check failed{' in ' + what if what else ''}: {desc}")
