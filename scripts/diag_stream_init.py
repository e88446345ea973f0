#!/usr/bin/env python3
"""Where does a fresh process's first-stream cost go? (plan cold start: `stream_ms` ~21 ms of
`upload_ms`, profiles/r4_final). Torch-free (ctypes HIP), each variant in fresh processes:

  stream: init -> hipStreamCreateWithFlags -> first memset + sync on it -> a second stream
  null:   init -> first memset + sync on the NULL stream -> then a created stream + first op
  malloc: init -> hipMalloc 64 MB -> hipStreamCreate -> first op (does an allocation pay it?)

Prints one JSON line per trial (ms per phase) and the per-variant medians.

    python scripts/diag_stream_init.py [--trials 5]
"""
import argparse
import ctypes as C
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(variant: str) -> dict:
    sys.path.insert(0, ROOT)
    from hipzap import hip
    h = hip.hip()
    out = {"variant": variant}
    t = time.perf_counter()

    def lap(name):
        nonlocal t
        now = time.perf_counter()
        out[name] = round((now - t) * 1e3, 3)
        t = now

    hip.check(h.hipSetDevice(0), "hipSetDevice")
    hip.check(h.hipFree(None), "hipFree")
    lap("init")
    buf = C.c_void_p()
    if variant == "malloc":
        hip.check(h.hipMalloc(C.byref(buf), 64 << 20), "hipMalloc")
        lap("malloc_64MB")
    else:
        hip.check(h.hipMalloc(C.byref(buf), 1 << 20), "hipMalloc")
        lap("malloc_1MB")
    if variant == "null":
        hip.check(h.hipMemsetAsync(buf, 0, 1 << 20, None), "memset")
        hip.check(h.hipStreamSynchronize(None), "sync")
        lap("null_first_op")
    s = C.c_void_p()
    hip.check(h.hipStreamCreateWithFlags(C.byref(s), 1), "create")
    lap("stream_create")
    hip.check(h.hipMemsetAsync(buf, 0, 1 << 20, s), "memset")
    hip.check(h.hipStreamSynchronize(s), "sync")
    lap("stream_first_op")
    s2 = C.c_void_p()
    hip.check(h.hipStreamCreateWithFlags(C.byref(s2), 1), "create2")
    lap("stream2_create")
    hip.check(h.hipMemsetAsync(buf, 0, 1 << 20, s2), "memset2")
    hip.check(h.hipStreamSynchronize(s2), "sync2")
    lap("stream2_first_op")
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=5)
    ap.add_argument("--child", default=None)
    a = ap.parse_args()
    if a.child:
        print(json.dumps(child(a.child)), flush=True)
        return 0
    res = {}
    for trial in range(a.trials):
        for v in ("stream", "null", "malloc"):
            r = subprocess.run([sys.executable, __file__, "--child", v], capture_output=True, text=True, timeout=120,
                               env=dict(os.environ, HSA_ENABLE_SDMA=os.environ.get("HSA_ENABLE_SDMA", "0")))
            line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            if r.returncode or not line:
                print(json.dumps({"variant": v, "error": r.stderr[-500:]}))
                return 1
            d = json.loads(line[-1])
            print(json.dumps(d), flush=True)
            res.setdefault(v, []).append(d)
    med = {v: {k: statistics.median(d[k] for d in ds) for k in ds[0] if k != "variant"} for v, ds in res.items()}
    print(json.dumps({"medians_ms": med}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
