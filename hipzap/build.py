"""Build the hipzap native library (HIP kernels + C++ runtime) for gfx950, in-tree.

``python -m hipzap.build`` (or ``__graft_entry__.build()``) compiles every source under
``hipzap/csrc`` with ``hipcc --offload-arch=gfx950`` into ``hipzap/_lib/libhipzap.so``.
Objects are cached by source-content hash under ``build/obj`` so a rebuild only recompiles
what changed. The library exposes a plain C ABI (``csrc/hipzap.h``) loaded with ctypes —
no torch headers, so a full rebuild takes seconds, and the same ``.so`` travels to the GPU
box inside the repo snapshot.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
LIBDIR = PKG / "_lib"
LIB = LIBDIR / "libhipzap.so"
LIB_DEBUG = LIBDIR / "libhipzap_debug.so"  # -DHZ_DEBUG: device-side HZ_DCHECK contracts (csrc/common.h)
# -DHZ_EXPERIMENTS=1: the measured-negative kernel variants (csrc/common.h); not part of the product
# build, built on demand for re-measurement and selected with HIPZAP_LIB
LIB_EXP = LIBDIR / "libhipzap_exp.so"
# the RCCL communicator is its own library: only multi-GPU processes map the 570 MB librccl
LIB_COMM = LIBDIR / "libhipzap_comm.so"
COMM_SRC = CSRC / "comm"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
OBJDIR = PKG.parent / "build" / "obj"
ARCH = os.environ.get("HIPZAP_ARCH", "gfx950")

HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")
# HIPZAP_CFLAGS: extra compile flags for experiments (e.g. -DHZ_RING_SHRINK=1); part of the object hash
COMMON = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wno-unused-result",
          "-munsafe-fp-atomics", "-I", str(CSRC), *os.environ.get("HIPZAP_CFLAGS", "").split()]


def sources() -> list[Path]:
    return sorted([p for p in CSRC.iterdir() if p.suffix in (".hip", ".cpp")])


def _flags(debug: bool, exp: bool = False) -> list[str]:
    return COMMON + (["-DHZ_DEBUG"] if debug else []) + (["-DHZ_EXPERIMENTS=1"] if exp else [])


def _variant(debug: bool, exp: bool) -> str:
    return "-dbg" if debug else "-exp" if exp else ""


def _hash(src: Path, debug: bool = False, exp: bool = False) -> str:
    h = hashlib.sha1()
    h.update(" ".join(_flags(debug, exp)).encode())
    h.update(src.read_bytes())
    for hdr in sorted(CSRC.glob("*.h")):  # headers are shared: any change invalidates all
        h.update(hdr.read_bytes())
    return h.hexdigest()[:16]


def _compile(src: Path, debug: bool = False, exp: bool = False) -> Path:
    obj = OBJDIR / f"{src.stem}{_variant(debug, exp)}-{_hash(src, debug, exp)}.o"
    if obj.exists():
        return obj
    tmp = obj.with_suffix(".o.tmp")
    cmd = [HIPCC, *_flags(debug, exp), "-c", str(src), "-o", str(tmp)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr[-6000:]}")
    os.replace(tmp, obj)
    return obj


def build(verbose: bool = True, jobs: int | None = None, debug: bool = False, experiments: bool = False) -> Path:
    """Release library (``libhipzap.so``); with ``debug`` the HZ_DEBUG variant
    (``libhipzap_debug.so``, loaded when ``HIPZAP_DEBUG=1``); with ``experiments`` the
    HZ_EXPERIMENTS variant (``libhipzap_exp.so``, ``HIPZAP_LIB=...``)."""
    OBJDIR.mkdir(parents=True, exist_ok=True)
    LIBDIR.mkdir(parents=True, exist_ok=True)
    srcs = sources()
    exp = experiments and not debug
    lib = LIB_DEBUG if debug else LIB_EXP if exp else LIB
    var = _variant(debug, exp)
    jobs = jobs or min(8, len(srcs), os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, debug, exp), srcs))
    live = {o.name for o in objs}
    stems = {s.stem for s in srcs}
    for stale in OBJDIR.glob("*.o"):  # objects of older source versions (of this variant)
        v = next((x for x in ("-dbg", "-exp") if f"{x}-" in stale.name), "")
        stem = stale.name.rsplit("-", 2 if v else 1)[0]
        if stale.name not in live and v == var and stem in stems:
            stale.unlink(missing_ok=True)
    key = hashlib.sha1("".join(o.name for o in objs).encode()).hexdigest()[:16]
    stamp = LIBDIR / (".buildkey_debug" if debug else ".buildkey_exp" if exp else ".buildkey")
    if lib.exists() and stamp.exists() and stamp.read_text() == key:
        if verbose:
            print(f"hipzap: {lib} up to date")
        return lib
    tmp = lib.with_suffix(".so.tmp")
    cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(tmp)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
    os.replace(tmp, lib)
    stamp.write_text(key)
    if verbose:
        print(f"hipzap: built {lib} from {len(objs)} sources")
    return lib


def build_comm(verbose: bool = True) -> Path:
    """``libhipzap_comm.so``: csrc/comm/*.cpp (host code over RCCL), linked against librccl."""
    OBJDIR.mkdir(parents=True, exist_ok=True)
    LIBDIR.mkdir(parents=True, exist_ok=True)
    objs = [_compile(src) for src in sorted(COMM_SRC.glob("*.cpp"))]
    key = hashlib.sha1("".join(o.name for o in objs).encode()).hexdigest()[:16]
    stamp = LIBDIR / ".buildkey_comm"
    if LIB_COMM.exists() and stamp.exists() and stamp.read_text() == key:
        if verbose:
            print(f"hipzap: {LIB_COMM} up to date")
        return LIB_COMM
    tmp = LIB_COMM.with_suffix(".so.tmp")
    cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-L", str(ROCM / "lib"), "-lrccl", "-ldl",
           f"-Wl,-rpath,{ROCM / 'lib'}", "-o", str(tmp)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"comm link failed:\n{r.stderr[-6000:]}")
    os.replace(tmp, LIB_COMM)
    stamp.write_text(key)
    if verbose:
        print(f"hipzap: built {LIB_COMM}")
    return LIB_COMM


TOOLS_SRC = CSRC / "tools"
SERVE_PLAN = LIBDIR / "hipzap-serve-plan"


def build_tools(verbose: bool = True) -> list[Path]:
    """Native executables (csrc/tools/*.cpp) linked against libhipzap.so (rpath $ORIGIN):
    ``hipzap-serve-plan``, the Python-free plan server / cold-start probe."""
    build(verbose=False)
    out = []
    for src in sorted(TOOLS_SRC.glob("*.cpp")):
        exe = LIBDIR / ("hipzap-" + src.stem.replace("_", "-"))
        h = hashlib.sha1(src.read_bytes() + (CSRC / "hipzap.h").read_bytes() + " ".join(COMMON).encode())
        key = h.hexdigest()[:16]
        stamp = LIBDIR / f".buildkey_tool_{src.stem}"
        if exe.exists() and stamp.exists() and stamp.read_text() == key:
            if verbose:
                print(f"hipzap: {exe} up to date")
            out.append(exe)
            continue
        tmp = exe.with_suffix(".tmp")
        cmd = [HIPCC, *COMMON, str(src), "-L", str(LIBDIR), "-lhipzap", "-Wl,-rpath,$ORIGIN", "-o", str(tmp)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"tool build failed for {src.name}:\n{r.stderr[-6000:]}")
        os.replace(tmp, exe)
        stamp.write_text(key)
        if verbose:
            print(f"hipzap: built {exe}")
        out.append(exe)
    return out


# weightless plan templates (engine/plan.py export_template): the torch-free .pth cold start of
# these architectures (hipzap/lite.py PlanEngine.from_checkpoint). (model, classes, batch, contexts)
TEMPLATES = [("resnet50", 1000, 1, 1), ("resnet18", 1000, 1, 1)]


def build_templates(verbose: bool = True) -> list[Path]:
    """Write the plan templates that are missing or stale (native ABI or lowering code changed).
    Needs torch on the build host (CPU only), never at serving time."""
    build(verbose=False)
    from .lite import code_stamp, lib, plan_usable, read_meta, template_path
    stamp = code_stamp()
    out = []
    for model, ncls, batch, ctx in TEMPLATES:
        p = Path(template_path(model, batch, ctx, ncls, True))
        if p.exists() and plan_usable(str(p)) and read_meta(str(p)).get("code_stamp") == stamp:
            if verbose:
                print(f"hipzap: {p} up to date")
            out.append(p)
            continue
        p.parent.mkdir(parents=True, exist_ok=True)
        from .engine.plan import export_template
        export_template(model, ncls, batch, ctx, True, str(p))
        if verbose:
            print(f"hipzap: built template {p} (abi {lib().hz_abi_version():x}, code {stamp})")
        out.append(p)
    return out


if __name__ == "__main__":
    if "--templates" in sys.argv[1:]:
        build_templates(verbose=True)
        sys.exit(0)
    if "--experiments" in sys.argv[1:]:
        build(verbose=True, experiments=True)
        sys.exit(0)
    build(verbose=True, debug="--debug" in sys.argv[1:])
    if "--debug" not in sys.argv[1:]:
        # an in-tree debug library is loaded by the GPU tests (HIPZAP_DEBUG=1): keep it on the
        # same sources as the product one (a stale one misses new entry points)
        if LIB_DEBUG.exists():
            build(verbose=True, debug=True)
        build_comm(verbose=True)
        build_tools(verbose=True)
        build_templates(verbose=True)
    sys.exit(0)
