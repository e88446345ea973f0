"""Process-group setup and RCCL collectives for data-parallel serving (one process per GPU).

Backend ``nccl`` on ROCm IS RCCL over xGMI; ``gloo`` is used for CPU tests. The collectives
follow SURVEY.md §2f:
* C1 weight broadcast at cold start: rank 0 packs the checkpoint once and broadcasts the
  packed blob (ONE large collective — per-link bound, ≈51 MB for ResNet-50 bf16); other
  ranks never touch the checkpoint file.
* C2/C3 scatter of a global batch / gather of logits (``dp.py``).
* C4 tiny all-reduce health check.
"""
from __future__ import annotations

import dataclasses
import datetime
import os

import torch
import torch.distributed as dist

from .loopback import default_comm


def env_rank() -> tuple[int, int, int]:
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def init_distributed(backend: str | None = None, device: torch.device | None = None, timeout_s: int = 600):
    """Init the default process group from torchrun env vars (no-op for world size 1)."""
    rank, world, local = env_rank()
    if world <= 1 or (dist.is_available() and dist.is_initialized()):
        return rank, world, local
    if backend is None:  # HIPZAP_DIST_BACKEND=gloo: multi-rank rehearsal on one GPU (HIPZAP_SHARE_GPU=1)
        backend = os.environ.get("HIPZAP_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
    if backend == "nccl" and device is not None:
        kw["device_id"] = device
    dist.init_process_group(**kw)
    return rank, world, local


def local_device(local: int) -> torch.device:
    """This rank's GPU: ``cuda:LOCAL_RANK``. ``HIPZAP_SHARE_GPU=1`` folds ranks onto the visible
    GPUs (``LOCAL_RANK % device_count``) so a multi-rank run can be rehearsed on one GPU with
    ``HIPZAP_DIST_BACKEND=gloo`` (RCCL refuses two ranks on one device)."""
    if os.environ.get("HIPZAP_SHARE_GPU") == "1":
        local = local % max(1, torch.cuda.device_count())
    return torch.device("cuda", local)


def max_over_ranks(x: float, device=None) -> float:
    """Slowest rank's value (bench timing). Host tensor under gloo, device tensor under RCCL."""
    if not is_dist():
        return x
    dev = "cpu" if dist.get_backend() == "gloo" else device
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def _tensor_fields(obj):
    if dataclasses.is_dataclass(obj):
        return [(f.name, getattr(obj, f.name)) for f in dataclasses.fields(obj)
                if torch.is_tensor(getattr(obj, f.name))]
    if torch.is_tensor(obj):
        return [(None, obj)]
    raise TypeError(type(obj))


def _rebuild(obj, new: dict):
    if torch.is_tensor(obj):
        return new[None]
    return dataclasses.replace(obj, **new)


def flat_layout(params: dict) -> tuple[list, int]:
    """[(key, field, dtype, shape, offset, nbytes)], total bytes (256-B aligned slots)."""
    out, off = [], 0
    for key in sorted(params):
        for name, t in _tensor_fields(params[key]):
            nb = t.numel() * t.element_size()
            out.append((key, name, t.dtype, tuple(t.shape), off, nb))
            off += (nb + 255) // 256 * 256
    return out, off


def pack_blob(params: dict, device) -> torch.Tensor:
    layout, total = flat_layout(params)
    blob = torch.empty(total, dtype=torch.uint8, device=device)
    for (key, name, dt, shape, off, nb) in layout:
        t = dict(_tensor_fields(params[key]))[name]
        blob[off: off + nb].copy_(t.contiguous().view(torch.uint8).reshape(-1))
    return blob


def unpack_blob(blob: torch.Tensor, meta_params: dict) -> dict:
    """Views into ``blob`` shaped like ``meta_params`` (zero-copy)."""
    layout, total = flat_layout(meta_params)
    assert blob.numel() >= total, (blob.numel(), total)
    fields: dict = {}
    for (key, name, dt, shape, off, nb) in layout:
        fields.setdefault(key, {})[name] = blob[off: off + nb].view(dt).view(shape)
    return {k: _rebuild(meta_params[k], fields[k]) for k in meta_params}


_NOTSET = object()


def broadcast_object(obj, device, src: int = 0, comm=None):
    """Broadcast a small JSON-serialisable object (length, then bytes) from ``src``."""
    import json
    comm = comm or default_comm()
    if comm.world <= 1:
        return obj
    dev = device if device is not None else "cpu"
    n = torch.zeros(1, dtype=torch.int64, device=dev)
    data = json.dumps(obj).encode() if comm.rank == src else b""
    if comm.rank == src:
        n.fill_(len(data))
    comm.broadcast(n, src=src)
    buf = torch.zeros(int(n.item()), dtype=torch.uint8, device=dev)
    if comm.rank == src:
        buf.copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    comm.broadcast(buf, src=src)
    return obj if comm.rank == src else json.loads(bytes(buf.cpu().tolist()).decode())


def broadcast_params(params: dict | None, meta_params, device, src: int = 0, group=None, comm=None,
                     arch_kw=_NOTSET):
    """C1: rank ``src`` sends its packed params; every rank returns params on ``device``.

    The blob is broadcast as one message, so it streams over every xGMI link at once
    instead of paying per-tensor launch latency 100+ times. ``meta_params`` (the shapes, as
    meta tensors) is only needed on the receiving ranks and may be a callable so the source
    rank and single-process runs never build it (it costs a model construction).

    ``arch_kw`` (the source's ``pack`` cfg): broadcast first, together with the blob size, so
    receivers build their layout from the SOURCE's architecture (``meta_params(arch_kw)``)
    instead of guessing defaults, and a layout mismatch fails loudly before any weight moves.
    Then the call returns ``(params, arch_kw)``; without it, just ``params``.
    ``comm``: a ``loopback.Comm`` (default: torch.distributed when initialised).
    """
    comm = comm or default_comm(group)
    with_meta = arch_kw is not _NOTSET
    if comm.world <= 1:
        return (params, arch_kw) if with_meta else params
    total_src = flat_layout(params)[1] if comm.rank == src else None
    if with_meta:
        hdr = broadcast_object({"arch_kw": arch_kw, "blob_bytes": total_src}, device, src, comm)
        arch_kw = hdr["arch_kw"]
    if comm.rank == src:
        blob = pack_blob(params, device)
        comm.broadcast(blob, src=src)
        return (params, arch_kw) if with_meta else params
    if callable(meta_params):
        meta = meta_params(arch_kw or {}) if with_meta else meta_params()
    else:
        meta = meta_params
    if isinstance(meta, tuple):  # adapter.meta_params() returns (params, cfg)
        meta = meta[0]
    _, total = flat_layout(meta)
    if with_meta and total != hdr["blob_bytes"]:
        raise ValueError(f"packed layout mismatch: source blob is {hdr['blob_bytes']} bytes, this rank's "
                         f"layout for {arch_kw} is {total}")
    blob = torch.empty(total, dtype=torch.uint8, device=device)
    comm.broadcast(blob, src=src)
    out = unpack_blob(blob, meta)
    return (out, arch_kw) if with_meta else out


def health_check(device=None, comm=None) -> int:
    """C4: 1-int all-reduce; returns the number of live ranks."""
    comm = comm or default_comm()
    if comm.world <= 1:
        return 1
    t = torch.ones(1, dtype=torch.int32, device=device if device is not None else "cpu")
    comm.all_reduce(t)
    return int(t.item())
