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


def broadcast_params(params: dict | None, meta_params, device, src: int = 0, group=None, comm=None) -> dict:
    """C1: rank ``src`` sends its packed params; every rank returns params on ``device``.

    The blob is broadcast as one message, so it streams over every xGMI link at once
    instead of paying per-tensor launch latency 100+ times. ``meta_params`` (the shapes, as
    meta tensors) is only needed on the receiving ranks and may be a zero-argument callable so
    the source rank and single-process runs never build it (it costs a model construction).
    ``comm``: a ``loopback.Comm`` (default: torch.distributed when initialised).
    """
    comm = comm or default_comm(group)
    if comm.world <= 1:
        return params
    if comm.rank == src:
        blob = pack_blob(params, device)
        comm.broadcast(blob, src=src)
        return params
    meta = meta_params() if callable(meta_params) else meta_params
    _, total = flat_layout(meta)
    blob = torch.empty(total, dtype=torch.uint8, device=device)
    comm.broadcast(blob, src=src)
    return unpack_blob(blob, meta)


def health_check(device=None, comm=None) -> int:
    """C4: 1-int all-reduce; returns the number of live ranks."""
    comm = comm or default_comm()
    if comm.world <= 1:
        return 1
    t = torch.ones(1, dtype=torch.int32, device=device if device is not None else "cpu")
    comm.all_reduce(t)
    return int(t.item())
