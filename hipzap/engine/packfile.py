"""Pre-packed weight files: the cold-start fast path (SURVEY.md §5 checkpoint/resume).

``torch.load`` of a standard state_dict stays the public format (reference parity:
main.py:99). ``hipzap pack`` additionally writes the *packed* device layout (BN folded,
fragment-major bf16/fp8, padded) as a safetensors file + JSON metadata next to the .pth, keyed
by the checkpoint's size, mtime and a sampled-content sha256, so a cold start can skip
folding/packing and stream the blob straight into device memory (safetensors: no pickle,
nothing executed on load). The torch-free plan image (engine/plan.py) uses the same key.
"""
from __future__ import annotations

import dataclasses
import json
import os

import torch


def _classes():
    from ..ops.conv import PackedConv
    from ..ops.fp8 import PackedFp8
    from ..ops.transformer import EmbedTables, NormParams
    return {c.__name__: c for c in (PackedConv, PackedFp8, NormParams, EmbedTables)}


PACK_SUFFIX = ".hzpack"


def packed_path(ckpt_path: str) -> str:
    """Where the pre-packed copy of a checkpoint lives: next to it (``m.pth`` -> ``m.pth.hzpack``)."""
    return ckpt_path + PACK_SUFFIX


def sampled_digest(path: str, chunks: int = 16, chunk: int = 65536) -> str:
    """sha256 over ``chunks`` evenly spaced 64-KiB windows of the file (plus its size): ~1 MiB
    read instead of the whole file, but a replaced checkpoint with the same size and a restored
    mtime still changes it (random-init or fine-tuned weights differ in every window)."""
    import hashlib
    h = hashlib.sha256()
    size = os.path.getsize(path)
    h.update(str(size).encode())
    with open(path, "rb") as f:
        if size <= chunks * chunk:
            h.update(f.read())
        else:
            step = (size - chunk) // (chunks - 1)
            for i in range(chunks):
                f.seek(i * step)
                h.update(f.read(chunk))
    return h.hexdigest()[:32]


def source_stamp(ckpt_path: str) -> dict:
    """Cheap identity of the source checkpoint: size + mtime + a sampled-content digest. A cold
    start must not hash a 100-MB file to validate its cache (sha256 of ResNet-50's .pth alone
    costs ~150 ms); the sampled digest reads ~1 MiB."""
    st = os.stat(ckpt_path)
    return {"size": st.st_size, "mtime_ns": st.st_mtime_ns, "sampled_sha256": sampled_digest(ckpt_path)}


def same_source(stamp: dict | None, ckpt_path: str, content_only: bool = False) -> bool:
    """``stamp`` (recorded when an artifact was derived) still describes ``ckpt_path``.
    ``content_only``: compare size + sampled digest but not mtime -- for a checkpoint and its
    derived artifact fetched together from an artifact store, where the local copies' mtimes are
    the download times."""
    if not stamp:
        return False
    cur = source_stamp(ckpt_path)
    if content_only:
        return stamp.get("size") == cur["size"] and stamp.get("sampled_sha256") == cur["sampled_sha256"]
    return stamp == cur


def find_packed(ckpt_path: str, model: str) -> str | None:
    """The packed file for ``ckpt_path`` if it exists, was packed for ``model`` and the source
    checkpoint is unchanged since; else None (the caller packs from the .pth)."""
    path = packed_path(ckpt_path)
    if not os.path.exists(path):
        return None
    try:
        meta = read_meta(path)
    except Exception:  # corrupt/partial file: ignore it, the .pth is the source of truth
        return None
    if meta.get("model") != model or meta.get("source_stamp") != source_stamp(ckpt_path):
        return None
    return path


def read_meta(path: str) -> dict:
    from safetensors import safe_open
    with safe_open(path, framework="pt", device="cpu") as f:
        return json.loads(f.metadata()["hipzap"])


def save_packed(params: dict, cfg: dict, path: str, source_sha256: str | None = None, model: str | None = None,
                stamp: dict | None = None) -> None:
    from safetensors.torch import save_file
    tensors, meta = {}, {"cfg": cfg, "source_sha256": source_sha256, "model": model, "source_stamp": stamp,
                         "entries": {}}
    for key, obj in params.items():
        if torch.is_tensor(obj):
            tensors[key] = obj.detach().contiguous().cpu()
            meta["entries"][key] = {"type": "tensor"}
            continue
        fields = {}
        for f in dataclasses.fields(obj):
            v = getattr(obj, f.name)
            if torch.is_tensor(v):
                tensors[f"{key}::{f.name}"] = v.detach().contiguous().cpu()
            else:
                fields[f.name] = v
        meta["entries"][key] = {"type": type(obj).__name__, "fields": fields}
    tmp = f"{path}.tmp{os.getpid()}"
    save_file(tensors, tmp, metadata={"hipzap": json.dumps(meta)})
    os.replace(tmp, path)


def load_packed(path: str, device="cpu") -> tuple[dict, dict]:
    """-> (packed params with every tensor on ``device``, arch cfg). safetensors reads straight
    into device memory; nothing in the file is executed."""
    from safetensors import safe_open
    classes = _classes()
    out = {}
    with safe_open(path, framework="pt", device=str(device)) as f:
        meta = json.loads(f.metadata()["hipzap"])
        for key, ent in meta["entries"].items():
            if ent["type"] == "tensor":
                out[key] = f.get_tensor(key)
                continue
            cls = classes[ent["type"]]
            kw = dict(ent["fields"])
            for fl in dataclasses.fields(cls):
                name = f"{key}::{fl.name}"
                if fl.name not in kw:
                    kw[fl.name] = f.get_tensor(name)
            out[key] = cls(**kw)
    return out, meta["cfg"]
