"""Read ``torch.save`` checkpoints without importing torch (the torch-free cold start from the
reference's own checkpoint format, ``torch.load(path, map_location='cpu')`` at
/root/reference/main.py:99; VERDICT r2 "next round" #4).

A ``torch.save`` file (zip format, torch >= 1.6) is a stored (uncompressed) zip archive:
``<name>/data.pkl`` (a protocol-2 pickle of the state_dict) plus one raw little-endian record
per tensor storage, ``<name>/data/<key>``, 64-byte aligned. The pickle is read with a
RESTRICTED unpickler, the way ``torch.load(weights_only=True)`` does it: ``find_class`` resolves
only an allowlist (``collections.OrderedDict``, the tensor/parameter rebuild functions and the
storage dtype markers) to local stand-ins, everything else raises, so nothing from the file is
executed. Storages are persistent ids ``('storage', <dtype marker>, key, location, numel)``
and become numpy views of the memory-mapped archive (zero copy; tensors that share a storage,
e.g. the tied embedding/decoder of the reference model, share the mapped bytes).

``load_state_dict`` returns ``{name: numpy.ndarray}`` (bfloat16 as :class:`BF16Array`, uint16
bit patterns); ``scan`` returns only where each tensor lives in the file (:class:`TensorRef`) and
needs no numpy at all -- the device-side packer (hipzap/lite.py ``PlanEngine.from_checkpoint``)
copies the raw records to the GPU. Legacy (pre-zip) files are refused: :class:`NotAZipCheckpoint`.
"""
from __future__ import annotations

import mmap
import os
import pickle
import struct
import zipfile
from collections import OrderedDict

# storage class -> (numpy dtype name, item size)
_STORAGE_DTYPES = {
    "FloatStorage": ("float32", 4), "DoubleStorage": ("float64", 8), "HalfStorage": ("float16", 2),
    "BFloat16Storage": ("uint16", 2), "LongStorage": ("int64", 8), "IntStorage": ("int32", 4),
    "ShortStorage": ("int16", 2), "CharStorage": ("int8", 1), "ByteStorage": ("uint8", 1), "BoolStorage": ("bool", 1),
}


class NotAZipCheckpoint(ValueError):
    pass


_BF16 = []


def _bf16_array_cls():
    if _BF16:
        return _BF16[0]
    import numpy as np

    class BF16Array(np.ndarray):
        """uint16 bit patterns of bfloat16 values (numpy has no bfloat16)."""

        def to_float32(self) -> np.ndarray:
            return (np.asarray(self, np.uint16).astype(np.uint32) << 16).view(np.float32)
    _BF16.append(BF16Array)
    return BF16Array


class _StorageType:
    """A storage dtype marker (``torch.FloatStorage`` ...). Immutable: a pickle BUILD opcode on it
    cannot rewrite its dtype or item size (they are looked up from the name, which is fixed)."""
    __slots__ = ("name",)

    def __init__(self, name: str):
        object.__setattr__(self, "name", name)

    def __setattr__(self, k, v):
        raise pickle.UnpicklingError("storage dtype markers are immutable")

    @property
    def dtype(self) -> str:
        return _STORAGE_DTYPES[self.name][0]

    @property
    def itemsize(self) -> int:
        return _STORAGE_DTYPES[self.name][1]


class StorageRef:
    """A storage record of the archive: ``file_off`` / ``nbytes`` in the checkpoint file."""
    __slots__ = ("key", "dtype", "itemsize", "numel", "file_off", "nbytes", "array", "bf16")

    def __init__(self, key, st: _StorageType, numel: int, file_off: int):
        self.key, self.dtype, self.itemsize, self.numel = key, st.dtype, st.itemsize, numel
        self.file_off, self.nbytes = file_off, numel * st.itemsize
        self.bf16 = st.name == "BFloat16Storage"
        self.array = None  # numpy view (load_state_dict)


class TensorRef:
    """A tensor as ``scan`` sees it: its storage record and view geometry (elements)."""
    __slots__ = ("storage", "offset", "shape", "stride")

    def __init__(self, storage: StorageRef, offset: int, shape: tuple, stride: tuple):
        self.storage, self.offset, self.shape, self.stride = storage, offset, shape, stride

    @property
    def dtype(self) -> str:
        return "bfloat16" if self.storage.bf16 else self.storage.dtype

    def numel(self) -> int:
        n = 1
        for s in self.shape:
            n *= s
        return n

    def is_contiguous(self) -> bool:
        expect = 1
        for n, s in zip(reversed(self.shape), reversed(self.stride)):
            if n != 1 and s != expect:
                return False
            expect *= n
        return True

    @property
    def file_off(self) -> int:
        return self.storage.file_off + self.offset * self.storage.itemsize


def _rebuild_tensor_v2(storage, storage_offset, size, stride, requires_grad=False, backward_hooks=None,
                       metadata=None):
    if not isinstance(storage, StorageRef):
        raise pickle.UnpicklingError("tensor rebuild without a storage record")
    size, stride = tuple(int(s) for s in size), tuple(int(s) for s in stride)
    storage_offset = int(storage_offset)
    # a view must stay inside its record: no negative offsets, sizes or strides (a negative one would
    # address bytes before the record -- on the host through numpy, on the device through the packer)
    if storage_offset < 0 or len(size) != len(stride) or any(n < 0 for n in size) or any(t < 0 for t in stride):
        raise pickle.UnpicklingError("tensor view with a negative offset, size or stride")
    if storage.array is None:  # scan: geometry only (a scalar spans one element)
        if not size or min(size) > 0:
            span = 1 + sum((n - 1) * s for n, s in zip(size, stride))
            if storage_offset + span > storage.numel:
                raise pickle.UnpicklingError("tensor view runs past its storage")
        return TensorRef(storage, int(storage_offset), size, stride)
    import numpy as np
    base = storage.array
    item = base.itemsize
    if len(size) == 0:
        if storage_offset >= base.size:
            raise pickle.UnpicklingError("tensor view runs past its storage")
        t = base[storage_offset: storage_offset + 1].reshape(())
    else:
        span = 1 + sum((n - 1) * s for n, s in zip(size, stride) if n > 0)
        if min(size) > 0 and storage_offset + span > base.size:
            raise pickle.UnpicklingError("tensor view runs past its storage")
        t = np.lib.stride_tricks.as_strided(base[storage_offset:], shape=size,
                                            strides=tuple(s * item for s in stride), writeable=False)
    return t.view(_bf16_array_cls()) if storage.bf16 else t


def _rebuild_parameter(data, requires_grad=False, backward_hooks=None):
    return data


def _rebuild_parameter_with_state(data, requires_grad, backward_hooks, state):
    return data


_ALLOWED = {
    ("collections", "OrderedDict"): OrderedDict,
    ("torch._utils", "_rebuild_tensor_v2"): _rebuild_tensor_v2,
    ("torch._utils", "_rebuild_parameter"): _rebuild_parameter,
    ("torch._utils", "_rebuild_parameter_with_state"): _rebuild_parameter_with_state,
}


class _RestrictedUnpickler(pickle.Unpickler):
    def __init__(self, f, load_storage):
        super().__init__(f)
        self._load_storage = load_storage

    def find_class(self, module, name):
        fn = _ALLOWED.get((module, name))
        if fn is not None:
            return fn
        if module == "torch" and name in _STORAGE_DTYPES:  # a dtype marker, never called
            return _StorageType(name)
        raise pickle.UnpicklingError(f"checkpoint references {module}.{name}: not allowed by the weights-only reader")

    def persistent_load(self, pid):  # ('storage', <dtype marker>, key, location, numel)
        if not (isinstance(pid, tuple) and len(pid) == 5 and pid[0] == "storage" and isinstance(pid[1], _StorageType)):
            raise pickle.UnpicklingError(f"unsupported persistent id {pid!r}")
        _, st, key, _location, numel = pid
        if int(numel) < 0:
            raise pickle.UnpicklingError("negative storage size")
        return self._load_storage(str(key), st, int(numel))


def _member_data_offset(mm, info: zipfile.ZipInfo) -> int:
    """Byte offset of a stored member's data inside the archive (local header is 30 bytes +
    name + extra; the extra field is what torch uses to 64-byte-align the records)."""
    hdr = mm[info.header_offset: info.header_offset + 30]
    if hdr[:4] != b"PK\x03\x04":
        raise NotAZipCheckpoint("bad local file header")
    name_len, extra_len = struct.unpack("<HH", hdr[26:30])
    return info.header_offset + 30 + name_len + extra_len


def _read(path: str, with_arrays: bool):
    if not zipfile.is_zipfile(path):
        raise NotAZipCheckpoint(f"{path}: not a zip-format torch checkpoint")
    fd = os.open(path, os.O_RDONLY)
    try:
        mm = mmap.mmap(fd, 0, access=mmap.ACCESS_READ)
    finally:
        os.close(fd)
    zf = zipfile.ZipFile(path)
    names = zf.namelist()
    pkl = [n for n in names if n.endswith("/data.pkl") or n == "data.pkl"]
    if len(pkl) != 1:
        raise NotAZipCheckpoint(f"{path}: expected one data.pkl, found {pkl}")
    prefix = pkl[0][: -len("data.pkl")]
    infos = {i.filename: i for i in zf.infolist()}
    bo = infos.get(prefix + "byteorder")
    if bo is not None and zf.read(bo).strip() not in (b"little", b""):
        raise ValueError(f"{path}: big-endian checkpoint")
    cache: dict = {}

    def load_storage(key: str, st: _StorageType, numel: int) -> StorageRef:
        s = cache.get(key)
        if s is None:
            info = infos.get(f"{prefix}data/{key}")
            if info is None or info.compress_type != zipfile.ZIP_STORED:
                raise pickle.UnpicklingError(f"storage {key}: missing or compressed record")
            if numel * st.itemsize > info.file_size:
                raise pickle.UnpicklingError(f"storage {key}: record shorter than {numel} elements")
            s = StorageRef(key, st, numel, _member_data_offset(mm, info))
            if s.file_off + s.nbytes > len(mm):
                raise pickle.UnpicklingError(f"storage {key}: record runs past the end of the file")
            cache[key] = s
            if with_arrays:
                import numpy as np
                s.array = np.frombuffer(mm, dtype=np.dtype(st.dtype), count=numel, offset=s.file_off)
        return s

    with zf.open(pkl[0]) as f:
        obj = _RestrictedUnpickler(f, load_storage).load()
    zf.close()
    if not with_arrays:
        mm.close()
    if isinstance(obj, dict) and "state_dict" in obj and isinstance(obj["state_dict"], dict):
        obj = obj["state_dict"]
    if not isinstance(obj, dict):
        raise pickle.UnpicklingError(f"{path}: checkpoint is a {type(obj).__name__}, not a state_dict")
    return dict(obj), mm


def load_state_dict(path: str) -> dict:
    """``torch.load(path, map_location="cpu", weights_only=True)`` without torch: a dict of
    numpy arrays backed by a read-only mmap of ``path`` (kept alive by the arrays). A checkpoint
    that wraps the state_dict (``{"state_dict": {...}}``) is unwrapped."""
    return _read(path, True)[0]


def scan(path: str) -> dict:
    """``{name: TensorRef}``: where every tensor of the checkpoint lives (no numpy, no torch)."""
    return _read(path, False)[0]
