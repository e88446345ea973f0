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


def _member_data_offset(mm, header_offset: int) -> int:
    """Byte offset of a stored member's data inside the archive (local header is 30 bytes +
    name + extra; the extra field is what torch uses to 64-byte-align the records)."""
    hdr = mm[header_offset: header_offset + 30]
    if hdr[:4] != b"PK\x03\x04":
        raise NotAZipCheckpoint("bad local file header")
    name_len, extra_len = struct.unpack("<HH", hdr[26:30])
    return header_offset + 30 + name_len + extra_len


def _zip_index(mm) -> dict | None:
    """{name: (method, compressed size, size, local header offset, flags)} from the archive's
    central directory, read straight from the memory map (zip64 records included) -- importing
    ``zipfile`` (pathlib, shutil, urllib.parse ...) cost ~1/3 of the torch-free cold-start
    child's imports. None when the archive has anything this reader does not handle; the caller
    then uses ``zipfile``."""
    n = len(mm)
    i = mm.rfind(b"PK\x05\x06", max(0, n - 22 - 65535))
    if i < 0 or i + 22 > n:
        return None
    _, disk, cd_disk, _, count, cd_size, cd_off, _ = struct.unpack("<IHHHHIIH", mm[i:i + 22])
    if disk != 0 or cd_disk != 0:
        return None
    if cd_off == 0xFFFFFFFF or count == 0xFFFF or cd_size == 0xFFFFFFFF:
        j = i - 20
        if j < 0 or mm[j:j + 4] != b"PK\x06\x07":
            return None
        eocd64 = struct.unpack("<IIQI", mm[j:j + 20])[2]
        if eocd64 + 56 > n or mm[eocd64:eocd64 + 4] != b"PK\x06\x06":
            return None
        count, cd_size, cd_off = struct.unpack("<IQHHIIQQQQ", mm[eocd64:eocd64 + 56])[7:10]
    members, p = {}, cd_off
    for _ in range(count):
        if p + 46 > n or mm[p:p + 4] != b"PK\x01\x02":
            return None
        f = struct.unpack("<IHHHHHHIIIHHHHHII", mm[p:p + 46])
        flags, method, csize, usize, nlen, xlen, clen, hoff = f[3], f[4], f[8], f[9], f[10], f[11], f[12], f[16]
        name = bytes(mm[p + 46:p + 46 + nlen]).decode("utf-8" if flags & 0x800 else "cp437")
        if 0xFFFFFFFF in (csize, usize, hoff):  # zip64 extended information (header id 1)
            extra, q, vals = mm[p + 46 + nlen:p + 46 + nlen + xlen], 0, None
            while q + 4 <= len(extra):
                hid, hlen = struct.unpack("<HH", extra[q:q + 4])
                if hid == 1:
                    vals = extra[q + 4:q + 4 + hlen]
                    break
                q += 4 + hlen
            if vals is None:
                return None
            k = 0
            if usize == 0xFFFFFFFF:
                usize, k = struct.unpack("<Q", vals[k:k + 8])[0], k + 8
            if csize == 0xFFFFFFFF:
                csize, k = struct.unpack("<Q", vals[k:k + 8])[0], k + 8
            if hoff == 0xFFFFFFFF:
                hoff = struct.unpack("<Q", vals[k:k + 8])[0]
        members[name] = (method, csize, usize, hoff, flags)
        p += 46 + nlen + xlen + clen
    return members


def _read(path: str, with_arrays: bool):
    fd = os.open(path, os.O_RDONLY)
    try:
        mm = mmap.mmap(fd, 0, access=mmap.ACCESS_READ) if os.fstat(fd).st_size else None
    finally:
        os.close(fd)
    idx = _zip_index(mm) if mm is not None else None
    if idx is None:  # not a zip, or a layout the direct reader does not handle: the zipfile module
        import zipfile
        if mm is None or not zipfile.is_zipfile(path):
            raise NotAZipCheckpoint(f"{path}: not a zip-format torch checkpoint")
        with zipfile.ZipFile(path) as zf:
            idx = {i.filename: (i.compress_type, i.compress_size, i.file_size, i.header_offset, i.flag_bits)
                   for i in zf.infolist()}
    pkl = [n for n in idx if n.endswith("/data.pkl") or n == "data.pkl"]
    if len(pkl) != 1:
        raise NotAZipCheckpoint(f"{path}: expected one data.pkl, found {pkl}")
    prefix = pkl[0][: -len("data.pkl")]

    def stored(name: str):  # (data offset, size) of an uncompressed, unencrypted member
        m = idx.get(name)
        if m is None or m[0] != 0 or m[4] & 1:
            return None
        return _member_data_offset(mm, m[3]), m[2]

    bo = stored(prefix + "byteorder")
    if bo is not None and bytes(mm[bo[0]:bo[0] + bo[1]]).strip() not in (b"little", b""):
        raise ValueError(f"{path}: big-endian checkpoint")
    cache: dict = {}

    def load_storage(key: str, st: _StorageType, numel: int) -> StorageRef:
        s = cache.get(key)
        if s is None:
            rec = stored(f"{prefix}data/{key}")
            if rec is None:
                raise pickle.UnpicklingError(f"storage {key}: missing or compressed record")
            if numel * st.itemsize > rec[1]:
                raise pickle.UnpicklingError(f"storage {key}: record shorter than {numel} elements")
            s = StorageRef(key, st, numel, rec[0])
            if s.file_off + s.nbytes > len(mm):
                raise pickle.UnpicklingError(f"storage {key}: record runs past the end of the file")
            cache[key] = s
            if with_arrays:
                import numpy as np
                s.array = np.frombuffer(mm, dtype=np.dtype(st.dtype), count=numel, offset=s.file_off)
        return s

    rec = stored(pkl[0])
    if rec is not None:
        import io
        data = io.BytesIO(mm[rec[0]:rec[0] + rec[1]])
    else:  # a compressed data.pkl: let zipfile inflate it
        import io
        import zipfile
        with zipfile.ZipFile(path) as zf:
            data = io.BytesIO(zf.read(pkl[0]))
    obj = _RestrictedUnpickler(data, load_storage).load()
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
