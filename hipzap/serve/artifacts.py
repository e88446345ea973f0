"""Model artifact store with an atomic local cache (the reference's S3 + /tmp scheme).

Reference behaviour (/root/reference/main.py:32-38): download ``s3://bucket/<key>`` to
``/tmp/<key>`` unless that file already exists. Its defects are fixed here: parent
directories are created, the download goes to a temp file that is fsync'ed and atomically
renamed (an interrupted download can never be mistaken for a complete file), and an
optional sha256 is verified. Backends:
  * ``file:///abs/dir`` or a plain directory path as the bucket -> local copy (the GPU box
    has no network);
  * ``s3://`` / a bare bucket name -> boto3 ``download_file`` when boto3 is importable.
"""
from __future__ import annotations

import hashlib
import os
import shutil
import tempfile
import threading

_locks: dict = {}
_glock = threading.Lock()


def _lock_for(path):
    with _glock:
        return _locks.setdefault(path, threading.Lock())


def sha256_file(path: str) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


class ArtifactStore:
    def __init__(self, bucket: str | None, cache_root: str = "/tmp"):
        self.bucket = bucket
        self.cache_root = cache_root

    @property
    def is_local(self) -> bool:
        b = self.bucket or ""
        return b.startswith("file://") or os.path.isdir(b)

    def _local_dir(self) -> str:
        b = self.bucket or ""
        return b[len("file://"):] if b.startswith("file://") else b

    def cache_path(self, key: str) -> str:
        return os.path.join(self.cache_root, key.lstrip("/"))

    def _download(self, key: str, dst: str):
        if self.bucket is None:
            raise FileNotFoundError(f"no models bucket configured and {dst} is not cached")
        if self.is_local:
            src = os.path.join(self._local_dir(), key)
            shutil.copyfile(src, dst)
            return
        try:
            import boto3  # noqa: F401
        except ImportError as e:
            raise RuntimeError(f"s3 bucket {self.bucket!r} needs boto3, which is not installed") from e
        import boto3
        bucket = self.bucket[len("s3://"):] if self.bucket.startswith("s3://") else self.bucket
        boto3.client("s3").download_file(bucket, key, dst)

    def fetch(self, key: str, sha256: str | None = None) -> str:
        """``maybe_fetch_s3`` with atomic caching; returns the local path."""
        path = self.cache_path(key)
        with _lock_for(path):
            if os.path.exists(path) and (sha256 is None or sha256_file(path) == sha256):
                return path
            os.makedirs(os.path.dirname(path), exist_ok=True)
            fd, tmp = tempfile.mkstemp(prefix=".part-", dir=os.path.dirname(path))
            os.close(fd)
            try:
                self._download(key, tmp)
                if sha256 is not None and sha256_file(tmp) != sha256:
                    raise IOError(f"sha256 mismatch for {key}")
                with open(tmp, "rb") as f:
                    os.fsync(f.fileno())
                os.replace(tmp, path)
            finally:
                if os.path.exists(tmp):
                    os.unlink(tmp)
        return path

    def upload_dir(self, local_models_dir: str, prefix: str = "models") -> list[str]:
        """``scripts/upload_models.py`` parity (``aws s3 sync ./models s3://bucket/models``)."""
        copied = []
        if self.is_local:
            dst_root = os.path.join(self._local_dir(), prefix)
            for root, _, files in os.walk(local_models_dir):
                for fn in files:
                    src = os.path.join(root, fn)
                    rel = os.path.relpath(src, local_models_dir)
                    dst = os.path.join(dst_root, rel)
                    os.makedirs(os.path.dirname(dst), exist_ok=True)
                    if not os.path.exists(dst) or os.path.getsize(dst) != os.path.getsize(src):
                        shutil.copyfile(src, dst)
                        copied.append(rel)
            return copied
        aws = shutil.which("aws")
        if aws is None:
            raise RuntimeError("aws CLI not found for s3 upload")
        import subprocess
        bucket = self.bucket if self.bucket.startswith("s3://") else f"s3://{self.bucket}"
        subprocess.check_call([aws, "s3", "sync", local_models_dir, f"{bucket}/{prefix}"])
        return copied
