"""Model artifact fetch (reference python/seldon_core/storage.py:36-160 and the
operator's model-initializer init container, operator/controllers/
model_initializer_injector.go:65-209).

Local paths and ``file://`` URIs are resolved in place; ``pvc://<claim>/<path>``
maps to ``$SELDON_PVC_ROOT/<claim>/<path>`` (default ``/mnt``).  Object stores
(``gs://``, ``s3://``, Azure blob) need their SDKs and network access, neither
of which exists on this platform: they raise a clear error unless a local
mirror is configured with ``SELDON_STORAGE_MIRROR=<dir>`` (``<dir>/<bucket>/<key>``).
"""
from __future__ import annotations

import os
import shutil
import tempfile
from urllib.parse import urlparse

_REMOTE = ("gs://", "s3://", "https://", "http://")


class Storage:
    @staticmethod
    def download(uri: str, out_dir: str | None = None) -> str:
        if not uri:
            raise ValueError("empty model uri")
        if uri.startswith("file://"):
            return Storage._local(uri[len("file://"):], out_dir)
        if uri.startswith("pvc://"):
            root = os.environ.get("SELDON_PVC_ROOT", "/mnt")
            return Storage._local(os.path.join(root, uri[len("pvc://"):]), out_dir)
        if uri.startswith(_REMOTE) or ".blob.core.windows.net" in uri:
            mirror = os.environ.get("SELDON_STORAGE_MIRROR")
            if mirror:
                p = urlparse(uri)
                return Storage._local(os.path.join(mirror, p.netloc, p.path.lstrip("/")), out_dir)
            raise RuntimeError(f"cannot fetch {uri}: no network access; set SELDON_STORAGE_MIRROR to a local copy")
        return Storage._local(uri, out_dir)

    @staticmethod
    def _local(path: str, out_dir: str | None) -> str:
        if not os.path.exists(path):
            raise FileNotFoundError(f"model uri {path} does not exist")
        if out_dir is None:
            return path
        os.makedirs(out_dir, exist_ok=True)
        dst = os.path.join(out_dir, os.path.basename(path.rstrip("/")))
        if os.path.isdir(path):
            if os.path.exists(dst):
                shutil.rmtree(dst)
            shutil.copytree(path, dst)
        else:
            shutil.copy2(path, dst)
        return dst

    @staticmethod
    def tempdir() -> str:
        return tempfile.mkdtemp(prefix="sca-model-")
