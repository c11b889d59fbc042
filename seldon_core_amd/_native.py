"""Loader for the native core (``_C``).

The extension links ``libamdhip64.so.7``.  PyTorch-ROCm ships its own copy of
the HIP runtime (SONAME ``libamdhip64.so.7``) and loads it as
``libamdhip64.so``; importing torch first guarantees the process holds exactly
one HIP runtime, which both torch and ``_C`` then share.

On a machine with a GPU the extension is mandatory: if it is missing we fail
loudly instead of silently degrading to a Python path.
"""
from __future__ import annotations

import glob
import importlib.util
import os
import sys

_PKG = os.path.dirname(os.path.abspath(__file__))
_C = None
_ERR: Exception | None = None


def _gpu_present() -> bool:
    return os.path.exists("/dev/kfd") and bool(glob.glob("/dev/dri/renderD*"))


def _load():
    global _C, _ERR
    if _C is not None:
        return _C
    try:
        import torch  # noqa: F401  (must precede _C: shared HIP runtime)
    except Exception:  # pragma: no cover - torch is always present in this image
        pass
    try:
        mod = importlib.import_module(__package__ + "._C")
    except ImportError as exc:
        candidates = glob.glob(os.path.join(_PKG, "_C*.so"))
        if candidates:
            spec = importlib.util.spec_from_file_location("seldon_core_amd._C", candidates[0])
            mod = importlib.util.module_from_spec(spec)
            try:
                spec.loader.exec_module(mod)  # type: ignore[union-attr]
                sys.modules["seldon_core_amd._C"] = mod
            except Exception as exc2:  # pragma: no cover
                _ERR = exc2
                raise
        else:
            _ERR = exc
            raise ImportError(
                "seldon_core_amd native extension is not built; run `python tools/build_native.py`"
            ) from exc
    _C = mod
    return mod


def native():
    """Return the native module, building it on first use if sources exist."""
    try:
        return _load()
    except ImportError:
        build_script = os.path.join(os.path.dirname(_PKG), "tools", "build_native.py")
        if os.environ.get("SCA_NO_AUTOBUILD") or not os.path.exists(build_script):
            raise
        import subprocess

        subprocess.run([sys.executable, build_script], check=True)
        return _load()


def available() -> bool:
    try:
        native()
        return True
    except Exception:
        return False


def gpu_count() -> int:
    """Number of visible GPUs according to the native HIP runtime."""
    if not _gpu_present():
        return 0
    return int(native().gpu_device_count())


def require_gpu_native():
    """On a GPU machine the HIP path must be the one that runs."""
    mod = native()
    if _gpu_present() and mod.gpu_device_count() == 0:
        raise RuntimeError("GPU device nodes present but the native HIP runtime sees no device")
    return mod
