"""Loader for the native extension ``_pmx`` (C++/HIP core built by utils/build.py).

torch is imported first on purpose: the wheel ships its own libamdhip64.so.7/librccl.so.1 and
our extension must bind to the same runtime instance (same SONAME -> the loader reuses the
already-mapped copy), otherwise two HIP runtimes would coexist in one process.
"""
from __future__ import annotations

import importlib
import os

_NATIVE = None


def load(build_if_missing: bool | None = None):
    """Return the ``_pmx`` module, building it in-tree first if it is missing.

    Fails loudly (ImportError) when the extension cannot be built or imported: there is no
    silent pure-Python fallback for the GPU path.
    """
    global _NATIVE
    if _NATIVE is not None:
        return _NATIVE
    import torch  # noqa: F401  (see module docstring)

    pkg = __name__.rsplit(".", 2)[0]
    if build_if_missing is None:
        build_if_missing = os.environ.get("PMX_NO_AUTOBUILD", "0") != "1"
    try:
        _NATIVE = importlib.import_module(pkg + "._pmx")
    except ImportError:
        if not build_if_missing:
            raise
        from . import build

        build.build()
        _NATIVE = importlib.import_module(pkg + "._pmx")
    return _NATIVE


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available() and load().device_count() > 0
    except Exception:
        return False
