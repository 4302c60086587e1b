"""Loader for the in-tree gfx950 extension (``distributed_ml_pytorch_amd/_native*.so``).

GPU tensors ALWAYS go through the native kernels: if the extension is missing
or fails to load while a GPU tensor reaches a native op, we raise instead of
silently running an eager PyTorch fallback.  CPU tensors (gloo tests, CPU-only
plumbing runs) use the reference PyTorch formulation of the same op, which is
also the numerics oracle for the kernel tests.
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_mod = None
_err: Exception | None = None


def _load():
    global _mod, _err
    if _mod is not None or _err is not None:
        return
    with _lock:
        if _mod is not None or _err is not None:
            return
        try:
            import torch  # noqa: F401  (loads torch's HIP runtime first)

            _mod = importlib.import_module("distributed_ml_pytorch_amd._native")
        except Exception as e:  # pragma: no cover - depends on build state
            if os.environ.get("DMP_AUTOBUILD", "1") == "1":
                try:
                    from .. import _build

                    _build.build()
                    _mod = importlib.import_module("distributed_ml_pytorch_amd._native")
                    return
                except Exception as e2:
                    _err = e2
                    return
            _err = e


def available() -> bool:
    _load()
    return _mod is not None


def native():
    """Return the native module or raise (never a silent fallback on GPU)."""
    _load()
    if _mod is None:
        raise RuntimeError(
            "distributed_ml_pytorch_amd native extension is not available "
            f"({_err!r}); build it with `python -m distributed_ml_pytorch_amd._build`"
        )
    return _mod


def so_path() -> str | None:
    _load()
    return getattr(_mod, "__file__", None)
