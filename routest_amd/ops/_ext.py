"""Loader for the native extensions.

``_C`` (gfx950 HIP kernels) is REQUIRED whenever a GPU is visible: GPU code paths call
:func:`native` which raises instead of silently falling back to eager PyTorch.  On a CPU-only
machine the pure-PyTorch reference paths are used and ``native(required=False)`` returns None.
"""
from __future__ import annotations

import importlib
import os
from types import ModuleType
from typing import Optional

_C: Optional[ModuleType] = None
_C_err: Optional[BaseException] = None
_RT: Optional[ModuleType] = None
_RT_err: Optional[BaseException] = None


class NativeExtensionMissing(RuntimeError):
    pass


def native(required: bool = True) -> Optional[ModuleType]:
    """Return the ``routest_amd._C`` module (HIP kernels)."""
    global _C, _C_err
    if _C is not None:
        return _C
    try:
        import torch  # noqa: F401  (loads libtorch_hip / libamdhip64 first)
        _C = importlib.import_module("routest_amd._C")
        return _C
    except ImportError as e:  # pragma: no cover - depends on build state
        _C_err = e
    if required:
        raise NativeExtensionMissing(
            f"routest_amd._C (gfx950 HIP kernels) is not importable: {_C_err!r}. "
            "Build it with `python tools/build_ext.py`.")
    return None


def runtime(required: bool = True) -> Optional[ModuleType]:
    """Return the ``routest_amd._rt`` module (CPU C++ runtime)."""
    global _RT, _RT_err
    if _RT is not None:
        return _RT
    try:
        _RT = importlib.import_module("routest_amd._rt")
        return _RT
    except ImportError as e:  # pragma: no cover
        _RT_err = e
    if required:
        raise NativeExtensionMissing(
            f"routest_amd._rt (C++ runtime) is not importable: {_RT_err!r}. "
            "Build it with `python tools/build_ext.py --only rt`.")
    return None


def gpu_available() -> bool:
    import torch
    return torch.cuda.is_available()
