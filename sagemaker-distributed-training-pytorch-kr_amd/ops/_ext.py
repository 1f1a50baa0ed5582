"""Loader for the in-tree gfx950 kernel library ``smdt_amd/_C.so``.

Policy (no silent fallback on the GPU): a CPU tensor always takes the plain PyTorch reference
path; a GPU tensor must take the HIP path, and if the extension is missing or fails to load the
call raises instead of quietly running an eager PyTorch op. ``SMDT_DISABLE_KERNELS=1`` is the
one explicit, logged opt-out (used only by A/B benchmarks).
"""
from __future__ import annotations

import importlib
import os
import warnings

import torch

_C = None
_ERR: Exception | None = None
_TRIED = False


def _load():
    global _C, _ERR, _TRIED
    if _TRIED:
        return _C
    _TRIED = True
    try:
        _C = importlib.import_module("smdt_amd._C")
    except Exception as e:  # pragma: no cover - exercised when the .so is missing
        _ERR = e
        _C = None
    return _C


def kernels_disabled() -> bool:
    return os.environ.get("SMDT_DISABLE_KERNELS", "0") == "1"


def available() -> bool:
    return _load() is not None


def ext():
    """Return the extension module or raise with the load error."""
    m = _load()
    if m is None:
        raise RuntimeError(
            "smdt_amd: the gfx950 kernel library (_C.so) is not loadable: "
            f"{_ERR!r}. Build it with `python -m smdt_amd._build`.")
    return m


def use_kernels(*tensors) -> bool:
    """True when the HIP path must be used for these operands.

    GPU operands -> True (and the extension must load); CPU operands -> False.
    """
    on_gpu = any(t is not None and t.is_cuda for t in tensors)
    if not on_gpu:
        return False
    if kernels_disabled():
        warnings.warn("SMDT_DISABLE_KERNELS=1: running PyTorch reference ops on the GPU", stacklevel=3)
        return False
    ext()
    return True
