"""Loader for the in-tree gfx950 kernel library (``_hcb_kernels.so``).

bf16 GPU activations ALWAYS go through the hand-written HIP kernels: if the library is missing
on a machine with a GPU this raises instead of silently falling back to PyTorch/MIOpen (the
PyTorch path on the GPU is only the explicitly requested fp32 / fp16 reference-precision mode).
CPU tensors use the PyTorch reference implementations in ``functional.py`` (the
reference's ``--device=cpu`` path, BASELINE config 1).
"""
from __future__ import annotations

import os
import threading

import torch

_LOCK = threading.Lock()
_LOADED = False
_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# HCB_KERNELS_SO: load another build of the library (kernel-variant A/B runs, tools/build_variant.py)
KERNELS_SO = os.environ.get("HCB_KERNELS_SO") or os.path.join(_PKG, "_hcb_kernels.so")


def load(build_if_missing: bool = True) -> bool:
    """Load the kernel library (building it in-tree first if needed)."""
    global _LOADED
    if _LOADED:
        return True
    with _LOCK:
        if _LOADED:
            return True
        if not os.path.exists(KERNELS_SO) or os.environ.get("HCB_REBUILD") == "1":
            if not build_if_missing:
                return False
            from .. import _build

            _build.build_kernels()
        torch.ops.load_library(KERNELS_SO)
        _LOADED = True
        from . import functional

        if functional.deterministic():
            torch.ops.hcb.set_deterministic(True)
        return True


def ops():
    """torch.ops.hcb namespace, loading the library on first use (raises if unavailable)."""
    if not _LOADED:
        load()
    return torch.ops.hcb


def loaded() -> bool:
    return _LOADED
