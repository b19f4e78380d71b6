"""Loader for the in-tree gfx950 kernel libraries (``_hcb_kernels.so``: bf16 activations,
``_hcb_kernels_f16.so``: the same sources for IEEE-fp16 activations).

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
_LOADED = {}  # activation type -> library loaded
_ACT = ["bf16"]  # activation type of the ops() namespace: "bf16" (hcb) or "fp16" (hcb16)
_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# HCB_KERNELS_SO: load another build of the library (kernel-variant A/B runs, tools/build_variant.py)
KERNELS_SO = os.environ.get("HCB_KERNELS_SO") or os.path.join(_PKG, "_hcb_kernels.so")
# the same kernels built for IEEE-fp16 activations (--use_fp16), torch.ops.hcb16
KERNELS_F16_SO = os.path.join(_PKG, "_hcb_kernels_f16.so")
_SO = {"bf16": KERNELS_SO, "fp16": KERNELS_F16_SO}
_NS = {"bf16": "hcb", "fp16": "hcb16"}


def set_act(act: str) -> None:
    """Select the library ops() returns: the bf16 build or the IEEE-fp16 build."""
    assert act in _SO, act
    _ACT[0] = act


def load(build_if_missing: bool = True, act: str = None) -> bool:
    """Load the kernel library of activation type ``act`` (default: the current one), building
    it in-tree first if needed."""
    act = act or _ACT[0]
    if _LOADED.get(act):
        return True
    with _LOCK:
        if _LOADED.get(act):
            return True
        so = _SO[act]
        if not os.path.exists(so) or os.environ.get("HCB_REBUILD") == "1":
            if not build_if_missing:
                return False
            from .. import _build

            _build.build_kernels(f16=act == "fp16")
        torch.ops.load_library(so)
        _LOADED[act] = True
        from . import functional

        if functional.deterministic():
            getattr(torch.ops, _NS[act]).set_deterministic(True)
        return True


def ops():
    """torch.ops namespace of the current activation type (hcb: bf16, hcb16: IEEE fp16),
    loading the library on first use (raises if unavailable)."""
    act = _ACT[0]
    if not _LOADED.get(act):
        load(act=act)
    return getattr(torch.ops, _NS[act])


def loaded_namespaces():
    return [getattr(torch.ops, _NS[a]) for a, v in _LOADED.items() if v]


def loaded() -> bool:
    return any(_LOADED.values())
