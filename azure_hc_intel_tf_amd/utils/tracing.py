"""Tracing: ``--trace_file`` (Chrome trace of one step through torch.profiler, which on ROCm
records HIP kernels via roctracer) and roctx ranges around the phases of a step so
``rocprofv3 --marker-trace`` / ``--kernel-trace`` timelines are readable
(SURVEY.md §5 "Tracing / profiling")."""
from __future__ import annotations

import contextlib
import ctypes
import os

_roctx = None


def _load_roctx():
    global _roctx
    if _roctx is not None:
        return _roctx
    for name in ("libroctx64.so", "/opt/rocm/lib/librocprofiler-sdk-roctx.so", "/opt/rocm/lib/libroctx64.so"):
        try:
            _roctx = ctypes.CDLL(name)
            break
        except OSError:
            continue
    if _roctx is None:
        _roctx = False
    return _roctx


@contextlib.contextmanager
def range_(name: str):
    """roctx range (no-op when roctx is unavailable or HCB_ROCTX=0)."""
    lib = _load_roctx() if os.environ.get("HCB_ROCTX", "1") != "0" else False
    if lib:
        try:
            lib.roctxRangePushA(name.encode())
        except AttributeError:
            lib = False
    try:
        yield
    finally:
        if lib:
            lib.roctxRangePop()


def trace_step(fn, path: str, on_gpu: bool = True):
    """Run ``fn`` once under torch.profiler and export a Chrome trace to ``path``."""
    import torch
    from torch.profiler import ProfilerActivity, profile

    acts = [ProfilerActivity.CPU]
    if on_gpu:
        acts.append(ProfilerActivity.CUDA)
    with profile(activities=acts) as prof:
        fn()
        if on_gpu:
            torch.cuda.synchronize()
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    prof.export_chrome_trace(path)
    return path
