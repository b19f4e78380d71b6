"""Gradient reducers over the flat gradient buffer.

The flat gradient buffer IS the fusion buffer (see nn/params.py): buckets are contiguous
slices of it, so there is no memcpy-in/out (Horovod's MEMCPY_IN_FUSION_BUFFER /
MEMCPY_OUT_FUSION_BUFFER phases disappear). Bucket size follows
``HOROVOD_FUSION_THRESHOLD`` (the reference sets 128 MiB,
/root/reference/benchmark-scripts/run-tf-sing-ucx-openmpi.sh:105).

* ``TorchDistReducer``: torch.distributed all_reduce per bucket (RCCL when the process group
  backend is "nccl" on ROCm, gloo on CPU). Optional bf16/fp16 compression
  (Horovod ``Compression.fp16``): pack kernel (scale + cast) -> allreduce -> unpack kernel.
* The C++ RCCL bucket engine with a side HIP stream lives in ``parallel/native.py``.
"""
from __future__ import annotations

import os
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

from .monitor import monitor, tracked

DEFAULT_FUSION_BYTES = 128 * 1024 * 1024


def fusion_threshold_bytes() -> int:
    v = os.environ.get("HOROVOD_FUSION_THRESHOLD")
    if v is None or v == "":
        return DEFAULT_FUSION_BYTES
    return max(int(v), 4096)


def make_buckets(numel: int, bucket_elems: int, align: int = 64) -> List[Tuple[int, int]]:
    """Split [0, numel) into contiguous (offset, length) buckets, issued from the END of the
    buffer first (the classifier / last stage's gradients are produced first in backward)."""
    bucket_elems = max(align, bucket_elems // align * align)
    out = []
    end = numel
    while end > 0:
        start = max(0, end - bucket_elems)
        out.append((start, end - start))
        end = start
    return out


def split_ranges(ranges, bucket_elems: int, align: int = 64) -> List[Tuple[int, int]]:
    """Cut every (offset, length) range into equal pieces of at most ``bucket_elems`` elements,
    in order (the same rule as the C++ engine's plan_buckets, csrc/comm/engine.h), so the
    HOROVOD_FUSION_THRESHOLD bounds each collective on the overlapped path too."""
    out = []
    m = max(align, bucket_elems // align * align) if bucket_elems > 0 else 0
    for off, n in ranges:
        if n <= 0:
            continue
        if m <= 0:
            out.append((off, n))
            continue
        pieces = (n + m - 1) // m
        per = min(m, ((n + pieces - 1) // pieces + align - 1) // align * align)
        s = 0
        while s < n:
            out.append((off + s, min(per, n - s)))
            s += per
    return out


class TorchDistReducer:
    graph_safe = False

    def __init__(self, group=None, compression: Optional[str] = None, bucket_bytes: Optional[int] = None,
                 average: bool = False):
        self.group = group
        self.compression = compression  # None | "fp16" | "bf16"
        self.bucket_bytes = bucket_bytes or fusion_threshold_bytes()
        self.average = average  # the trainer folds 1/N into the optimizer by default
        self._buckets = None
        self._comm_buf = None

    def allreduce_(self, flat: torch.Tensor) -> torch.Tensor:
        world = dist.get_world_size(self.group)
        if world == 1:
            return flat
        esz = 2 if self.compression else 4
        if self._buckets is None:
            self._buckets = make_buckets(flat.numel(), self.bucket_bytes // esz)
        if self.compression:
            dt = torch.float16 if self.compression == "fp16" else torch.bfloat16
            if self._comm_buf is None or self._comm_buf.numel() != flat.numel():
                self._comm_buf = torch.empty(flat.numel(), dtype=dt, device=flat.device)
        for bi, (off, n) in enumerate(self._buckets):
            view = flat[off:off + n]
            with tracked(f"allreduce.bucket{bi}", n * esz):
                if self.compression:
                    cb = self._comm_buf[off:off + n]
                    cb.copy_(view)
                    dist.all_reduce(cb, group=self.group)
                    view.copy_(cb)
                else:
                    dist.all_reduce(view, group=self.group)
        if self.average:
            flat.mul_(1.0 / world)
        return flat

    # -- overlap interface (trainer: reduce finished gradient ranges while backward continues)
    def allreduce_ranges_async_(self, flat: torch.Tensor, ranges) -> None:
        if dist.get_world_size(self.group) == 1:
            return
        pend = getattr(self, "_pending", None)
        if pend is None:
            pend = self._pending = []
        if self.compression and (self._comm_buf is None or self._comm_buf.numel() != flat.numel()):
            dt = torch.float16 if self.compression == "fp16" else torch.bfloat16
            self._comm_buf = torch.empty(flat.numel(), dtype=dt, device=flat.device)
        esz = 2 if self.compression else 4
        for off, n in split_ranges(ranges, self.bucket_bytes // esz):
            view = flat[off:off + n]
            tid = monitor().begin(f"allreduce.range{off}", n * esz)
            if self.compression:
                cb = self._comm_buf[off:off + n]
                cb.copy_(view)
                pend.append((view, cb, dist.all_reduce(cb, group=self.group, async_op=True), tid))
            else:
                pend.append((view, None, dist.all_reduce(view, group=self.group, async_op=True), tid))

    def join(self) -> None:
        for view, cb, work, tid in getattr(self, "_pending", None) or []:
            work.wait()
            monitor().end(tid)
            if cb is not None:
                view.copy_(cb)
        self._pending = []

    def broadcast_(self, t: torch.Tensor, root: int = 0) -> torch.Tensor:
        if dist.get_world_size(self.group) > 1:
            dist.broadcast(t, src=root, group=self.group)
        return t
