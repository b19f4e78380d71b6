"""Gradient compression (horovod ``Compression.none / fp16``; plus bf16, which keeps the fp32
exponent range and needs no loss-scale interplay on MI355X)."""
from __future__ import annotations

import torch


class _NoneCompressor:
    name = None

    @staticmethod
    def compress(t):
        return t, None

    @staticmethod
    def decompress(t, ctx):
        return t


class _CastCompressor:
    dtype = torch.float16
    name = "fp16"

    @classmethod
    def compress(cls, t):
        if t.dtype.is_floating_point and t.dtype != cls.dtype:
            return t.to(cls.dtype), t.dtype
        return t, None

    @classmethod
    def decompress(cls, t, ctx):
        return t.to(ctx) if ctx is not None else t


class _FP16(_CastCompressor):
    dtype = torch.float16
    name = "fp16"


class _BF16(_CastCompressor):
    dtype = torch.bfloat16
    name = "bf16"


class Compression:
    none = _NoneCompressor
    fp16 = _FP16
    bf16 = _BF16

    @staticmethod
    def by_name(name):
        return {None: Compression.none, "none": Compression.none, "fp16": Compression.fp16,
                "bf16": Compression.bf16}[name]
