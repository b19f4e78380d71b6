"""Data-parallel communication: Horovod-compatible API (``hvd``), gradient reducers and the
native C++ RCCL bucket engine."""
from .reducer import TorchDistReducer, fusion_threshold_bytes, make_buckets, split_ranges


def make_reducer(engine: str = "torch", compression=None, group=None, **kw):
    """engine: 'native' (C++ RCCL bucket engine on a side HIP stream) or 'torch'
    (torch.distributed all_reduce per bucket)."""
    if engine == "native":
        from .native import NativeReducer

        return NativeReducer(compression=compression, **kw)
    if engine == "torch":
        return TorchDistReducer(group=group, compression=compression, **kw)
    raise ValueError(f"unknown engine {engine!r}")


__all__ = ["make_reducer", "TorchDistReducer", "fusion_threshold_bytes", "make_buckets", "split_ranges"]
