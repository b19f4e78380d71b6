"""Model base class: a ParamStore plus explicit forward / backward over NHWC activations."""
from __future__ import annotations

import os
from typing import Callable, List, Sequence, Tuple

import torch

from ..nn.layers import act_dtype
from ..nn.params import ParamStore


# activation / GEMM-operand precisions the GPU path implements (the CPU path is fp32/fp64)
GPU_COMPUTE_DTYPES = ("bf16", "fp32", "fp16")
TORCH_DTYPES = {"bf16": torch.bfloat16, "fp32": torch.float32, "fp16": torch.float16}


def check_compute_dtype(compute_dtype, device) -> str:
    """Validate a requested compute precision; never substitute one precision for another. The
    default is fp32 on every device: the reference's precision (tf_cnn_benchmarks with MKL-DNN,
    /root/reference/benchmark-scripts/run-tf-sing-ucx-openmpi.sh:62-81 passes no --use_fp16), the
    same default as tf_cnn_benchmarks.py, the runners and bench.py; bf16 / fp16 are opt-in."""
    if torch.device(device).type != "cuda":
        if compute_dtype not in (None, "fp32"):
            raise ValueError(f"the CPU path computes in fp32, not {compute_dtype}")
        return "fp32"
    cd = compute_dtype or "fp32"
    if cd not in GPU_COMPUTE_DTYPES:
        raise NotImplementedError(f"compute dtype {cd!r} is not implemented on the GPU path "
                                  f"(available: {', '.join(GPU_COMPUTE_DTYPES)})")
    return cd


class CNNModel:
    """Subclasses build their layers in ``build()`` using ``self.ps`` and implement
    ``forward(images) -> logits`` and ``backward(dlogits)``.

    ``image_channels`` is what the input tensor carries: on the GPU the 3 RGB channels are
    zero-padded to 8 so every conv operand is a whole number of 16-byte vectors.
    """

    name = "model"
    # every op of the model has an fp32 HIP kernel: --compute_dtype fp32 runs natively (bf16x6
    # GEMMs + fp32 BN / pool / loss); otherwise fp32 takes the PyTorch (MIOpen) path
    F32_NATIVE_OK = False
    default_image_size = 224
    default_batch_size = 64
    default_lr_per_256 = 0.1  # tf_cnn_benchmarks: lr = 0.1 * global_batch / 256 for ResNets

    def __init__(self, num_classes: int = 1001, image_size: int = None, device="cpu", seed: int = 1234,
                 image_channels: int = None, compute_dtype: str = None):
        self.num_classes = num_classes
        self.compute_dtype = check_compute_dtype(compute_dtype, device)
        self.image_size = image_size or self.default_image_size
        self.device = torch.device(device)
        # native: the hand-written HIP kernels (bf16, or the IEEE-fp16 build); otherwise (CPU, or
        # a GPU in the fp32 reference-precision mode) the PyTorch path of ops/functional.py
        from ..ops import functional as Fn

        # HCB_F32_NATIVE=0: fp32 through the PyTorch (MIOpen / rocBLAS) path even where the HIP
        # kernels exist -- the comparison point of the fp32 numbers
        f32_ok = self.F32_NATIVE_OK and os.environ.get("HCB_F32_NATIVE", "1") != "0"
        self.native = self.device.type == "cuda" and (
            self.compute_dtype == "bf16" or (self.compute_dtype == "fp16" and Fn.F16_NATIVE)
            or (self.compute_dtype == "fp32" and f32_ok))
        if image_channels is None:
            image_channels = 8 if self.native else 3
        assert image_channels in (3, 8) and (not self.native or image_channels == 8)
        self.image_channels = image_channels
        self.activate()
        self.ps = ParamStore(seed=seed)
        self.layers: List = []
        self.build()
        f32n = self.native and self.compute_dtype == "fp32"
        self.ps.finalize(self.device, dtype_pack=torch.bfloat16 if f32n or not self.native
                         else TORCH_DTYPES[self.compute_dtype], pack=self.native, pack_lo=f32n)

    # -- to implement
    def build(self):
        raise NotImplementedError

    def forward(self, images: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def backward(self, dlogits: torch.Tensor) -> None:
        raise NotImplementedError

    def backward_segments(self, dlogits: torch.Tensor):
        """Backward in segments, for overlapping the gradient allreduce with the rest of the
        backward pass: yields ``(layers, last)`` after each segment, where every parameter
        gradient of ``layers`` is final. Default: one segment (the whole backward)."""
        self.backward(dlogits)
        yield None, True  # None: every gradient

    @staticmethod
    def _param_count(layers) -> int:
        return sum(p.numel for l in layers for p in getattr(l, "params", lambda: [])())

    def _segments_from_units(self, dx, head: Sequence, units: Sequence[Tuple[Callable, Sequence]],
                             tail: Sequence = ()):
        """Generic segmented backward. ``head``: layers whose backward already ran (their
        gradients are final); ``units``: (fn(dx) -> dx, layers) in backward order; ``tail``:
        parameter-free layers that are never back-propagated through. A segment is closed
        (yielded) once it owns >= HCB_SEGMENT_PARAMS parameters (default 2M = 8 MB fp32), so
        the first reductions start while most of the backward is still ahead."""
        thr = int(os.environ.get("HCB_SEGMENT_PARAMS", 2_000_000))
        seg, n = list(head), self._param_count(head)
        for i, (fn, layers) in enumerate(units):
            dx = fn(dx)
            seg += list(layers)
            n += self._param_count(layers)
            if i < len(units) - 1 and n >= thr:
                yield seg, False
                seg, n = [], 0
        yield seg + list(tail), True

    def activate(self) -> None:
        """Make this model's activation dtype current for the layer helpers (GPU models of
        different compute dtypes can coexist in one process)."""
        if self.device.type == "cuda":
            from ..nn.layers import set_gpu_compute_dtype
            from ..ops import functional as Fn

            set_gpu_compute_dtype(TORCH_DTYPES[self.compute_dtype])
            Fn.set_f32_native(self.compute_dtype == "fp32" and self.native)

    # -- helpers
    @property
    def act_dtype(self):
        self.activate()
        return act_dtype(self.device)

    def input_shape(self, batch: int):
        return (batch, self.image_size, self.image_size, self.image_channels)

    def num_params(self) -> int:
        return self.ps.num_params()

    def flops_per_image(self) -> float:
        """Forward FLOPs per image (multiply-adds x 2) of the conv / affine layers."""
        tot = 0
        for l in self.all_layers():
            if hasattr(l, "flops"):
                tot += l.flops(1)
        return float(tot)

    def all_layers(self):
        return list(self.layers)

    def grad_ranges(self, layers):
        """Merged (offset, length) ranges of the flat gradient buffer owned by ``layers``."""
        spans = sorted((p.offset, p.numel) for l in layers for p in getattr(l, "params", lambda: [])())
        out = []
        for off, n in spans:
            if out and out[-1][0] + out[-1][1] == off:
                out[-1] = (out[-1][0], out[-1][1] + n)
            else:
                out.append((off, n))
        return out

    def set_training(self, training: bool) -> None:
        """Training (batch-statistics BN, dropout on) or inference mode (moving-statistics BN,
        dropout off) -- tf_cnn_benchmarks' phase_train, False under ``--forward_only``."""
        todo = list(self.all_layers())
        while todo:
            l = todo.pop()
            if hasattr(l, "layers") and callable(l.layers):
                todo += l.layers()
            if hasattr(l, "training"):
                l.training = training

    def clear(self):
        for l in self.all_layers():
            if hasattr(l, "clear"):
                l.clear()
