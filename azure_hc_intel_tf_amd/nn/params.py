"""Flat parameter / gradient / optimizer-state storage.

All trainable variables live in ONE fp32 buffer (decayed variables first, then the
BatchNorm scale/offset that tf_cnn_benchmarks excludes from the L2 loss), with one matching
momentum buffer and one gradient buffer. This is what makes the hot paths single-launch:

* the fused SGD-momentum kernel updates every parameter in one launch (ApplyMomentum role,
  SURVEY.md §2.6);
* the gradient allreduce works on contiguous slices of one buffer -- the Horovod fusion
  buffer (HOROVOD_FUSION_THRESHOLD=128 MiB, /root/reference/benchmark-scripts/
  run-tf-sing-ucx-openmpi.sh:105) without any memcpy-in/out: weight-gradient kernels write
  straight into their slot;
* broadcast_global_variables / checkpointing are one tensor each.

BatchNorm running statistics live in a second flat buffer (``buffers``), and the bf16 GEMM
operands of every conv (packed [Cout][Kpad] + flipped/transposed [Cin][Kpad_t]) in a bf16
``pack`` buffer regenerated from the masters by one multi-tensor kernel per step.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, List, Optional

import torch

ALIGN = 64  # elements; keeps every slot 256-byte aligned


def _align(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


@dataclass
class ParamRef:
    name: str
    shape: tuple
    decay: bool
    init: Callable[[torch.Tensor], None]
    logical_numel: int = 0
    offset: int = -1
    data: Optional[torch.Tensor] = None
    grad: Optional[torch.Tensor] = None

    @property
    def numel(self) -> int:
        return int(math.prod(self.shape))


@dataclass
class BufferRef:
    name: str
    shape: tuple
    fill: float
    offset: int = -1
    data: Optional[torch.Tensor] = None

    @property
    def numel(self) -> int:
        return int(math.prod(self.shape))


@dataclass
class PackRef:
    """bf16 GEMM operands of one conv weight."""
    param: ParamRef
    Nout: int
    R: int
    S: int
    C: int
    Kpad: int
    Kpad_t: int
    want_tr: bool
    pack_off: int = -1
    tr_off: int = -1
    pack: Optional[torch.Tensor] = None
    tr: Optional[torch.Tensor] = None


class ParamStore:
    def __init__(self, seed: int = 1234):
        self.params: List[ParamRef] = []
        self.buffers: List[BufferRef] = []
        self.stats: List[BufferRef] = []
        self.persist: List[BufferRef] = []
        self.packs: List[PackRef] = []
        self.gen = torch.Generator().manual_seed(seed)
        self.finalized = False

    # ------------------------------------------------------------------ registration
    def add(self, name, shape, decay: bool, init, logical_numel: Optional[int] = None) -> ParamRef:
        p = ParamRef(name, tuple(shape), decay, init)
        p.logical_numel = logical_numel if logical_numel is not None else p.numel
        self.params.append(p)
        return p

    def add_buffer(self, name, shape, fill: float) -> BufferRef:
        b = BufferRef(name, tuple(shape), fill)
        self.buffers.append(b)
        return b

    def add_stat(self, name, shape) -> BufferRef:
        """Per-step scratch (BN statistic accumulators, saved mean/invstd): one flat fp32
        buffer, zeroed once per step together with the gradients."""
        b = BufferRef(name, tuple(shape), 0.0)
        self.stats.append(b)
        return b

    def add_persist(self, name, shape) -> BufferRef:
        """Cross-step scratch (the BN statistic shifts): zero at finalize, never zeroed per step
        and not part of the checkpoint state (any value is numerically valid)."""
        b = BufferRef(name, tuple(shape), 0.0)
        self.persist.append(b)
        return b

    def add_pack(self, p: ParamRef, Nout, R, S, C, Kpad, Kpad_t, want_tr=True) -> PackRef:
        pk = PackRef(p, Nout, R, S, C, Kpad, Kpad_t, want_tr)
        self.packs.append(pk)
        return pk

    # ------------------------------------------------------------------ init helpers
    def trunc_normal(self, std: float):
        gen = self.gen

        def f(t):
            v = torch.empty(t.shape, dtype=torch.float32)
            v.normal_(0.0, 1.0, generator=gen)
            # resample outside 2 sigma (tf.truncated_normal)
            for _ in range(8):
                bad = v.abs() > 2
                if not bool(bad.any()):
                    break
                v[bad] = torch.empty(int(bad.sum()), dtype=torch.float32).normal_(0.0, 1.0, generator=gen)
            v.clamp_(-2, 2)
            t.copy_(v * std)

        return f

    def variance_scaling(self, fan_in: int, logical_c: int = -1):
        """tf.variance_scaling_initializer() (scale 1, fan_in, truncated normal); channels
        beyond ``logical_c`` (input padding of the stem) are zero."""
        std = math.sqrt(1.0 / fan_in) / 0.87962566103423978
        tn = self.trunc_normal(std)

        def f(t):
            tn(t)
            if logical_c > 0 and t.dim() == 4 and t.shape[3] > logical_c:
                t[..., logical_c:] = 0

        return f

    def glorot_uniform(self, fan_in: int, fan_out: int, logical_c: int = -1):
        """tf.glorot_uniform_initializer() -- the tf.layers default kernel initializer, which
        tf_cnn_benchmarks' convnet_builder uses for the conv / affine layers of the models
        without batch norm (VGG, AlexNet, OverFeat, LeNet, GoogLeNet)."""
        limit = math.sqrt(6.0 / (fan_in + fan_out))
        gen = self.gen

        def f(t):
            v = torch.empty(t.shape, dtype=torch.float32).uniform_(-limit, limit, generator=gen)
            if logical_c > 0 and t.dim() == 4 and t.shape[3] > logical_c:
                v[..., logical_c:] = 0
            t.copy_(v)

        return f

    @staticmethod
    def const(v: float):
        return lambda t: t.fill_(v)

    # ------------------------------------------------------------------ finalize
    def finalize(self, device, dtype_pack=torch.bfloat16, pack: bool = True, pack_lo: bool = False):
        """Allocate the flat buffers on ``device``; ``pack``: also the bf16 GEMM operands of the
        HIP kernels (GPU; not in the PyTorch path); ``pack_lo``: also the mid and lo terms of
        the three-way bf16 split w = hi + mid + lo, the weight operands of the fp32 path's bf16x6
        GEMMs (pack_buf_lo [2][pack_total], same layout; each pack's [2][n] view registered with
        ops.functional.register_lo)."""
        order = [p for p in self.params if p.decay] + [p for p in self.params if not p.decay]
        off = 0
        self.n_decay = 0
        for p in order:
            p.offset = off
            off += _align(p.numel)
            if p.decay:
                self.n_decay = off
        self.total = off
        master_cpu = torch.zeros(self.total, dtype=torch.float32)
        for p in order:
            view = master_cpu[p.offset:p.offset + p.numel].view(p.shape)
            p.init(view)
        self.master = master_cpu.to(device)
        self.momentum = torch.zeros_like(self.master)
        self.grad = torch.zeros_like(self.master)
        for p in order:
            p.data = self.master[p.offset:p.offset + p.numel].view(p.shape)
            p.grad = self.grad[p.offset:p.offset + p.numel].view(p.shape)
        boff = 0
        for b in self.buffers:
            b.offset = boff
            boff += _align(b.numel)
        bcpu = torch.zeros(max(boff, ALIGN), dtype=torch.float32)
        for b in self.buffers:
            bcpu[b.offset:b.offset + b.numel] = b.fill
        self.buf = bcpu.to(device)
        for b in self.buffers:
            b.data = self.buf[b.offset:b.offset + b.numel].view(b.shape)
        soff = 0
        for b in self.stats:
            b.offset = soff
            soff += _align(b.numel)
        self.statbuf = torch.zeros(max(soff, ALIGN), dtype=torch.float32, device=device)
        for b in self.stats:
            b.data = self.statbuf[b.offset:b.offset + b.numel].view(b.shape)
        poff = 0
        for b in self.persist:
            b.offset = poff
            poff += _align(b.numel)
        self.persistbuf = torch.zeros(max(poff, ALIGN), dtype=torch.float32, device=device)
        for b in self.persist:
            b.data = self.persistbuf[b.offset:b.offset + b.numel].view(b.shape)
        # bf16 GEMM operands (GPU only)
        poff = 0
        rows = []
        self.pack_max_work = 1
        for pk in self.packs:
            pk.pack_off = poff
            poff += _align(pk.Nout * pk.Kpad)
            if pk.want_tr:
                pk.tr_off = poff
                poff += _align(pk.C * pk.Kpad_t)
            rows.append([pk.param.offset, pk.pack_off, pk.tr_off, pk.Nout, pk.R, pk.S, pk.C, pk.Kpad, pk.Kpad_t])
            work = pk.Nout * pk.Kpad + (pk.C * pk.Kpad_t if pk.want_tr else 0)
            self.pack_max_work = max(self.pack_max_work, work)
        self.pack_total = poff
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.packs and pack:
            # the pack kernel moves 8-channel vectors (fp32 float4 pairs -> one 16-byte bf16 store)
            for pk in self.packs:
                assert pk.C % 8 == 0 and pk.Kpad % 64 == 0, f"pack of {pk.param.name}: C % 8, Kpad % 64"
            self.pack_table = torch.tensor(rows, dtype=torch.int64, device=device)
            if pack_lo:  # fp32 path: the hi / mid / lo planes of every pack in one [3][n] buffer
                self.pack_planes = torch.zeros((3, max(poff, ALIGN)), dtype=dtype_pack, device=device)
                self.pack_buf = self.pack_planes[0]
                self.pack_buf_lo = self.pack_planes[1:]
            else:
                self.pack_planes = None
                self.pack_buf = torch.zeros(max(poff, ALIGN), dtype=dtype_pack, device=device)
                self.pack_buf_lo = None
            from ..ops import functional as Fn

            for pk in self.packs:
                pk.pack = self.pack_buf[pk.pack_off:pk.pack_off + pk.Nout * pk.Kpad]
                if pk.want_tr:
                    pk.tr = self.pack_buf[pk.tr_off:pk.tr_off + pk.C * pk.Kpad_t]
                # always (re)register: a pack without lo terms clears whatever an earlier, freed
                # pack at the same address left behind
                lo = self.pack_buf_lo
                Fn.register_lo(pk.pack, None if lo is None else lo[:, pk.pack_off:pk.pack_off + pk.Nout * pk.Kpad])
                if pk.want_tr:
                    Fn.register_lo(pk.tr, None if lo is None else lo[:, pk.tr_off:pk.tr_off + pk.C * pk.Kpad_t])
        else:
            self.pack_buf = None
            self.pack_buf_lo = None
            self.pack_planes = None
            self.pack_table = None
        self.finalized = True
        return self

    # ------------------------------------------------------------------ per step
    def repack(self):
        """fp32 masters -> bf16 GEMM operands of every conv (one launch)."""
        if self.pack_buf is None:
            return
        from ..ops import _ext

        if self.pack_planes is not None:  # fp32 path: hi / mid / lo planes in one launch
            _ext.ops().weight_pack(self.master, self.pack_planes, self.pack_table, self.pack_max_work, 3)
            return
        _ext.ops().weight_pack(self.master, self.pack_buf, self.pack_table, self.pack_max_work)

    def zero_grad(self):
        self.grad.zero_()

    def zero_stats(self):
        self.statbuf.zero_()

    def num_params(self) -> int:
        return sum(p.logical_numel for p in self.params)

    def num_tensors(self) -> int:
        return len(self.params)

    # ------------------------------------------------------------------ state
    def state_dict(self):
        return {"master": self.master.detach().cpu(), "momentum": self.momentum.detach().cpu(),
                "buffers": self.buf.detach().cpu(),
                "names": [p.name for p in self.params], "offsets": [p.offset for p in self.params]}

    def load_state_dict(self, sd):
        assert sd["names"] == [p.name for p in self.params], "checkpoint / model mismatch"
        self.master.copy_(sd["master"].to(self.master.device))
        self.momentum.copy_(sd["momentum"].to(self.momentum.device))
        self.buf.copy_(sd["buffers"].to(self.buf.device))
