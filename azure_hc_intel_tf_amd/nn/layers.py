"""Layer DSL with explicit forward / backward (the convnet_builder role of tf_cnn_benchmarks,
SURVEY.md §2.2 "convnet_builder.py": conv(+BN+ReLU), mpool, apool, affine, spatial_mean,
inception concat).

Layers run on NHWC activations and call the primitive ops of ``ops.functional`` (HIP
kernels on the GPU, PyTorch on the CPU). Backward is written out by hand instead of using
autograd so that
  * BN statistics come fused from the conv epilogue,
  * the ReLU mask / residual-gradient fan-out is produced by the BN-backward kernel,
  * the residual add of a bottleneck block becomes the beta-accumulate of the data-grad
    GEMM epilogue (no separate add kernel),
  * weight gradients land directly in the flat gradient (allreduce) buffer, and
  * the whole step (fwd + bwd + optimizer) is a fixed kernel sequence that is captured in
    a HIP graph.
"""
from __future__ import annotations

import math
import os
from typing import List, Optional, Tuple

import torch

from ..ops import functional as Fn
from ..ops.functional import ConvSpec, same_pads
from .params import ParamStore


_GPU_ACT_DTYPE = [torch.bfloat16]


def set_gpu_compute_dtype(dt: torch.dtype) -> None:
    """Activation dtype of GPU models built / stepped from now on: bf16 or IEEE fp16 (the
    hand-written HIP kernels, bf16 / fp16 builds) or fp32 (the reference-precision PyTorch
    path, --compute_dtype)."""
    from ..ops import _ext

    _GPU_ACT_DTYPE[0] = dt
    _ext.set_act("fp16" if dt == torch.float16 else "bf16")


def act_dtype(device) -> torch.dtype:
    """bf16 activations on the GPU (or the reference-precision dtype); fp32 on the CPU
    (HCB_CPU_DTYPE=float64 for exact tests)."""
    if torch.device(device).type == "cuda":
        return _GPU_ACT_DTYPE[0]
    return torch.float64 if os.environ.get("HCB_CPU_DTYPE") == "float64" else torch.float32


def empty_act(shape, device, zero=False):
    f = torch.zeros if zero else torch.empty
    return f(shape, dtype=act_dtype(device), device=device)


def empty_op(shape, device):
    """A tensor that a GEMM consumes next (a BN output, a BN-backward dz): on the fp32 path the
    Planes format the bf16x6 GEMMs read (written by the producing kernel); otherwise empty_act."""
    if torch.device(device).type == "cuda" and Fn.planes_mode():
        return Fn.Planes.empty(tuple(shape), device)
    return empty_act(shape, device)


def resolve_pads(mode, H, W, kh, kw, sh, sw, dh=1, dw=1):
    """Padding (pt, pb, pl, pr) for tf_cnn_benchmarks modes 'SAME', 'VALID', 'SAME_RESNET'."""
    if isinstance(mode, (tuple, list)):
        return tuple(mode)
    if mode == "VALID":
        return (0, 0, 0, 0)
    if mode == "SAME_RESNET":  # explicit symmetric (k-1)//2 padding then VALID
        ph = (dh * (kh - 1)) // 2
        pw = (dw * (kw - 1)) // 2
        return (ph, dh * (kh - 1) - ph, pw, dw * (kw - 1) - pw)
    if mode == "SAME":
        pt, pb = same_pads(H, kh, sh, dh)
        pl, pr = same_pads(W, kw, sw, dw)
        return (pt, pb, pl, pr)
    raise ValueError(mode)


# Fusion switches (module attributes, set before a model is built; the tests flip them to
# compare against the unfused forms):
# ResNet stem: BN+ReLU+max pool in one kernel on the GPU
FUSE_STEM_POOL = True
# replicas of the BN statistic accumulators (spreads the fp32 atomic contention)
STAT_R = 8
# fold a BN layer's backward reduction into the data-grad GEMM that produces its dy
FUSE_BN_BWD = True
# projection blocks: the shortcut's BN is applied inside the block output's BN pass
# (act(BN3(z3) + BN_sc(z_sc)) in one kernel), so the shortcut's normalised tensor is never written
FUSE_RES_BN = True
# shifted single-pass BN statistics: the conv epilogue sums (v - K), (v - K)^2 with K = the
# layer's previous batch mean, so E[x^2] - E[x]^2 does not cancel in fp32 when |mean| >> std
# (False: K = 0, the plain single-pass form)
BN_SHIFT = True
class _FixedParam:
    """A non-trainable per-channel constant with a scratch gradient sink (BN scale=False)."""

    def __init__(self, value_buf, sink_buf):
        self._v = value_buf
        self._g = sink_buf

    @property
    def data(self):
        return self._v.data

    @property
    def grad(self):
        return self._g.data


class Layer:
    in_shape: Tuple[int, int, int]
    out_shape: Tuple[int, int, int]

    def clear(self):
        pass


class ConvBN(Layer):
    """conv(k x k, stride, padding) -> BatchNorm(train) -> [residual add] -> [ReLU]."""

    _pool_fused = None  # the Pool whose forward ran fused into this layer's BN (forward_maxpool)

    def __init__(self, ps: ParamStore, name: str, in_shape, cout: int, kh: int, kw: int, sh: int = 1,
                 sw: int = 1, mode="SAME", relu: bool = True, bn: bool = True, need_dx: bool = True,
                 eps: float = 1e-5, decay: float = 0.9, logical_cin: Optional[int] = None,
                 dilation: int = 1, scale: bool = True, init: str = "variance_scaling", bias: bool = True):
        H, W, cin = in_shape
        self.name = name
        self.in_shape = in_shape
        pt, pb, pl, pr = resolve_pads(mode, H, W, kh, kw, sh, sw, dilation, dilation)
        self.spec = ConvSpec(cin=logical_cin or cin, cin_pad=cin, cout=cout, kh=kh, kw=kw, sh=sh, sw=sw,
                             pt=pt, pl=pl, pb=pb, pr=pr, dh=dilation, dw=dilation)
        P, Q = self.spec.out_hw(H, W)
        assert P > 0 and Q > 0, f"{name}: empty output"
        self.out_shape = (P, Q, cout)
        self.relu = relu
        self.bn = bn
        self.need_dx = need_dx
        self.eps = eps
        self.decay = decay
        lc = logical_cin or cin
        fan_in = kh * kw * lc
        winit = (ps.glorot_uniform(fan_in, kh * kw * cout, lc if lc != cin else -1) if init == "glorot"
                 else ps.variance_scaling(fan_in, lc if lc != cin else -1))
        self.w = ps.add(f"{name}/conv2d/kernel", (cout, kh, kw, cin), True, winit, logical_numel=cout * kh * kw * lc)
        self.pack = ps.add_pack(self.w, cout, kh, kw, cin, self.spec.Kpad, self.spec.Kpad_t, want_tr=need_dx)
        if bn:
            if scale:
                self.gamma = ps.add(f"{name}/batchnorm/gamma", (cout,), False, ParamStore.const(1.0))
            else:  # tf batch_norm(scale=False): gamma fixed at 1, not a variable
                self.gamma = _FixedParam(ps.add_buffer(f"{name}/batchnorm/gamma_fixed", (cout,), 1.0),
                                         ps.add_buffer(f"{name}/batchnorm/gamma_grad_sink", (cout,), 0.0))
            self.beta = ps.add(f"{name}/batchnorm/beta", (cout,), False, ParamStore.const(0.0))
            self.rmean = ps.add_buffer(f"{name}/batchnorm/moving_mean", (cout,), 0.0)
            self.rvar = ps.add_buffer(f"{name}/batchnorm/moving_variance", (cout,), 1.0)
            # GPU: statistic accumulators (R replicas of [2][C]) and saved batch moments
            self.acc_f = ps.add_stat(f"{name}/bn_acc_fwd", (STAT_R, 2, cout))
            self.acc_b = ps.add_stat(f"{name}/bn_acc_bwd", (STAT_R, 2, cout))
            self.sv_mean = ps.add_stat(f"{name}/bn_mean", (cout,))
            self.sv_invstd = ps.add_stat(f"{name}/bn_invstd", (cout,))
            # statistics shift K: the previous step's batch mean (written by the BN backward); the
            # epilogue accumulates (v - K) so the single-pass variance does not cancel (|mean| >> std)
            self.shift = ps.add_persist(f"{name}/bn_shift", (cout,)) if BN_SHIFT else None
        else:
            # ResNet-v2's un-normalised convs (shortcut, conv3) have no bias in tf_cnn_benchmarks
            self.bias = ps.add(f"{name}/conv2d/bias", (cout,), True, ParamStore.const(0.0)) if bias else None
        self._saved = None
        self._acc = None  # (fwd acc, bwd acc, replicas) of the current step
        self._pre_reduced = False
        self.training = True  # False: inference BN from the moving statistics (forward-only)

    def flops(self, batch: int) -> int:
        P, Q, C = self.out_shape
        return 2 * batch * P * Q * C * self.spec.kh * self.spec.kw * self.spec.cin

    def _stat_bufs(self, N: int, dev):
        """(forward acc, backward acc, replicas) of this step's BN statistics: the persistent
        STAT_R-replica buffers, or in deterministic mode fresh ones with a replica per 64 rows
        (each fp32 slot then receives a single add)."""
        if not Fn.deterministic():
            self._acc = (self.acc_f.data, self.acc_b.data, STAT_R)
        else:
            P, Q, C = self.out_shape
            R = Fn.det_replicas(N * P * Q)
            self._acc = (torch.zeros((R, 2, C), dtype=torch.float32, device=dev),
                         torch.zeros((R, 2, C), dtype=torch.float32, device=dev), R)
        return self._acc

    def params(self):
        """Trainable ParamRefs of this layer (gradient slots in the flat buffer)."""
        if not self.bn:
            return [self.w, self.bias] if self.bias is not None else [self.w]
        out = [self.w, self.beta]
        if not isinstance(self.gamma, _FixedParam):
            out.append(self.gamma)
        return out

    # ------------------------------------------------------------------ forward
    def forward_deferred(self, x):
        """GPU training forward of a conv + BN whose BN apply is left to the consumer (a
        projection shortcut: the block output's BN pass normalises z_sc on the fly, see
        ``forward(residual_bn=)``). Returns z; the saved batch moments are written by that pass."""
        assert self.bn and not self.relu and self.training and Fn.native(x)
        P, Q, C = self.out_shape
        z = empty_act((x.shape[0], P, Q, C), x.device)
        x = self._conv_fwd_stats(x, z)
        self._saved = (x, z, None, Fn.BNSaved(self.sv_mean.data, self.sv_invstd.data), False)
        return z

    def res_bn_args(self):
        """The residual-BN operands of a deferred BN (bn_forward_acc res_bn)."""
        acc_f, _, _ = self._acc
        return (acc_f, self.gamma.data, self.beta.data, self.sv_mean.data, self.sv_invstd.data, self.rmean.data,
                self.rvar.data, self._shift())

    def forward(self, x, out=None, residual=None, residual_bn=None):
        """``residual_bn``: the ConvBN (run with forward_deferred) whose raw output ``residual``
        is BN-normalised inside this layer's BN pass before the add."""
        N = x.shape[0]
        P, Q, C = self.out_shape
        dev = x.device
        if self.bn and not self.training:
            z = empty_act((N, P, Q, C), dev)
            y = out if out is not None else empty_act((N, P, Q, C), dev)
            if Fn.planes_mode() and Fn.native(x) and not Fn.is_planes(x):  # fp32 path: the GEMM operand as planes
                x = Fn.to_planes(x)
            Fn.conv_forward(x, self.spec, self.pack.pack if Fn.native(x) else None, self.w.data, z)
            Fn.bn_inference(z, self.gamma.data, self.beta.data, self.rmean.data, self.rvar.data, self.eps, y,
                            self.relu, residual=residual)
            self._saved = None
            return y
        if self.bn:
            z = empty_act((N, P, Q, C), dev)
            if Fn.native(x):
                y = out if out is not None else empty_op((N, P, Q, C), dev)
                # conv epilogue accumulates the batch statistics; the apply kernel finalizes them
                x = self._conv_fwd_stats(x, z)
                acc_f, _, R = self._acc
                if residual_bn is not None:
                    assert residual_bn._acc[2] == R, "residual BN accumulators must match the replica count"
                saved = Fn.bn_forward_acc(z, self.gamma.data, self.beta.data, self.rmean.data, self.rvar.data,
                                          self.decay, self.eps, y, self.relu, acc_f, R,
                                          self.sv_mean.data, self.sv_invstd.data, residual=residual,
                                          shift=self._shift(),
                                          res_bn=residual_bn.res_bn_args() if residual_bn is not None else None)
            else:
                y = out if out is not None else empty_act((N, P, Q, C), dev)
                Fn.conv_forward(x, self.spec, None, self.w.data, z)
                saved = Fn.bn_forward(z, self.gamma.data, self.beta.data, self.rmean.data, self.rvar.data,
                                      self.decay, self.eps, y, self.relu, residual=residual)
            self._saved = (x, z, y, saved, residual is not None)
            return y
        assert residual is None or not self.relu, "conv without BN: residual add only without ReLU"
        y = out if out is not None else empty_act((N, P, Q, C), dev)
        if Fn.planes_mode() and Fn.native(x) and not Fn.is_planes(x):
            # fp32 path, conv + bias + ReLU layers (the zoo): the fp32 input split into the GEMM's
            # planes once, for the forward and the weight gradient
            x = Fn.to_planes(x)
        Fn.conv_forward(x, self.spec, self.pack.pack if Fn.native(x) else None, self.w.data, y,
                        bias=self.bias.data if self.bias is not None else None, relu=self.relu, residual=residual)
        self._saved = (x, None, y, None, False)
        return y

    def forward_maxpool(self, x, pool: "Pool", out_planes: bool = True):
        """GPU training forward of conv -> BN -> ReLU -> max pool (the ResNet stem) in two
        launches: the conv (BN statistics in its epilogue) and one BN+ReLU+pool kernel. The
        full-size BN+ReLU activation is never written; ``pool`` keeps the argmax for its
        backward and this layer recomputes the ReLU mask from z. ``out_planes=False``: on the fp32
        path the pooled map is written as an fp32 tensor, not as GEMM planes (its consumer is a
        BN -- ResNet v2's first pre-activation)."""
        assert self.bn and self.relu and Fn.native(x) and pool.is_max and self.training
        N = x.shape[0]
        P, Q, C = self.out_shape
        z = empty_act((N, P, Q, C), x.device)
        x = self._conv_fwd_stats(x, z)
        y = (empty_op if out_planes else empty_act)((N,) + tuple(pool.out_shape), x.device)
        amax = torch.empty((N,) + tuple(pool.out_shape), dtype=torch.uint8, device=x.device)
        acc_f, _, R = self._acc
        saved = Fn.bn_relu_maxpool_acc(z, self.gamma.data, self.beta.data, self.rmean.data, self.rvar.data, self.decay,
                                       self.eps, acc_f, R, self.sv_mean.data, self.sv_invstd.data, y,
                                       amax, *pool.k, *pool.s, pool.pads, shift=self._shift())
        self._saved = (x, z, None, saved, False)
        pool._saved = (z, y, amax)  # the argmax backward reads only shapes from x / y
        self._pool_fused = pool
        return y

    def backward_from_maxpool(self, dyp, pool: "Pool"):
        """Backward of forward_maxpool without the full-size BN output gradient: the BN backward
        reduce and apply gather it from the pool's gradient ``dyp`` through the saved argmax
        (bn.hip pool_gather), so the max-pool backward kernel and its conv-sized output (written
        once, read twice) are gone. Then the weight gradient; the stem needs no dx."""
        assert self._pool_fused is pool and not self.need_dx
        x, z, _, saved, _ = self._saved
        _, _, amax = pool._saved
        N = dyp.shape[0]
        H, W, C = self.out_shape
        P, Q, _ = pool.out_shape
        pt, _, pl, _ = pool.pads
        dz = empty_op((N, H, W, C), dyp.device)
        _, acc_b, R = self._acc
        Fn.bn_backward_acc(dyp, None, z, saved, self.gamma.data, self.beta.data, 2, self.gamma.grad, self.beta.grad,
                           dz, acc_b, R, None, shift_out=self._shift(),
                           pool=(amax, [H, W, P, Q, pool.k[0], pool.s[0], pt, pl]))
        run_wgrad(self, dz, x)
        self._saved = None
        self._pool_fused = None
        pool._saved = None

    def _conv_fwd_stats(self, x, z):
        """GPU conv with the BN statistics in its epilogue; returns the tensor the weight
        gradient will read (the conv's GEMM input)."""
        acc_f, _, R = self._stat_bufs(x.shape[0], x.device)
        if Fn.planes_mode() and not Fn.is_planes(x):  # fp32 path: the GEMM (and wgrad) operand as planes
            x = Fn.to_planes(x)
        Fn.conv_forward(x, self.spec, self.pack.pack, self.w.data, z, stats=acc_f, stats_R=R,
                        stats_shift=self._shift())
        return x

    def _shift(self):
        return self.shift.data if self.shift is not None else None

    def _wgrad(self, dz, x):
        Fn.conv_wgrad(dz, x, self.spec, self.w.grad.view(dz.shape[-1], -1) if Fn.native(dz) else self.w.grad)

    # ------------------------------------------------------------------ backward
    def bwd_fuse_request(self) -> Optional[Fn.BNBwdFuse]:
        """BN-backward reduction of this layer, to be fused into the GEMM producing its dy."""
        if not (self.bn and FUSE_BN_BWD) or self._saved is None:
            return None
        x, z, y, saved, had_res = self._saved
        if z.dtype == torch.float32 and not (Fn.planes_mode() and z.is_cuda):
            return None  # fp32 fusion runs on the plane GEMMs (conv_p3.hip) only
        mode = (1 if had_res else 2) if self.relu else 0
        self._pre_reduced = True
        _, acc_b, R = self._acc if self._acc is not None else (None, self.acc_b.data, STAT_R)
        return Fn.BNBwdFuse(z, y, saved, self.gamma.data, self.beta.data, mode, acc_b, R)

    def backward(self, dy, dx=None, accumulate: bool = False, want_gres: bool = False, dx_bn=None):
        """Returns (dx or None, gres or None). gres = gradient w.r.t. the residual input.
        ``dx_bn``: the ConvBN layer whose BN consumes dx; its backward reduction (and ReLU
        gating) is fused into this layer's data-grad GEMM."""
        x, z, y, saved, had_res = self._saved
        dev = dy.device
        N = dy.shape[0]
        P, Q, C = self.out_shape
        gres = None
        if self.bn and self._pre_reduced:
            # dy is already g = dy * mask and (GPU) acc_b holds sum(g), sum(g*xhat)
            self._pre_reduced = False
            dz = empty_op((N, P, Q, C), dev) if Fn.native(dy) else empty_act((N, P, Q, C), dev)
            if Fn.native(dy):
                _, acc_b, R = self._acc
                Fn.bn_backward_acc(dy, None, z, saved, self.gamma.data, self.beta.data, 0, self.gamma.grad,
                                   self.beta.grad, dz, acc_b, R, None, pre_reduced=True, shift_out=self._shift())
            else:
                Fn.bn_backward(dy, y, z, saved, self.gamma.data, self.beta.data, 0, self.gamma.grad,
                               self.beta.grad, dz, None)
            if want_gres:
                gres = dy
        elif self.bn:
            dz = empty_op((N, P, Q, C), dev) if Fn.native(dy) else empty_act((N, P, Q, C), dev)
            if want_gres:
                gres = empty_act((N, P, Q, C), dev)
            relu_mode = (1 if had_res else 2) if self.relu else 0
            if Fn.native(dy):
                _, acc_b, R = self._acc
                Fn.bn_backward_acc(dy, y, z, saved, self.gamma.data, self.beta.data, relu_mode, self.gamma.grad,
                                   self.beta.grad, dz, acc_b, R, gres, shift_out=self._shift())
            else:
                Fn.bn_backward(dy, y, z, saved, self.gamma.data, self.beta.data, relu_mode, self.gamma.grad,
                               self.beta.grad, dz, gres)
        else:
            if self.relu:
                if Fn.native(dy) and not (dy.is_contiguous() and y.is_contiguous()):
                    dy, y = dy.contiguous(), y.contiguous()  # concat-window views (GoogLeNet)
                dz = Fn.relu_backward(dy, y, empty_act((N, P, Q, C), dev))
            else:
                dz = dy if dy.is_contiguous() else dy.contiguous()
            if self.bias is not None:
                Fn.colsum(dz.reshape(-1, C), N * P * Q, C, self.bias.grad)
            if want_gres:
                gres = dz
            if Fn.planes_mode() and Fn.native(dz) and not Fn.is_planes(dz):
                dz = Fn.to_planes(dz)  # one split for the data- and the weight-gradient GEMM
        run_wgrad(self, dz, x)
        if self.need_dx:
            H, W, Cin = self.in_shape
            if dx is None:  # (a strided 1x1 data gradient writes its stride cells' gaps itself)
                dx = empty_act((N, H, W, Cin), dev)
                accumulate = False
            bnb = dx_bn.bwd_fuse_request() if dx_bn is not None else None
            Fn.conv_dgrad(dz, self.spec, self.pack.tr, self.w.data, dx, accumulate, bnb=bnb)
        self._saved = None
        return dx, gres

    def clear(self):
        self._saved = None
        self._pre_reduced = False


# Weight-gradient GEMMs on a side stream (set by the Trainer around a step, HCB_WGRAD_STREAM=1):
# layer i's dW GEMM forks off the main stream right after its dz exists and runs beside the data-
# gradient chain, filling the CUs the dgrad grid leaves idle (e.g. 196 tiles on 256 CUs); the
# Trainer joins before a segment's gradients are reduced / the optimizer runs. The operands are
# kept referenced until the join, so the caching allocator cannot hand their memory to a later
# main-stream tensor while the side stream still reads it.
WGRAD_SIDE = {"stream": None, "keep": []}


def run_wgrad(layer, dz, x):
    s = WGRAD_SIDE["stream"]
    if s is None or not Fn.native(dz):
        layer._wgrad(dz, x)
        return
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        layer._wgrad(dz, x)
    WGRAD_SIDE["keep"].append((dz, x))


def wgrad_join():
    """The main stream waits for every weight-gradient GEMM issued on the side stream."""
    s = WGRAD_SIDE["stream"]
    if s is not None and WGRAD_SIDE["keep"]:
        torch.cuda.current_stream().wait_stream(s)
        WGRAD_SIDE["keep"].clear()


# GPU ResNet stem as a space-to-depth 4x4/1 GEMM (False: the direct padded 7x7/2 form)
STEM_S2D = True


# ResNet stem: the BN backward gathers dy from the max pool's gradient (ConvBN.backward_from_maxpool).
# Bitwise equal (tests/test_stem_pool_bwd_gpu.py). The per-pixel window gather (<= 4 argmax /
# gradient loads + index math per 8 channels) costs about what the removed round trip saves: bf16
# 0.5-0.7% slower (16-bit: the round trip is only 103 MB), fp32 +0.3% in round 5's A/B
# (profiles/r4sp_stem_pool_bwd_ab.txt, profiles/r5_stem_pool_bwd_fp32.txt). None = on for the fp32
# (planes) path only; HCB_FUSE_STEM_POOL_BWD=1 / 0 forces it.
_SPB = os.environ.get("HCB_FUSE_STEM_POOL_BWD")
FUSE_STEM_POOL_BWD = None if _SPB is None else _SPB == "1"


def fuse_stem_pool_bwd() -> bool:
    return FUSE_STEM_POOL_BWD if FUSE_STEM_POOL_BWD is not None else Fn.planes_mode()


class StemS2D(ConvBN):
    """The 7x7/2 'SAME_RESNET' stem conv (3 input channels, stored padded) computed on the GPU as
    a stride-1 4x4 conv over the 2x2 space-to-depth fold of the image (csrc/kernels/stem.hip):
    K = 256 instead of the padded direct form's 448. The fp32 master weight, its gradient, the
    BN and the CPU path are exactly those of the 7x7 layer; only the GEMM operands are folded."""

    PAD = 4  # X'(P) = x(2P + a - 4): the 3-pixel SAME_RESNET pad plus the fold's half step

    def __init__(self, ps: ParamStore, name: str, in_shape, cout: int, **kw):
        super().__init__(ps, name, in_shape, cout, 7, 7, 2, 2, "SAME_RESNET", **kw)
        assert self.spec.pt == 3 and self.spec.pl == 3 and not self.need_dx
        P, Q, _ = self.out_shape
        self.fold_shape = (P + 3, Q + 3, 16)
        # the GEMM of the 4x4 / stride-1 conv over the 16-channel fold, read as a 4x1 conv over ROW
        # WINDOWS of 64 channels (pixel w's window = the 16 channels of pixels w .. w+3, the input's
        # pixel stride staying 16; csrc/bindings.cpp x_span_bytes): K = 4 x 64 keeps the weight layout
        # [cout][r][s][16] = [cout][r][64], and every k-step reads one contiguous 64-channel row (the
        # kernels' channels-multiple-of-64 fast path) instead of a gather of 16-channel pieces of two
        # or four taps. pr = -3: the windows of the last three fold columns reach past the row and are
        # never an output's.
        self.fold_spec = ConvSpec(cin=64, cin_pad=64, cout=cout, kh=4, kw=1, sh=1, sw=1, pt=0, pl=0, pb=0, pr=-3)
        self._wfold = None
        self._wpack = None
        # the folded weight gradient [cout][256]: per-step scratch in the statistics buffer, so the
        # step-start clear zeroes it (no allocation + fill per step)
        self.dwfold = ps.add_stat(f"{name}/dw_fold", (cout, 256))

    def _folded_weight(self, dev):
        """The folded GEMM weight [cout][256]: the 16-bit pack, or on the fp32 path the hi pack of
        its three planes (mid / lo attached as the pack's ``hcb_lo``, ops.functional.lo_pack)."""
        from ..ops import _ext

        p3 = Fn.lo_pack(self.pack.pack) is not None  # this model's packs carry planes: the fp32 path
        if self._wfold is None or self._wfold.device != dev or (self._wfold.dim() == 3) != p3:
            if p3:
                self._wfold = torch.empty((3, self.spec.cout, 256), dtype=torch.bfloat16, device=dev)
                self._wpack = self._wfold[0]
                Fn.register_lo(self._wpack, self._wfold[1:].reshape(2, -1))
            else:
                self._wfold = torch.empty((self.spec.cout, 256), dtype=act_dtype(dev), device=dev)
                self._wpack = self._wfold
        _ext.ops().stem_wfold(self.w.data, self._wfold)
        return self._wpack

    def fold_input(self, x):
        """2x2 space-to-depth fold of the padded image; on the fp32 path the image is split into its
        bf16 planes first and the three planes are folded as one batch of 3N images."""
        from ..ops import _ext

        if Fn.is_planes(x) or (x.is_cuda and x.dtype == torch.float32):
            N = x.shape[0]
            xf = Fn.Planes.empty((N,) + self.fold_shape, x.device)
            if not Fn.is_planes(x) and x.is_contiguous():  # split while folding: one pass over the image
                _ext.ops().stem_s2d(x, xf.t, self.PAD)
                return xf
            xp = Fn.to_planes(x)
            _ext.ops().stem_s2d(xp.t.view((3 * N,) + tuple(xp.shape[1:])), xf.t.view((3 * N,) + self.fold_shape),
                                self.PAD)
            return xf
        xf = torch.empty((x.shape[0],) + self.fold_shape, dtype=x.dtype, device=x.device)
        _ext.ops().stem_s2d(x, xf, self.PAD)
        return xf

    def _conv_fwd_stats(self, x, z):
        xf = self.fold_input(x)
        acc_f, _, R = self._stat_bufs(x.shape[0], x.device)
        Fn.conv_forward(xf, self.fold_spec, self._folded_weight(x.device), self.w.data, z, stats=acc_f, stats_R=R,
                        stats_shift=self._shift())
        return xf

    def _wgrad(self, dz, x):
        if not Fn.native(dz):
            return super()._wgrad(dz, x)
        from ..ops import _ext

        if x.shape[1:] != self.fold_shape:  # direct-form training path (forward() not forward_maxpool)
            x = self.fold_input(x)
        dwf = self.dwfold.data.view(self.spec.cout, 256)
        Fn.conv_wgrad(dz, x, self.fold_spec, dwf)
        _ext.ops().stem_wgrad_unfold(dwf, self.w.grad)

    def forward(self, x, out=None, residual=None):
        if not Fn.native(x):
            return super().forward(x, out, residual)
        N = x.shape[0]
        P, Q, C = self.out_shape
        z = empty_act((N, P, Q, C), x.device)
        y = out if out is not None else empty_act((N, P, Q, C), x.device)
        if not self.training:
            xf = self.fold_input(x)
            Fn.conv_forward(xf, self.fold_spec, self._folded_weight(x.device), self.w.data, z)
            Fn.bn_inference(z, self.gamma.data, self.beta.data, self.rmean.data, self.rvar.data, self.eps, y,
                            self.relu, residual=residual)
            self._saved = None
            return y
        xf = self._conv_fwd_stats(x, z)
        acc_f, _, R = self._acc
        saved = Fn.bn_forward_acc(z, self.gamma.data, self.beta.data, self.rmean.data, self.rvar.data, self.decay,
                                  self.eps, y, self.relu, acc_f, R, self.sv_mean.data,
                                  self.sv_invstd.data, residual=residual, shift=self._shift())
        self._saved = (xf, z, y, saved, residual is not None)
        return y

    def tune_view(self):
        """The GEMM problem the autotuner must time for this layer (the folded one)."""
        from types import SimpleNamespace

        dev = self.w.data.device
        return SimpleNamespace(spec=self.fold_spec, in_shape=self.fold_shape, out_shape=self.out_shape,
                               need_dx=False, pack=SimpleNamespace(pack=self._folded_weight(dev), tr=None),
                               name=self.name)


class Pool(Layer):
    def __init__(self, name, in_shape, kh, kw, sh, sw, mode="VALID", is_max=True, incl_pad=False):
        H, W, C = in_shape
        self.name = name
        self.in_shape = in_shape
        self.k = (kh, kw)
        self.s = (sh, sw)
        self.pads = resolve_pads(mode, H, W, kh, kw, sh, sw)
        pt, pb, pl, pr = self.pads
        P = (H + pt + pb - kh) // sh + 1
        Q = (W + pl + pr - kw) // sw + 1
        self.out_shape = (P, Q, C)
        self.is_max = is_max
        self.incl_pad = incl_pad
        self._saved = None

    def forward(self, x, out=None):
        N = x.shape[0]
        if Fn.planes_mode() and Fn.native(x) and not Fn.is_planes(x) and (out is None or Fn.is_planes(out)):
            # fp32 path after a BN-free conv (the zoo): the fp32 map split into planes here, where the
            # consuming GEMM would split the pooled map anyway; the pool then runs on planes
            x = Fn.to_planes(x)
        if out is not None:
            y = out
        elif Fn.is_planes(x):  # fp32 path: the pooled tensor is the next GEMM's operand
            y = Fn.Planes.empty((N,) + self.out_shape, x.device)
        else:
            y = empty_act((N,) + self.out_shape, x.device)
        amax = None
        if self.is_max and Fn.native(x):
            amax = torch.empty((N,) + self.out_shape, dtype=torch.uint8, device=x.device)
        Fn.pool_forward(x, y, *self.k, *self.s, self.pads, self.is_max, self.incl_pad, argmax=amax)
        self._saved = (x, y, amax)
        return y

    def backward(self, dy, dx=None, accumulate=False):
        x, y, amax = self._saved
        if dx is None:
            dx = empty_act(x.shape, dy.device)
            accumulate = False
        Fn.pool_backward(dy, x, y, dx, *self.k, *self.s, self.pads, self.is_max, self.incl_pad, accumulate,
                         argmax=amax)
        self._saved = None
        return dx

    def clear(self):
        self._saved = None


class BNReLU(Layer):
    """Standalone training-mode BatchNorm (+ ReLU) on an activation: the pre-activation of
    ResNet v2 blocks (tf_cnn_benchmarks ``bottleneck_block_v2``: preact = relu(batch_norm(x)))
    and its final BN. There is no producing GEMM epilogue to fuse the statistics into: on the GPU
    one reduction pass accumulates them (shifted sums into the R replicas, ``bn_stats_acc``) and
    the finalize-free apply writes the next GEMMs' operand (Planes on the fp32 path); the backward
    is the acc-replica reduce + apply, with the identity shortcut's gradient added in the apply
    (``backward(dy, add=)``)."""

    def __init__(self, ps: ParamStore, name: str, in_shape, relu: bool = True, eps: float = 1e-5,
                 decay: float = 0.9):
        self.name = name
        self.in_shape = in_shape
        self.out_shape = in_shape
        C = in_shape[2]
        self.relu = relu
        self.eps = eps
        self.decay = decay
        self.gamma = ps.add(f"{name}/batchnorm/gamma", (C,), False, ParamStore.const(1.0))
        self.beta = ps.add(f"{name}/batchnorm/beta", (C,), False, ParamStore.const(0.0))
        self.rmean = ps.add_buffer(f"{name}/batchnorm/moving_mean", (C,), 0.0)
        self.rvar = ps.add_buffer(f"{name}/batchnorm/moving_variance", (C,), 1.0)
        self.acc_f = ps.add_stat(f"{name}/bn_acc_fwd", (STAT_R, 2, C))
        self.acc_b = ps.add_stat(f"{name}/bn_acc_bwd", (STAT_R, 2, C))
        self.sv_mean = ps.add_stat(f"{name}/bn_mean", (C,))
        self.sv_invstd = ps.add_stat(f"{name}/bn_invstd", (C,))
        self.shift = ps.add_persist(f"{name}/bn_shift", (C,)) if BN_SHIFT else None
        self._saved = None
        self._acc = None
        self.training = True

    def params(self):
        return [self.beta, self.gamma]

    _stat_bufs = ConvBN._stat_bufs
    _shift = ConvBN._shift

    def forward(self, x):
        if Fn.is_planes(x):  # (the fp32 path's pooled stem output when not produced in fp32)
            x = Fn.from_planes(x)
        if not self.training:
            y = empty_act(tuple(x.shape), x.device)
            return Fn.bn_inference(x, self.gamma.data, self.beta.data, self.rmean.data, self.rvar.data, self.eps, y,
                                   self.relu)
        if Fn.native(x):
            N, H, W, C = x.shape
            acc_f, _, R = self._stat_bufs(N, x.device)
            Fn.bn_stats_acc(x, acc_f, R, self._shift())
            y = empty_op(tuple(x.shape), x.device)
            saved = Fn.bn_forward_acc(x, self.gamma.data, self.beta.data, self.rmean.data, self.rvar.data, self.decay,
                                      self.eps, y, self.relu, acc_f, R, self.sv_mean.data, self.sv_invstd.data,
                                      shift=self._shift())
        else:
            y = empty_act(tuple(x.shape), x.device)
            saved = Fn.bn_forward(x, self.gamma.data, self.beta.data, self.rmean.data, self.rvar.data, self.decay,
                                  self.eps, y, self.relu)
        self._saved = (x, y, saved)
        return y

    def backward(self, dy, add=None):
        """dx = BN'(dy) (+ ``add``, the identity shortcut's gradient, summed in the same pass)."""
        x, y, saved = self._saved
        dx = empty_act(tuple(x.shape), dy.device)
        dy = dy if dy.is_contiguous() else dy.contiguous()
        if Fn.native(dy):
            _, acc_b, R = self._acc
            Fn.bn_backward_acc(dy, None, x, saved, self.gamma.data, self.beta.data, 2 if self.relu else 0,
                               self.gamma.grad, self.beta.grad, dx, acc_b, R, None, shift_out=self._shift(),
                               add=add)
        else:
            Fn.bn_backward(dy, y, x, saved, self.gamma.data, self.beta.data, 1 if self.relu else 0, self.gamma.grad,
                           self.beta.grad, dx)
            if add is not None:
                dx.add_(add)
        self._saved = None
        return dx

    def clear(self):
        self._saved = None


class Dropout(Layer):
    """tf_cnn_benchmarks ``cnn.dropout(keep_prob=0.5)`` after the hidden affine layers of
    AlexNet / VGG / OverFeat. Identity when ``keep == 1`` or in forward-only mode."""

    def __init__(self, name, in_shape, keep: float = 0.5, seed: int = 0):
        self.name = name
        self.in_shape = in_shape
        self.out_shape = in_shape
        self.keep = keep
        self.seed = seed
        self.training = True
        self._step = None
        self._mask = None

    def forward(self, x):
        if self.keep >= 1.0 or not self.training:
            self._mask = None
            return x
        if self._step is None or self._step.device != x.device:
            self._step = torch.zeros(1, dtype=torch.int64, device=x.device)
        y = torch.empty_like(x)
        if Fn.native(x):
            mask = torch.empty((x.numel() + 7) // 8, dtype=torch.uint8, device=x.device)
        else:
            mask = torch.empty(x.shape, dtype=torch.bool, device=x.device)
        Fn.dropout_forward(x, y, mask, self.keep, self.seed, self._step)
        self._step.add_(1)  # device-side: a replayed graph advances it too
        self._mask = mask
        return y

    def backward(self, dy):
        if self._mask is None:
            return dy
        dx = torch.empty_like(dy)
        Fn.dropout_backward(dy.contiguous(), self._mask, dx, self.keep)
        self._mask = None
        return dx

    def clear(self):
        self._mask = None


class GlobalAvgPool(Layer):
    def __init__(self, name, in_shape):
        self.name = name
        self.in_shape = in_shape
        self.out_shape = (1, 1, in_shape[2])

    def forward(self, x):
        N = x.shape[0]
        if Fn.is_planes(x):  # fp32 path: the pooled features feed the classifier GEMM as planes
            y = Fn.Planes.empty((N, self.in_shape[2]), x.device)
        else:
            y = torch.empty((N, self.in_shape[2]), dtype=x.dtype, device=x.device)
        return Fn.gap_forward(x, y)

    def backward(self, dy):
        N = dy.shape[0]
        dx = empty_act((N,) + tuple(self.in_shape), dy.device)
        Fn.gap_backward(dy, dx)
        return dx


class Logits(Layer):
    """Final affine layer: logits[B, ncls] (fp32, row stride padded to 8) = x W^T + b."""

    def __init__(self, ps: ParamStore, name, in_features: int, ncls: int, stddev: float = 0.01):
        self.name = name
        self.cin = in_features
        self.ncls = ncls
        self.ld = (ncls + 7) // 8 * 8
        self.spec = ConvSpec(cin=in_features, cin_pad=in_features, cout=ncls, kh=1, kw=1)
        self.w = ps.add(f"{name}/affine/weights", (ncls, 1, 1, in_features), True, ps.trunc_normal(stddev))
        self.b = ps.add(f"{name}/affine/biases", (ncls,), True, ParamStore.const(0.0))
        # dgrad operand uses the padded logits width as its reduction length
        kt = (self.ld + 63) // 64 * 64
        self.pack = ps.add_pack(self.w, ncls, 1, 1, in_features, self.spec.Kpad, kt, want_tr=True)
        self._x = None
        # fp32 copy of 16-bit dlogits (Trainer): the bias gradient's source -- only for the exact
        # dlogits tensor it was written with (dl32_src), never for another caller's dlogits
        self.dl32 = None
        self.dl32_src = None

    def forward(self, x):
        B = x.shape[0]
        x4 = x.view(B, 1, 1, self.cin)
        logits = torch.empty((B, self.ld), dtype=torch.float32, device=x.device)
        if Fn.native(x):
            Fn.conv_forward(x4, self.spec, self.pack.pack, None, logits.view(B, 1, 1, self.ld)[..., :self.ld],
                            bias=self.b.data)
        else:
            logits.zero_()
            logits[:, :self.ncls] = (x @ self.w.data.view(self.ncls, self.cin).t().to(x.dtype)
                                     + self.b.data.to(x.dtype)).float()
        self._x = x
        return logits

    def backward(self, dlogits):
        """dlogits: [B, ld] (bf16 on GPU, zero in the padding columns)."""
        x = self._x
        B = x.shape[0]
        if (self.dl32 is not None and dlogits is self.dl32_src and self.dl32.shape[0] == B and Fn.native(x)
                and dlogits.dtype != torch.float32):
            Fn._ext.ops().colsum(self.dl32, self.ld, B, self.ncls, self.b.grad)
        else:
            Fn.colsum(dlogits, B, self.ncls, self.b.grad)
        if Fn.native(x) and x.dtype == torch.float32:  # fp32 path: Planes operands (conv_p3.hip)
            dlp = Fn.to_planes(dlogits)
            Fn.conv_wgrad(dlp.view(B, 1, 1, self.ld), x.view(B, 1, 1, self.cin), self._wgrad_spec(),
                          self.w.grad.view(self.ncls, self.cin))
            dx = torch.empty((B, self.cin), dtype=torch.float32, device=x.device)
            Fn.conv_dgrad(dlp.view(B, 1, 1, self.ld), self._dgrad_spec(), self.pack.tr, None,
                          dx.view(B, 1, 1, self.cin), False)
        elif Fn.native(x):
            hcb = Fn._ext.ops()
            geom = [B, 1, 1, self.cin, self.cin, 1, 1, 1, 1, 1, 1, 0, 0, 1, 1, self.ncls, self.ld]
            cfg, splits = 2, 1
            hcb.conv_wgrad(dlogits, x, self.w.grad.view(self.ncls, self.cin), geom, cfg, splits)
            dx = torch.empty((B, self.cin), dtype=x.dtype, device=x.device)
            C = self.ld
            geom = [B, 1, 1, C, C, 1, 1, 1, 1, 1, 1, 0, 0, 1, 1, 1, 1, self.cin, C, self.pack.Kpad_t, self.cin,
                    0, 1, 1, 1, 1, 0, Fn._f32o(dx)]
            cfgd = Fn.conv_plan(B, self.cin, C)[0]
            hcb.conv_igemm(dlogits, self.pack.tr, dx, None, None, None, geom, cfgd, None, None)
        else:
            g = dlogits[:, :self.ncls]
            self.w.grad.view(self.ncls, self.cin).add_((g.t() @ x).float())
            dx = g @ self.w.data.view(self.ncls, self.cin).to(x.dtype)
        self._x = None
        return dx

    def _wgrad_spec(self):
        """dW[ncls, cin] = dlogits^T x as a 1x1 conv's weight gradient (dz rows of ld columns)."""
        return ConvSpec(cin=self.cin, cin_pad=self.cin, cout=self.ncls, kh=1, kw=1)

    def _dgrad_spec(self):
        """dx = dlogits W as a 1x1 conv's data gradient: the reduction runs over the padded logits
        width (the transposed pack's Kpad_t covers it)."""
        return ConvSpec(cin=self.cin, cin_pad=self.cin, cout=self.ld, kh=1, kw=1)

    def flops(self, batch):
        return 2 * batch * self.cin * self.ncls

    def params(self):
        return [self.w, self.b]
