"""Inception-v3 as trained by tf_cnn_benchmarks ``--model=inception3`` (BASELINE config 4;
SURVEY.md §2.6 "Inception-v3 adds these kernel shapes").

299x299 input; stem conv 3x3/2 V(32), 3x3 V(32), 3x3 S(64), maxpool 3x3/2 V, 1x1 V(80),
3x3 V(192), maxpool 3x3/2 V; modules A(32), A(64), A(64), B, C(128), C(160), C(160), C(192),
D, E(avg), E(max); 8x8 average pool; affine -> 1001 classes. Every conv is conv + BN + ReLU
with tf_cnn_benchmarks' default batch-norm config (decay 0.999, epsilon 0.001, scale=False).

MI355X specifics: asymmetric 1x7 / 7x1 / 1x3 / 3x1 filters and VALID / SAME padding go
through the same implicit-GEMM kernels (rectangular taps are just a different R x S); the
channel concat of the branches is free -- each branch's last layer writes its BN/ReLU output
directly into its channel window of the module output (strided NHWC view), and in backward
each branch reads its window of the concat gradient in place.
"""
from __future__ import annotations

from typing import List

import torch

from ..nn.layers import ConvBN, GlobalAvgPool, Logits, Pool, empty_act, empty_op
from ..ops import functional as Fn
from .base import CNNModel

BN_KW = dict(eps=1e-3, decay=0.999, scale=False)


class _Node:
    def __init__(self, layer, src):
        self.layer = layer
        self.src = src  # None = module input, else _Node
        self.out = None


class InceptionModule:
    """Columns of ('conv', C, kh, kw[, sh, sw, mode]) / ('mpool'|'apool', kh, kw, sh, sw, mode) /
    ('share',) -- the convnet_builder.inception_module DSL. Column outputs are concatenated."""

    def __init__(self, ps, name, in_shape, cols, conv_kw=None):
        conv_kw = dict(relu=True, **BN_KW) if conv_kw is None else conv_kw
        self.name = name
        self.in_shape = in_shape
        self.nodes: List[_Node] = []
        self.terminals: List[_Node] = []
        prev_col: List[_Node] = []
        for ci, col in enumerate(cols):
            cur: List[_Node] = []
            src = None
            shape = in_shape
            for li, spec in enumerate(col):
                kind = spec[0]
                if kind == "share":
                    node = prev_col[li]
                else:
                    lname = f"{name}/col{ci}/{li}"
                    if kind == "conv":
                        _, c, kh, kw = spec[:4]
                        sh, sw, mode = (spec[4], spec[5], spec[6]) if len(spec) > 4 else (1, 1, "SAME")
                        layer = ConvBN(ps, lname, shape, c, kh, kw, sh, sw, mode, **conv_kw)
                    elif kind in ("mpool", "apool"):
                        _, kh, kw, sh, sw, mode = spec
                        layer = Pool(lname, shape, kh, kw, sh, sw, mode, is_max=(kind == "mpool"))
                    else:
                        raise ValueError(kind)
                    node = _Node(layer, src)
                    self.nodes.append(node)
                cur.append(node)
                src = node
                shape = node.layer.out_shape
            self.terminals.append(cur[-1])
            prev_col = cur
        # consumers of every node's output (a terminal's concat slice counts as one): a conv whose
        # input comes from a single-consumer conv produces that conv's whole dy, so the
        # producer's BN-backward reduction is fused into the consumer's data-grad epilogue
        cons = {}
        for n in self.nodes:
            if n.src is not None:
                cons[id(n.src)] = cons.get(id(n.src), 0) + 1
        for t in self.terminals:
            cons[id(t)] = cons.get(id(t), 0) + 1
        self._fuse_src = {id(n) for n in self.nodes
                          if n.src is not None and cons.get(id(n.src)) == 1
                          and isinstance(n.layer, ConvBN) and isinstance(n.src.layer, ConvBN) and n.src.layer.bn}
        self._fp32_out = any(isinstance(t.layer, ConvBN) and not t.layer.bn for t in self.terminals)
        outs = [t.layer.out_shape for t in self.terminals]
        H, W = outs[0][0], outs[0][1]
        assert all(o[0] == H and o[1] == W for o in outs), f"{name}: branch spatial mismatch {outs}"
        self.offsets = []
        c = 0
        for o in outs:
            self.offsets.append(c)
            c += o[2]
        self.out_shape = (H, W, c)

    def layers(self):
        return [n.layer for n in self.nodes]

    def forward(self, x):
        N = x.shape[0]
        # the concat buffer: bf16, or on the fp32 path the Planes the next module's GEMMs read -- fp32
        # when a branch ends in a conv without BN (GoogLeNet: its conv epilogue writes fp32)
        out = (empty_act if self._fp32_out else empty_op)((N,) + self.out_shape, x.device)
        term_slot = {id(t): (off, t.layer.out_shape[2]) for t, off in zip(self.terminals, self.offsets)}
        heads = [n for n in self.nodes if n.src is None]
        if len(heads) > 1 and Fn.planes_mode() and Fn.native(x) and not Fn.is_planes(x) and not (
                self._fp32_out and any(isinstance(n.layer, Pool) and id(n) in term_slot for n in heads)):
            # fp32 path, an fp32 module input (GoogLeNet: the previous concat is fp32) read by several
            # branch heads: split it into the GEMM planes once instead of once per branch
            x = Fn.to_planes(x)
        for n in self.nodes:
            inp = x if n.src is None else n.src.out
            slot = term_slot.get(id(n))
            view = out[..., slot[0]:slot[0] + slot[1]] if slot is not None else None
            n.out = n.layer.forward(inp, out=view)
        self._x = x
        return out

    def backward(self, dy):
        grads = {}
        for t, off in zip(self.terminals, self.offsets):
            c = t.layer.out_shape[2]
            grads[id(t)] = (dy[..., off:off + c], False)  # (grad, owned)
        dx = None
        for n in reversed(self.nodes):
            g = grads.pop(id(n), None)
            if g is None:
                continue
            g = g[0]
            if n.src is None:
                if isinstance(n.layer, ConvBN):
                    dx, _ = n.layer.backward(g, dx=dx, accumulate=dx is not None)
                else:
                    dx = n.layer.backward(g, dx=dx, accumulate=dx is not None)
            elif id(n) in self._fuse_src:
                r, _ = n.layer.backward(g, dx_bn=n.src.layer)
                grads[id(n.src)] = (r, True)
            else:
                prev = grads.get(id(n.src))
                tgt = prev[0] if prev is not None else None
                if isinstance(n.layer, ConvBN):
                    r, _ = n.layer.backward(g, dx=tgt, accumulate=tgt is not None)
                else:
                    r = n.layer.backward(g, dx=tgt, accumulate=tgt is not None)
                grads[id(n.src)] = (r, True)
            n.out = None
        self._x = None
        return dx


class InceptionV3(CNNModel):
    name = "inception3"
    # --compute_dtype fp32 on the HIP kernels: bf16x6 plane GEMMs for every filter shape (1x1, 3x3,
    # 5x5, 1x7 / 7x1, 1x3 / 3x1; SAME and VALID), max / average pools on planes, concat windows of
    # a Planes buffer (each branch's BN writes its channel window)
    F32_NATIVE_OK = True
    default_image_size = 299
    default_batch_size = 32

    def build(self):
        ps = self.ps
        S = self.image_size
        c = lambda name, shape, co, kh, kw, sh=1, sw=1, mode="SAME", **extra: ConvBN(
            ps, name, shape, co, kh, kw, sh, sw, mode, relu=True, **BN_KW, **extra)
        stem = []
        stem.append(c("conv0", (S, S, self.image_channels), 32, 3, 3, 2, 2, "VALID", need_dx=False, logical_cin=3))
        stem.append(c("conv1", stem[-1].out_shape, 32, 3, 3, 1, 1, "VALID"))
        stem.append(c("conv2", stem[-1].out_shape, 64, 3, 3, 1, 1, "SAME"))
        stem.append(Pool("mpool0", stem[-1].out_shape, 3, 3, 2, 2, "VALID", is_max=True))
        stem.append(c("conv3", stem[-1].out_shape, 80, 1, 1, 1, 1, "VALID"))
        stem.append(c("conv4", stem[-1].out_shape, 192, 3, 3, 1, 1, "VALID"))
        stem.append(Pool("mpool1", stem[-1].out_shape, 3, 3, 2, 2, "VALID", is_max=True))
        self.stem = stem
        shape = stem[-1].out_shape
        mods = []

        def A(n):
            return [[("conv", 64, 1, 1)], [("conv", 48, 1, 1), ("conv", 64, 5, 5)],
                    [("conv", 64, 1, 1), ("conv", 96, 3, 3), ("conv", 96, 3, 3)],
                    [("apool", 3, 3, 1, 1, "SAME"), ("conv", n, 1, 1)]]

        B = [[("conv", 384, 3, 3, 2, 2, "VALID")],
             [("conv", 64, 1, 1), ("conv", 96, 3, 3), ("conv", 96, 3, 3, 2, 2, "VALID")],
             [("mpool", 3, 3, 2, 2, "VALID")]]

        def C(n):
            return [[("conv", 192, 1, 1)],
                    [("conv", n, 1, 1), ("conv", n, 1, 7), ("conv", 192, 7, 1)],
                    [("conv", n, 1, 1), ("conv", n, 7, 1), ("conv", n, 1, 7), ("conv", n, 7, 1), ("conv", 192, 1, 7)],
                    [("apool", 3, 3, 1, 1, "SAME"), ("conv", 192, 1, 1)]]

        D = [[("conv", 192, 1, 1), ("conv", 320, 3, 3, 2, 2, "VALID")],
             [("conv", 192, 1, 1), ("conv", 192, 1, 7), ("conv", 192, 7, 1), ("conv", 192, 3, 3, 2, 2, "VALID")],
             [("mpool", 3, 3, 2, 2, "VALID")]]

        def E(pool):
            return [[("conv", 320, 1, 1)], [("conv", 384, 1, 1), ("conv", 384, 1, 3)],
                    [("share",), ("conv", 384, 3, 1)],
                    [("conv", 448, 1, 1), ("conv", 384, 3, 3), ("conv", 384, 1, 3)],
                    [("share",), ("share",), ("conv", 384, 3, 1)],
                    [(pool, 3, 3, 1, 1, "SAME"), ("conv", 192, 1, 1)]]

        plan = [("incept_v3_a0", A(32)), ("incept_v3_a1", A(64)), ("incept_v3_a2", A(64)), ("incept_v3_b", B),
                ("incept_v3_c0", C(128)), ("incept_v3_c1", C(160)), ("incept_v3_c2", C(160)),
                ("incept_v3_c3", C(192)), ("incept_v3_d", D), ("incept_v3_e0", E("apool")),
                ("incept_v3_e1", E("mpool"))]
        for name, cols in plan:
            m = InceptionModule(ps, name, shape, cols)
            mods.append(m)
            shape = m.out_shape
        self.modules = mods
        self.gap = GlobalAvgPool("apool_final", shape)
        self.fc = Logits(ps, "logits", shape[2], self.num_classes)
        self.layers = list(stem) + [l for m in mods for l in m.layers()] + [self.gap, self.fc]

    def forward(self, images):
        x = images
        for l in self.stem:
            x = l.forward(x)
        for m in self.modules:
            x = m.forward(x)
        return self.fc.forward(self.gap.forward(x))

    def backward_segments(self, dlogits):
        """Segments of whole inception modules (last first; the 8x8 'E' modules and the
        logits hold most of the parameters), then the stem."""
        dx = self.gap.backward(self.fc.backward(dlogits))
        units = [(m.backward, m.layers()) for m in reversed(self.modules)]
        for i in range(len(self.stem) - 1, -1, -1):
            l, below = self.stem[i], self._stem_bn_below(i)
            if isinstance(l, ConvBN):
                units.append((lambda d, l=l, b=below: l.backward(d, dx_bn=b)[0], [l]))
            else:
                units.append((l.backward, [l]))
        yield from self._segments_from_units(dx, [self.fc, self.gap], units)

    def backward(self, dlogits):
        dx = self.gap.backward(self.fc.backward(dlogits))
        for m in reversed(self.modules):
            dx = m.backward(dx)
        for i in range(len(self.stem) - 1, -1, -1):
            l = self.stem[i]
            if isinstance(l, ConvBN):
                dx, _ = l.backward(dx, dx_bn=self._stem_bn_below(i))
            else:
                dx = l.backward(dx)

    def _stem_bn_below(self, i):
        """The conv+BN feeding stem layer i directly (its BN-backward reduction is fused into
        layer i's data-grad epilogue), else None."""
        l = self.stem[i]
        if i > 0 and isinstance(l, ConvBN) and l.need_dx and isinstance(self.stem[i - 1], ConvBN) \
                and self.stem[i - 1].bn:
            return self.stem[i - 1]
        return None
