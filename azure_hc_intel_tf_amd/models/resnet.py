"""ResNet v1 / v1.5 (50 / 101 / 152) as trained by tf_cnn_benchmarks ``--model=resnet50``
(the reference's hard-coded model, /root/reference/benchmark-scripts/
run-tf-sing-ucx-openmpi.sh:34,66).

Architecture (tf_cnn_benchmarks resnet_model semantics):
  conv 7x7/2 'SAME_RESNET' (64) + BN + ReLU -> max-pool 3x3/2 'SAME'
  -> bottleneck stages [3,4,6,3] (50) / [3,4,23,3] (101) / [3,8,36,3] (152),
     depths 256/512/1024/2048, bottleneck widths 64/128/256/512,
     v1: stride on the first 1x1 of the first block of stages 2-4,
     v1.5: stride on the 3x3 instead; projection shortcut (1x1 conv + BN) when the
     channel count changes; v2 (``ResNetV2``): pre-activation blocks
  -> spatial mean -> affine 2048 -> 1001 classes (ImageNet + background).
BN: decay 0.9, epsilon 1e-5, scale=True. ResNet-50 v1: 25,559,081 trainable params.
"""
from __future__ import annotations

from ..nn import layers as L
from ..nn.layers import BNReLU, ConvBN, GlobalAvgPool, Logits, Pool, StemS2D
from ..ops import functional as Fn
from .base import CNNModel

LAYER_COUNTS = {18: None, 50: (3, 4, 6, 3), 101: (3, 4, 23, 3), 152: (3, 8, 36, 3)}


class Bottleneck:
    def __init__(self, ps, name, in_shape, depth, bottleneck, stride, v15: bool):
        H, W, C = in_shape
        self.proj = C != depth
        s1, s2 = (1, stride) if v15 else (stride, 1)
        if self.proj:
            self.sc = ConvBN(ps, f"{name}/shortcut", in_shape, depth, 1, 1, stride, stride, "SAME", relu=False)
        else:
            assert stride == 1, "identity shortcut with stride is not used by these ResNets"
            self.sc = None
        self.c1 = ConvBN(ps, f"{name}/conv1", in_shape, bottleneck, 1, 1, s1, s1, "SAME")
        self.c2 = ConvBN(ps, f"{name}/conv2", self.c1.out_shape, bottleneck, 3, 3, s2, s2, "SAME_RESNET")
        self.c3 = ConvBN(ps, f"{name}/conv3", self.c2.out_shape, depth, 1, 1, 1, 1, "SAME", relu=True)
        self.in_shape = in_shape
        self.out_shape = self.c3.out_shape

    def layers(self):
        return [l for l in (self.sc, self.c1, self.c2, self.c3) if l is not None]

    def forward(self, x):
        if self.proj and L.FUSE_RES_BN and self.sc.training and Fn.native(x):
            # the shortcut's BN is applied inside conv3's BN pass (its output never stored)
            z_sc = self.sc.forward_deferred(x)
            a = self.c1.forward(x)
            b = self.c2.forward(a)
            return self.c3.forward(b, residual=z_sc, residual_bn=self.sc)
        sc = self.sc.forward(x) if self.proj else x
        a = self.c1.forward(x)
        b = self.c2.forward(a)
        return self.c3.forward(b, residual=sc)

    def backward(self, dy, prev_bn=None):
        """``prev_bn``: the ConvBN producing this block's input (the previous block's conv3), whose
        BN backward is fused into the last data-grad GEMM that completes dx."""
        db, gres = self.c3.backward(dy, want_gres=True, dx_bn=self.c2)
        da, _ = self.c2.backward(db, dx_bn=self.c1)
        if self.proj:
            # shortcut first: the fused GEMM must be the one that visits every dx pixel (v1.5's
            # strided 1x1 shortcut only writes the strided ones; v1's two strided 1x1s cover the
            # same pixels and leave the rest zero)
            dx, _ = self.sc.backward(gres)
            self.c1.backward(da, dx=dx, accumulate=True, dx_bn=prev_bn)
        else:
            # identity shortcut: dx = gres + dgrad(c1), accumulated in place by the GEMM epilogue
            dx, _ = self.c1.backward(da, dx=gres, accumulate=True, dx_bn=prev_bn)
        return dx


class ResNet(CNNModel):
    default_image_size = 224
    F32_NATIVE_OK = True  # --compute_dtype fp32 on the HIP kernels (bf16x6 GEMMs, fp32 BN / pool)
    # gradient-reduction granularity of the overlapped multi-GPU step (backward_segments):
    # "stage" (default) or "block" (per block in stages 3-4, stage 1 split from the stem)
    segments = "stage"

    def __init__(self, depth: int = 50, version: str = "v1", **kw):
        self.depth = depth
        self.version = version
        self.name = f"resnet{depth}" + ("_v1.5" if version == "v1.5" else "")
        super().__init__(**kw)

    def build(self):
        ps = self.ps
        S = self.image_size
        v15 = self.version == "v1.5"
        if self.native and L.STEM_S2D:  # fp32: the fold runs on the image's bf16 planes
            self.stem = StemS2D(ps, "conv0", (S, S, self.image_channels), 64, relu=True, need_dx=False,
                                logical_cin=3)
        else:
            self.stem = ConvBN(ps, "conv0", (S, S, self.image_channels), 64, 7, 7, 2, 2, "SAME_RESNET",
                               relu=True, need_dx=False, logical_cin=3)
        self.pool = Pool("mpool0", self.stem.out_shape, 3, 3, 2, 2, "SAME", is_max=True)
        shape = self.pool.out_shape
        self.blocks = []
        counts = LAYER_COUNTS[self.depth]
        for si, (n, depth, bott) in enumerate(zip(counts, (256, 512, 1024, 2048), (64, 128, 256, 512))):
            for bi in range(n):
                stride = 2 if (si > 0 and bi == 0) else 1
                blk = Bottleneck(ps, f"stage{si + 1}/block{bi + 1}", shape, depth, bott, stride, v15)
                blk.stage = si
                self.blocks.append(blk)
                shape = blk.out_shape
        self.gap = GlobalAvgPool("spatial_mean", shape)
        self.fc = Logits(ps, "logits", shape[2], self.num_classes)
        self.layers = [self.stem, self.pool] + [l for b in self.blocks for l in b.layers()] + [self.gap, self.fc]

    def _stem_pool(self, images):
        if Fn.native(images) and L.FUSE_STEM_POOL and self.stem.training:
            return self.stem.forward_maxpool(images, self.pool)
        return self.pool.forward(self.stem.forward(images))

    def forward(self, images):
        x = self._stem_pool(images)
        for b in self.blocks:
            x = b.forward(x)
        self._last = x
        feat = self.gap.forward(x)
        return self.fc.forward(feat)

    def backward(self, dlogits):
        for _ in self.backward_segments(dlogits):
            pass

    def backward_segments(self, dlogits):
        """One segment per stage, last stage first (its ~60 % of the parameters are reduced
        while stages 3..1 are still in backward). segments == "block": every block of stages
        3-4 is its own segment (ResNet-50: stage 4's 15 M parameters go out in three ~20 MB
        pieces, the first while blocks 2..1 still run), and stage 1 is cut from the stem so
        only the stem's 9.4 k parameters are reduced after the last backward kernel."""
        fine = self.segments == "block"
        dfeat = self.fc.backward(dlogits)
        dx = self.gap.backward(dfeat)
        seg = [self.fc, self.gap]
        for i in range(len(self.blocks) - 1, -1, -1):
            dx = self.blocks[i].backward(dx, self.blocks[i - 1].c3 if i > 0 else None)
            seg += self.blocks[i].layers()
            cut = i > 0 and self.blocks[i].stage != self.blocks[i - 1].stage
            if fine and (self.blocks[i].stage >= 2 or i == 0):
                cut = True
            if cut:
                yield seg, False
                seg = []
        if L.fuse_stem_pool_bwd() and getattr(self.stem, "_pool_fused", None) is self.pool and Fn.native(dx):
            self.stem.backward_from_maxpool(dx, self.pool)  # no max-pool backward kernel
        else:
            dx = self.pool.backward(dx)
            self.stem.backward(dx)
        self._last = None
        yield seg + [self.pool, self.stem], True


class PreActBottleneck:
    """tf_cnn_benchmarks ``bottleneck_block_v2`` (pre-activation ResNet): preact = relu(BN(x));
    shortcut = x (identity) or a bias-free 1x1 projection of preact; 1x1 (stride) conv+BN+ReLU
    -> 3x3 conv+BN+ReLU -> bias-free 1x1 conv whose GEMM epilogue adds the shortcut.

    Backward as the v1 block: conv2's / conv1's BN-backward reductions run in the epilogues of the
    data-grad GEMMs of conv3 / conv2 (``dx_bn``); the projection's data gradient and conv1's are
    summed by beta-accumulate; the identity shortcut's gradient is added inside the pre-activation
    BN's backward apply."""

    def __init__(self, ps, name, in_shape, depth, bottleneck, stride):
        H, W, C = in_shape
        self.pre = BNReLU(ps, f"{name}/preact", in_shape)
        self.proj = C != depth
        if self.proj:
            self.sc = ConvBN(ps, f"{name}/shortcut", in_shape, depth, 1, 1, stride, stride, "SAME", relu=False,
                             bn=False, bias=False)
        else:
            assert stride == 1, "identity shortcut with stride is not used by these ResNets"
            self.sc = None
        self.c1 = ConvBN(ps, f"{name}/conv1", in_shape, bottleneck, 1, 1, stride, stride, "SAME")
        self.c2 = ConvBN(ps, f"{name}/conv2", self.c1.out_shape, bottleneck, 3, 3, 1, 1, "SAME_RESNET")
        self.c3 = ConvBN(ps, f"{name}/conv3", self.c2.out_shape, depth, 1, 1, 1, 1, "SAME", relu=False, bn=False,
                         bias=False)
        self.in_shape = in_shape
        self.out_shape = self.c3.out_shape

    def layers(self):
        return [l for l in (self.pre, self.sc, self.c1, self.c2, self.c3) if l is not None]

    def forward(self, x):
        a = self.pre.forward(x)
        sc = self.sc.forward(a) if self.proj else x
        h = self.c2.forward(self.c1.forward(a))
        return self.c3.forward(h, residual=sc)

    def backward(self, dy):
        d2, gres = self.c3.backward(dy, want_gres=True, dx_bn=self.c2)  # gres = dy: the shortcut's gradient
        d1, _ = self.c2.backward(d2, dx_bn=self.c1)
        if self.proj:
            da, _ = self.sc.backward(gres)
            self.c1.backward(d1, dx=da, accumulate=True)
            return self.pre.backward(da)
        da, _ = self.c1.backward(d1)
        return self.pre.backward(da, add=gres)  # identity shortcut: d(x) = BN'(da) + dy, one pass


class ResNetV2(CNNModel):
    """ResNet v2 (``--model=resnet50_v2`` / 101 / 152): stem conv+BN+ReLU, max pool, the
    pre-activation bottleneck stages (stride on the first 1x1, as tf_cnn_benchmarks), a final
    BN + ReLU, spatial mean, affine. fp32 (``--compute_dtype fp32``) runs on the HIP kernels like
    v1: plane GEMMs, the S2D stem, acc-replica BN passes."""

    default_image_size = 224
    F32_NATIVE_OK = True

    def __init__(self, depth: int = 50, **kw):
        self.depth = depth
        self.name = f"resnet{depth}_v2"
        super().__init__(**kw)

    def build(self):
        ps = self.ps
        S = self.image_size
        if self.native and L.STEM_S2D:
            self.stem = StemS2D(ps, "conv0", (S, S, self.image_channels), 64, relu=True, need_dx=False,
                                logical_cin=3)
        else:
            self.stem = ConvBN(ps, "conv0", (S, S, self.image_channels), 64, 7, 7, 2, 2, "SAME_RESNET", relu=True,
                               need_dx=False, logical_cin=3)
        self.pool = Pool("mpool0", self.stem.out_shape, 3, 3, 2, 2, "SAME", is_max=True)
        shape = self.pool.out_shape
        self.blocks = []
        for si, (n, depth, bott) in enumerate(zip(LAYER_COUNTS[self.depth], (256, 512, 1024, 2048),
                                                  (64, 128, 256, 512))):
            for bi in range(n):
                stride = 2 if (si > 0 and bi == 0) else 1
                blk = PreActBottleneck(ps, f"stage{si + 1}/block{bi + 1}", shape, depth, bott, stride)
                self.blocks.append(blk)
                shape = blk.out_shape
        self.post = BNReLU(ps, "postnorm", shape)
        self.gap = GlobalAvgPool("spatial_mean", shape)
        self.fc = Logits(ps, "logits", shape[2], self.num_classes)
        self.layers = ([self.stem, self.pool] + [l for b in self.blocks for l in b.layers()]
                       + [self.post, self.gap, self.fc])

    def _stem_pool(self, images):
        if Fn.native(images) and L.FUSE_STEM_POOL and self.stem.training:
            # the pooled map feeds a BN (the first pre-activation), not a GEMM: fp32, not planes
            return self.stem.forward_maxpool(images, self.pool, out_planes=False)
        return self.pool.forward(self.stem.forward(images))

    def forward(self, images):
        x = self._stem_pool(images)
        for b in self.blocks:
            x = b.forward(x)
        return self.fc.forward(self.gap.forward(self.post.forward(x)))

    def _stem_backward(self, dx):
        if L.fuse_stem_pool_bwd() and getattr(self.stem, "_pool_fused", None) is self.pool and Fn.native(dx):
            self.stem.backward_from_maxpool(dx, self.pool)  # no max-pool backward kernel
        else:
            self.stem.backward(self.pool.backward(dx))
        return None

    def backward_segments(self, dlogits):
        dx = self.post.backward(self.gap.backward(self.fc.backward(dlogits)))
        units = [(b.backward, b.layers()) for b in reversed(self.blocks)]
        units.append((self._stem_backward, [self.pool, self.stem]))
        yield from self._segments_from_units(dx, [self.fc, self.gap, self.post], units)

    def backward(self, dlogits):
        for _ in self.backward_segments(dlogits):
            pass
