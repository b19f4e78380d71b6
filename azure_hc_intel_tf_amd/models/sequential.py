"""The plain feed-forward models of the tf_cnn_benchmarks zoo (``--model=vgg16`` etc.; SURVEY.md
§2.2 "models/model_config.py ... (+ alexnet/vgg/googlenet/...)"): VGG-11/16/19, AlexNet,
OverFeat, LeNet and GoogLeNet (Inception-v1), built from the same layer DSL as ResNet.

Layer semantics follow tf_cnn_benchmarks' convnet_builder defaults for these models: conv =
conv + bias + ReLU without batch norm ('SAME' unless given; Glorot-uniform kernels, zero
biases), mpool / apool 'VALID', affine =
fully connected + bias + ReLU, dropout keep_prob 0.5 after the hidden affine layers, then the
1001-way logits. On the MI355X every conv / affine layer is the implicit-GEMM HIP kernel with
the bias + ReLU epilogue (an affine layer is a 1x1 conv over a [B, 1, 1, F] activation), the
channel concat of the GoogLeNet modules is the strided-window write of the Inception-v3
modules, and dropout is a counter-hash kernel whose step lives on the device (fresh masks on
every replay of the captured graph).
"""
from __future__ import annotations

from typing import List, Tuple

from ..nn.layers import ConvBN, Dropout, GlobalAvgPool, Layer, Logits, Pool
from .base import CNNModel
from .inception import InceptionModule


class Flatten(Layer):
    """[B, H, W, C] -> [B, 1, 1, H*W*C] (a view; NHWC order)."""

    def __init__(self, name, in_shape):
        self.name = name
        self.in_shape = in_shape
        H, W, C = in_shape
        self.out_shape = (1, 1, H * W * C)

    def forward(self, x):
        return x.reshape(x.shape[0], 1, 1, -1)

    def backward(self, dy):
        return dy.reshape((dy.shape[0],) + tuple(self.in_shape))


def inception_v1_cols(k, l, m, n, p, q):
    """convnet_builder.inception_module columns of GoogLeNet's inception_v1(k, l, m, n, p, q)."""
    return [[("conv", k, 1, 1)], [("conv", l, 1, 1), ("conv", m, 3, 3)],
            [("conv", n, 1, 1), ("conv", p, 5, 5)], [("mpool", 3, 3, 1, 1, "SAME"), ("conv", q, 1, 1)]]


class SequentialCNN(CNNModel):
    """A model given as a list of layer specs:
    ('conv', C, kh, kw[, sh, sw, mode]) | ('mpool'|'apool', kh, kw, sh, sw[, mode]) |
    ('inception', cols) | ('gap',) | ('flatten',) | ('affine', N) | ('dropout',)."""

    specs: List[Tuple] = []
    # --compute_dtype fp32 on the HIP kernels: bf16x6 plane GEMMs with the bias + ReLU epilogue (fp32
    # output; each fp32 activation / gradient split into planes once per consuming GEMM pair), fp32
    # pools, dropout, ReLU backward and bias column sums
    F32_NATIVE_OK = True
    dropout_keep = 0.5
    default_batch_size = 32
    default_lr = 0.005

    def build(self):
        ps = self.ps
        shape = (self.image_size, self.image_size, self.image_channels)
        self.seq = []
        first = True
        for i, op in enumerate(self.specs):
            kind = op[0]
            name = f"v{i}_{kind}"
            if kind == "conv":
                c, kh, kw = op[1:4]
                sh, sw, mode = (op[4], op[5], op[6]) if len(op) > 4 else (1, 1, "SAME")
                layer = ConvBN(ps, name, shape, c, kh, kw, sh, sw, mode, relu=True, bn=False, need_dx=not first,
                               logical_cin=3 if first else None, init="glorot")
                first = False
            elif kind in ("mpool", "apool"):
                kh, kw, sh, sw = op[1:5]
                mode = op[5] if len(op) > 5 else "VALID"
                layer = Pool(name, shape, kh, kw, sh, sw, mode, is_max=(kind == "mpool"))
            elif kind == "inception":
                layer = InceptionModule(ps, name, shape, op[1], conv_kw=dict(relu=True, bn=False, init="glorot"))
            elif kind == "gap":
                layer = GlobalAvgPool(name, shape)
            elif kind == "flatten":
                layer = Flatten(name, shape)
            elif kind == "affine":
                assert shape[0] == 1 and shape[1] == 1, f"{name}: affine needs a flattened input"
                layer = ConvBN(ps, name, shape, op[1], 1, 1, relu=True, bn=False, init="glorot")
            elif kind == "dropout":
                layer = Dropout(name, shape, self.dropout_keep, seed=len(self.seq))
            else:
                raise ValueError(kind)
            self.seq.append(layer)
            shape = layer.out_shape
        self.feat_dim = shape[2]
        self.fc = Logits(ps, "logits", self.feat_dim, self.num_classes)
        self.layers = list(self.seq) + [self.fc]

    def all_layers(self):
        out = []
        for l in self.seq:
            out += l.layers() if isinstance(l, InceptionModule) else [l]
        return out + [self.fc]

    def forward(self, images):
        x = images
        for l in self.seq:
            x = l.forward(x)
        self._last_shape = tuple(x.shape)
        return self.fc.forward(x.reshape(x.shape[0], -1))

    def backward_segments(self, dlogits):
        dx = self.fc.backward(dlogits).reshape(self._last_shape)
        units, rest = [], list(reversed(self.seq))
        while rest:
            l = rest.pop(0)
            if isinstance(l, ConvBN):
                units.append((lambda d, l=l: l.backward(d)[0], [l]))
                if not l.need_dx:
                    break  # the input conv: nothing below it needs a gradient
            else:
                units.append((l.backward, l.layers() if isinstance(l, InceptionModule) else [l]))
        yield from self._segments_from_units(dx, [self.fc], units, tail=rest)

    def backward(self, dlogits):
        dx = self.fc.backward(dlogits).reshape(self._last_shape)
        for l in reversed(self.seq):
            if isinstance(l, ConvBN):
                dx, _ = l.backward(dx)
                if not l.need_dx:
                    break
            else:
                dx = l.backward(dx)



def _vgg_specs(counts):
    out = []
    for n, c in zip(counts, (64, 128, 256, 512, 512)):
        out += [("conv", c, 3, 3)] * n + [("mpool", 2, 2, 2, 2)]
    return out + [("flatten",), ("affine", 4096), ("dropout",), ("affine", 4096), ("dropout",)]


class VGG(SequentialCNN):
    default_image_size = 224

    def __init__(self, depth: int = 16, **kw):
        self.name = f"vgg{depth}"
        self.specs = _vgg_specs({11: (1, 1, 2, 2, 2), 16: (2, 2, 3, 3, 3), 19: (2, 2, 4, 4, 4)}[depth])
        super().__init__(**kw)


class AlexNet(SequentialCNN):
    name = "alexnet"
    default_image_size = 224 + 3
    default_batch_size = 512
    specs = [("conv", 64, 11, 11, 4, 4, "VALID"), ("mpool", 3, 3, 2, 2), ("conv", 192, 5, 5), ("mpool", 3, 3, 2, 2),
             ("conv", 384, 3, 3), ("conv", 384, 3, 3), ("conv", 256, 3, 3), ("mpool", 3, 3, 2, 2), ("flatten",),
             ("affine", 4096), ("dropout",), ("affine", 4096), ("dropout",)]


class OverFeat(SequentialCNN):
    name = "overfeat"
    default_image_size = 231
    specs = [("conv", 96, 11, 11, 4, 4, "VALID"), ("mpool", 2, 2, 2, 2), ("conv", 256, 5, 5, 1, 1, "VALID"),
             ("mpool", 2, 2, 2, 2), ("conv", 512, 3, 3), ("conv", 1024, 3, 3), ("conv", 1024, 3, 3),
             ("mpool", 2, 2, 2, 2), ("flatten",), ("affine", 3072), ("dropout",), ("affine", 4096), ("dropout",)]


class LeNet(SequentialCNN):
    name = "lenet"
    default_image_size = 28
    specs = [("conv", 32, 5, 5), ("mpool", 2, 2, 2, 2), ("conv", 64, 5, 5), ("mpool", 2, 2, 2, 2), ("flatten",),
             ("affine", 512)]


class GoogLeNet(SequentialCNN):
    name = "googlenet"
    default_image_size = 224
    specs = [("conv", 64, 7, 7, 2, 2, "SAME"), ("mpool", 3, 3, 2, 2, "SAME"), ("conv", 64, 1, 1), ("conv", 192, 3, 3),
             ("mpool", 3, 3, 2, 2, "SAME"),
             ("inception", inception_v1_cols(64, 96, 128, 16, 32, 32)),
             ("inception", inception_v1_cols(128, 128, 192, 32, 96, 64)), ("mpool", 3, 3, 2, 2, "SAME"),
             ("inception", inception_v1_cols(192, 96, 208, 16, 48, 64)),
             ("inception", inception_v1_cols(160, 112, 224, 24, 64, 64)),
             ("inception", inception_v1_cols(128, 128, 256, 24, 64, 64)),
             ("inception", inception_v1_cols(112, 144, 288, 32, 64, 64)),
             ("inception", inception_v1_cols(256, 160, 320, 32, 128, 128)), ("mpool", 3, 3, 2, 2, "SAME"),
             ("inception", inception_v1_cols(256, 160, 320, 32, 128, 128)),
             ("inception", inception_v1_cols(384, 192, 384, 48, 128, 128)), ("gap",)]
