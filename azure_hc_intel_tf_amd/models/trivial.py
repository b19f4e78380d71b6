"""tf_cnn_benchmarks ``--model=trivial`` (the tool's default model): flatten the 227x227x3 image,
affine(1) + ReLU, affine(4096) + ReLU, affine -> 1001 classes. Used to measure pipeline and
framework overhead rather than compute. On the GPU the 1-unit layer is stored 8 wide (the
7 extra units have zero weights/bias, so they stay exactly zero and receive zero gradient);
the image's 3 channels are padded to 8 the same way as for the CNNs."""
from __future__ import annotations

from ..nn.layers import ConvBN, Logits
from ..nn.params import ParamStore
from .base import CNNModel


class Trivial(CNNModel):
    name = "trivial"
    default_image_size = 227
    default_batch_size = 32
    F32_NATIVE_OK = True  # the affine layers are 1x1 plane GEMMs with the bias + ReLU epilogue

    def build(self):
        ps = self.ps
        S = self.image_size
        feat = S * S * self.image_channels
        self.a1 = ConvBN(ps, "affine0", (1, 1, feat), 8, 1, 1, relu=True, bn=False, logical_cin=S * S * 3)
        self._zero_units(self.a1, 1)
        self.a2 = ConvBN(ps, "affine1", (1, 1, 8), 4096, 1, 1, relu=True, bn=False, logical_cin=1)
        self.fc = Logits(ps, "logits", 4096, self.num_classes)
        self.a1.w.logical_numel = S * S * 3
        self.layers = [self.a1, self.a2, self.fc]

    @staticmethod
    def _zero_units(layer, keep):
        init = layer.w.init

        def f(t, init=init):
            init(t)
            t[keep:] = 0

        layer.w.init = f
        layer.bias.logical_numel = keep

    def forward(self, images):
        B = images.shape[0]
        x = images.reshape(B, 1, 1, -1)
        h = self.a1.forward(x)
        h = self.a2.forward(h)
        return self.fc.forward(h.view(B, -1))

    def backward(self, dlogits):
        B = dlogits.shape[0]
        dh = self.fc.backward(dlogits).view(B, 1, 1, -1)
        dh, _ = self.a2.backward(dh)
        self.a1.need_dx = False
        self.a1.backward(dh)
