"""The ResNet stem's BN backward fed straight from the max-pool gradient (nn/layers.py
ConvBN.backward_from_maxpool, bn.hip pool_gather: the full-size dy is gathered through the pool's
argmax instead of being written by the max-pool backward kernel and read back) is bitwise equal to
the unfused max-pool backward + BN backward, in bf16 and at fp32 (planes), in deterministic mode."""
import pytest
import torch

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.nn import layers as L
from azure_hc_intel_tf_amd.ops import functional as Fn
from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch

pytestmark = pytest.mark.gpu


def _grads(dtype, fused):
    keep = L.FUSE_STEM_POOL_BWD
    L.FUSE_STEM_POOL_BWD = fused
    try:
        m = create_model("resnet50", image_size=64, device="cuda", compute_dtype=dtype, seed=11)
        img, lab = synthetic_batch(m, 4, seed=2)
        t = Trainer(m, 4, constant_lr(0.0), use_graph=False)
        t.step(img, lab)
        torch.cuda.synchronize()
        return m.ps.grad.clone(), {p.name: p.grad.clone() for p in m.ps.params if p.name.startswith("conv0")}
    finally:
        L.FUSE_STEM_POOL_BWD = keep


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_stem_bn_backward_from_pool_gradient_matches_unfused(dtype):
    Fn.set_deterministic(True)
    try:
        ga, sa = _grads(dtype, True)
        gb, sb = _grads(dtype, False)
    finally:
        Fn.set_deterministic(False)
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k
    assert torch.equal(ga, gb)
    assert float(sa["conv0/batchnorm/gamma"].abs().sum()) > 0
