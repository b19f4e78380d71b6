"""Inception-v3 (tf_cnn_benchmarks inception3): structure + hand-written backward vs autograd."""
import torch

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch
from reference_models import inception_ref, reference_grads


def test_inception3_shapes_and_params():
    m = create_model("inception3", device="cpu")
    assert m.image_size == 299
    shapes = [mod.out_shape for mod in m.modules]
    assert shapes[0] == (35, 35, 256) and shapes[2] == (35, 35, 288) and shapes[3] == (17, 17, 768)
    assert shapes[8] == (8, 8, 1280) and shapes[-1] == (8, 8, 2048)
    # conv weights + BN betas (scale=False) + affine 2048x1001+1001
    n = m.num_params()
    assert 23_000_000 < n < 24_500_000, n
    assert abs(m.flops_per_image() / 1e9 - 11.4) < 1.0  # ~5.7 GMAC forward


def test_inception3_grads_match_autograd(monkeypatch):
    monkeypatch.setenv("HCB_CPU_DTYPE", "float64")
    m = create_model("inception3", image_size=107, device="cpu")
    img, lab = synthetic_batch(m, 2)
    img = ((img - 127.0) / 60.0).double()
    loss_ref, grads_ref, _ = reference_grads(m, img, lab, inception_ref)
    t = Trainer(m, 2, constant_lr(0.0), weight_decay=0.0)
    t._forward_backward(img, lab)
    assert torch.allclose(t.row_loss.mean().double(), loss_ref, rtol=1e-6)
    for p in m.ps.params:
        r = grads_ref[p.name]
        err = (p.grad.double() - r).abs().max().item()
        assert err <= 1e-4 * (r.abs().max().item() + 1e-6) + 1e-7, p.name
