"""Hand-written ResNet forward/backward (CPU path) vs a PyTorch autograd reference."""
import pytest
import torch

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch
from reference_models import reference_grads, resnet_ref


@pytest.mark.parametrize("name", ["resnet50", "resnet50_v1.5"])
def test_resnet_grads_match_autograd(name, monkeypatch):
    monkeypatch.setenv("HCB_CPU_DTYPE", "float64")
    torch.manual_seed(0)
    m = create_model(name, image_size=64, device="cpu")
    img, lab = synthetic_batch(m, 4)
    img = ((img - 127.0) / 60.0).double()
    loss_ref, grads_ref, logits_ref = reference_grads(m, img, lab, resnet_ref)
    t = Trainer(m, 4, constant_lr(0.0), weight_decay=0.0)
    t._forward_backward(img, lab)
    assert torch.allclose(t.row_loss.mean().double(), loss_ref, rtol=1e-5, atol=1e-6)
    for p in m.ps.params:
        g = p.grad
        r = grads_ref[p.name]
        err = (g - r).abs().max().item()
        scale = r.abs().max().item() + 1e-6
        assert err <= 1e-4 * scale + 1e-6, f"{p.name}: max err {err} vs scale {scale}"


def test_resnet50_param_count():
    m = create_model("resnet50", device="cpu")
    assert m.num_params() == 25_559_081
    assert m.ps.num_tensors() == 161


def test_resnet152_param_count():
    m = create_model("resnet152", image_size=64, device="cpu")
    assert m.num_params() == 60_194_857


def test_training_reduces_loss():
    m = create_model("resnet50", image_size=64, device="cpu")
    img, lab = synthetic_batch(m, 8)
    img = (img - 127.0) / 60.0
    t = Trainer(m, 8, constant_lr(0.01), weight_decay=4e-5)
    first = float(t.step(img, lab))
    for _ in range(6):
        last = float(t.step(img, lab))
    assert last < first
