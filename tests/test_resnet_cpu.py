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


def _bnrelu_ref(layer, x, params, relu=True):
    z = torch.nn.functional.batch_norm(x, None, None, params[layer.gamma.name], params[layer.beta.name],
                                       training=True, eps=layer.eps)
    return torch.relu(z) if relu else z


def resnet_v2_ref(model, images_nhwc, params):
    from reference_models import conv_ref, convbn_ref, pool_ref

    x = images_nhwc.permute(0, 3, 1, 2)
    x = pool_ref(model.pool, convbn_ref(model.stem, x, params))
    for b in model.blocks:
        a = _bnrelu_ref(b.pre, x, params)
        sc = conv_ref(b.sc, a, params) if b.proj else x
        h = convbn_ref(b.c2, convbn_ref(b.c1, a, params), params)
        x = conv_ref(b.c3, h, params) + sc
    x = _bnrelu_ref(model.post, x, params)
    feat = x.mean(dim=(2, 3))
    w = params[model.fc.w.name].view(model.fc.ncls, -1)
    return feat @ w.t() + params[model.fc.b.name]


def test_resnet_v2_grads_match_autograd(monkeypatch):
    """Pre-activation ResNet-50 v2: standalone BN+ReLU layers, bias-free convs, shortcut
    added in the last conv's epilogue, identity-shortcut gradient fan-in."""
    monkeypatch.setenv("HCB_CPU_DTYPE", "float64")
    torch.manual_seed(0)
    m = create_model("resnet50_v2", image_size=64, device="cpu")
    img, lab = synthetic_batch(m, 4)
    img = ((img - 127.0) / 60.0).double()
    loss_ref, grads_ref, _ = reference_grads(m, img, lab, resnet_v2_ref)
    t = Trainer(m, 4, constant_lr(0.0), weight_decay=0.0)
    t._forward_backward(img, lab)
    assert torch.allclose(t.row_loss.mean().double(), loss_ref, rtol=1e-5, atol=1e-6)
    for p in m.ps.params:
        r = grads_ref[p.name]
        err = (p.grad - r).abs().max().item()
        scale = r.abs().max().item() + 1e-6
        assert err <= 1e-4 * scale + 1e-6, f"{p.name}: max err {err} vs scale {scale}"


def test_forward_only_uses_moving_statistics(monkeypatch):
    """--forward_only: BN runs in inference mode from the moving statistics (phase_train=False)."""
    monkeypatch.setenv("HCB_CPU_DTYPE", "float64")
    from reference_models import conv_ref, pool_ref

    torch.manual_seed(2)
    m = create_model("resnet50", image_size=64, device="cpu")
    # non-trivial moving statistics
    for l in m.all_layers():
        if getattr(l, "bn", False):
            l.rmean.data.normal_(0.0, 0.1)
            l.rvar.data.uniform_(0.5, 2.0)
    img, lab = synthetic_batch(m, 2)
    img = ((img - 127.0) / 60.0).double()
    t = Trainer(m, 2, constant_lr(0.0), forward_only=True)
    t._forward(img, lab)
    params = {p.name: p.data.double() for p in m.ps.params}

    def cbn(layer, x, residual=None):
        z = conv_ref(layer, x, params)
        z = torch.nn.functional.batch_norm(z, layer.rmean.data.double(), layer.rvar.data.double(),
                                           params[layer.gamma.name], params[layer.beta.name], training=False,
                                           eps=layer.eps)
        if residual is not None:
            z = z + residual
        return torch.relu(z) if layer.relu else z

    x = pool_ref(m.pool, cbn(m.stem, img.permute(0, 3, 1, 2)))
    for b in m.blocks:
        sc = cbn(b.sc, x) if b.proj else x
        x = cbn(b.c3, cbn(b.c2, cbn(b.c1, x)), residual=sc)
    logits = x.mean(dim=(2, 3)) @ params[m.fc.w.name].view(m.fc.ncls, -1).t() + params[m.fc.b.name]
    ref = torch.nn.functional.cross_entropy(logits, lab, reduction="none")
    assert torch.allclose(t.row_loss.double(), ref, rtol=1e-6, atol=1e-7)


def test_cpu_training_is_bitwise_deterministic():
    """Same seed, same data -> bitwise-identical losses and weights (fp32 CPU path; the GPU
    path reduces BN statistics / weight gradients with fp32 atomics, so it is reproducible to
    rounding, not bitwise)."""
    def run():
        torch.manual_seed(0)
        m = create_model("resnet50", image_size=32, device="cpu", seed=7)
        img, lab = synthetic_batch(m, 4, seed=3)
        img = (img - 127.0) / 60.0
        t = Trainer(m, 4, constant_lr(0.05))
        losses = [float(t.step(img, lab)) for _ in range(3)]
        return losses, m.ps.master.clone()

    (l1, w1), (l2, w2) = run(), run()
    assert l1 == l2 and torch.equal(w1, w2)
