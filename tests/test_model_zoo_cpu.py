"""The feed-forward zoo (VGG / AlexNet / OverFeat / LeNet / GoogLeNet): hand-written backward
on the CPU path vs a PyTorch autograd reference (fp64), parameter counts, dropout semantics and
a few training steps through the Trainer."""
import pytest
import torch
import torch.nn.functional as F

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.models.inception import InceptionModule
from azure_hc_intel_tf_amd.models.sequential import Flatten
from azure_hc_intel_tf_amd.nn.layers import ConvBN, Dropout, GlobalAvgPool, Pool
from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch
from reference_models import conv_ref, pool_ref

SIZES = {"vgg11": 32, "vgg16": 32, "alexnet": 99, "overfeat": 91, "lenet": 28, "googlenet": 64}


def _layer_ref(l, x, params):
    if isinstance(l, ConvBN):
        z = conv_ref(l, x, params) + params[l.bias.name].view(1, -1, 1, 1)
        return torch.relu(z) if l.relu else z
    if isinstance(l, Pool):
        return pool_ref(l, x)
    if isinstance(l, InceptionModule):
        outs = {}
        for n in l.nodes:
            inp = x if n.src is None else outs[id(n.src)]
            outs[id(n)] = _layer_ref(n.layer, inp, params)
        return torch.cat([outs[id(t)] for t in l.terminals], dim=1)
    if isinstance(l, GlobalAvgPool):
        return x.mean(dim=(2, 3), keepdim=True)
    if isinstance(l, Flatten):  # NHWC flatten order
        return x.permute(0, 2, 3, 1).reshape(x.shape[0], -1, 1, 1)
    if isinstance(l, Dropout):
        return x
    raise TypeError(type(l))


def seq_ref(model, images_nhwc, params):
    x = images_nhwc.permute(0, 3, 1, 2)
    for l in model.seq:
        x = _layer_ref(l, x, params)
    feat = x.reshape(x.shape[0], -1)
    w = params[model.fc.w.name].view(model.fc.ncls, -1)
    return feat @ w.t() + params[model.fc.b.name]


@pytest.mark.parametrize("name", ["vgg11", "alexnet", "overfeat", "lenet", "googlenet"])
def test_zoo_grads_match_autograd(name, monkeypatch):
    monkeypatch.setenv("HCB_CPU_DTYPE", "float64")
    torch.manual_seed(0)
    m = create_model(name, image_size=SIZES[name], device="cpu")
    for l in m.seq:
        if isinstance(l, Dropout):
            l.keep = 1.0  # deterministic for the gradient comparison
    img, lab = synthetic_batch(m, 3)
    img = ((img - 127.0) / 60.0).double()
    params = {p.name: p.data.detach().clone().double().requires_grad_(True) for p in m.ps.params}
    logits = seq_ref(m, img, params)
    loss = F.cross_entropy(logits, lab)
    loss.backward()
    t = Trainer(m, 3, constant_lr(0.0), weight_decay=0.0)
    t._forward_backward(img, lab)
    assert torch.allclose(t.row_loss.mean().double(), loss.detach(), rtol=1e-6, atol=1e-7)
    for p in m.ps.params:
        r = params[p.name].grad
        err = (p.grad.double() - r).abs().max().item()
        scale = r.abs().max().item() + 1e-8
        assert err <= 1e-5 * scale + 1e-9, f"{p.name}: max err {err} vs {scale}"


def test_zoo_param_counts():
    # 1001-way logits (ImageNet + background), tf_cnn_benchmarks layouts
    assert create_model("vgg16", device="cpu").num_params() == 138_361_641
    assert create_model("vgg19", device="cpu").num_params() == 143_671_337
    assert create_model("alexnet", device="cpu").image_size == 227
    g = create_model("googlenet", device="cpu")
    assert g.feat_dim == 1024 and 6_900_000 < g.num_params() < 7_100_000


def test_dropout_semantics_cpu():
    d = Dropout("d", (1, 1, 4096), keep=0.5, seed=3)
    x = torch.randn(64, 1, 1, 4096)
    y = d.forward(x)
    kept = y != 0
    assert abs(kept.float().mean().item() - 0.5) < 0.02
    assert torch.allclose(y[kept], 2.0 * x[kept])
    dy = torch.randn_like(x)
    dx = d.backward(dy)
    assert torch.equal(dx, torch.where(kept, 2.0 * dy, torch.zeros_like(dy)))
    y2 = d.forward(x)  # the device-side step advanced: a new mask
    assert not torch.equal(y2 != 0, kept)
    d.training = False
    assert d.forward(x) is x


@pytest.mark.parametrize("name", ["vgg16", "googlenet"])
def test_zoo_training_reduces_loss(name):
    torch.manual_seed(1)
    m = create_model(name, image_size=SIZES[name], device="cpu")
    img, lab = synthetic_batch(m, 8)
    img = (img - 127.0) / 60.0
    t = Trainer(m, 8, constant_lr(0.01), weight_decay=4e-5)
    first = float(t.step(img, lab))
    for _ in range(8):
        last = float(t.step(img, lab))
    assert last < first
