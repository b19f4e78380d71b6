"""The feed-forward zoo on the MI355X: forward / classifier gradient vs the fp32 CPU path,
descent of the hand-written HIP backward, the dropout kernel, and full-size captured steps."""
import pytest
import torch

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.nn.layers import Dropout
from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch

pytestmark = pytest.mark.gpu

SIZES = {"vgg16": 32, "alexnet": 99, "overfeat": 91, "lenet": 28, "googlenet": 64}


def _no_dropout(m):
    for l in m.seq:
        if isinstance(l, Dropout):
            l.keep = 1.0


@pytest.mark.parametrize("name", sorted(SIZES))
def test_zoo_gpu_forward_and_descent(name):
    kw = dict(image_size=SIZES[name], image_channels=8, seed=3)
    mg = create_model(name, device="cuda", compute_dtype="bf16", **kw)
    mc = create_model(name, device="cpu", **kw)
    _no_dropout(mg)
    _no_dropout(mc)
    B = 8
    img_c, lab_c = synthetic_batch(mc, B, seed=2)
    img_c = ((img_c - 127.0) / 60.0).to(torch.bfloat16).float()
    img_g, lab_g = img_c.to("cuda", torch.bfloat16), lab_c.cuda()
    tg = Trainer(mg, B, constant_lr(0.0), weight_decay=0.0, use_graph=False)
    tc = Trainer(mc, B, constant_lr(0.0), weight_decay=0.0)
    tg._forward_backward(img_g, lab_g)
    tc._forward_backward(img_c, lab_c)
    torch.cuda.synchronize()
    lg, lc = tg.row_loss.mean().item(), tc.row_loss.mean().item()
    assert abs(lg - lc) < 0.05, (lg, lc)
    fg = [p for p in mg.ps.params if p.name == "logits/affine/weights"][0].grad.float().cpu().flatten()
    fc = [p for p in mc.ps.params if p.name == "logits/affine/weights"][0].grad.float().flatten()
    assert (fg @ fc / (fg.norm() * fc.norm() + 1e-12)).item() > 0.97
    g = mg.ps.grad.clone()
    base = tg.row_loss.mean().item()
    mg.ps.master.sub_(0.05 * g / g.norm() * mg.ps.master.norm() * 1e-2)
    tg._forward_backward(img_g, lab_g)
    torch.cuda.synchronize()
    assert tg.row_loss.mean().item() < base


def test_dropout_kernel():
    d = Dropout("d", (1, 1, 4096), keep=0.5, seed=7)
    x = torch.randn(64, 1, 1, 4096, device="cuda").bfloat16()
    y = d.forward(x)
    kept = y != 0
    assert abs(kept.float().mean().item() - 0.5) < 0.02
    assert torch.equal(y[kept].float(), (2.0 * x[kept].float()).bfloat16().float())
    dy = torch.randn_like(x)
    dx = d.backward(dy)
    assert torch.equal(dx.float(), torch.where(kept, 2.0 * dy.float(), torch.zeros_like(dy.float())))
    y2 = d.forward(x)
    assert not torch.equal(y2 != 0, kept)  # step counter advanced on the device


@pytest.mark.parametrize("name,batch", [("vgg16", 16), ("googlenet", 32), ("alexnet", 64)])
def test_zoo_full_size_graph_steps(name, batch):
    m = create_model(name, device="cuda", compute_dtype="bf16")
    img, lab = synthetic_batch(m, batch)
    t = Trainer(m, batch, constant_lr(1e-4), use_graph=True)
    losses = [float(t.step(img, lab)) for _ in range(5)]
    torch.cuda.synchronize()
    assert all(l == l and l < 1e4 for l in losses), losses
