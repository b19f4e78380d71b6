"""Whole-model checks on the MI355X: hand-written HIP fwd/bwd vs the fp32 CPU path, and the
HIP-graph captured training step."""
import pytest
import torch

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    a = a.float().cpu()
    b = b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("name,size,batch", [("resnet50", 128, 16), ("resnet50_v1.5", 128, 16),
                                             ("inception3", 299, 4), ("trivial", 64, 16),
                                             ("resnet50_v2", 128, 16)])
def test_model_gpu_forward_and_descent(name, size, batch):
    """At random init the gradients of this BN network are chaotic in the rounding (an fp32
    CPU run already differs from fp64 autograd by ~1% and bf16 rounding decorrelates deep
    layers), so whole-network grads are not compared elementwise. Checked instead: the
    forward (loss, logits) against the fp32 CPU path, the classifier gradient (depends on the
    forward only), and that the hand-written GPU gradient is a descent direction."""
    kw = dict(image_size=size, image_channels=8, seed=11)
    mg = create_model(name, device="cuda", compute_dtype="bf16", **kw)
    mc = create_model(name, device="cpu", **kw)
    assert torch.equal(mg.ps.master.cpu(), mc.ps.master)
    img_c, lab_c = synthetic_batch(mc, batch, seed=5)
    img_c = ((img_c - 127.0) / 60.0).to(torch.bfloat16).float()
    img_g = img_c.to("cuda", torch.bfloat16)
    lab_g = lab_c.cuda()
    tg = Trainer(mg, batch, constant_lr(0.0), weight_decay=0.0, use_graph=False)
    tc = Trainer(mc, batch, constant_lr(0.0), weight_decay=0.0)
    tg._forward_backward(img_g, lab_g)
    tc._forward_backward(img_c, lab_c)
    torch.cuda.synchronize()
    lg, lc = tg.row_loss.mean().item(), tc.row_loss.mean().item()
    assert abs(lg - lc) < 0.05, (lg, lc)
    fcg = [p for p in mg.ps.params if p.name == "logits/affine/weights"][0]
    fcc = [p for p in mc.ps.params if p.name == "logits/affine/weights"][0]
    a, b = fcg.grad.float().cpu().flatten(), fcc.grad.float().flatten()
    if b.norm() == 0:  # trivial: its 1-unit ReLU layer is dead at this init (as in TF): no signal
        assert a.norm() == 0
        return
    assert (a @ b / (a.norm() * b.norm())).item() > 0.97  # bf16 features through 50 layers
    # descent: a small step along -grad lowers the loss of the same batch
    g = mg.ps.grad.clone()
    base = tg.row_loss.mean().item()
    mg.ps.master.sub_(0.05 * g / g.norm() * mg.ps.master.norm() * 1e-2)
    tg._forward_backward(img_g, lab_g)
    torch.cuda.synchronize()
    assert tg.row_loss.mean().item() < base


def test_graph_training_step_runs_and_learns():
    # Loss on one repeated batch plateaus near ln(#labels in batch) for a few steps before it
    # drops; seed the init and run long enough to leave the plateau.
    torch.manual_seed(0)
    m = create_model("resnet50", image_size=96, device="cuda", compute_dtype="bf16")
    img, lab = synthetic_batch(m, 16)
    t = Trainer(m, 16, constant_lr(0.02), use_graph=True, graph_warmup=2)
    losses = [float(t.step(img, lab)) for _ in range(28)]
    assert all(torch.isfinite(torch.tensor(losses)))
    assert t._g_all is not None
    # (the plateau's length varies with the rounding of the run: 28 steps clear it)
    assert min(losses[-3:]) < 0.8 * losses[2], losses


def test_full_size_resnet50_step_bs64():
    m = create_model("resnet50", device="cuda", compute_dtype="bf16")
    img, lab = synthetic_batch(m, 64)
    t = Trainer(m, 64, constant_lr(0.01), use_graph=True)
    for _ in range(4):
        loss = float(t.step(img, lab))
    assert loss == loss and loss < 20
