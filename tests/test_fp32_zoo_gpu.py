"""fp32 (the reference's precision) for the rest of the tf_cnn_benchmarks zoo on the hand-written HIP
kernels: VGG, AlexNet, OverFeat, LeNet, GoogLeNet and `trivial` run their conv / affine layers as
bf16x6 plane GEMMs with the bias + ReLU epilogue, fp32 pools, dropout, ReLU backward and bias column
sums -- no F.conv2d / F.*pool2d call in the step. One GPU step against the fp32 CPU step of the same
weights (dropout off for the comparison: the GPU mask is a counter hash, the CPU one a generator),
and a few training steps with dropout on."""
import pytest
import torch
import torch.nn.functional as F

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.models import sequential
from azure_hc_intel_tf_amd.nn.layers import set_gpu_compute_dtype
from azure_hc_intel_tf_amd.ops import functional as Fn
from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch

pytestmark = pytest.mark.gpu

# (model, image size, batch): small images that keep every layer's output non-empty
ZOO = [("vgg11", 32, 4), ("alexnet", 67, 4), ("overfeat", 95, 4), ("lenet", 28, 8), ("googlenet", 64, 4),
       ("trivial", 32, 8)]


def _reset():
    Fn.set_f32_native(False)
    set_gpu_compute_dtype(torch.bfloat16)


@pytest.mark.parametrize("name,size,batch", ZOO, ids=[z[0] for z in ZOO])
def test_fp32_zoo_gpu_step_matches_fp32_cpu_step(name, size, batch, monkeypatch):
    monkeypatch.setattr(sequential.SequentialCNN, "dropout_keep", 1.0)
    kw = dict(image_size=size, seed=9, image_channels=8)  # the GPU layout: image channels padded to 8
    try:
        mg = create_model(name, device="cuda", compute_dtype="fp32", **kw)
        mc = create_model(name, device="cpu", **kw)
        assert mg.native and mg.act_dtype == torch.float32
        assert torch.equal(mg.ps.master.cpu(), mc.ps.master)
        img_c, lab_c = synthetic_batch(mc, batch, seed=4)
        img_c[..., :3] = (img_c[..., :3] - 127.0) / 60.0
        calls = []
        for fn in ("conv2d", "max_pool2d", "avg_pool2d"):
            real = getattr(F, fn)
            monkeypatch.setattr(F, fn, lambda *a, _n=fn, _r=real, **k: (calls.append(_n), _r(*a, **k))[1])
        tg = Trainer(mg, batch, constant_lr(0.01), use_graph=False)
        lg = float(tg.step(img_c.cuda(), lab_c.cuda()))
        torch.cuda.synchronize()
        assert calls == [], calls
        monkeypatch.undo()
        monkeypatch.setattr(sequential.SequentialCNN, "dropout_keep", 1.0)
        tc = Trainer(mc, batch, constant_lr(0.01))
        lc = float(tc.step(img_c, lab_c))
        assert abs(lg - lc) <= 1e-4 * abs(lc), (lg, lc)
        gg, gc = mg.ps.grad.cpu(), mc.ps.grad
        assert float(gg @ gc / (gg.norm() * gc.norm())) > 0.9999
        if name not in MIRRORED:
            assert ((gg - gc).norm() / gc.norm()).item() < 1e-3
        # (the plain sequential nets are held to fp32 rounding given their ReLU / max-pool decisions
        # by test_fp32_zoo_gpu_gradient_given_its_decisions below: AlexNet / LeNet each flip ONE ReLU
        # decision against the CPU, which alone moves the whole gradient by 5.2e-3 / 1.4e-3)
    finally:
        _reset()


# the sequential nets the fp64 decision-forced mirror of tools/zoo_flip_probe.py covers
MIRRORED = {"vgg11", "alexnet", "overfeat", "lenet"}


@pytest.mark.parametrize("name,size,batch", [z for z in ZOO if z[0] in MIRRORED], ids=[z[0] for z in ZOO if z[0] in MIRRORED])
def test_fp32_zoo_gpu_gradient_given_its_decisions(name, size, batch):
    """The GPU gradient against an fp64 autograd mirror of the network whose ReLU masks and
    max-pool argmaxes are forced to the GPU's own decisions: what remains is the kernels' fp32
    rounding (measured 3.5e-7 - 7.1e-7). The GPU-vs-CPU gap is then bounded GIVEN the number of
    decisions that differ from the CPU's (profiles/r6_zoo_fp32_flip_probe.txt: one ReLU flip in
    AlexNet's last affine layer / LeNet's second conv accounts for the whole 5.2e-3 / 1.4e-3)."""
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import zoo_flip_probe as ZP

    r = ZP.probe(name, size, batch, seed=9, img_seed=4)  # the inputs of the step test above
    flips = sum(f for _, _, f, _ in r["flips"])
    assert r["gpu_vs_mirror_gpu"] < 1e-5, r
    assert r["cpu_vs_mirror_cpu"] < 1e-5, r  # the mirror itself reproduces the CPU step
    assert flips <= 2, r["flips"]
    if flips == 0:
        assert r["gpu_vs_cpu"] < 1e-5, r


@pytest.mark.parametrize("name,size,batch", [("alexnet", 67, 8), ("googlenet", 64, 8)], ids=["alexnet", "googlenet"])
def test_fp32_zoo_trains_in_the_step_graph(name, size, batch):
    """The captured fp32 step (dropout on for AlexNet: fresh device-side masks every replay)."""
    try:
        m = create_model(name, image_size=size, device="cuda", compute_dtype="fp32", seed=3)
        img, lab = synthetic_batch(m, batch, seed=1)
        img[..., :3] = (img[..., :3] - 127.0) / 60.0
        t = Trainer(m, batch, constant_lr(0.02))
        assert t.use_graph
        losses = [float(t.step(img, lab)) for _ in range(12)]
        assert all(l == l for l in losses), losses
        assert min(losses[-3:]) < losses[0], losses
    finally:
        _reset()
