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
        # fp32-level agreement except where a ReLU / max-pool decision sits within rounding of its
        # threshold and flips between the two summation orders (measured: 5.2e-3 AlexNet, 1.4e-3
        # LeNet, < 1e-3 the others; cosine > 0.9999 everywhere)
        assert float(gg @ gc / (gg.norm() * gc.norm())) > 0.9999
        assert ((gg - gc).norm() / gc.norm()).item() < 1e-2
    finally:
        _reset()


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
