"""fp32 (the reference's precision) for the ResNet v2 family on the hand-written HIP kernels
(VERDICT r5 item 4): the pre-activation BN (statistics pass ``bn_stats_acc`` + the finalize-free
apply writing GEMM planes), the bias-free 1x1 conv whose fp32 epilogue adds the shortcut, the
identity shortcut's gradient added inside the pre-activation BN's backward apply, the S2D stem.

* kernels: ``bn_stats_acc`` (fp32 and bf16 input, shifted sums, replicas) and the ADD form of
  ``bn_bwd_apply_acc`` against fp64 references;
* model: one fp32 GPU step against the fp32 CPU step of the same weights, with a spy that sees no
  F.conv2d / F.max_pool2d / F.avg_pool2d call (no MIOpen); the captured step trains.
"""
import pytest
import torch
import torch.nn.functional as F

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.nn.layers import set_gpu_compute_dtype
from azure_hc_intel_tf_amd.ops import _ext
from azure_hc_intel_tf_amd.ops import functional as Fn
from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch

pytestmark = pytest.mark.gpu


def _reset():
    Fn.set_f32_native(False)
    set_gpu_compute_dtype(torch.bfloat16)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,C,R", [(1000, 64, 8), (3136, 256, 8), (50, 2048, 1), (777, 24, 3)])
def test_bn_stats_acc_matches_fp64(M, C, R, dtype):
    g = torch.Generator().manual_seed(M + C)
    x = (torch.randn(M, C, generator=g, dtype=torch.float64) * 2.0 + 5.0)
    shift = torch.randn(C, generator=g, dtype=torch.float64) + 5.0
    xd = x.to(dtype)
    acc = torch.zeros(R, 2, C, dtype=torch.float32, device="cuda")
    _ext.load()
    _ext.ops().bn_stats_acc(xd.cuda(), C, M, C, acc, R, shift.float().cuda())
    s = acc.double().sum(0).cpu()
    d = xd.double() - shift.float().double()
    ref1, ref2 = d.sum(0), (d * d).sum(0)
    assert torch.allclose(s[0], ref1, rtol=1e-5, atol=1e-3 * M ** 0.5), (s[0] - ref1).abs().max()
    assert torch.allclose(s[1], ref2, rtol=1e-5, atol=1e-3), (s[1] - ref2).abs().max()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_bn_bwd_apply_acc_add_matches_fp64(dtype):
    """dx = BN-ReLU backward(dy) + add in one pass, against fp64 (mode 2: mask recomputed from z)."""
    M, C, R = 2000, 128, 8
    g = torch.Generator().manual_seed(5)
    z = torch.randn(M, C, generator=g, dtype=torch.float64) * 1.5 + 0.3
    dy = torch.randn(M, C, generator=g, dtype=torch.float64)
    add = torch.randn(M, C, generator=g, dtype=torch.float64)
    gamma = torch.rand(C, generator=g, dtype=torch.float64) + 0.5
    beta = torch.randn(C, generator=g, dtype=torch.float64) * 0.1
    zd, dyd, addd = z.to(dtype), dy.to(dtype), add.to(dtype)
    zz = zd.double()
    mean = zz.mean(0)
    invstd = (zz.var(0, unbiased=False) + 1e-5).rsqrt()
    xhat = (zz - mean) * invstd
    mask = (xhat * gamma + beta) > 0
    gg = dyd.double() * mask
    db, dgm = gg.sum(0), (gg * xhat).sum(0)
    ref = gamma * invstd * (gg - db / M - xhat * dgm / M) + addd.double()
    # the reduce pass (acc replicas), then the apply with the addend
    dev = "cuda"
    acc = torch.zeros(R, 2, C, dtype=torch.float32, device=dev)
    mean_f, inv_f = mean.float().to(dev), invstd.float().to(dev)
    gam, bet = gamma.float().to(dev), beta.float().to(dev)
    dgamma = torch.empty(C, dtype=torch.float32, device=dev)
    dbeta = torch.empty_like(dgamma)
    dx = torch.empty(M, C, dtype=dtype, device=dev)
    _ext.load()
    hcb = _ext.ops()
    zg, dyg, addg = zd.to(dev), dyd.to(dev), addd.to(dev)
    hcb.bn_bwd_reduce_acc(dyg, C, None, 0, zg, C, M, C, mean_f, inv_f, gam, bet, 2, acc, R, None, 0)
    hcb.bn_bwd_apply_acc(dyg, C, None, 0, zg, C, dx, C, M, C, mean_f, inv_f, gam, bet, acc, R, dgamma, dbeta, 2,
                         None, None, None, addg, C)
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    err = ((dx.double().cpu() - ref).abs().max() / ref.abs().max()).item()
    assert err < tol, err
    assert torch.allclose(dbeta.double().cpu(), db, rtol=1e-4, atol=1e-3)


def test_fp32_resnet50_v2_step_matches_fp32_cpu_step(monkeypatch):
    kw = dict(image_size=64, seed=7, image_channels=8)
    try:
        mg = create_model("resnet50_v2", device="cuda", compute_dtype="fp32", **kw)
        mc = create_model("resnet50_v2", device="cpu", **kw)
        assert mg.native and mg.act_dtype == torch.float32
        assert torch.equal(mg.ps.master.cpu(), mc.ps.master)
        img_c, lab_c = synthetic_batch(mc, 4, seed=3)
        img_c[..., :3] = (img_c[..., :3] - 127.0) / 60.0
        calls = []
        for fn in ("conv2d", "max_pool2d", "avg_pool2d"):
            real = getattr(F, fn)
            monkeypatch.setattr(F, fn, lambda *a, _n=fn, _r=real, **k: (calls.append(_n), _r(*a, **k))[1])
        tg = Trainer(mg, 4, constant_lr(0.05), use_graph=False)
        lg = float(tg.step(img_c.cuda(), lab_c.cuda()))
        torch.cuda.synchronize()
        assert calls == [], calls  # every conv / pool of the fp32 step on the HIP kernels
        monkeypatch.undo()
        tc = Trainer(mc, 4, constant_lr(0.05))
        lc = float(tc.step(img_c, lab_c))
        assert abs(lg - lc) <= 1e-4 * abs(lc), (lg, lc)
        # random-init BN net: compared as a whole (test_precision_modes_gpu.py's v1 bound)
        gg, gc = mg.ps.grad.cpu(), mc.ps.grad
        assert (gg - gc).norm() / gc.norm() < 5e-2
        assert float(gg @ gc / (gg.norm() * gc.norm())) > 0.999
    finally:
        _reset()


def test_fp32_resnet50_v2_trains_in_the_step_graph():
    try:
        m = create_model("resnet50_v2", image_size=64, device="cuda", compute_dtype="fp32", seed=3)
        assert m.native
        img, lab = synthetic_batch(m, 8, seed=1)
        img[..., :3] = (img[..., :3] - 127.0) / 60.0
        t = Trainer(m, 8, constant_lr(0.02))
        assert t.use_graph
        losses = [float(t.step(img, lab)) for _ in range(12)]
        assert all(l == l for l in losses), losses
        assert min(losses[-3:]) < 0.8 * losses[0], losses
    finally:
        _reset()


def test_bf16_resnet50_v2_trains_in_the_step_graph():
    """The bf16 build of the same v2 path (acc-replica pre-activation BN, fused identity add)."""
    try:
        m = create_model("resnet50_v2", image_size=64, device="cuda", compute_dtype="bf16", seed=3)
        img, lab = synthetic_batch(m, 8, seed=1)
        img[..., :3] = (img[..., :3] - 127.0) / 60.0
        t = Trainer(m, 8, constant_lr(0.02))
        losses = [float(t.step(img, lab)) for _ in range(12)]
        assert all(l == l for l in losses), losses
        assert min(losses[-3:]) < 0.8 * losses[0], losses
    finally:
        _reset()
