"""The projection shortcut's BN-backward reduction fused into the data-grad epilogue that produces the
block output's gradient (nn.layers.FUSE_RES_BN_BWD, ConvParams::bnb2_*): ResNet v1's block output
is relu(bn3(z3) + bn_sc(z_sc)), so both BNs see the same g, and the epilogue that already reduces
sum(g), sum(g * xhat3) for bn3 adds sum(g * xhat_sc) for the shortcut -- its separate reduce pass
(4 per ResNet-50 step) disappears. Fused against unfused, bf16 and fp32 paths."""
import pytest
import torch

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.nn import layers as L
from azure_hc_intel_tf_amd.nn.layers import set_gpu_compute_dtype
from azure_hc_intel_tf_amd.ops import functional as Fn
from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_shortcut_bn_reduction_rides_in_the_dgrad_epilogue(dtype, monkeypatch):
    """Deterministic mode (this tiny-batch net amplifies atomic-order noise: two default-mode runs of
    the SAME code differ by 100% (bf16) / 1.5% (fp32) in these gradients, tools/diag/res_bn_probe.py,
    profiles/r5_res_bn_fusion.txt). fp32: fused = unfused to ~1e-6. bf16: the fused sums take the
    epilogue's unrounded fp32 g where the separate pass reads the bf16-rounded tensor; the difference
    (2e-3 on the first fused shortcut in backward order, stage 4) grows through the later BN
    backwards to ~1.5e-2 on stage 1."""
    out = {}
    Fn.set_deterministic(True)
    try:
        for fuse in (False, True):
            monkeypatch.setattr(L, "FUSE_RES_BN_BWD", fuse)
            m = create_model("resnet50", image_size=64, device="cuda", seed=11,
                             compute_dtype=None if dtype == "bf16" else "fp32")
            img, lab = synthetic_batch(m, 8, seed=2)
            if dtype == "fp32":
                img[..., :3] = (img[..., :3] - 127.0) / 60.0
            t = Trainer(m, 8, constant_lr(0.0), weight_decay=0.0, use_graph=False)
            unfused = [0]
            real = Fn.bn_backward_acc

            def spy(*a, pre_reduced=False, **k):
                if not pre_reduced:
                    unfused[0] += 1
                return real(*a, pre_reduced=pre_reduced, **k)

            monkeypatch.setattr(Fn, "bn_backward_acc", spy)
            t._forward_backward(img, lab)
            torch.cuda.synchronize()
            monkeypatch.setattr(Fn, "bn_backward_acc", real)
            sc = {p.name: p.grad.float().cpu().clone() for p in m.ps.params if "shortcut/batchnorm" in p.name}
            out[fuse] = (m.ps.grad.float().cpu().clone(), sc, unfused[0])
            del m, t
    finally:
        Fn.set_deterministic(False)
        Fn.set_f32_native(False)
        set_gpu_compute_dtype(torch.bfloat16)
    g0, sc0, n0 = out[False]
    g1, sc1, n1 = out[True]
    assert n0 - n1 == 4, (n0, n1)  # ResNet-50's four projection shortcuts
    assert len(sc0) == 8
    for name in sc0:
        rel = ((sc1[name] - sc0[name]).norm() / sc0[name].norm()).item()
        tol = 1e-5 if dtype == "fp32" else (1e-2 if name.startswith("stage4") else 5e-2)
        assert rel < tol, (name, rel)
    rel = ((g1 - g0).norm() / g0.norm()).item()
    assert rel < (1e-4 if dtype == "fp32" else 5e-2), rel
