"""Projection-shortcut BN fused into the block output's BN pass (nn.layers.FUSE_RES_BN, ResBN in
csrc/kernels/bn.hip): act(BN3(z3) + BN_sc(z_sc)) in one kernel, the shortcut's normalised
tensor never written. Checked against the unfused path (shortcut BN apply, then the add)."""
import pytest
import torch

from azure_hc_intel_tf_amd.nn import layers as L
from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch

pytestmark = pytest.mark.gpu


def _step(fused, monkeypatch):
    from test_determinism_gpu import _shallow

    monkeypatch.setattr(L, "FUSE_RES_BN", fused)
    m = _shallow("cuda", image_size=32, seed=5, num_classes=11)
    img, lab = synthetic_batch(m, 32, seed=7)
    img = ((img.float() - 127.0) / 60.0).to(img.dtype)
    t = Trainer(m, 32, constant_lr(0.0), weight_decay=0.0, use_graph=False)
    t._forward_backward(img, lab)
    torch.cuda.synchronize()
    sc = next(l for l in m.all_layers() if l.name.endswith("/shortcut"))
    return (t.row_loss.clone(), m.ps.grad.clone(), sc.rmean.data.clone(), sc.rvar.data.clone(),
            sc.sv_mean.data.clone(), sc.sv_invstd.data.clone())


def test_fused_shortcut_bn_matches_unfused(monkeypatch):
    lu, gu, rmu, rvu, smu, siu = _step(False, monkeypatch)
    lf, gf, rmf, rvf, smf, sif = _step(True, monkeypatch)
    # the shortcut's batch moments come from the same epilogue sums (fp32 atomics: up to the
    # accumulation order)
    for a, b in ((smu, smf), (siu, sif), (rmu, rmf), (rvu, rvf)):
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-5), float((a - b).abs().max())
    # the output differs only by the bf16 rounding of the (unfused) normalised shortcut
    assert torch.allclose(lu, lf, rtol=1e-2, atol=1e-2), (lu[:4].tolist(), lf[:4].tolist())
    rel = ((gu - gf).norm() / gu.norm()).item()
    cos = float(gu @ gf / (gu.norm() * gf.norm()))
    assert rel < 0.05 and cos > 0.998, (rel, cos)
