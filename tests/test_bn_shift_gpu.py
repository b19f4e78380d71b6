"""Shifted single-pass BN statistics (nn.layers.BN_SHIFT, ConvParams::stats_shift): the conv epilogue
sums (v - K) and (v - K)^2 with K = the layer's previous batch mean (written by its BN backward),
so the variance E[(v-K)^2] - E[v-K]^2 does not cancel in fp32 when |mean| >> std. Checked against
an fp64 reference of the same GEMM (bf16 operands)."""
import pytest
import torch

from azure_hc_intel_tf_amd.nn import layers as L
from azure_hc_intel_tf_amd.nn.layers import ConvBN
from azure_hc_intel_tf_amd.nn.params import ParamStore

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _layer(cin=64, cout=64, hw=28):
    ps = ParamStore(seed=3)
    layer = ConvBN(ps, "c", (hw, hw, cin), cout, 1, 1, 1, 1, "SAME", relu=False, need_dx=False)
    ps.finalize(DEV)
    g = torch.Generator().manual_seed(7)
    # positive weights on a positive input: the output's |mean| / std is ~40
    layer.w.data.copy_((0.2 + 0.01 * torch.randn(layer.w.data.shape, generator=g)).to(DEV))
    ps.repack()
    return layer, ps


def _ref_moments(x, layer):
    cout = layer.out_shape[2]
    w = layer.w.data.bfloat16().double().reshape(cout, -1)
    z = x.double().reshape(-1, w.shape[1]) @ w.t()
    return z.mean(0), z.var(0, unbiased=False)


def _forward(layer, ps, x):
    ps.zero_stats()
    layer.forward(x)
    torch.cuda.synchronize()
    mean = layer.sv_mean.data.double().clone()
    var = layer.sv_invstd.data.double().pow(-2) - layer.eps
    return mean, var


@pytest.mark.skipif(not L.BN_SHIFT, reason="BN_SHIFT off")
def test_shifted_statistics_match_fp64_when_mean_dominates():
    layer, ps = _layer()
    g = torch.Generator().manual_seed(11)
    x = (1.0 + torch.rand(64, 28, 28, 64, generator=g)).bfloat16().to(DEV)
    rmean, rvar = _ref_moments(x, layer)
    assert (rmean.abs() / rvar.sqrt()).min() > 20  # the regime the shift is for

    assert torch.count_nonzero(layer.shift.data) == 0  # first step: K = 0, the plain form
    m0, v0 = _forward(layer, ps, x)
    err0 = ((v0 - rvar).abs() / rvar).max().item()

    # the BN backward hands this step's batch mean to the next step as K
    ps.zero_grad()
    layer.backward(torch.randn(x.shape[:3] + (64,), device=DEV).bfloat16())
    torch.cuda.synchronize()
    assert torch.equal(layer.shift.data, layer.sv_mean.data)

    m1, v1 = _forward(layer, ps, x)
    err1 = ((v1 - rvar).abs() / rvar).max().item()
    print(f"max relative variance error: unshifted {err0:.2e}, shifted {err1:.2e}")
    assert ((m1 - rmean).abs() / rvar.sqrt()).max().item() < 1e-4
    assert err1 < 2e-4, err1
    assert err1 <= err0


def test_shift_keeps_training_forward_exact_for_centered_data():
    """Zero-mean data: the shift (K ~ 0) changes nothing measurable."""
    layer, ps = _layer()
    layer.w.data.normal_(0.0, 0.05)
    ps.repack()
    x = torch.randn(16, 28, 28, 64, device=DEV).bfloat16()
    rmean, rvar = _ref_moments(x, layer)
    m, v = _forward(layer, ps, x)
    assert ((m - rmean).abs() / rvar.sqrt()).max().item() < 1e-4
    assert ((v - rvar).abs() / rvar).max().item() < 1e-4
