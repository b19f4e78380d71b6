"""The 3x3 / stride-1 conv kernels with the input patch resident in LDS (cfg 17-21,
csrc/kernels/conv3x3_patch.hip) against the fp32 PyTorch reference: forward + fused BN
statistics, data gradient (plain, beta-accumulate, fused BN-backward epilogue), split-K over
channel slabs, tiles that straddle image boundaries, Nout not a multiple of the tile, and the
fallback of an ineligible problem (stride 2) to a generic kernel of the same row tile."""
import math

import pytest
import torch

from azure_hc_intel_tf_amd.ops import functional as Fn

from test_kernels_gpu import bf, cpu_ref_conv, make_conv, rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda"
PATCH_CFGS = [17, 18, 19, 20, 21]
# cin, cout, H, N: the ResNet-50 bottleneck conv2 shapes at small batch, odd image sizes
# (tiles cross rows and images at every offset) and a cout that no tile divides
CASES = [(64, 64, 56, 1), (128, 128, 28, 2), (256, 256, 14, 3), (512, 512, 7, 4), (64, 192, 9, 5),
         (128, 64, 13, 3)]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0]}x{c[1]}h{c[2]}n{c[3]}")
@pytest.mark.parametrize("cfg", PATCH_CFGS)
def test_patch_fwd_and_stats(case, cfg):
    cin, cout, H, N = case
    torch.manual_seed(cfg)
    spec, p, pk = make_conv(cin, cout, 3, 3, 1, 1, (1, 1, 1, 1))
    assert Fn.patch_eligible(spec) and Fn.patch_eligible(spec, dgrad=cout % 64 == 0) == (cout % 64 == 0)
    x = bf(torch.randn(N, H, H, cin, device=DEV))
    y = torch.empty(N, H, H, cout, dtype=torch.bfloat16, device=DEV)
    T = math.ceil(N * H * H / Fn._CONV_TILES[cfg][0])
    slab = torch.empty(T * 2 * cout, device=DEV)
    Fn.conv_forward(x, spec, pk.pack, p.data, y, stats=slab, cfg=cfg)
    ref = cpu_ref_conv(x, spec, bf(p.data))
    assert rel_err(y, ref) < 1e-2
    s = slab.view(T, 2, cout).sum(0).cpu()
    assert rel_err(s[0], ref.reshape(-1, cout).sum(0)) < 2e-2
    assert rel_err(s[1], (ref * ref).reshape(-1, cout).sum(0)) < 2e-2
    # replica statistics with a shift K: sums of (v - K) and (v - K)^2
    R = 8
    acc = torch.zeros(R * 2 * cout, device=DEV)
    shift = torch.randn(cout, device=DEV) * 0.1
    Fn.conv_forward(x, spec, pk.pack, p.data, y, stats=acc, stats_R=R, cfg=cfg, stats_shift=shift)
    d = ref.reshape(-1, cout) - shift.cpu()
    a = acc.view(R, 2, cout).sum(0).cpu()
    assert rel_err(a[0], d.sum(0)) < 2e-2 and rel_err(a[1], (d * d).sum(0)) < 2e-2


@pytest.mark.parametrize("case", [c for c in CASES if c[1] % 64 == 0], ids=lambda c: f"{c[0]}x{c[1]}h{c[2]}n{c[3]}")
@pytest.mark.parametrize("cfg", PATCH_CFGS)
def test_patch_dgrad(case, cfg):
    cin, cout, H, N = case
    torch.manual_seed(40 + cfg)
    spec, p, pk = make_conv(cin, cout, 3, 3, 1, 1, (1, 1, 1, 1))
    dz = bf(torch.randn(N, H, H, cout, device=DEV))
    ref = torch.empty(N, H, H, cin)
    Fn.conv_dgrad(dz.float().cpu(), spec, None, bf(p.data).float().cpu(), ref, False)
    dx = torch.empty(N, H, H, cin, dtype=torch.bfloat16, device=DEV)
    Fn.conv_dgrad(dz, spec, pk.tr, p.data, dx, False, cfg=cfg)
    assert rel_err(dx, ref) < 1e-2
    base = bf(torch.randn(N, H, H, cin, device=DEV))
    dx = base.clone()
    Fn.conv_dgrad(dz, spec, pk.tr, p.data, dx, True, cfg=cfg)
    assert rel_err(dx, ref + base.float().cpu()) < 1e-2


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("cfg", PATCH_CFGS)
def test_patch_dgrad_fused_bn_backward(mode, cfg):
    cin, cout, H, N = 128, 128, 14, 3
    torch.manual_seed(60 + mode)
    spec, p, pk = make_conv(cin, cout, 3, 3, 1, 1, (1, 1, 1, 1))
    dz = bf(torch.randn(N, H, H, cout, device=DEV))
    base = bf(torch.randn(N, H, H, cin, device=DEV))
    z = bf(torch.randn(N, H, H, cin, device=DEV) * 1.5 + 0.2)
    yact = bf(torch.relu(torch.randn(N, H, H, cin, device=DEV)))
    mean = torch.randn(cin, device=DEV) * 0.1 + 0.2
    invstd = torch.rand(cin, device=DEV) + 0.5
    gamma = torch.rand(cin, device=DEV) + 0.5
    beta = torch.randn(cin, device=DEV) * 0.2
    R = 8
    acc = torch.zeros(R * 2 * cin, device=DEV)
    dx = base.clone()
    bnb = Fn.BNBwdFuse(z, yact, Fn.BNSaved(mean, invstd), gamma, beta, mode, acc, R)
    Fn.conv_dgrad(dz, spec, pk.tr, p.data, dx, True, cfg=cfg, bnb=bnb)
    ref = torch.empty(N, H, H, cin)
    Fn.conv_dgrad(dz.float().cpu(), spec, None, bf(p.data).float().cpu(), ref, False)
    ref = ref + base.float().cpu()
    zc = z.float().cpu()
    cpu_bnb = Fn.BNBwdFuse(zc, yact.float().cpu(), Fn.BNSaved(mean.cpu(), invstd.cpu()), gamma.cpu(), beta.cpu(),
                           mode, None, R)
    g = cpu_bnb.gate_cpu(ref.clone())
    assert rel_err(dx, g) < 1e-2
    xhat = (zc - mean.cpu()) * invstd.cpu()
    sums = acc.view(R, 2, cin).sum(0).cpu()
    assert rel_err(sums[0], g.reshape(-1, cin).sum(0)) < 2e-2
    assert rel_err(sums[1], (g * xhat).reshape(-1, cin).sum(0)) < 2e-2


@pytest.mark.parametrize("plan", [(17, 2), (18, 4), (19, 2), (20, 4), (21, 3), (18, 8)])
def test_patch_split_k_over_channel_slabs(plan):
    cfg, s = plan
    torch.manual_seed(80 + s)
    cin, cout, H, N = 512, 512, 7, 4
    spec, p, pk = make_conv(cin, cout, 3, 3, 1, 1, (1, 1, 1, 1))
    assert s in Fn.splitk_candidates(cfg, N * H * H, cout, spec.K) or s == 8
    x = bf(torch.randn(N, H, H, cin, device=DEV))
    y = torch.empty(N, H, H, cout, dtype=torch.bfloat16, device=DEV)
    acc = torch.zeros(8 * 2 * cout, device=DEV)
    ref = cpu_ref_conv(x, spec, bf(p.data))
    for rep in range(2):  # the second pass checks that the tickets were left re-armed
        acc.zero_()
        Fn.conv_forward(x, spec, pk.pack, p.data, y, stats=acc, stats_R=8, cfg=list(plan))
        assert rel_err(y, ref) < 1e-2, rep
        assert rel_err(acc.view(8, 2, cout).sum(0)[0], ref.reshape(-1, cout).sum(0)) < 2e-2
    dz = bf(torch.randn(N, H, H, cout, device=DEV))
    dref = torch.empty(N, H, H, cin)
    Fn.conv_dgrad(dz.float().cpu(), spec, None, bf(p.data).float().cpu(), dref, False)
    dx = torch.empty(N, H, H, cin, dtype=torch.bfloat16, device=DEV)
    Fn.conv_dgrad(dz, spec, pk.tr, p.data, dx, False, cfg=list(plan))
    assert rel_err(dx, dref) < 1e-2
    assert int(Fn._splitk["cnt"].abs().sum().item()) == 0


@pytest.mark.parametrize("cfg", PATCH_CFGS)
def test_patch_cfg_on_ineligible_problem_falls_back(cfg):
    """a tuned patch cfg handed a stride-2 3x3 (or a channel count off the 64 grid) runs a
    generic kernel of the same row tile: correct output and per-tile statistics slab size"""
    torch.manual_seed(90 + cfg)
    for cin, s, H in ((128, 2, 14), (96, 1, 9)):
        spec, p, pk = make_conv(cin, 128, 3, 3, s, s, (1, 1, 1, 1))
        assert not Fn.patch_eligible(spec)
        N = 2
        P, Q = spec.out_hw(H, H)
        x = bf(torch.randn(N, H, H, cin, device=DEV))
        y = torch.empty(N, P, Q, 128, dtype=torch.bfloat16, device=DEV)
        T = math.ceil(N * P * Q / Fn._CONV_TILES[cfg][0])
        slab = torch.empty(T * 2 * 128, device=DEV)
        Fn.conv_forward(x, spec, pk.pack, p.data, y, stats=slab, cfg=cfg)
        ref = cpu_ref_conv(x, spec, bf(p.data))
        assert rel_err(y, ref) < 1e-2
        assert rel_err(slab.view(T, 2, 128).sum(0)[0].cpu(), ref.reshape(-1, 128).sum(0)) < 2e-2
