"""fp32 (the reference's precision: /root/reference/benchmark-scripts/run-tf-sing-ucx-openmpi.sh:62-81
passes no --use_fp16) through the hand-written HIP kernels: --compute_dtype fp32 on ResNet runs
bf16x3 GEMMs (every fp32 operand split into bf16 hi + lo while staged to LDS, hi*hi + hi*lo + lo*hi
MFMAs, fp32 accumulation; csrc/kernels/conv_igemm.hip / conv_wgrad.hip) and the fp32
instantiations of the BN / pool / loss kernels. Every kernel is checked against an fp64 CPU
reference of the same fp32 operands; the full step against the fp32 CPU step."""
import pytest
import torch

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.nn.layers import set_gpu_compute_dtype
from azure_hc_intel_tf_amd.nn.params import ParamStore
from azure_hc_intel_tf_amd.ops import functional as Fn
from azure_hc_intel_tf_amd.ops.functional import ConvSpec
from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel_err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


@pytest.fixture
def fp32_mode():
    set_gpu_compute_dtype(torch.float32)
    Fn.set_f32_native(True)
    yield
    Fn.set_f32_native(False)
    set_gpu_compute_dtype(torch.bfloat16)


def _conv(cin, cout, k, s, pad):
    spec = ConvSpec(cin=cin, cin_pad=cin, cout=cout, kh=k, kw=k, sh=s, sw=s, pt=pad, pl=pad, pb=pad, pr=pad)
    ps = ParamStore(seed=5)
    p = ps.add("w", (cout, k, k, cin), True, ps.variance_scaling(k * k * cin))
    pk = ps.add_pack(p, cout, k, k, cin, spec.Kpad, spec.Kpad_t, want_tr=True)
    ps.finalize(DEV, dtype_pack=torch.bfloat16, pack_lo=True)
    ps.repack()
    return spec, p, pk, ps


CASES = [(64, 256, 1, 1, 0, 14), (64, 64, 3, 1, 1, 14), (128, 128, 3, 2, 1, 14), (256, 64, 1, 1, 0, 7),
         (256, 512, 1, 2, 0, 14), (80, 96, 3, 1, 1, 9)]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0]}x{c[1]}k{c[2]}s{c[3]}")
@pytest.mark.parametrize("cfg", [None, 0, 2, 12])
def test_fp32_conv_fwd_dgrad_wgrad_match_fp64(fp32_mode, case, cfg):
    """bf16x6 reproduces the fp32 convolution to fp32 accuracy (~1e-6): fwd, data grad
    (incl. the stride-phase and strided-1x1 remap forms) and weight grad (incl. split-K); an
    LDS-DMA cfg (12) is mapped to the register-staged kernel of its tile."""
    cin, cout, k, s, pad, H = case
    spec, p, pk, ps = _conv(cin, cout, k, s, pad)
    assert Fn.lo_pack(pk.pack) is not None and Fn.lo_pack(pk.tr) is not None
    torch.manual_seed(0)
    N = 4
    x = torch.randn(N, H, H, cin, device=DEV)
    P, Q = spec.out_hw(H, H)
    xd = x.double().cpu().permute(0, 3, 1, 2)
    wd = p.data.double().cpu().permute(0, 3, 1, 2)
    ref = torch.nn.functional.conv2d(xd, wd, stride=s, padding=pad).permute(0, 2, 3, 1)
    y = torch.empty(N, P, Q, cout, dtype=torch.float32, device=DEV)
    Fn.conv_forward(x, spec, pk.pack, p.data, y, cfg=cfg)
    assert rel_err(y, ref) < 3e-6
    dz = torch.randn(N, P, Q, cout, device=DEV)
    xr = xd.clone().requires_grad_(True)
    wr = wd.clone().requires_grad_(True)
    torch.nn.functional.conv2d(xr, wr, stride=s, padding=pad).backward(dz.double().cpu().permute(0, 3, 1, 2))
    dx = torch.zeros(N, H, H, cin, dtype=torch.float32, device=DEV)
    Fn.conv_dgrad(dz, spec, pk.tr, p.data, dx, False, cfg=cfg)
    assert rel_err(dx, xr.grad.permute(0, 2, 3, 1)) < 3e-6
    for wcfg in ((2, 1), (0, 4), (10, 8)):
        dw = torch.zeros(cout, spec.K, device=DEV)
        Fn.conv_wgrad(dz, x, spec, dw, cfg=wcfg)
        assert rel_err(dw.view(cout, k, k, cin), wr.grad.permute(0, 2, 3, 1)) < 3e-6, wcfg


@pytest.mark.parametrize("C", [64, 256, 2048])
@pytest.mark.parametrize("relu,residual", [(True, False), (True, True), (False, False)])
def test_fp32_bn_kernels_match_cpu(fp32_mode, C, relu, residual):
    """conv-epilogue statistics -> bn_apply_acc, then the backward reduce / apply pair, fp32
    tensors end to end, against the CPU fp32 path."""
    torch.manual_seed(13)
    spec, p, pk, ps = _conv(64, C, 3, 1, 1)
    N, H = 4, 9
    x = torch.randn(N, H, H, 64, device=DEV)
    z = torch.empty(N, H, H, C, dtype=torch.float32, device=DEV)
    R = 8
    acc_f = torch.zeros(R * 2 * C, device=DEV)
    Fn.conv_forward(x, spec, pk.pack, p.data, z, stats=acc_f, stats_R=R, cfg=2)
    gamma = torch.rand(C, device=DEV) + 0.5
    beta = torch.randn(C, device=DEV) * 0.1
    res = torch.randn(N, H, H, C, device=DEV) if residual else None
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    mean, invstd = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
    y = torch.empty_like(z)
    saved = Fn.bn_forward_acc(z, gamma, beta, rm, rv, 0.9, 1e-5, y, relu, acc_f, R, mean, invstd, residual=res)
    zc = z.cpu()
    yc = torch.empty(N, H, H, C)
    rmc, rvc = torch.zeros(C), torch.ones(C)
    sc = Fn.bn_forward(zc, gamma.cpu(), beta.cpu(), rmc, rvc, 0.9, 1e-5, yc, relu,
                       residual=None if res is None else res.cpu())
    assert rel_err(y, yc) < 1e-5
    assert rel_err(saved.mean, sc.mean) < 1e-5 and rel_err(saved.invstd, sc.invstd) < 1e-4
    assert rel_err(rv, rvc) < 1e-5
    dy = torch.randn(N, H, H, C, device=DEV)
    mode = (1 if residual else 2) if relu else 0
    dz = torch.empty_like(z)
    dg, db = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
    acc_b = torch.zeros(R * 2 * C, device=DEV)
    gres = torch.empty_like(z) if residual else None
    Fn.bn_backward_acc(dy, y, z, saved, gamma, beta, mode, dg, db, dz, acc_b, R, gres)
    dzc, dgc, dbc = torch.empty(N, H, H, C), torch.empty(C), torch.empty(C)
    gresc = torch.empty(N, H, H, C) if residual else None
    Fn.bn_backward(dy.cpu(), yc, zc, sc, gamma.cpu(), beta.cpu(), mode, dgc, dbc, dzc, gresc)
    assert rel_err(dz, dzc) < 1e-4
    assert rel_err(dg, dgc) < 1e-4 and rel_err(db, dbc) < 1e-4
    if residual:
        assert rel_err(gres, gresc) < 1e-6


def test_fp32_model_runs_the_hip_kernels():
    m = create_model("resnet50", image_size=64, device=DEV, compute_dtype="fp32", seed=3)
    try:
        assert m.native and m.image_channels == 8 and m.act_dtype == torch.float32
        assert m.ps.pack_buf.dtype == torch.bfloat16 and m.ps.pack_buf_lo.shape[0] == 2
        img, lab = synthetic_batch(m, 8)
        assert img.dtype == torch.float32
        img = (img - 127.0) / 60.0
        t = Trainer(m, 8, constant_lr(0.02))
        assert t.use_graph
        losses = [float(t.step(img, lab)) for _ in range(12)]
        assert all(l == l for l in losses)
        assert min(losses[-3:]) < 0.8 * losses[0], losses
    finally:
        Fn.set_f32_native(False)
        set_gpu_compute_dtype(torch.bfloat16)
