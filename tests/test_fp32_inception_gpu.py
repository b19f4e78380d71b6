"""fp32 Inception-v3 on the hand-written HIP kernels (BASELINE config 4 at the reference's precision:
/root/reference/benchmark-scripts/run-tf-sing-ucx-openmpi.sh:34,66 trains whatever MODEL names in fp32).
Every conv shape class Inception adds beyond ResNet -- 1x7 / 7x1 and 1x3 / 3x1 rectangular filters, 5x5,
3x3/2 and 3x3/1 VALID -- through the bf16x6 plane GEMMs (forward, data gradient incl. the stride-phase
form, weight gradient) against an fp64 reference; the max / average pools on planes (into a concat
window) and their fp32 backward; and the whole fp32 step: no PyTorch conv / pool call, planes end to
end, training."""
import pytest
import torch
import torch.nn.functional as F

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.nn.layers import resolve_pads, set_gpu_compute_dtype
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


# (cin, cout, kh, kw, stride, mode, H): the Inception-v3 conv classes (models/inception.py)
CASES = [
    (64, 80, 1, 1, 1, "VALID", 17),     # stem 1x1 VALID
    (32, 64, 3, 3, 1, "VALID", 19),     # stem 3x3/1 VALID
    (64, 96, 3, 3, 2, "VALID", 17),     # reduction 3x3/2 VALID (B / D modules)
    (48, 64, 5, 5, 1, "SAME", 13),      # A modules 5x5
    (128, 128, 1, 7, 1, "SAME", 17),    # C modules 1x7
    (128, 192, 7, 1, 1, "SAME", 17),    # C modules 7x1
    (384, 384, 1, 3, 1, "SAME", 8),     # E modules 1x3
    (448, 384, 3, 1, 1, "SAME", 8),     # E modules 3x1
]


def _conv(cin, cout, kh, kw, s, mode, H):
    pt, pb, pl, pr = resolve_pads(mode, H, H, kh, kw, s, s)
    spec = ConvSpec(cin=cin, cin_pad=cin, cout=cout, kh=kh, kw=kw, sh=s, sw=s, pt=pt, pl=pl, pb=pb, pr=pr)
    ps = ParamStore(seed=5)
    p = ps.add("w", (cout, kh, kw, cin), True, ps.variance_scaling(kh * kw * cin))
    pk = ps.add_pack(p, cout, kh, kw, cin, spec.Kpad, spec.Kpad_t, want_tr=True)
    ps.finalize(DEV, dtype_pack=torch.bfloat16, pack_lo=True)
    ps.repack()
    return spec, p, pk


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0]}x{c[1]}k{c[2]}x{c[3]}s{c[4]}{c[5]}")
@pytest.mark.parametrize("cfg", [None, 4, 7, 14, 17, (2, 3), (13, 2)], ids=str)
def test_fp32_inception_conv_classes_match_fp64(fp32_mode, case, cfg):
    cin, cout, kh, kw, s, mode, H = case
    spec, p, pk = _conv(cin, cout, kh, kw, s, mode, H)
    torch.manual_seed(0)
    N = 4
    x = torch.randn(N, H, H, cin, device=DEV)
    P, Q = spec.out_hw(H, H)
    xd = F.pad(x.double().cpu().permute(0, 3, 1, 2), (spec.pl, spec.pr, spec.pt, spec.pb))
    wd = p.data.double().cpu().permute(0, 3, 1, 2)
    ref = F.conv2d(xd, wd, stride=s).permute(0, 2, 3, 1)
    assert ref.shape[1:3] == (P, Q)
    y = torch.empty(N, P, Q, cout, dtype=torch.float32, device=DEV)
    Fn.conv_forward(x, spec, pk.pack, p.data, y, cfg=cfg)
    assert rel_err(y, ref) < 3e-6
    dz = torch.randn(N, P, Q, cout, device=DEV)
    xr = x.double().cpu().permute(0, 3, 1, 2).requires_grad_(True)
    wr = wd.clone().requires_grad_(True)
    F.conv2d(F.pad(xr, (spec.pl, spec.pr, spec.pt, spec.pb)), wr, stride=s).backward(
        dz.double().cpu().permute(0, 3, 1, 2))
    dx = torch.zeros(N, H, H, cin, dtype=torch.float32, device=DEV)
    Fn.conv_dgrad(dz, spec, pk.tr, p.data, dx, False, cfg=cfg)
    assert rel_err(dx, xr.grad.permute(0, 2, 3, 1)) < 3e-6
    if cfg is None:
        for wcfg in (None, (2, 1), (0, 4), (13, 2), (15, 3)):
            dw = torch.zeros(cout, spec.K, device=DEV)
            Fn.conv_wgrad(dz, x, spec, dw, cfg=wcfg)
            assert rel_err(dw.view(cout, kh, kw, cin), wr.grad.permute(0, 2, 3, 1)) < 3e-6, wcfg


@pytest.mark.parametrize("kind", ["max3s2V", "max3s1S", "avg3s1S"])
def test_fp32_pools_on_planes_into_a_concat_window(fp32_mode, kind):
    """pool_fwd_p3: planes in, planes written into a channel window of a wider Planes buffer (an
    Inception branch's slot of the concat), exact fp32 max / the fp32 average (TF 'SAME': padding
    excluded from the count); the fp32 backward (argmax gather / 3x3/1 average gather, accumulated
    into an existing gradient) against fp64 autograd."""
    torch.manual_seed(3)
    N, H, C = 4, 17, 96
    is_max = kind.startswith("max")
    s = 2 if "s2" in kind else 1
    mode = "VALID" if kind.endswith("V") else "SAME"
    pads = resolve_pads(mode, H, H, 3, 3, s, s)
    pt, pb, pl, pr = pads
    P = (H + pt + pb - 3) // s + 1
    x = torch.randn(N, H, H, C, device=DEV) * 3
    xp = Fn.to_planes(x)
    wide = Fn.Planes.empty((N, P, P, C + 64), DEV)
    wide.t.zero_()
    out = wide[..., 32:32 + C]
    amax = torch.empty(N, P, P, C, dtype=torch.uint8, device=DEV) if is_max else None
    Fn.pool_forward(xp, out, 3, 3, s, s, pads, is_max, argmax=amax)
    xd = x.double().cpu().permute(0, 3, 1, 2).requires_grad_(True)
    if is_max:
        ref = F.max_pool2d(F.pad(xd, (pl, pr, pt, pb), value=-float("inf")), 3, s)
    else:
        ones = torch.ones_like(xd[:, :1])
        ref = (F.avg_pool2d(F.pad(xd, (pl, pr, pt, pb)), 3, s, divisor_override=1)
               / F.avg_pool2d(F.pad(ones, (pl, pr, pt, pb)), 3, s, divisor_override=1))
    got = out.float()
    if is_max:
        assert torch.equal(got.cpu().double(), ref.detach().permute(0, 2, 3, 1))  # exact
        assert torch.equal(out.t, Fn.to_planes(got).t)  # the winner's planes, canonical split
    else:
        assert rel_err(got, ref.detach().permute(0, 2, 3, 1)) < 3e-7
    assert float(wide.t[..., :32].abs().sum()) == 0 and float(wide.t[..., 32 + C:].abs().sum()) == 0
    dy = torch.randn(N, P, P, C, device=DEV)
    ref.backward(dy.double().cpu().permute(0, 3, 1, 2))
    base = torch.randn(N, H, H, C, device=DEV)
    dx = base.clone()
    Fn.pool_backward(dy, xp, out, dx, 3, 3, s, s, pads, is_max, accumulate=True, argmax=amax)
    assert rel_err(dx - base, xd.grad.permute(0, 2, 3, 1)) < 3e-7


def test_fp32_inception_step_runs_native_planes_no_torch_conv_or_pool(monkeypatch):
    """The fp32 Inception-v3 training step runs entirely on the HIP kernels: no F.conv2d /
    F.max_pool2d / F.avg_pool2d call, every GEMM operand produced as planes (the only fp32 -> plane
    splits are the input image's and the classifier's dlogits), finite losses that fall."""
    m = create_model("inception3", image_size=139, device=DEV, compute_dtype="fp32", seed=3)
    try:
        assert m.native and m.act_dtype == torch.float32 and m.ps.pack_buf_lo.shape[0] == 2
        torch_calls = []
        for name in ("conv2d", "max_pool2d", "avg_pool2d", "conv_transpose2d"):
            real = getattr(F, name)
            monkeypatch.setattr(F, name, lambda *a, _n=name, _r=real, **k: (torch_calls.append(_n), _r(*a, **k))[1])
        splits = []
        real_split = Fn.to_planes

        def spy(t):
            if not Fn.is_planes(t):
                splits.append(tuple(t.shape))
            return real_split(t)

        monkeypatch.setattr(Fn, "to_planes", spy)
        img, lab = synthetic_batch(m, 4)
        img[..., :3] = (img[..., :3] - 127.0) / 60.0
        t = Trainer(m, 4, constant_lr(0.02), use_graph=False)
        t.step(img, lab)
        torch.cuda.synchronize()
        assert torch_calls == [], torch_calls
        assert sorted(splits) == sorted([tuple(img.shape), (4, m.fc.ld)]), splits
        monkeypatch.undo()
        t = Trainer(m, 4, constant_lr(0.02))
        assert t.use_graph
        losses = [float(t.step(img, lab)) for _ in range(10)]
        assert all(l == l for l in losses)
        assert min(losses[-3:]) < 0.8 * losses[0], losses
    finally:
        Fn.set_f32_native(False)
        set_gpu_compute_dtype(torch.bfloat16)


def test_fp32_inception_gpu_matches_fp32_cpu_step():
    """One fp32 Inception-v3 step on the GPU (HIP kernels) equals the fp32 CPU step: the loss to fp32
    tolerance, the gradient as a whole (direction and norm; see test_precision_modes_gpu.py)."""
    kw = dict(image_size=139, seed=7, image_channels=8)
    mg = create_model("inception3", device="cuda", compute_dtype="fp32", **kw)
    mc = create_model("inception3", device="cpu", **kw)
    try:
        assert mg.native
        assert torch.equal(mg.ps.master.cpu(), mc.ps.master)
        img_c, lab_c = synthetic_batch(mc, 4, seed=3)
        img_c[..., :3] = (img_c[..., :3] - 127.0) / 60.0
        tg = Trainer(mg, 4, constant_lr(0.05))
        tc = Trainer(mc, 4, constant_lr(0.05))
        lg = float(tg.step(img_c.cuda(), lab_c.cuda()))
        lc = float(tc.step(img_c, lab_c))
        torch.cuda.synchronize()
        assert abs(lg - lc) <= 1e-4 * abs(lc), (lg, lc)
        gg, gc = mg.ps.grad.cpu(), mc.ps.grad
        assert (gg - gc).norm() / gc.norm() < 5e-2
        assert float(gg @ gc / (gg.norm() * gc.norm())) > 0.999
    finally:
        Fn.set_f32_native(False)
        set_gpu_compute_dtype(torch.bfloat16)
