"""fp32 (the reference's precision: /root/reference/benchmark-scripts/run-tf-sing-ucx-openmpi.sh:62-81
passes no --use_fp16) through the hand-written HIP kernels: --compute_dtype fp32 on ResNet holds every
GEMM operand as three bf16 planes hi / mid / lo (``Fn.Planes``, written by the producing BN / split
kernel) and runs bf16x6 GEMMs on them (six MFMA products, fp32 accumulation;
csrc/kernels/conv_p3.hip), with the fp32 instantiations of the BN / pool / loss kernels. Every kernel
is checked against an fp64 CPU reference of the same fp32 operands; the full step against the fp32
CPU step."""
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
@pytest.mark.parametrize("cfg", [None, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22,
                                 23, 24, 25, 26, 27, 28, 31, 32, 33, 34, 35, 36, (0, 2), (4, 3), (7, 2), (10, 3), (14, 3),
                                 (16, 5), (17, 6)],
                         ids=str)
def test_fp32_conv_fwd_dgrad_wgrad_match_fp64(fp32_mode, case, cfg):
    """bf16x6 on planes reproduces the fp32 convolution to fp32 accuracy (~1e-6): fwd, data grad
    (incl. the stride-phase and strided-1x1 remap forms) and weight grad (incl. split-K), every
    plane-GEMM tile config (conv_p3.hip cfg 0-6) and in-launch split-K; fp32 inputs are split into
    planes by the ops themselves. cfg 7-13: 32-deep slots (64-byte LDS rows) and 128x128 / 256x128
    block tiles; (cfg, S): in-launch split-K (fixed-order slab sum); weight-grad cfg 6-11: 32-deep slots, up to 256x128 / 128x256; fwd cfg 14-17 / weight-grad 12-15: two or
    three workgroups per CU; 18-22: the persistent short-K kernel (conv_p3_persist.h; the strided
    data gradients' remap form runs its twin); 23-27: its stream-K form; 31-34: its weights-resident
    form (falling back where it does not fit)."""
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
    dx = torch.full((N, H, H, cin), float("nan"), dtype=torch.float32, device=DEV)  # every pixel written
    Fn.conv_dgrad(dz, spec, pk.tr, p.data, dx, False, cfg=cfg)
    assert rel_err(dx, xr.grad.permute(0, 2, 3, 1)) < 3e-6
    if isinstance(cfg, tuple):  # split-K case: the weight-gradient configs once
        return
    for wcfg in ((2, 1), (0, 4), (3, 8), (1, 2), (4, 1), (5, 2), (6, 1), (7, 2), (8, 1), (9, 3), (10, 4), (11, 2),
                 (12, 1), (13, 2), (14, 3), (15, 2), (16, 1), (16, 3), (17, 2), (18, 5)):
        dw = torch.zeros(cout, spec.K, device=DEV)
        Fn.conv_wgrad(dz, x, spec, dw, cfg=wcfg)
        assert rel_err(dw.view(cout, k, k, cin), wr.grad.permute(0, 2, 3, 1)) < 3e-6, wcfg


@pytest.mark.parametrize("H", [13, 14])
@pytest.mark.parametrize("f32", [True, False], ids=["fp32", "bf16"])
def test_strided_1x1_dgrad_zeroes_its_cells(H, f32):
    """A strided 1x1 data gradient (remap 2) writes ALL of dx: the GEMM row of dz pixel (p, q) also
    zeroes the other pixels of its 2x2 stride cell (odd H: the last cell is cut by the border), so
    the step allocates dx without a fill kernel. dx starts as NaN."""
    if f32:
        set_gpu_compute_dtype(torch.float32)
        Fn.set_f32_native(True)
    try:
        spec, p, pk, ps = _conv(64, 128, 1, 2, 0)
        N = 3
        P, Q = spec.out_hw(H, H)
        torch.manual_seed(6)
        dz = torch.randn(N, P, Q, 128, device=DEV)
        dt = torch.float32 if f32 else torch.bfloat16
        dz = dz.to(dt)
        dx = torch.full((N, H, H, 64), float("nan"), dtype=dt, device=DEV)
        Fn.conv_dgrad(dz, spec, pk.tr, p.data, dx, False)
        wd = p.data.double().cpu().permute(0, 3, 1, 2)
        if not f32:
            wd = wd.to(torch.bfloat16).double()
        xr = torch.zeros(N, 64, H, H, dtype=torch.float64, requires_grad=True)
        torch.nn.functional.conv2d(xr, wd, stride=2).backward(dz.double().cpu().permute(0, 3, 1, 2))
        ref = xr.grad.permute(0, 2, 3, 1)
        assert not torch.isnan(dx).any()
        assert float(dx[:, 1::2].abs().max()) == 0.0 and float(dx[:, :, 1::2].abs().max()) == 0.0
        assert rel_err(dx, ref) < (3e-6 if f32 else 1e-2)
    finally:
        Fn.set_f32_native(False)
        set_gpu_compute_dtype(torch.bfloat16)


@pytest.mark.parametrize("cfg", [18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 31, 32, 33, 34, 35, 36])
@pytest.mark.parametrize("shape", [(64, 256, 1, 56, 16), (256, 96, 1, 23, 5), (64, 64, 3, 30, 3), (256, 256, 3, 14, 4),
                                   (64, 40, 1, 23, 5), (256, 64, 1, 23, 5)],
                         ids=lambda c: f"{c[0]}x{c[1]}k{c[2]}H{c[3]}N{c[4]}")
def test_fp32_persistent_short_k_gemm(fp32_mode, cfg, shape):
    """The persistent plane GEMM (conv_p3_persist.h): each workgroup walks several tiles with the
    LDS-DMA ring running across tile boundaries (16 x 56 x 56 rows: 3-6 tiles per workgroup), row
    and column tails (2645 rows, 96 outputs against 64 / 128-wide tiles), a 3x3 (18 k-steps); the
    register epilogue's output, ReLU and BN statistics (shifted sums in STAT_R replicas) against
    fp64, and the deterministic mode's one-replica-per-64-rows statistics bitwise reproducible.
    cfg 23-27: the stream-K form -- equal (tile, k-step) shares per workgroup, split tiles summed
    through the workspace (256x256 3x3 at 14 x 14 x 4: 14 tiles x 72 k-steps over the grid, up to
    ~20 shares per tile), bitwise reproducible output and statistics. cfg 31-36: each workgroup's
    weight slice resident in LDS (one or several N tiles: 40 / 64 / 96 / 256 outputs, K = 64 / 256),
    the others falling back."""
    cin, cout, k, H, N = shape
    pad = k // 2
    spec, p, pk, ps = _conv(cin, cout, k, 1, pad)
    torch.manual_seed(4)
    x = torch.randn(N, H, H, cin, device=DEV)
    xd = x.double().cpu().permute(0, 3, 1, 2)
    wd = p.data.double().cpu().permute(0, 3, 1, 2)
    ref = torch.nn.functional.conv2d(xd, wd, padding=pad).permute(0, 2, 3, 1)
    M = N * H * H
    shift = (torch.randn(cout) * 0.1).to(DEV)
    R = 8
    acc = torch.zeros(R * 2 * cout, device=DEV)
    y = torch.empty(N, H, H, cout, device=DEV)
    Fn.conv_forward(x, spec, pk.pack, p.data, y, stats=acc, stats_R=R, cfg=cfg, stats_shift=shift)
    assert rel_err(y, ref) < 3e-6
    st = acc.view(R, 2, cout).double().sum(0).cpu()
    d = ref.reshape(M, cout) - shift.double().cpu()
    assert rel_err(st[0], d.sum(0)) < 1e-5 and rel_err(st[1], (d * d).sum(0)) < 1e-5
    y2 = torch.empty_like(y)
    Fn.conv_forward(x, spec, pk.pack, p.data, y2, cfg=cfg, relu=True)
    assert rel_err(y2, ref.clamp(min=0)) < 3e-6
    if cfg == 18:  # the persistent weight gradient (wgrad cfg 16-18): many (tile, split) items per workgroup
        dz = torch.randn(N, H, H, cout, device=DEV)
        xr = xd.clone().requires_grad_(True)
        wr = wd.clone().requires_grad_(True)
        torch.nn.functional.conv2d(xr, wr, padding=pad).backward(dz.double().cpu().permute(0, 3, 1, 2))
        ksteps = (M + 63) // 64
        for wc in (16, 17, 18):
            for sp in (1, max(1, ksteps // 2), 7):
                dw = torch.zeros(cout, spec.K, device=DEV)
                Fn.conv_wgrad(dz, x, spec, dw, cfg=(wc, sp))
                # (one split sums up to 50,176 rows in one fp32 chain: ~sqrt(n) * 2^-24 = 1.3e-5)
                assert rel_err(dw.view(cout, k, k, cin), wr.grad.permute(0, 2, 3, 1)) < 2e-5, (wc, sp)
    Rd = Fn.det_replicas(M)
    runs = []
    for _ in range(2):
        a = torch.zeros(Rd * 2 * cout, device=DEV)
        Fn.conv_forward(x, spec, pk.pack, p.data, y2, stats=a, stats_R=Rd, cfg=cfg, stats_shift=shift)
        runs.append((a, y2.clone()))
    assert torch.equal(runs[0][0], runs[1][0]) and torch.equal(runs[0][1], runs[1][1])


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
        img[..., :3] = (img[..., :3] - 127.0) / 60.0  # padded channels stay zero
        t = Trainer(m, 8, constant_lr(0.02))
        assert t.use_graph
        losses = [float(t.step(img, lab)) for _ in range(12)]
        assert all(l == l for l in losses)
        assert min(losses[-3:]) < 0.8 * losses[0], losses
    finally:
        Fn.set_f32_native(False)
        set_gpu_compute_dtype(torch.bfloat16)


def test_planes_split_is_exact():
    """x == hi + mid + lo for every fp32 value whose lo term is a normal number (random magnitudes
    over 2^-60..2^60, signs, zeros), and the GPU split equals the CPU split bit for bit."""
    torch.manual_seed(1)
    x = torch.randn(1000, 64) * torch.exp2(torch.randint(-60, 60, (1000, 64)).float())
    x[0, :8] = 0.0
    xg = x.to(DEV)
    pg = Fn.to_planes(xg)
    pc = Fn.to_planes(x)
    assert torch.equal(pg.t.cpu(), pc.t)
    assert torch.equal(pg.float().cpu(), x)
    y = torch.empty_like(xg)
    Fn._ext.ops().merge_planes(pg.t, 64, 1000, 64, y, 64)
    assert torch.equal(y.cpu(), x)
    # strided rows (a channel window of a wider buffer)
    wide = torch.randn(50, 96, device=DEV)
    pw = Fn.to_planes(wide[:, 16:80])
    assert torch.equal(pw.float(), wide[:, 16:80])


@pytest.mark.parametrize("relu,residual", [(True, False), (True, True), (False, False), (True, "bn")])
def test_fp32_bn_planes_match_fp32_kernels(fp32_mode, relu, residual):
    """The plane-writing BN kernels equal the fp32-output ones bit for bit after the split: forward
    apply (plain / ReLU / planes residual / fused residual BN), the backward pair (hi-plane ReLU
    mask, planes dz), and the stem's BN+ReLU+max-pool."""
    torch.manual_seed(21)
    C, N, H, R = 256, 4, 9, 8
    spec, p, pk, ps = _conv(64, C, 3, 1, 1)
    x = torch.randn(N, H, H, 64, device=DEV)
    z = torch.empty(N, H, H, C, device=DEV)
    acc_f = torch.zeros(R * 2 * C, device=DEV)
    Fn.conv_forward(x, spec, pk.pack, p.data, z, stats=acc_f, stats_R=R)
    gamma = torch.rand(C, device=DEV) + 0.5
    beta = torch.randn(C, device=DEV) * 0.1
    res = res_bn = None
    if residual is True:
        res = torch.randn(N, H, H, C, device=DEV)
    elif residual == "bn":
        res = torch.randn(N, H, H, C, device=DEV) * 3 + 1
        racc = torch.zeros(R, 2, C, device=DEV)
        rf = res.view(-1, C)
        racc[0, 0] = rf.sum(0)
        racc[0, 1] = (rf * rf).sum(0)

        def res_bn():
            return (racc, torch.ones(C, device=DEV), torch.zeros(C, device=DEV), torch.empty(C, device=DEV),
                    torch.empty(C, device=DEV), None, None, None)
    outs = []
    for planes in (False, True):
        y = Fn.Planes.empty((N, H, H, C), DEV) if planes else torch.empty_like(z)
        r = Fn.to_planes(res) if (planes and residual is True) else res
        mean, invstd = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
        Fn.bn_forward_acc(z, gamma, beta, None, None, 0.9, 1e-5, y, relu, acc_f, R, mean, invstd, residual=r,
                          res_bn=res_bn() if res_bn else None)
        outs.append((y, Fn.BNSaved(mean, invstd)))
    (y32, sv), (yp, _) = outs
    assert torch.equal(yp.t, Fn.to_planes(y32).t)
    dy = torch.randn(N, H, H, C, device=DEV)
    mode = (1 if residual else 2) if relu else 0
    dzs = []
    Fn.set_deterministic(True)  # one add per accumulator slot: the two backward runs sum identically
    for planes in (False, True):
        dz = Fn.Planes.empty((N, H, H, C), DEV) if planes else torch.empty_like(z)
        dg, db = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
        acc_b = torch.zeros(R * 2 * C, device=DEV)
        Fn.bn_backward_acc(dy, yp if planes else y32, z, sv, gamma, beta, mode, dg, db, dz, acc_b, R)
        dzs.append((dz, dg, db))
    Fn.set_deterministic(False)
    # the two kernel instantiations may contract one FMA differently: 1 ulp
    assert torch.allclose(dzs[1][0].float(), dzs[0][0], rtol=3e-7, atol=1e-7 * float(dzs[0][0].abs().max()))
    assert torch.equal(dzs[1][1], dzs[0][1]) and torch.equal(dzs[1][2], dzs[0][2])
    # stem: BN + ReLU + 3x3/2 max pool into planes
    Pp = (H + 1) // 2
    pooled = []
    for planes in (False, True):
        out = Fn.Planes.empty((N, Pp, Pp, C), DEV) if planes else torch.empty(N, Pp, Pp, C, device=DEV)
        amax = torch.empty(N, Pp, Pp, C, dtype=torch.uint8, device=DEV)
        Fn.bn_relu_maxpool_acc(z, gamma, beta, torch.zeros(C, device=DEV), torch.ones(C, device=DEV), 0.9, 1e-5,
                               acc_f, R, torch.empty(C, device=DEV), torch.empty(C, device=DEV), out, amax, 3, 3, 2,
                               2, (1, 1, 1, 1))
        pooled.append((out, amax))
    assert torch.equal(pooled[1][0].t, Fn.to_planes(pooled[0][0]).t) and torch.equal(pooled[1][1], pooled[0][1])


def test_fp32_gap_planes():
    torch.manual_seed(2)
    x = torch.randn(4, 7, 7, 2048, device=DEV)
    xp = Fn.to_planes(x)
    y = Fn.Planes.empty((4, 2048), DEV)
    Fn.gap_forward(xp, y)
    assert rel_err(y.float(), x.double().mean(dim=(1, 2))) < 2e-7


def test_fp32_model_activations_are_planes():
    """The ResNet fp32 step keeps its GEMM operands as planes end to end: no fp32 -> plane split
    launch inside the step (the producers write planes; the input image is split by the stem's
    space-to-depth fold itself, stem_s2d_f32_kernel) except the classifier's tiny dlogits."""
    m = create_model("resnet50", image_size=64, device=DEV, compute_dtype="fp32", seed=3)
    try:
        img, lab = synthetic_batch(m, 4)
        calls = []
        real = Fn.to_planes

        def spy(t):
            if not Fn.is_planes(t):
                calls.append(tuple(t.shape))
            return real(t)

        Fn.to_planes = spy
        try:
            t = Trainer(m, 4, constant_lr(0.01), use_graph=False)
            t.step(img, lab)
        finally:
            Fn.to_planes = real
        # the classifier's dlogits (tiny) is the only split
        assert calls == [(4, m.fc.ld)], calls
    finally:
        Fn.set_f32_native(False)
        set_gpu_compute_dtype(torch.bfloat16)


@pytest.mark.parametrize("mode", [0, 1, 2])
# (a strided 1x1 data gradient visits only the strided pixels: the models never fuse into it)
@pytest.mark.parametrize("case", [(256, 64, 1, 1, 0, 14, False), (64, 64, 3, 1, 1, 14, True),
                                  (128, 256, 1, 1, 0, 7, True), (128, 128, 3, 2, 1, 14, False)],
                         ids=lambda c: f"{c[0]}x{c[1]}k{c[2]}s{c[3]}acc{int(c[6])}")
def test_fp32_fused_bn_backward_matches_unfused(fp32_mode, case, mode):
    """conv_p3_bnb: the fp32 data-grad GEMM with the consuming BN's backward reduction fused into its
    epilogue stores g = dx * relu_mask (mask from the hi plane of y, or recomputed from z) and adds
    sum(g), sum(g * xhat) -- against the unfused GEMM plus an fp64 reduction."""
    cin, cout, k, s, pad, H, accumulate = case
    spec, p, pk, ps = _conv(cin, cout, k, s, pad)
    torch.manual_seed(7)
    N = 4
    P, Q = spec.out_hw(H, H)
    dz = Fn.to_planes(torch.randn(N, P, Q, cout, device=DEV))
    z = torch.randn(N, H, H, cin, device=DEV) * 1.5 + 0.2
    mean, invstd = torch.randn(cin, device=DEV) * 0.1, torch.rand(cin, device=DEV) + 0.5
    gamma, beta = torch.rand(cin, device=DEV) + 0.5, torch.randn(cin, device=DEV) * 0.1
    yf = torch.relu(torch.randn(N, H, H, cin, device=DEV))
    y = Fn.to_planes(yf)
    base = torch.randn(N, H, H, cin, device=DEV) if accumulate else None
    dx_u = base.clone() if accumulate else torch.zeros(N, H, H, cin, device=DEV)
    Fn.conv_dgrad(dz, spec, pk.tr, p.data, dx_u, accumulate)
    R = 8
    acc = torch.zeros(R, 2, cin, device=DEV)
    dx_f = base.clone() if accumulate else torch.zeros(N, H, H, cin, device=DEV)
    bnb = Fn.BNBwdFuse(z, y, Fn.BNSaved(mean, invstd), gamma, beta, mode, acc, R)
    Fn.conv_dgrad(dz, spec, pk.tr, p.data, dx_f, accumulate, bnb=bnb)
    g = dx_u.double()
    if mode == 1:
        g = g * (yf > 0).double()
    elif mode == 2:
        xh = (z.double() - mean.double()) * invstd.double()
        g = g * ((xh * gamma.double() + beta.double()) > 0).double()
    assert rel_err(dx_f, g) < 1e-6
    xhat = ((z.double() - mean.double()) * invstd.double()).view(-1, cin)
    s1 = g.view(-1, cin).sum(0)
    s2 = (g.view(-1, cin) * xhat).sum(0)
    a = acc.double().sum(0)
    assert rel_err(a[0], s1) < 1e-5 and rel_err(a[1], s2) < 1e-5


@pytest.mark.parametrize("cfg", [18, 19, 20, 21, 22, 23])
@pytest.mark.parametrize("case", [(96, 64, 1, 23, 5, False), (64, 64, 3, 30, 3, True), (256, 128, 1, 14, 4, True)],
                         ids=lambda c: f"{c[0]}x{c[1]}k{c[2]}H{c[3]}N{c[4]}acc{int(c[5])}")
def test_fp32_persistent_fused_bn_backward(fp32_mode, cfg, case):
    """The persistent plane GEMM's BNB register epilogue (conv_p3_persist.h, a fused BN-backward data
    gradient walking several tiles per workgroup; cfg 23 -- stream-K -- falls back to it): g for
    modes 0 / 1 / 2 with and without the beta source, row tails (2645 rows) and a 96-column tail,
    sum(g) / sum(g * xhat) against fp64, and the deterministic replicas bitwise reproducible."""
    cin, cout, k, H, N, accumulate = case
    pad = k // 2
    spec, p, pk, ps = _conv(cin, cout, k, 1, pad)
    torch.manual_seed(11)
    dzf = torch.randn(N, H, H, cout, device=DEV)
    dz = Fn.to_planes(dzf)
    wd = p.data.double().cpu().permute(0, 3, 1, 2)
    xr = torch.zeros(N, cin, H, H, dtype=torch.float64, requires_grad=True)
    torch.nn.functional.conv2d(xr, wd, padding=pad).backward(dzf.double().cpu().permute(0, 3, 1, 2))
    ref = xr.grad.permute(0, 2, 3, 1)
    z = torch.randn(N, H, H, cin, device=DEV) * 1.5 + 0.2
    mean, invstd = torch.randn(cin, device=DEV) * 0.1, torch.rand(cin, device=DEV) + 0.5
    gamma, beta = torch.rand(cin, device=DEV) + 0.5, torch.randn(cin, device=DEV) * 0.1
    yf = torch.relu(torch.randn(N, H, H, cin, device=DEV))
    y = Fn.to_planes(yf)
    base = torch.randn(N, H, H, cin, device=DEV) if accumulate else None
    M = N * H * H
    xh = ((z.double() - mean.double()) * invstd.double()).cpu()
    Fn.set_p3p_bnb(2)  # every mode on the persistent kernel (the default, 0, runs the twin)
    for mode in (0, 1, 2):
        g = ref + (base.double().cpu() if accumulate else 0)
        if mode == 1:
            g = g * (yf.cpu() > 0).double()
        elif mode == 2:
            g = g * ((xh * gamma.double().cpu() + beta.double().cpu()) > 0).double()
        R = 8
        acc = torch.zeros(R, 2, cin, device=DEV)
        dx = base.clone() if accumulate else torch.zeros(N, H, H, cin, device=DEV)
        bnb = Fn.BNBwdFuse(z, y, Fn.BNSaved(mean, invstd), gamma, beta, mode, acc, R)
        Fn.conv_dgrad(dz, spec, pk.tr, p.data, dx, accumulate, cfg=(cfg, 1), bnb=bnb)
        assert rel_err(dx, g) < 3e-6, mode
        a = acc.double().sum(0).cpu()
        assert rel_err(a[0], g.reshape(-1, cin).sum(0)) < 1e-5, mode
        assert rel_err(a[1], (g.reshape(-1, cin) * xh.reshape(-1, cin)).sum(0)) < 1e-5, mode
    Rd = Fn.det_replicas(M)
    runs = []
    for _ in range(2):
        a = torch.zeros(Rd, 2, cin, device=DEV)
        dx = base.clone() if accumulate else torch.zeros(N, H, H, cin, device=DEV)
        Fn.conv_dgrad(dz, spec, pk.tr, p.data, dx, accumulate, cfg=(cfg, 1),
                      bnb=Fn.BNBwdFuse(z, y, Fn.BNSaved(mean, invstd), gamma, beta, 2, a, Rd))
        runs.append((a, dx))
    Fn.set_p3p_bnb(0)
    assert torch.equal(runs[0][0], runs[1][0]) and torch.equal(runs[0][1], runs[1][1])
