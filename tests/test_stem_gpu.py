"""Space-to-depth ResNet stem (csrc/kernels/stem.hip + nn/layers.StemS2D) against the plain fp32
7x7/2 convolution: forward output, folded-weight consistency and the weight gradient mapped
back into the 7x7 master layout."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _stem(size):
    from azure_hc_intel_tf_amd.nn.layers import StemS2D
    from azure_hc_intel_tf_amd.nn.params import ParamStore

    ps = ParamStore(seed=3)
    st = StemS2D(ps, "conv0", (size, size, 8), 64, relu=True, need_dx=False, logical_cin=3)
    ps.finalize(torch.device("cuda"))
    return st, ps


@pytest.mark.parametrize("size,cfg", [(224, None), (64, None), (30, None), (64, 4), (64, 11), (64, 16), (64, 7)],
                         ids=str)
def test_s2d_forward_matches_direct_conv(size, cfg):
    import azure_hc_intel_tf_amd.ops.functional as Fn

    st, ps = _stem(size)
    torch.manual_seed(0)
    x = torch.zeros(4, size, size, 8, device="cuda")
    x[..., :3] = torch.randn(4, size, size, 3, device="cuda")
    x = x.bfloat16()
    P, Q, C = st.out_shape
    z = torch.empty(4, P, Q, C, device="cuda", dtype=torch.bfloat16)
    xf = st.fold_input(x)
    Fn.conv_forward(xf, st.fold_spec, st._folded_weight(x.device), st.w.data, z, cfg=cfg)
    w = st.w.data[..., :3].permute(0, 3, 1, 2).float().cpu()
    ref = F.conv2d(x[..., :3].permute(0, 3, 1, 2).float().cpu(), w.bfloat16().float(), stride=2, padding=3)
    got = z.float().permute(0, 3, 1, 2).cpu()
    assert got.shape == ref.shape
    err = (got - ref).abs().max() / ref.abs().max()
    assert err < 1e-2, float(err)


def test_s2d_weight_gradient_maps_back_to_7x7():
    st, ps = _stem(64)
    torch.manual_seed(1)
    x = torch.zeros(2, 64, 64, 8, device="cuda")
    x[..., :3] = torch.randn(2, 64, 64, 3, device="cuda")
    x = x.bfloat16()
    P, Q, C = st.out_shape
    dz = torch.randn(2, P, Q, C, device="cuda").bfloat16()
    st.w.grad.zero_()
    st._wgrad(dz, st.fold_input(x))
    torch.cuda.synchronize()
    ref = torch.nn.grad.conv2d_weight(x[..., :3].permute(0, 3, 1, 2).float().cpu(), (64, 3, 7, 7),
                                      dz.permute(0, 3, 1, 2).float().cpu(), stride=2, padding=3)
    got = st.w.grad[..., :3].permute(0, 3, 1, 2).cpu()
    err = (got - ref).abs().max() / ref.abs().max()
    assert err < 1e-2, float(err)
    assert torch.all(st.w.grad[..., 3:] == 0), "padded input channels must get no gradient"


@pytest.fixture
def fp32_stem():
    from azure_hc_intel_tf_amd.nn.layers import StemS2D, set_gpu_compute_dtype
    from azure_hc_intel_tf_amd.nn.params import ParamStore
    import azure_hc_intel_tf_amd.ops.functional as Fn

    set_gpu_compute_dtype(torch.float32)
    Fn.set_f32_native(True)
    ps = ParamStore(seed=3)
    st = StemS2D(ps, "conv0", (64, 64, 8), 64, relu=True, need_dx=False, logical_cin=3)
    ps.finalize(torch.device("cuda"), pack_lo=True)
    ps.repack()
    yield st
    Fn.set_f32_native(False)
    set_gpu_compute_dtype(torch.bfloat16)


@pytest.mark.parametrize("cfg", [None, 14, 7, 16, 10, 4], ids=str)
def test_s2d_fp32_planes_match_fp64(fp32_stem, cfg):
    """fp32 path: the image split into planes and folded (three planes as one 3N batch), the folded
    weight as planes, the bf16x6 plane GEMM over 64-channel row windows (fold_spec: a 4x1 conv whose
    pixel stride, 16, is below its channel count) -- forward (every tile shape class) and weight
    gradient (the tuned plan and the candidate tiles) to fp32 accuracy."""
    import azure_hc_intel_tf_amd.ops.functional as Fn

    st = fp32_stem
    assert st.fold_spec.cin_pad == 64 and st.fold_spec.kh * st.fold_spec.kw == 4
    torch.manual_seed(2)
    x = torch.zeros(2, 64, 64, 8, device="cuda")
    x[..., :3] = torch.randn(2, 64, 64, 3, device="cuda")
    P, Q, C = st.out_shape
    xf = st.fold_input(x)
    assert Fn.is_planes(xf)
    z = torch.empty(2, P, Q, C, device="cuda")
    Fn.conv_forward(xf, st.fold_spec, st._folded_weight(x.device), st.w.data, z, cfg=cfg)
    xd = x[..., :3].permute(0, 3, 1, 2).double().cpu()
    wd = st.w.data[..., :3].permute(0, 3, 1, 2).double().cpu()
    ref = F.conv2d(xd, wd, stride=2, padding=3)
    got = z.permute(0, 3, 1, 2).double().cpu()
    assert ((got - ref).norm() / ref.norm()).item() < 3e-6
    dz = torch.randn(2, P, Q, C, device="cuda")
    gref = torch.nn.grad.conv2d_weight(xd, (64, 3, 7, 7), dz.permute(0, 3, 1, 2).double().cpu(), stride=2, padding=3)
    st.w.grad.zero_()
    st._wgrad(Fn.to_planes(dz), xf)
    torch.cuda.synchronize()
    g = st.w.grad[..., :3].permute(0, 3, 1, 2).double().cpu()
    assert ((g - gref).norm() / gref.norm()).item() < 3e-6
    if cfg is None:  # the weight-gradient tiles over the row windows, split-K included
        fs = st.fold_spec
        per_tile = {}
        for c, sp in Fn.wgrad_p3_candidates(C, fs.K, 2 * P * Q):
            per_tile[c] = (c, sp)  # each tile class with its largest split
        for wcfg in per_tile.values():
            dwf = torch.zeros(C, fs.K, device="cuda")
            Fn.conv_wgrad(Fn.to_planes(dz), xf, fs, dwf, cfg=tuple(wcfg))
            st.w.grad.zero_()
            Fn._ext.ops().stem_wgrad_unfold(dwf, st.w.grad)
            g = st.w.grad[..., :3].permute(0, 3, 1, 2).double().cpu()
            assert ((g - gref).norm() / gref.norm()).item() < 3e-6, wcfg


def test_resnet_uses_s2d_stem_and_trains():
    from azure_hc_intel_tf_amd.models import create_model
    from azure_hc_intel_tf_amd.nn.layers import StemS2D
    from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch

    torch.manual_seed(0)
    m = create_model("resnet50", image_size=96, device="cuda", compute_dtype="bf16")
    assert isinstance(m.stem, StemS2D)
    img, lab = synthetic_batch(m, 16)
    t = Trainer(m, 16, constant_lr(0.02), use_graph=True, graph_warmup=2)
    # 24 steps: the bf16 loss sits on a ~3.3 plateau for a few steps before it falls again, and how
    # long depends on the summation order of the kernels earlier tests' autotuning picked in this
    # process (16 steps: passes alone and after the forward-only tests, 2.80 vs 0.8 * 3.36 once in
    # the full GPU tier)
    losses = [float(t.step(img, lab)) for _ in range(24)]
    assert all(l == l for l in losses) and min(losses[-4:]) < 0.8 * losses[2], losses
