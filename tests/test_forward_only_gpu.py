"""``--forward_only`` (tf_cnn_benchmarks' phase_train=False: BN from the moving statistics) on the
hand-written kernels at fp32 -- the default precision -- and bf16: the GPU logits against the CPU
logits of the same weights and moving statistics. At fp32 the inference BN is the training apply
kernel (bn_apply_acc, fp32 z / out) fed the moving statistics as one replica of shifted sums
(ops/functional.py bn_inference); the conv operands are split into planes as in training."""
import pytest
import torch

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.nn.layers import set_gpu_compute_dtype
from azure_hc_intel_tf_amd.ops import functional as Fn
from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch

pytestmark = pytest.mark.gpu


def _reset():
    Fn.set_f32_native(False)
    set_gpu_compute_dtype(torch.bfloat16)


def _bn_layers(m):
    todo, out = list(m.all_layers()), []
    while todo:
        l = todo.pop()
        if hasattr(l, "layers") and callable(l.layers):
            todo += l.layers()
        if hasattr(l, "rmean") and hasattr(l, "rvar"):
            out.append(l)
    return out


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("name,size", [("resnet50", 64), ("resnet50_v2", 64), ("inception3", 75)])
def test_forward_only_gpu_logits_match_cpu(name, size, dtype):
    kw = dict(image_size=size, seed=11, image_channels=8)
    try:
        mg = create_model(name, device="cuda", compute_dtype=dtype, **kw)
        mc = create_model(name, device="cpu", **kw)
        assert mg.native
        assert torch.equal(mg.ps.master.cpu(), mc.ps.master)
        g = torch.Generator().manual_seed(5)
        lg_, lc_ = _bn_layers(mg), _bn_layers(mc)
        assert len(lg_) == len(lc_) > 0
        for a, b in zip(lg_, lc_):  # non-trivial moving statistics, the same on both
            b.rmean.data.copy_(torch.randn(b.rmean.data.shape, generator=g) * 0.1)
            b.rvar.data.copy_(torch.rand(b.rvar.data.shape, generator=g) * 1.5 + 0.5)
            a.rmean.data.copy_(b.rmean.data)
            a.rvar.data.copy_(b.rvar.data)
        img_c, lab_c = synthetic_batch(mc, 4, seed=3)
        img_c[..., :3] = (img_c[..., :3] - 127.0) / 60.0
        tg = Trainer(mg, 4, constant_lr(0.0), forward_only=True, use_graph=False)
        tc = Trainer(mc, 4, constant_lr(0.0), forward_only=True)
        img_g = img_c.to("cuda", mg.act_dtype)
        tg.step(img_g, lab_c.cuda())
        tc.step(img_c, lab_c)
        torch.cuda.synchronize()
        out_g = Fn.from_planes(tg.logits).float().cpu()
        out_c = Fn.from_planes(tc.logits).float()
        rel = ((out_g - out_c).norm() / out_c.norm()).item()
        assert rel < (1e-4 if dtype == "fp32" else 5e-2), rel
        # moving statistics untouched by the inference passes
        for a, b in zip(lg_, lc_):
            assert torch.equal(a.rmean.data.cpu(), b.rmean.data) and torch.equal(a.rvar.data.cpu(), b.rvar.data)
    finally:
        _reset()
