"""Reference-precision compute modes on the GPU. fp32 is the reference's precision
(run-tf-sing-ucx-openmpi.sh:62-81 passes no --use_fp16) and the default of create_model on every
device: every model of the zoo runs it on the HIP kernels (bf16x6 plane GEMMs, fp32 BN / pool;
kernel checks in test_fp32_native_gpu.py, models in test_fp32_zoo_gpu.py / test_fp32_inception_gpu.py
/ test_fp32_resnet_v2_gpu.py). The PyTorch path (MIOpen / rocBLAS) of ops/functional.py is only the
comparison arm (HCB_F32_NATIVE=0, or F32_NATIVE_OK patched off as below) -- as is IEEE fp16 with
Fn.F16_NATIVE off (the default fp16 mode runs the HIP kernels: test_fp16_native_gpu.py)."""
import pytest
import torch

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch

pytestmark = pytest.mark.gpu


def test_fp32_gpu_matches_fp32_cpu_step():
    """One fp32 training step on the GPU (HIP kernels: bf16x6 GEMMs) equals the fp32 CPU step:
    the loss to fp32 tolerance, the gradient as a whole (direction and norm)."""
    kw = dict(image_size=64, seed=7, image_channels=8)
    mg = create_model("resnet50", device="cuda", compute_dtype="fp32", **kw)
    mc = create_model("resnet50", device="cpu", **kw)
    assert mg.native and mg.image_channels == 8
    assert torch.equal(mg.ps.master.cpu(), mc.ps.master)
    img_c, lab_c = synthetic_batch(mc, 4, seed=3)
    img_c[..., :3] = (img_c[..., :3] - 127.0) / 60.0  # the padded channels stay zero (the S2D stem's contract)
    tg = Trainer(mg, 4, constant_lr(0.05))
    tc = Trainer(mc, 4, constant_lr(0.05))
    lg = float(tg.step(img_c.cuda(), lab_c.cuda()))
    lc = float(tc.step(img_c, lab_c))
    torch.cuda.synchronize()
    assert abs(lg - lc) <= 1e-4 * abs(lc), (lg, lc)
    # whole-network gradients of a random-init BN net are chaotic in the rounding order
    # (bf16x6 MFMA vs oneDNN accumulation): compared as a whole, not elementwise. Measured floor of
    # this configuration on the CPU alone: fp32 vs fp64 2.9%, fp32 vs fp32 with the input scaled by
    # (1 + 1e-7) 2.7% (the GPU step lands at ~3.6%)
    gg, gc = mg.ps.grad.cpu(), mc.ps.grad
    assert (gg - gc).norm() / gc.norm() < 5e-2
    assert float(gg @ gc / (gg.norm() * gc.norm())) > 0.999


@pytest.mark.parametrize("dtype", ["fp32", "fp16"])
def test_reference_precision_training_learns(dtype, monkeypatch):
    """The PyTorch (MIOpen) path: ResNet-50 with the fp32 / fp16 HIP paths switched off."""
    from azure_hc_intel_tf_amd.models.resnet import ResNet
    from azure_hc_intel_tf_amd.ops import functional as Fn

    monkeypatch.setattr(Fn, "F16_NATIVE", False)  # fp16 through MIOpen, not the fp16 kernel build
    monkeypatch.setattr(ResNet, "F32_NATIVE_OK", False)  # fp32 through MIOpen, not bf16x6
    torch.manual_seed(0)
    m = create_model("resnet50", image_size=64, device="cuda", compute_dtype=dtype)
    assert not m.native
    img, lab = synthetic_batch(m, 8)
    assert img.dtype == {"fp32": torch.float32, "fp16": torch.float16}[dtype]
    img = (img.float() - 127.0).div(60.0).to(img.dtype)
    # (lr 0.02 on this 8-image batch occasionally diverged after learning on the fp16 MIOpen path:
    # 6.99 -> 3.20 by step 3, then 10.9 at step 9; 0.01 learns as fast without the overshoot)
    t = Trainer(m, 8, constant_lr(0.01), dynamic_loss_scale=(dtype == "fp16"))
    losses = [float(t.step(img, lab)) for _ in range(12)]
    assert all(l == l for l in losses)
    assert min(losses[-3:]) < 0.8 * losses[0], losses


def test_bf16_and_fp32_models_coexist():
    """A bf16 (HIP) and an fp32 (reference) GPU model in one process keep their own
    activation dtypes."""
    a = create_model("resnet50", image_size=64, device="cuda", compute_dtype="fp32")
    b = create_model("resnet50", image_size=64, device="cuda", compute_dtype="bf16")
    assert b.native and b.act_dtype == torch.bfloat16 and a.act_dtype == torch.float32
