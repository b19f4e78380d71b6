"""Loss scaling (tf_cnn_benchmarks --use_fp16 / --fp16_loss_scale / --fp16_enable_auto_loss_scale):
static scaling must not change the update; an Inf/NaN gradient must skip the step and halve
the dynamic scale; clean steps double it after the interval. CPU path (the GPU ops are the
same math: tests/test_kernels_gpu.py::test_loss_scale_ops_gpu)."""
import torch

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.ops import functional as Fn
from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch


def _train(loss_scale=None, dynamic=False, steps=2):
    m = create_model("trivial", image_size=32, device="cpu", seed=5)
    img, lab = synthetic_batch(m, 4, seed=1)
    img = (img - 127) / 60
    t = Trainer(m, 4, constant_lr(0.05), loss_scale=loss_scale, dynamic_loss_scale=dynamic)
    for _ in range(steps):
        t.step(img, lab)
    return m, t


def test_static_loss_scale_is_transparent():
    m0, _ = _train()
    m1, t1 = _train(loss_scale=256.0)
    assert torch.allclose(m0.ps.master, m1.ps.master, rtol=1e-4, atol=1e-6)
    assert float(t1.hyper[5]) == 256.0 and abs(float(t1.hyper[3]) - 1 / 256.0) < 1e-12


def test_overflow_skips_step_and_halves_dynamic_scale():
    h = torch.tensor([0.1, 0.9, 0.0, 1.0 / 1024, 0.0, 1024.0, 5.0, 1000.0])
    w = torch.ones(8)
    mom = torch.zeros(8)
    g = torch.ones(8)
    g[3] = float("inf")
    Fn.nonfinite(g, h[4:5])
    assert float(h[4]) == 1.0
    Fn.sgd_momentum(w, mom, g, 0, h)
    assert torch.equal(w, torch.ones(8)) and torch.equal(mom, torch.zeros(8))  # skipped
    Fn.loss_scale_update(h, 1, True)
    assert float(h[5]) == 512.0 and float(h[6]) == 0.0 and abs(float(h[3]) - 1 / 512.0) < 1e-12


def test_dynamic_scale_grows_after_clean_interval():
    h = torch.tensor([0.1, 0.9, 0.0, 1.0 / 8, 0.0, 8.0, 0.0, 3.0])
    for _ in range(3):
        h[4] = 0.0
        Fn.loss_scale_update(h, 2, True)
    assert float(h[5]) == 16.0 and abs(float(h[3]) - 1 / 32.0) < 1e-12


def test_dynamic_training_runs_and_matches_unscaled():
    m0, _ = _train()
    m1, t1 = _train(dynamic=True)
    assert torch.allclose(m0.ps.master, m1.ps.master, rtol=1e-4, atol=1e-6)
    assert float(t1.hyper[4]) == 0.0
