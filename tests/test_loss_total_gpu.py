"""Fused step-loss kernel (csrc/kernels/misc.hip loss_total_kernel) vs the PyTorch fp32 expression it
replaces in the trainer: mean(row_loss) + 0.5 * wd * l2 (tf_cnn_benchmarks' total_loss)."""
import pytest
import torch

from azure_hc_intel_tf_amd.ops import functional as Fn


@pytest.mark.gpu
@pytest.mark.parametrize("B", [1, 7, 64, 256, 1000])
@pytest.mark.parametrize("with_l2", [False, True])
def test_loss_total_matches_torch(B, with_l2):
    g = torch.Generator().manual_seed(B)
    row = (torch.rand(B + 5, generator=g) * 8).cuda()  # tail past B must be ignored
    l2 = torch.tensor([123.456]).cuda() if with_l2 else None
    out = torch.full((1,), float("nan")).cuda()
    Fn.loss_total(row, B, l2, 0.5 * 1e-4, out)
    torch.cuda.synchronize()
    ref = row[:B].double().mean() + (0.5 * 1e-4 * 123.456 if with_l2 else 0.0)
    assert abs(out.item() - ref.item()) <= 1e-6 * abs(ref.item()) + 1e-7


def test_loss_total_cpu():
    row = torch.arange(10, dtype=torch.float32)
    out = torch.zeros(1)
    Fn.loss_total(row, 8, torch.tensor([2.0]), 0.25, out)
    assert out.item() == pytest.approx(3.5 + 0.5)
    Fn.loss_total(row, 4, None, 0.0, out)
    assert out.item() == pytest.approx(1.5)
