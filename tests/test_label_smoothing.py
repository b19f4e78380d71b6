"""--label_smoothing (tf_cnn_benchmarks: tf.losses.softmax_cross_entropy with targets
(1 - ls) * onehot + ls / num_classes): the loss + dlogits of ops/functional.py softmax_xent against
torch's cross_entropy(label_smoothing=) and its autograd gradient -- the CPU path here, the HIP kernel
(fp32 and bf16 dlogits) on the GPU."""
import pytest
import torch
import torch.nn.functional as F

from azure_hc_intel_tf_amd.ops import functional as Fn


def _reference(logits, labels, ncls, ls):
    lg = logits[:, :ncls].double().clone().requires_grad_(True)
    loss = F.cross_entropy(lg, labels, label_smoothing=ls, reduction="none")
    loss.sum().backward()
    return loss.detach(), lg.grad  # d(sum of rows)/dlogits = softmax - target


def _check(dev, ls, dl_dtype, tol):
    g = torch.Generator().manual_seed(int(ls * 100) + 1)
    B, ncls, ldl = 8, 1001, 1008
    logits = torch.randn(B, ldl, generator=g) * 3
    labels = torch.randint(0, ncls, (B,), generator=g)
    rl = torch.empty(B, device=dev)
    dl = torch.zeros(B, ldl, dtype=dl_dtype, device=dev)
    Fn.softmax_xent(logits.to(dev), labels.to(dev), ncls, rl, dl, 1.0, label_smoothing=ls)
    ref_loss, ref_grad = _reference(logits, labels, ncls, ls)
    assert torch.allclose(rl.double().cpu(), ref_loss, rtol=1e-5, atol=1e-5), (rl.cpu(), ref_loss)
    err = (dl.double().cpu()[:, :ncls] - ref_grad).abs().max().item()
    assert err < tol, err
    assert dl.cpu()[:, ncls:].abs().max().item() == 0


@pytest.mark.parametrize("ls", [0.0, 0.1, 0.5])
def test_label_smoothing_cpu_matches_torch(ls):
    _check("cpu", ls, torch.float32, 1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("dl_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("ls", [0.0, 0.1, 0.5])
def test_label_smoothing_kernel_matches_torch(ls, dl_dtype):
    from azure_hc_intel_tf_amd.ops import _ext

    _ext.load()
    _check("cuda", ls, dl_dtype, 1e-5 if dl_dtype == torch.float32 else 4e-3)


def test_label_smoothing_flag_reaches_the_trainer():
    from azure_hc_intel_tf_amd.bench.flags import parse_flags

    assert parse_flags(["--label_smoothing=0.1"]).label_smoothing == 0.1
