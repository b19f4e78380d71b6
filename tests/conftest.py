import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs via gpurun)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(autouse=True)
def _default_gpu_compute_dtype():
    """Every test starts with the default (bf16 HIP-kernel) GPU activation dtype; models of the
    reference-precision mode switch it while they step."""
    import torch

    from azure_hc_intel_tf_amd.nn.layers import set_gpu_compute_dtype

    set_gpu_compute_dtype(torch.bfloat16)
    yield


def gpu_available():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
