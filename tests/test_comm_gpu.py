"""Native C++ RCCL engine on one MI355X (a 1-rank communicator: RCCL refuses two ranks on
one GPU; multi-rank semantics are covered on CPU/gloo by tests/test_hvd_dist.py)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_native_comm_one_rank(tmp_path, monkeypatch):
    monkeypatch.setenv("HOROVOD_TIMELINE", str(tmp_path / "timeline.json"))
    from azure_hc_intel_tf_amd.parallel.native import Communicator, NativeReducer, rccl_version

    assert rccl_version() >= 22000
    c = Communicator()
    t = torch.arange(1000, dtype=torch.float32, device="cuda")
    c.allreduce_(t)
    c.broadcast_(t, 0)
    out = torch.empty(1000, device="cuda")
    c.allgather_(t, out)
    torch.cuda.synchronize()
    assert torch.equal(out, torch.arange(1000, dtype=torch.float32, device="cuda"))
    flat = torch.randn(300_000, device="cuda")
    ref = flat.clone()
    buckets = torch.tensor([[200_000, 100_000], [0, 200_000]], dtype=torch.int64)
    c.bucket_allreduce_(flat, buckets, 0, 1.0, False)
    torch.cuda.synchronize()
    assert torch.equal(flat, ref)
    c.bucket_allreduce_(flat, buckets, 1, 1.0, False)  # bf16 wire format
    torch.cuda.synchronize()
    assert torch.allclose(flat, ref.bfloat16().float())
    c.barrier()
    c.close()
    assert (tmp_path / "timeline.json").read_text().strip().startswith("[")
    r = NativeReducer(compression="bf16", bucket_bytes=1 << 20)
    g = torch.randn(1_000_003, device="cuda")
    g0 = g.clone()
    r.allreduce_(g)
    torch.cuda.synchronize()
    assert torch.allclose(g, g0.bfloat16().float())
    r.close()


def test_native_async_range_allreduce_overlap_one_rank():
    """the overlap interface: async range reductions forked off the compute stream, one join"""
    from azure_hc_intel_tf_amd.parallel.native import NativeReducer

    r = NativeReducer(compression="bf16")
    g = torch.randn(500_000, device="cuda")
    g0 = g.clone()
    r.allreduce_ranges_async_(g, [(300_000, 200_000)])
    g[:1000].mul_(2.0)  # compute-stream work between the two hand-offs
    r.allreduce_ranges_async_(g, [(0, 100_000), (100_000, 200_000)])
    r.join()
    torch.cuda.synchronize()
    ref = g0.clone()
    ref[:1000] *= 2.0
    assert torch.allclose(g, ref.bfloat16().float())
    r.close()
