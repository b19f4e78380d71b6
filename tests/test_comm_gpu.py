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


@pytest.mark.parametrize("model_name", ["resnet50", "inception3"])
def test_segmented_overlap_step_matches_single_graph(model_name):
    """The multi-GPU training step (one graph per backward segment, each segment's gradient
    ranges handed to the C++ RCCL engine asynchronously, join, optimizer graph) on a forced
    1-rank communicator must train like the single-graph step: the same losses up to the
    GPU's run-to-run noise (fp32 atomics in the fused BN statistics reorder between runs,
    ~0.3% on the first loss at this tiny batch), and the segments' gradient ranges must
    cover the flat gradient buffer exactly once."""
    from azure_hc_intel_tf_amd.models import create_model
    from azure_hc_intel_tf_amd.parallel.native import NativeReducer
    from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch

    size = 96 if model_name == "resnet50" else 139
    runs = []
    for seg in (False, True):
        torch.manual_seed(0)
        m = create_model(model_name, image_size=size, device="cuda")
        img, lab = synthetic_batch(m, 8)
        red = NativeReducer(force=True) if seg else None
        t = Trainer(m, 8, constant_lr(0.002), reducer=red, world_size=1, use_graph=True, graph_warmup=2,
                    force_overlap=seg)
        # no host sync between steps (as in bench.py): losses are traced device-side
        tr = torch.zeros(8, device="cuda")
        for i in range(8):
            tr[i:i + 1].copy_(t.step(img, lab))
        losses = tr.tolist()
        if seg:
            # collectives captured in the step graph: one graph, >= 2 segments reduced in it
            assert t._g_all is not None and t._segs is None and len(t._seg_ranges) >= 2
            cover = torch.zeros(m.ps.grad.numel(), dtype=torch.int32)
            for rng in t._seg_ranges.values():
                for off, n in rng:
                    cover[off:off + n] += 1
            # every gradient exactly once (the buffer carries alignment padding between tensors)
            assert int(cover.max()) == 1 and int(cover.sum()) >= m.num_params() - 64
            red.close()
        else:
            assert t._g_all is not None
        runs.append(losses)
    a, b = torch.tensor(runs[0]), torch.tensor(runs[1])
    assert torch.isfinite(b).all()
    assert torch.allclose(a[:4], b[:4], rtol=3e-2, atol=3e-2), (runs[0], runs[1])
    assert b[-1] < 0.9 * b[0] and a[-1] < 0.9 * a[0], (runs[0], runs[1])
