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
    1-rank communicator must train EXACTLY like the single-graph step: both run in deterministic
    mode (no split-K, one accumulator replica per tile), where the 1-rank reduction is the
    identity, so losses and master weights are compared bitwise -- a segment reduced before all
    of its gradients were written would show up here (no tolerance that could absorb
    a partial race). The segments' gradient ranges must cover the flat gradient buffer exactly once."""
    from azure_hc_intel_tf_amd.models import create_model
    from azure_hc_intel_tf_amd.ops import functional as Fn
    from azure_hc_intel_tf_amd.parallel.native import NativeReducer
    from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch

    size = 96 if model_name == "resnet50" else 139
    runs, masters = [], []
    Fn.set_deterministic(True)
    try:
        for seg in (False, True):
            torch.manual_seed(0)
            m = create_model(model_name, image_size=size, device="cuda", compute_dtype="bf16")
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
            masters.append(m.ps.master.detach().cpu().clone())
    finally:
        Fn.set_deterministic(False)
    a, b = torch.tensor(runs[0]), torch.tensor(runs[1])
    assert torch.isfinite(b).all()
    assert torch.equal(a, b), (runs[0], runs[1])
    assert torch.equal(masters[0], masters[1])
    assert b[-1] < 0.9 * b[0], runs[1]


def _xgmi_worker(rank, world, port, q):
    import os

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)  # every rank on the one GPU of the box: IPC maps within the device
    from azure_hc_intel_tf_amd.parallel.xgmi import XgmiAllreduce

    x = XgmiAllreduce(capacity_bytes=1 << 20)
    ok = True
    for it, n in enumerate([1, 7, 4096, 100_003, 262_144, 5, 65_536]):  # > 2 epochs per slot
        t = torch.arange(n, dtype=torch.float32, device="cuda") * (rank + 1) + it
        x.allreduce_(t, average=(it % 2 == 1))
        ref = torch.arange(n, dtype=torch.float32, device="cuda") * sum(range(1, world + 1)) + it * world
        if it % 2 == 1:
            ref /= world
        torch.cuda.synchronize()
        ok = ok and torch.allclose(t, ref, rtol=1e-6, atol=1e-3)
    err = x.error()
    x.close()
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, bool(ok), err))


@pytest.mark.parametrize("world", [2, 3])
def test_xgmi_one_shot_allreduce_two_processes_one_gpu(world):
    """The IPC one-shot allreduce protocol (publish / bounded wait / system-scope reads, slot
    alternation across epochs, in-place, average) with `world` processes sharing the GPU."""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_xgmi_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    try:
        res = [q.get(timeout=100) for _ in range(world)]
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert all(ok and err == 0 for _, ok, err in res), res


def test_fp16_wire_and_threshold_split_one_rank():
    """IEEE fp16 wire format (Horovod Compression.fp16) through the engine, every range cut
    into buckets of at most the fusion threshold, and the rank count read back from RCCL."""
    from azure_hc_intel_tf_amd.parallel.native import NativeReducer

    r = NativeReducer(compression="fp16", bucket_bytes=256 << 10, force=True)
    assert r.comm.size() == 1
    g = torch.randn(1_000_003, device="cuda")
    g0 = g.clone()
    b0 = r.comm.buckets_issued()
    r.allreduce_ranges_async_(g, [(0, 600_000), (600_000, 400_003)])
    r.join()
    torch.cuda.synchronize()
    assert torch.equal(g, g0.half().float())
    issued = r.comm.buckets_issued() - b0
    assert issued == -(-600_000 // (128 << 10)) + -(-400_003 // (128 << 10))  # 2-byte wire
    r.close()


def test_bucket_pack_unpack_wire_formats():
    import azure_hc_intel_tf_amd.ops._ext as ext

    hcb = ext.ops()
    for n in (1, 3, 4, 1027, 262_147):
        x = torch.randn(n, device="cuda") * 100
        for dt in (torch.float32, torch.bfloat16, torch.float16):
            w = torch.empty(n, dtype=dt, device="cuda")
            hcb.bucket_pack(x, w, 0.5)
            torch.cuda.synchronize()
            assert torch.equal(w, (x * 0.5).to(dt)), (n, dt)
            y = torch.empty(n, device="cuda")
            hcb.bucket_unpack(w, y, 2.0)
            torch.cuda.synchronize()
            assert torch.equal(y, w.float() * 2.0), (n, dt)


def test_comm_profile_on_forced_dp_path():
    """allreduce ms / exposed ms / overlap % of the captured multi-GPU step (1-rank engine)"""
    from azure_hc_intel_tf_amd.models import create_model
    from azure_hc_intel_tf_amd.parallel.native import NativeReducer
    from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch

    m = create_model("resnet50", image_size=64, device="cuda", compute_dtype="bf16")
    img, lab = synthetic_batch(m, 8)
    red = NativeReducer(force=True, bucket_bytes=4 << 20)
    t = Trainer(m, 8, constant_lr(0.01), reducer=red, world_size=1, use_graph=True, force_overlap=True)
    for _ in range(4):
        t.step(img, lab)
    prof = t.comm_profile(img, lab, iters=3)
    assert prof is not None and prof["allreduce_ms"] > 0 and prof["compute_ms"] > 0
    assert 0.0 <= prof["overlap_pct"] <= 100.0
    # 102 MB of fp32 gradients in buckets of <= 4 MiB
    assert prof["buckets_per_step"] >= m.num_params() * 4 // (4 << 20)
    t1, t5 = t.accuracy(lab)
    assert 0.0 <= float(t1) <= float(t5) <= 1.0
    red.close()
