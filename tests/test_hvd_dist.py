"""Horovod-compatible API and gradient reducers on CPU with gloo, world_size 2, 4 and 8."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fn, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    try:
        from azure_hc_intel_tf_amd.parallel import hvd

        hvd.init(backend="gloo")
        fn(hvd)
        hvd.shutdown()
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback

        q.put((rank, traceback.format_exc()))


def run(world, fn):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, fn, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    errs = [r for r in res if r[1] != "ok"]
    assert not errs, errs


def _collectives(hvd):
    r, n = hvd.rank(), hvd.size()
    t = torch.full((5,), float(r + 1))
    assert torch.allclose(hvd.allreduce(t), torch.full((5,), (n + 1) / 2))
    assert torch.allclose(hvd.allreduce(t, average=False), torch.full((5,), n * (n + 1) / 2))
    from azure_hc_intel_tf_amd.parallel.compression import Compression

    c = hvd.allreduce(t, compression=Compression.fp16)
    assert c.dtype == torch.float32 and torch.allclose(c, torch.full((5,), (n + 1) / 2))
    g = hvd.allgather(torch.full((r + 1, 2), float(r)))
    assert g.shape == (n * (n + 1) // 2, 2)
    b = hvd.broadcast(torch.full((3,), float(r)), root_rank=n - 1)
    assert torch.all(b == n - 1)
    assert hvd.broadcast_object({"r": r}, 0) == {"r": 0}
    assert hvd.local_rank() == r and hvd.local_size() == n and hvd.cross_size() == 1
    ts = [torch.full((7,), float(r)), torch.full((3, 3), 2.0 * r)]
    hvd.grouped_allreduce_(ts)
    assert torch.allclose(ts[0], torch.full((7,), (n - 1) / 2))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_hvd_collectives(world):
    run(world, _collectives)


def _dist_optimizer(hvd):
    torch.manual_seed(hvd.rank())
    model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))
    hvd.broadcast_parameters(model.state_dict(), root_rank=0)
    opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9)
    opt = hvd.DistributedOptimizer(opt, named_parameters=model.named_parameters())
    hvd.broadcast_optimizer_state(opt, root_rank=0)
    x = torch.randn(4, 8)
    for _ in range(3):
        opt.zero_grad()
        model(x).pow(2).mean().backward()
        opt.step()
    # every rank must hold identical weights after averaged updates
    w = torch.cat([p.detach().flatten() for p in model.parameters()])
    allw = hvd.allgather(w.view(1, -1))
    assert torch.allclose(allw[0], allw[-1], atol=1e-6)


def test_distributed_optimizer_keeps_replicas_in_sync():
    run(2, _dist_optimizer)


def _dist_optimizer_unused_param(hvd):
    """A parameter that receives no gradient (unused branch) must not leave its bucket
    unreduced: the others in that bucket still get averaged (Horovod semantics: zeros)."""
    torch.manual_seed(0)
    used = torch.nn.Linear(4, 4)
    unused = torch.nn.Linear(4, 4)
    hvd.broadcast_parameters(dict(list(used.state_dict().items())), root_rank=0)
    params = list(used.parameters()) + list(unused.parameters())
    opt = hvd.DistributedOptimizer(torch.optim.SGD(params, lr=1.0))
    x = torch.full((2, 4), float(hvd.rank() + 1))
    opt.zero_grad()
    used(x).sum().backward()
    opt.step()
    w = used.weight.detach().flatten()
    allw = hvd.allgather(w.view(1, -1))
    assert torch.allclose(allw[0], allw[-1], atol=1e-6), "replicas diverged: a bucket was never reduced"
    assert unused.weight.grad is not None and torch.all(unused.weight.grad == 0)


def test_distributed_optimizer_reduces_buckets_with_unused_params(monkeypatch):
    monkeypatch.setenv("HOROVOD_FUSION_THRESHOLD", "4096")  # one bucket holds used + unused params
    run(2, _dist_optimizer_unused_param)


def _dist_optimizer_rank_dependent_branch(hvd):
    """A data-dependent branch unused on SOME ranks only: the buckets must still go out in the
    same order on every rank (a rank whose middle bucket is incomplete must not launch the later
    ones first), or the collectives pair up mismatched buffers / hang."""
    torch.manual_seed(0)
    a, b, c = torch.nn.Linear(32, 32), torch.nn.Linear(32, 32), torch.nn.Linear(32, 32)
    params = list(a.parameters()) + list(b.parameters()) + list(c.parameters())
    hvd.broadcast_parameters([p.data for p in params], root_rank=0)
    opt = hvd.DistributedOptimizer(torch.optim.SGD(params, lr=0.05))
    assert len(opt._buckets) >= 3, "one bucket per layer expected"
    for step in range(3):
        opt.zero_grad()
        x = torch.full((2, 32), 0.1 * float(hvd.rank() + step + 1))
        h = a(x)
        if (hvd.rank() + step) % 2 == 0:  # b used on half of the ranks only
            h = b(h)
        c(h).sum().backward()
        opt.step()
    w = torch.cat([p.detach().flatten() for p in params])
    allw = hvd.allgather(w.view(1, -1))
    for r in range(1, hvd.size()):
        assert torch.allclose(allw[0], allw[r], atol=1e-5), "replicas diverged"


def test_distributed_optimizer_rank_dependent_unused_branch(monkeypatch):
    monkeypatch.setenv("HOROVOD_FUSION_THRESHOLD", "4096")  # the floor: ~one bucket per tensor (32x32 fp32 = 4 KiB)
    run(4, _dist_optimizer_rank_dependent_branch)


def _engine_training_world8(hvd):
    """world 8: overlapped, threshold-split range reductions keep every replica identical."""
    from azure_hc_intel_tf_amd.models import create_model
    from azure_hc_intel_tf_amd.parallel import make_reducer
    from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch

    torch.set_num_threads(1)
    m = create_model("trivial", image_size=16, device="cpu", seed=300 + hvd.rank())
    hvd.broadcast_global_variables(m, 0)
    red = make_reducer("torch", bucket_bytes=64 << 10)
    img, lab = synthetic_batch(m, 2, seed=hvd.rank())
    img = (img - 127) / 60
    t = Trainer(m, 2, constant_lr(0.01), reducer=red, world_size=hvd.size(), force_overlap=True)
    for _ in range(2):
        t.step(img, lab)
    allw = hvd.allgather(m.ps.master.view(1, -1))
    for r in range(1, hvd.size()):
        assert torch.allclose(allw[0], allw[r])


def test_reducer_training_in_sync_world8():
    run(8, _engine_training_world8)


def _engine_training(hvd):
    from azure_hc_intel_tf_amd.models import create_model
    from azure_hc_intel_tf_amd.parallel import make_reducer
    from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch

    m = create_model("resnet50", image_size=32, device="cpu", seed=100 + hvd.rank())
    hvd.broadcast_global_variables(m, 0)
    red = make_reducer("torch", bucket_bytes=1 << 20)
    img, lab = synthetic_batch(m, 2, seed=hvd.rank())
    img = (img - 127) / 60
    t = Trainer(m, 2, constant_lr(0.01), reducer=red, world_size=hvd.size())
    for _ in range(2):
        t.step(img, lab)
    allw = hvd.allgather(m.ps.master.view(1, -1))
    assert torch.allclose(allw[0], allw[1])


def test_flat_buffer_reducer_training_in_sync():
    run(2, _engine_training)


def test_make_buckets_cover_buffer_in_reverse():
    from azure_hc_intel_tf_amd.parallel import make_buckets

    b = make_buckets(1000, 256)
    assert b[0] == (744, 256) and sum(n for _, n in b) == 1000 and b[-1][0] == 0


def _overlap_matches_serial(hvd):
    """segmented backward + async range allreduce == one allreduce after the whole backward"""
    from azure_hc_intel_tf_amd.models import create_model
    from azure_hc_intel_tf_amd.parallel import make_reducer
    from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch

    masters = []
    for overlap in (True, False):
        m = create_model("resnet50", image_size=32, device="cpu", seed=7 + hvd.rank())
        hvd.broadcast_global_variables(m, 0)
        img, lab = synthetic_batch(m, 2, seed=hvd.rank())
        img = (img - 127) / 60
        t = Trainer(m, 2, constant_lr(0.05), reducer=make_reducer("torch", bucket_bytes=1 << 20),
                    world_size=hvd.size())
        t.overlap = overlap
        for _ in range(2):
            t.step(img, lab)
        masters.append(m.ps.master.clone())
    assert torch.allclose(masters[0], masters[1], rtol=1e-5, atol=1e-6)


def test_overlapped_allreduce_matches_serial():
    run(2, _overlap_matches_serial)


def test_backward_segments_cover_every_gradient_once():
    from azure_hc_intel_tf_amd.models import create_model

    for name in ("resnet50", "resnet50_v1.5"):
        m = create_model(name, image_size=32, device="cpu")
        # the segment ranges only depend on which layers each segment lists
        layers_all = []
        for blk in reversed(m.blocks):
            layers_all.append(blk.layers())
        cover = torch.zeros(m.ps.grad.numel(), dtype=torch.int32)
        ranges = m.grad_ranges([l for ls in layers_all for l in ls] + [m.fc, m.stem])
        for off, n in ranges:
            cover[off:off + n] += 1
        # every parameter exactly once (the buffer may carry alignment padding between tensors)
        assert int(cover.max()) == 1 and int(cover.sum()) == sum(p.numel for l in m.all_layers()
                                                                  for p in getattr(l, "params", lambda: [])()), name
        assert int(cover.sum()) >= m.num_params() - 64, name


def _stall_and_timeline(hvd):
    import time

    r = hvd.rank()
    if r == 1:
        time.sleep(2.5)  # fault injection: rank 1 joins the collective late
    t = torch.full((1000,), float(r))
    hvd.allreduce_(t, average=False, name="grad")
    assert torch.all(t == 1.0)
    from azure_hc_intel_tf_amd.parallel.monitor import monitor

    if r == 0:
        assert monitor().stalls >= 1
        assert monitor().timeline is not None


def test_stall_inspector_and_timeline(tmp_path, monkeypatch, capfd):
    """Horovod's stall inspector / HOROVOD_TIMELINE on the gloo path: a late rank is reported
    while the collective is outstanding, and every collective lands in the Chrome trace."""
    tl = tmp_path / "timeline.json"
    monkeypatch.setenv("HOROVOD_TIMELINE", str(tl))
    monkeypatch.setenv("HOROVOD_STALL_CHECK_TIME_SECONDS", "0.5")
    run(2, _stall_and_timeline)
    import json

    ev = json.loads(tl.read_text())
    assert any(e["name"] == "allreduce.grad" and e["ph"] == "X" and e["args"]["bytes"] == 4000 for e in ev)
    assert json.loads((tmp_path / "timeline.json.rank1").read_text())
    assert "stall inspector" in capfd.readouterr().err


def _stall_abort(hvd):
    import time

    if hvd.rank() == 1:
        time.sleep(30)  # never joins in time
    hvd.allreduce_(torch.ones(4))


def test_stall_abort_exits_the_stuck_rank(monkeypatch):
    """HCB_STALL_ABORT_SECONDS: the waiting rank exits with the stall code instead of hanging."""
    import multiprocessing

    monkeypatch.setenv("HOROVOD_STALL_CHECK_TIME_SECONDS", "0.3")
    monkeypatch.setenv("HCB_STALL_ABORT_SECONDS", "1.5")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    p0 = ctx.Process(target=_worker, args=(0, 2, port, _stall_abort, q))
    p1 = ctx.Process(target=_worker, args=(1, 2, port, _stall_abort, q))
    p0.start()
    p1.start()
    p0.join(timeout=60)
    from azure_hc_intel_tf_amd.parallel.monitor import STALL_EXIT_CODE

    assert p0.exitcode == STALL_EXIT_CODE
    p1.kill()
    p1.join(timeout=30)


@pytest.mark.parametrize("name,size", [("resnet50", 32), ("resnet50_v2", 32), ("inception3", 107), ("vgg11", 32),
                                       ("googlenet", 64), ("alexnet", 99)])
def test_segmented_backward_equals_plain_backward(name, size, monkeypatch):
    """backward_segments (the multi-GPU overlap path) computes the same gradients as the plain
    backward, closes more than one segment for the large models, and its segments own every
    parameter exactly once."""
    monkeypatch.setenv("HCB_SEGMENT_PARAMS", "500000")
    from azure_hc_intel_tf_amd.models import create_model
    from azure_hc_intel_tf_amd.nn.layers import Dropout
    from azure_hc_intel_tf_amd.trainer import synthetic_batch

    torch.manual_seed(0)
    m = create_model(name, image_size=size, device="cpu")
    for l in getattr(m, "seq", []):
        if isinstance(l, Dropout):
            l.keep = 1.0
    img, lab = synthetic_batch(m, 2)
    dl = torch.randn(2, m.num_classes, dtype=torch.float32).to(m.act_dtype) * 0.1
    if dl.shape[1] != getattr(m.fc, "ld", dl.shape[1]):
        dl = torch.nn.functional.pad(dl, (0, m.fc.ld - dl.shape[1]))
    m.ps.zero_grad()
    m.forward(img)
    m.backward(dl)
    g_plain = m.ps.grad.clone()
    m.ps.zero_grad()
    m.forward(img)
    cover = torch.zeros(m.ps.grad.numel(), dtype=torch.int32)
    nseg = 0
    for layers, last in m.backward_segments(dl):
        nseg += 1
        rng = [(0, m.ps.grad.numel())] if layers is None else m.grad_ranges(layers)
        for off, n in rng:
            cover[off:off + n] += 1
    assert last
    assert int(cover.max()) == 1 and int(cover.sum()) >= m.num_params() - 64
    if name != "alexnet":
        assert nseg >= 2
    assert torch.allclose(m.ps.grad, g_plain, rtol=1e-4, atol=1e-6)


def test_resnet_block_segments():
    """segments="block" (bench.py --backward_segments block): one segment per block of stages
    3-4, stage 2 whole, stage 1 cut from the stem -- ResNet-50: 3 + 6 + 1 + 1 + stem = 12
    segments, the same gradients as the plain backward, every parameter exactly once."""
    from azure_hc_intel_tf_amd.models import create_model
    from azure_hc_intel_tf_amd.trainer import synthetic_batch

    torch.manual_seed(0)
    m = create_model("resnet50", image_size=32, device="cpu")
    img, lab = synthetic_batch(m, 2)
    dl = torch.randn(2, m.num_classes) * 0.1
    if dl.shape[1] != getattr(m.fc, "ld", dl.shape[1]):
        dl = torch.nn.functional.pad(dl, (0, m.fc.ld - dl.shape[1]))
    m.ps.zero_grad()
    m.forward(img)
    m.backward(dl)
    g_plain = m.ps.grad.clone()
    m.segments = "block"
    m.ps.zero_grad()
    m.forward(img)
    cover = torch.zeros(m.ps.grad.numel(), dtype=torch.int32)
    sizes = []
    for layers, last in m.backward_segments(dl):
        rng = m.grad_ranges(layers)
        sizes.append(sum(n for _, n in rng))
        for off, n in rng:
            cover[off:off + n] += 1
    assert last and len(sizes) == 12, sizes
    assert sizes[-1] < 10_000  # only the stem (conv 7x7x3x64 + BN) after the last block
    assert int(cover.max()) == 1 and int(cover.sum()) >= m.num_params() - 64
    assert torch.allclose(m.ps.grad, g_plain, rtol=1e-4, atol=1e-6)


def test_rccl_env_plumbing(monkeypatch):
    from azure_hc_intel_tf_amd.launch.launcher import rccl_env, worker_env

    monkeypatch.delenv("NCCL_ALGO", raising=False)
    e = rccl_env(channels=16, algo="Ring", proto=None, base={"NCCL_MAX_NCHANNELS": "8"})
    assert e == {"NCCL_MIN_NCHANNELS": "16", "NCCL_ALGO": "Ring"}  # a value already set wins
    w = worker_env({}, 1, 1, 2, 2, 0, "127.0.0.1", 29500, "ib", None, rccl=e)
    assert w["NCCL_ALGO"] == "Ring" and w["NCCL_MIN_NCHANNELS"] == "16" and w["RANK"] == "1"


def _comm_check(hvd, compression=None):
    """The overlapped-allreduce race detector (Trainer comm_check) passes on a correct engine and
    fails loudly when a reduction reads gradients that are not final -- also with a 16-bit wire,
    whose bound is per element (2 ulp * world * sum_r |g_r|), not relative to a range's max."""
    from azure_hc_intel_tf_amd.models import create_model
    from azure_hc_intel_tf_amd.parallel import make_reducer
    from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch

    m = create_model("resnet50", image_size=32, device="cpu", seed=3 + hvd.rank())
    hvd.broadcast_global_variables(m, 0)
    img, lab = synthetic_batch(m, 2, seed=hvd.rank())
    img = (img - 127) / 60
    red = make_reducer("torch", compression=compression, bucket_bytes=1 << 20)
    t = Trainer(m, 2, constant_lr(0.01), reducer=red, world_size=hvd.size(), comm_check=True)
    assert t.overlap and not t.use_graph
    t.step(img, lab)
    assert len(t.comm_check_errs) == 1 and t.comm_check_errs[0] < (1e-6 if compression is None else 0.05)
    # a broken engine: one range reduction per segment sees this rank's gradients scaled by 1.25
    # (on rank 0 only, a quarter of one contribution: under the old range-max bound a bf16 wire let
    # this through)
    real = red.allreduce_ranges_async_

    def stale(flat, ranges):
        if hvd.rank() == 0:
            off, n = ranges[0]
            flat[off:off + n].mul_(1.25)
        return real(flat, ranges)

    red.allreduce_ranges_async_ = stale
    try:
        t.step(img, lab)
    except RuntimeError as e:
        assert "comm check" in str(e)
    else:
        raise AssertionError("comm check missed a corrupted reduction")


def test_comm_check_race_detector():
    run(2, _comm_check)


def _comm_check_bf16(hvd):
    _comm_check(hvd, "bf16")


def test_comm_check_race_detector_bf16_wire():
    run(2, _comm_check_bf16)


def _xgmi_validation(hvd):
    """The one-shot xGMI allreduce's startup cross-check (parallel/native.py validate_xgmi), with a
    fake one-shot on gloo: a correct one-shot is turned on; a mismatch, a peer time-out or an
    exception on ANY rank disables it on EVERY rank, with the reason."""
    from azure_hc_intel_tf_amd.parallel.native import validate_xgmi, xgmi_probe

    def agree_min(v):
        t = torch.tensor([v], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return int(t.item())

    def rccl(t):
        dist.all_reduce(t)

    def exact(t):  # what a working one-shot computes, without a gloo collective of its own
        t.copy_(sum(xgmi_probe(t.numel(), r) for r in range(hvd.size())))

    good = lambda t: (exact(t), 0)[1]  # noqa: E731
    assert validate_xgmi(good, rccl, agree_min, 4096, hvd.rank()) == "on"

    def wrong_on_rank1(t):
        exact(t)
        if hvd.rank() == 1:
            t[7] += 1.0
        return 0

    st = validate_xgmi(wrong_on_rank1, rccl, agree_min, 4096, hvd.rank())
    assert st.startswith("disabled("), st
    assert ("mismatch" in st) if hvd.rank() == 1 else ("another rank" in st), st
    timeout = lambda t: (exact(t), 1)[1]  # noqa: E731
    assert validate_xgmi(timeout, rccl, agree_min, 256, hvd.rank()) == "disabled(peer timeout)"

    def boom_on_rank0(t):
        if hvd.rank() == 0:
            raise RuntimeError("hipIpcOpenMemHandle failed")
        exact(t)
        return 0

    st = validate_xgmi(boom_on_rank0, rccl, agree_min, 256, hvd.rank())
    assert st.startswith("disabled(RuntimeError: hipIpcOpenMemHandle" if hvd.rank() == 0 else
                         "disabled(failed on another rank"), st


def test_xgmi_startup_validation_disables_on_any_rank_failure():
    run(2, _xgmi_validation)


def _xgmi_construction_failure(hvd):
    """XgmiAllreduce construction when the region export fails on ONE rank: every rank
    still joins the handle all-gather and every rank raises, so the next collective (the startup
    cross-check's RCCL reduction) is issued by all ranks -- no rank left waiting in a collective
    its peers never enter. Fake native library on gloo."""
    from azure_hc_intel_tf_amd.parallel import xgmi

    class FakeCC:
        def xgmi_create(self, rank, world, cap, dev):
            if rank == 1:
                raise RuntimeError("hipIpcGetMemHandle: invalid argument")
            return 7

        def xgmi_handle(self, h):
            return torch.arange(64, dtype=torch.uint8)

        def xgmi_open(self, h, handles):
            raise AssertionError("must not open after a failed exchange")

        def xgmi_destroy(self, h):
            pass

    xgmi.load = lambda: FakeCC()
    xgmi.torch.cuda.current_device = lambda: 0
    with pytest.raises(RuntimeError, match=r"rank\(s\) \[1\]"):
        xgmi.XgmiAllreduce(capacity_bytes=1024)
    t = torch.ones(3)
    dist.all_reduce(t)  # both ranks arrive here: the collectives stayed matched
    assert torch.all(t == hvd.size())


def test_xgmi_construction_failure_keeps_collectives_matched():
    run(2, _xgmi_construction_failure)
