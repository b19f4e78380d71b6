"""The C++ gradient bucket engine (csrc/comm/engine.h -- the code _hcb_comm.so runs on RCCL)
on its in-process fake backend: W ranks emulated by threads, each with its own engine, comm
thread and stall watchdog, collectives done by a shared fake fabric.

Checks: identical bucket schedule on every rank, HOROVOD_FUSION_THRESHOLD splitting of
backward-segment ranges, sum / average numerics for fp32 and the bf16 / IEEE fp16 wire
formats, and the stall watchdog naming the stalled cycle when one rank falls behind."""
import struct

import numpy as np
import pytest

from azure_hc_intel_tf_amd import _build

_build.build_engine_cpu()
from azure_hc_intel_tf_amd import _hcb_engine_cpu as E  # noqa: E402

N = 40_003


def _init(world, n=N):
    i = np.arange(n, dtype=np.float64)
    return [((r + 1) * ((i % 97) - 48) * 0.0625 + 0.001 * r).astype(np.float32) for r in range(world)]


def _wire(x, wire):
    x = np.asarray(x, dtype=np.float32)
    if wire == 1:  # bf16 RNE
        u = x.view(np.uint32).astype(np.uint64)
        u = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
        return u.astype(np.uint32).view(np.float32)
    if wire == 2:
        return x.astype(np.float16).astype(np.float32)
    return x


def _expected(init, wire, avg):
    acc = np.zeros_like(init[0])
    for x in init:
        acc = (acc + _wire(x, wire)).astype(np.float32)
    if avg:
        acc = (acc / np.float32(len(init))).astype(np.float32)
    return _wire(acc, wire)


CYCLES = [[30_000, 10_003], [10_000, 20_000], [0, 10_000]]  # backward order: last layers first


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("wire,avg", [(0, False), (0, True), (1, False), (2, True)])
def test_fake_world_sums_and_identical_schedule(world, wire, avg):
    init = _init(world)
    thr = 16 * 1024  # bytes of wire buffer per bucket
    r = E.run(world, [x.tolist() for x in init], CYCLES, wire=wire, average=avg, threshold_bytes=thr)
    assert r["size_mismatches"] == 0
    sched = r["buckets"]
    assert all(s == sched[0] for s in sched), "every rank must issue the same bucket schedule"
    seqs = [b[0] for b in sched[0]]
    assert seqs == list(range(len(seqs)))
    esz = 4 if wire == 0 else 2
    assert all(b[2] * esz <= thr for b in sched[0])
    # buckets tile each cycle's range, in order
    covered = sorted((b[1], b[2]) for b in sched[0])
    pos = 0
    for off, n in covered:
        assert off == pos
        pos += n
    assert pos == N
    exp = _expected(init, wire, avg)
    for buf in r["buffers"]:
        np.testing.assert_allclose(np.asarray(buf, np.float32), exp, rtol=1e-6, atol=1e-6)
    assert r["cycles"] == [len(CYCLES)] * world


def test_threshold_split_is_equal_sized_and_aligned():
    # a 60 MB stage-4 range under an 8 MiB fp32 threshold: equal pieces, none above it
    b = E.plan([1000, 15_000_000], 8 << 20, 0)
    lens = [n for _, n in b]
    assert len(b) == 8 and max(lens) * 4 <= 8 << 20 and max(lens) - min(lens) <= 64
    assert b[0][0] == 1000 and sum(lens) == 15_000_000
    assert all((off - 1000) % 64 == 0 for off, _ in b)
    # no threshold: one bucket per range
    assert E.plan([0, 10, 10, 20], 0, 0) == [(0, 10), (10, 20)]
    # the threshold counts WIRE bytes: bf16 allows twice the elements
    assert len(E.plan([0, 4_000_000], 8 << 20, 1)) == 1 and len(E.plan([0, 4_000_000], 8 << 20, 0)) == 2


def test_stall_watchdog_names_the_stalled_cycle():
    world = 4
    init = _init(world, 4096)
    # rank 2's comm thread stalls 400 ms before bucket #1; every rank's watchdog must warn
    r = E.run(world, [x.tolist() for x in init], [[2048, 2048], [0, 2048]], threshold_bytes=4096,
              stall_rank=2, stall_seq=1, stall_ms=400, warn_s=0.1)
    warned = {w[0] for w in r["warnings"]}
    assert warned == set(range(world)), r["warnings"]
    for rank, cycle, last_seq, waited in r["warnings"]:
        assert cycle == 1 and last_seq >= 1 and waited > 0.1
    exp = _expected(init, 0, False)
    for buf in r["buffers"]:  # the stall delays, it does not corrupt
        np.testing.assert_allclose(np.asarray(buf, np.float32), exp, rtol=1e-6)


def test_graph_replay_heartbeat_lets_the_watchdog_see_captured_collectives():
    """The default multi-GPU step replays a captured graph: its collectives make no engine call,
    so the watchdog only learns about them through the per-step heartbeat (step_mark, called by
    trainer.py after each replay). Rank 1 stalls in replayed step 2: with the heartbeat every
    rank's watchdog warns and names step 3 (1-based watch cycle); without it the stall is
    invisible -- the blind spot the heartbeat closes."""
    world = 3
    init = _init(world, 4096)
    cycles = [[2048, 2048], [0, 2048]]
    r = E.run(world, [x.tolist() for x in init], cycles, threshold_bytes=4096, replay_steps=4, stall_rank=1,
              stall_step=2, stall_ms=400, warn_s=0.1)
    warned = {w[0] for w in r["warnings"]}
    assert warned == set(range(world)), r["warnings"]
    for rank, cycle, last_seq, waited in r["warnings"]:
        assert cycle == 3 and waited > 0.1, r["warnings"]
    assert r["cycles"] == [4] * world
    # four replays of the full-buffer sum: x_r -> sum over ranks, then world^k growth
    exp = _expected(init, 0, False) * world ** 3
    for buf in r["buffers"]:
        np.testing.assert_allclose(np.asarray(buf, np.float32), exp, rtol=1e-5)
    blind = E.run(world, [x.tolist() for x in init], cycles, threshold_bytes=4096, replay_steps=4, stall_rank=1,
                  stall_step=2, stall_ms=400, warn_s=0.1, heartbeat=False)
    assert blind["warnings"] == []


def test_no_warning_without_stall():
    init = _init(2, 2048)
    r = E.run(2, [x.tolist() for x in init], [[0, 2048]], warn_s=0.2)
    assert r["warnings"] == []


def test_stall_decision_logic():
    # (t, enqueued, completed): idle, then a cycle waits, warns once after 1 s, progresses,
    # stalls again, aborts after 3 s
    acts = E.stall_decisions(1.0, 3.0, [(0.0, 0, 0), (0.1, 1, 0), (0.5, 1, 0), (1.2, 1, 0), (1.5, 1, 0),
                                         (1.6, 2, 1), (2.0, 2, 1), (5.0, 2, 1)])
    IDLE, PROGRESS, WAITING, WARN, ABORT = range(5)
    assert acts == [IDLE, WAITING, WAITING, WARN, WAITING, PROGRESS, WAITING, ABORT]


def test_wire_conversions_match_numpy():
    xs = np.array([0.0, 1.0, -2.5, 65504.0, 65520.0, 1e-8, 3.0e-5, 6.1e-5, 123.456, -7.77e4], dtype=np.float32)
    for x in xs:
        assert E.f32_to_f16_bits(float(x)) == int(np.float16(x).view(np.uint16)), x
    u = struct.unpack("<I", struct.pack("<f", 1.00390625))[0]
    assert E.f32_to_bf16_bits(1.00390625) == ((u + 0x7FFF + ((u >> 16) & 1)) >> 16)


def test_comm_engine_and_host_bookkeeping_under_sanitizers(tmp_path):
    """tools/sanitize/run_engine_sanitizers.sh: the bucket engine with its fake 8-rank fabric
    AND the RCCL runtime's HIP-free host bookkeeping (csrc/comm/host.h, the header comm.cpp
    compiles: handle tables, event pool / timeline, watch state, xGMI checks), each built with
    ASan + UBSan and with TSan and stress-driven."""
    import os
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run(["bash", os.path.join(root, "tools", "sanitize", "run_engine_sanitizers.sh")], cwd=root,
                       env=dict(os.environ, OUT=str(tmp_path)), capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert r.stdout.count("comm_host_stress: ok") == 2 and r.stdout.count("ENGINE STRESS OK") == 2
