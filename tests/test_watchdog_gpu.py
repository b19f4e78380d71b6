"""Stall watchdog on the DEFAULT multi-GPU step path: one replayed HIP graph whose RCCL
collectives run on a forked comm branch and make no host call per reduction (trainer.py). The
trainer's per-step heartbeat (hcb_comm.step_mark) is what lets the native engine's watchdog see
them (csrc/comm/comm.cpp; Horovod's stall inspector role, SURVEY.md §5 "Failure detection",
/root/reference/benchmark-scripts/run-tf-sing-ucx-openmpi.sh:105-106).

Staged on one GPU: bench.py --force_dp_path runs that exact graph on a 1-rank communicator and
HCB_COMM_DEBUG_SLEEP_MS puts a bounded device sleep on the comm stream INSIDE the captured graph
(eager warm-up steps do not sleep), so every replayed step's reductions finish seconds late."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _run(extra, steps=3):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE")}
    env.update(HOROVOD_STALL_CHECK_TIME_SECONDS="1", HCB_COMM_DEBUG_SLEEP_MS="2500", HCB_BENCH_COMM_PROFILE="0")
    env.update(extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--model", "trivial", "--batch_size", "8",
                           "--compute_dtype", "bf16", "--force_dp_path", "--steps", str(steps), "--warmup", "3",
                           "--no_tune"], env=env, capture_output=True, text=True, timeout=150)


def test_watchdog_warns_on_a_stalled_replayed_step():
    r = _run({})
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stderr.splitlines() if l.startswith("[hcb watchdog]")]
    assert any("has not completed" in l and "(graph-replayed step)" in l for l in lines), r.stderr[-3000:]


def test_stall_abort_exits_nonzero_on_the_graph_path():
    r = _run({"HCB_STALL_ABORT_SECONDS": "1.5"})
    assert r.returncode != 0, r.stderr[-3000:]
    assert "aborting" in r.stderr, r.stderr[-3000:]
    assert '"n_gpus"' not in r.stdout  # no result line from an aborted run


def test_no_false_stall_when_the_host_runs_ahead():
    """Healthy but slow replayed steps queued without any host sync (the host runs many steps ahead
    of the device) for longer than the stall threshold: every step's own watch event completes in
    turn, so the watchdog sees progress and neither warns nor aborts (one re-recorded event would be
    overwritten before completing and report a stall of a healthy job)."""
    r = _run({"HOROVOD_STALL_CHECK_TIME_SECONDS": "3", "HCB_STALL_ABORT_SECONDS": "4", "HCB_COMM_DEBUG_SLEEP_MS": "500"},
             steps=12)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "[hcb watchdog]" not in r.stderr, r.stderr[-3000:]
