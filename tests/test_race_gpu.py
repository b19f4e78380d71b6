"""Race detection on the GPU: the same deterministic-mode training run with every kernel and copy
serialised by the HIP runtime (AMD_SERIALIZE_KERNEL=3, AMD_SERIALIZE_COPY=3, HIP_LAUNCH_BLOCKING=1)
must be bitwise equal to the normal asynchronous run -- graph replays, the forked comm-stream
branches of the multi-GPU step (1-rank RCCL communicator) and the weight-gradient side work
included. A missing stream / event dependency makes the asynchronous run read data early and
diverge. (race detection.)"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import hashlib, json, os, sys
sys.path.insert(0, sys.argv[1])
import torch
from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.ops import functional as Fn
from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch

Fn.set_deterministic(True)
from azure_hc_intel_tf_amd.nn import layers as L
for kv in filter(None, os.environ.get("RACE_SWITCHES", "").split(",")):  # e.g. L.FUSE_BN_BWD=0 (bisection)
    k, v = kv.split("=")
    mod, attr = k.split(".")
    setattr({"L": L, "Fn": Fn}[mod], attr, type(getattr({"L": L, "Fn": Fn}[mod], attr))(int(v)))
dp = sys.argv[2] == "dp"
size, batch = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (64, 8)
if len(sys.argv) > 5 and sys.argv[5] == "tuned":  # the autotuned kernel configs bench.py runs
    from azure_hc_intel_tf_amd.ops import autotune
    autotune.load_cache()
dt = os.environ.get("RACE_DTYPE")  # fp32: the headline precision (plane GEMMs, persistent kernels)
m = create_model("resnet50", image_size=size, device="cuda", seed=5, **({"compute_dtype": dt} if dt else {}))
img, lab = synthetic_batch(m, batch, seed=3)
red = None
if dp:
    from azure_hc_intel_tf_amd.parallel.native import NativeReducer
    red = NativeReducer(force=True)
t = Trainer(m, batch, constant_lr(0.02), use_graph=True, graph_warmup=1, reducer=red, force_overlap=dp)
rows = []
for _ in range(int(os.environ.get("RACE_STEPS", "4"))):
    t.step(img, lab)
    rows.append(t.row_loss.clone())
torch.cuda.synchronize()
# per-row cross entropies (the reported total adds an atomically accumulated L2 term)
losses = [hashlib.sha256(r.cpu().numpy().tobytes()).hexdigest() for r in rows]
print(json.dumps({"losses": losses, "graph": t._g_all is not None or t._g_fb is not None,
                  "overlap": t.overlap,
                  "master": hashlib.sha256(m.ps.master.cpu().numpy().tobytes()).hexdigest()}))
if red is not None:
    red.close()
"""


def _run(mode, serialize, extra_env=None):
    env = dict(os.environ)
    env.update(extra_env or {})
    if serialize:
        env.update(AMD_SERIALIZE_KERNEL="3", AMD_SERIALIZE_COPY="3", HIP_LAUNCH_BLOCKING="1")
    if mode.startswith("dp"):
        env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29650 + int(serialize)), RANK="0", WORLD_SIZE="1",
                   LOCAL_RANK="0", LOCAL_WORLD_SIZE="1")
    out = subprocess.run([sys.executable, "-c", SCRIPT, ROOT, mode.split("+")[0]], env=env, capture_output=True, text=True,
                         timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("mode", ["single", "dp", "single+fp32", "dp+fp32"])
def test_serialised_run_equals_async_run(mode):
    """bf16 and the fp32 headline path (plane GEMMs incl. the persistent short-K kernels, fp32 BN)."""
    env = {"RACE_DTYPE": "fp32"} if mode.endswith("+fp32") else None
    a = _run(mode, serialize=False, extra_env=env)
    s = _run(mode, serialize=True, extra_env=env)
    assert a["graph"] and a["overlap"] == mode.startswith("dp")
    assert a["losses"] == s["losses"], (a["losses"], s["losses"])
    assert a["master"] == s["master"], "weights differ between the asynchronous and the serialised run"


@pytest.mark.parametrize("mode", ["single", "dp"])
def test_wgrad_side_stream_equals_serialised_and_main_stream(mode):
    """HCB_WGRAD_STREAM=1 (weight-gradient GEMMs forked onto a side stream beside the data-gradient
    chain, joined per backward segment): bitwise equal to its kernel-serialised run AND to the
    main-stream run -- the fork / join and the operand lifetimes (nn/layers.py run_wgrad) leave
    no race."""
    side = {"HCB_WGRAD_STREAM": "1"}
    a = _run(mode, serialize=False, extra_env=side)
    s = _run(mode, serialize=True, extra_env=side)
    m = _run(mode, serialize=False)
    assert a["graph"]
    assert a["losses"] == s["losses"] == m["losses"], (a["losses"], s["losses"], m["losses"])
    assert a["master"] == s["master"] == m["master"]
