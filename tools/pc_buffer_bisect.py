#!/usr/bin/env python3
"""Buffer-level bisection of the DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 divergence.

One child process per run replays the deterministic single-graph step (tests/test_race_gpu.py
setup: ResNet-50, 64 px, batch 8, seed 5) and, after EVERY replay, hashes every device buffer the
step leaves behind, in execution order: per layer (forward order) the tensors it holds (GEMM
input, conv output z, BN output y, batch moments, BN statistics accumulators, ...), then the
flat gradient / master / momentum / weight-pack buffers and the row losses. The parent runs
packet capture OFF twice (the determinism baseline: every hash must agree) and ON twice, then
reports, per ON run, the first step with any difference and, in that step, the first buffers
(in execution order) that differ -- the first producer whose output differs while everything it
read before it is equal.

    python tools/pc_buffer_bisect.py [steps=4] [single|dp] [out.jsonl] [runs per setting=2]
"""
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import hashlib, json, os, sys
sys.path.insert(0, sys.argv[1])
import torch
from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.ops import functional as Fn
from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch

# the package forces packet capture off at import; re-set the requested value before the GPU is touched
os.environ["DEBUG_CLR_GRAPH_PACKET_CAPTURE"] = os.environ["HCB_PC_WANT"]
Fn.set_deterministic(True)
steps = int(sys.argv[2])
dp = sys.argv[3] == "dp"
m = create_model("resnet50", image_size=64, device="cuda", seed=5, compute_dtype="bf16")
img, lab = synthetic_batch(m, 8, seed=3)
red = None
if dp:  # the data-parallel step graph: forked comm branch, 1-rank RCCL communicator
    from azure_hc_intel_tf_amd.parallel.native import NativeReducer
    red = NativeReducer(force=True)
t = Trainer(m, 8, constant_lr(0.02), use_graph=True, graph_warmup=1, reducer=red, force_overlap=dp)


def tensors(name, v, out, seen):
    if isinstance(v, torch.Tensor):
        if v.is_cuda and v.numel() and v.data_ptr() not in seen:
            seen.add(v.data_ptr())
            out.append((name, v))
    elif isinstance(v, (tuple, list)):
        for i, e in enumerate(v):
            tensors(f"{name}[{i}]", e, out, seen)
    elif hasattr(v, "t") and isinstance(getattr(v, "t"), torch.Tensor):  # Fn.Planes
        tensors(name + ".planes", v.t, out, seen)
    elif hasattr(v, "mean") and hasattr(v, "invstd"):  # Fn.BNSaved
        tensors(name + ".mean", v.mean, out, seen)
        tensors(name + ".invstd", v.invstd, out, seen)


def buffers():
    out, seen = [], set()
    for li, l in enumerate(m.all_layers()):
        for k in sorted(vars(l)):
            if k in ("w", "gamma", "beta", "bias", "pack"):  # views of the flat buffers below
                continue
            tensors(f"{li:03d}:{getattr(l, 'name', type(l).__name__)}.{k}", getattr(l, k), out, seen)
    ps = m.ps
    for p in reversed(ps.params):  # per-parameter gradients, in backward (reverse creation) order
        tensors("grad:" + p.name, p.grad, out, set())
    for k in ("grad", "master", "momentum", "pack_buf", "pack_buf_lo"):
        tensors("ps." + k, getattr(ps, k, None), out, seen)
    tensors("trainer.row_loss", t.row_loss, out, seen)
    return out  # (trainer.loss adds an atomically accumulated L2 term: not bitwise reproducible)


for s in range(steps):
    t.step(img, lab)
    torch.cuda.synchronize()
    for name, v in buffers():
        c = v.detach().contiguous()
        h = hashlib.sha256(c.view(torch.uint8).cpu().numpy().tobytes()).hexdigest()[:16]
        row = {"step": s, "buf": name, "shape": list(v.shape), "h": h}
        if c.dtype == torch.float32:
            row["sum"], row["abssum"] = float(c.double().sum()), float(c.double().abs().sum())
        print(json.dumps(row), flush=True)
    for p in m.ps.params:  # anomalous gradient elements of this step (bit patterns)
        gp = p.grad.detach().reshape(-1)
        bad = (gp.abs() > 1e6).nonzero().reshape(-1)[:8].tolist()
        if bad:
            vals = gp[bad].cpu()
            print(json.dumps({"step": s, "anomaly": p.name, "idx": bad, "n": int((gp.abs() > 1e6).sum()),
                              "hex": [hex(int(v)) for v in vals.view(torch.int32).tolist()]}), flush=True)
print(json.dumps({"done": True, "graph": t._g_all is not None or t._g_fb is not None}), flush=True)
if red is not None:
    red.close()
"""


def run(pc: str, steps: int, mode: str):
    env = dict(os.environ, HCB_PC_WANT=pc)
    if mode == "dp":
        env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29671", RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
                   LOCAL_WORLD_SIZE="1")
    out = subprocess.run([sys.executable, "-c", CHILD, ROOT, str(steps), mode], env=env, capture_output=True,
                         text=True, timeout=400)
    if out.returncode != 0:
        raise SystemExit(f"child (pc={pc}) failed:\n{out.stderr[-3000:]}")
    rows = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    for r in rows:
        if "anomaly" in r:
            print(f"[pc_buffer_bisect] pc={pc} {mode}: {json.dumps(r)}", flush=True)
    assert rows and rows[-1].get("done") and rows[-1]["graph"], rows[-1:]
    return [r for r in rows if "buf" in r]


def first_diffs(a, b, limit=16):
    """Rows of b that differ from a, in (step, execution) order, within the first differing step
    (with the relative change of the fp32 sums)."""
    diffs = [(x, y) for x, y in zip(a, b) if x["h"] != y["h"]]
    assert all(x["buf"] == y["buf"] for x, y in zip(a, b)), "buffer lists differ"
    if not diffs:
        return None, []
    s0 = diffs[0][0]["step"]
    out = []
    for x, y in diffs:
        if x["step"] != s0:
            continue
        d = x["buf"]
        if "abssum" in x:
            d += f" (abssum {x['abssum']:.6g} -> {y['abssum']:.6g})"
        out.append(d)
    return s0, out[:limit]


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    mode = sys.argv[2] if len(sys.argv) > 2 else "single"
    path = sys.argv[3] if len(sys.argv) > 3 else None
    nrun = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    runs = {}
    for pc, name in (("0", "off"), ("1", "on")):
        for i in range(1, nrun + 1):
            tag = f"{name}{i}"
            runs[tag] = run(pc, steps, mode)
            print(f"[pc_buffer_bisect] {mode} {tag}: {len(runs[tag])} buffer hashes over {steps} replays", flush=True)
    if path:
        with open(path, "w") as f:
            for tag, rows in runs.items():
                for r in rows:
                    f.write(json.dumps(dict(r, run=tag)) + "\n")
    n_per = len(runs["off1"]) // steps
    print(json.dumps({"buffers_per_step": n_per}))
    for tag in runs:
        if tag == "off1":
            continue
        s0, bufs = first_diffs(runs["off1"], runs[tag])
        print(json.dumps({"mode": mode, "run": tag, "vs": "off1", "first_diff_step": s0, "first_diff_buffers": bufs}),
              flush=True)
    digest = hashlib.sha256(json.dumps([r["h"] for r in runs["off1"]]).encode()).hexdigest()[:16]
    print(json.dumps({"off1_digest": digest}))


if __name__ == "__main__":
    main()
