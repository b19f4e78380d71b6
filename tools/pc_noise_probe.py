#!/usr/bin/env python3
"""Run-to-run loss spread of the (non-deterministic) 96 px / batch 8 ResNet-50 graph step, single
graph and data-parallel graph (1-rank RCCL), with graph packet capture on and off: one child per
run, losses of 8 steps. python tools/pc_noise_probe.py [runs=3]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import json, os, sys
sys.path.insert(0, sys.argv[1])
import torch
from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch
os.environ["DEBUG_CLR_GRAPH_PACKET_CAPTURE"] = os.environ["HCB_PC_WANT"]
seg = sys.argv[2] == "dp"
torch.manual_seed(0)
m = create_model("resnet50", image_size=96, device="cuda", compute_dtype="bf16")
img, lab = synthetic_batch(m, 8)
red = None
if seg:
    from azure_hc_intel_tf_amd.parallel.native import NativeReducer
    red = NativeReducer(force=True)
t = Trainer(m, 8, constant_lr(0.002), reducer=red, world_size=1, use_graph=True, graph_warmup=2, force_overlap=seg)
tr = torch.zeros(8, device="cuda")
for i in range(8):
    tr[i:i + 1].copy_(t.step(img, lab))
print(json.dumps([round(v, 4) for v in tr.tolist()]))
if red is not None:
    red.close()
"""
runs = int(sys.argv[1]) if len(sys.argv) > 1 else 3
for pc in ("0", "1"):
    for mode in ("single", "dp"):
        for r in range(runs):
            env = dict(os.environ, HCB_PC_WANT=pc, MASTER_ADDR="127.0.0.1", MASTER_PORT="29681", RANK="0",
                       WORLD_SIZE="1", LOCAL_RANK="0", LOCAL_WORLD_SIZE="1")
            out = subprocess.run([sys.executable, "-c", CHILD, ROOT, mode], env=env, capture_output=True, text=True,
                                 timeout=300)
            if out.returncode != 0:
                raise SystemExit(out.stderr[-2000:])
            print(f"pc={pc} {mode:6s} run{r}: {out.stdout.strip().splitlines()[-1]}", flush=True)
