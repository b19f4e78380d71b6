#!/usr/bin/env python3
"""Bisect the DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 divergence of the data-parallel step graph.

bench.py --force_dp_path with HCB_DETERMINISTIC=1 and packet capture on diverged 4/4 while the
race detector (tests/test_race_gpu.py SCRIPT: the same Trainer / graph, driven directly) replays
bitwise-exact (profiles/r2f_graph_packet_capture.txt). This script is bench.py's single-GPU
--force_dp_path run with each of its additions behind a switch, so one GPU call can remove them
one at a time:

  --tune        run autotune.tune_model() as bench.py does (else only load the cache)
  --lr sched    bench.py's resnet_lr_schedule (else constant 0.02, the race script's)
  --warmup N    untimed steps (bench.py 10; the graph is captured at step graph_warmup)
  --graph_warmup N   eager steps before capture (bench.py 2, race script 1)
  --trace       device copy of the loss after every replay (HCB_BENCH_LOSS_TRACE)
  --clone       row_loss.clone() after every replay (the race script's per-step read)
  --sync_each   torch.cuda.synchronize() after every replay
  --seed S      model seed (bench.py: default, race script 5)

Prints one JSON line: per-step losses (host floats, read after the run), finite flag."""
import argparse
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import azure_hc_intel_tf_amd  # noqa: E402,F401


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tune", action="store_true")
    ap.add_argument("--lr", default="const", choices=["const", "sched"])
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--graph_warmup", type=int, default=2)
    ap.add_argument("--trace", action="store_true")
    ap.add_argument("--clone", action="store_true")
    ap.add_argument("--sync_each", action="store_true")
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--single", action="store_true", help="no reducer (single-GPU graph, no fork)")
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29671")
    for k, v in (("RANK", "0"), ("WORLD_SIZE", "1"), ("LOCAL_RANK", "0"), ("LOCAL_WORLD_SIZE", "1")):
        os.environ.setdefault(k, v)
    import torch

    from azure_hc_intel_tf_amd.models import create_model
    from azure_hc_intel_tf_amd.ops import _ext, autotune
    from azure_hc_intel_tf_amd.ops import functional as Fn
    from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, resnet_lr_schedule, synthetic_batch

    _ext.load()
    Fn.set_deterministic(True)
    dev = torch.device("cuda", 0)
    red = None
    if not a.single:
        from azure_hc_intel_tf_amd.parallel.native import NativeReducer

        red = NativeReducer(force=True)
    kw = {} if a.seed is None else {"seed": a.seed}
    m = create_model("resnet50", device=dev, compute_dtype="bf16", **kw)
    autotune.load_cache()
    if a.tune:
        autotune.tune_model(m, a.batch, save=False)
    img, lab = synthetic_batch(m, a.batch, seed=0)
    lr = resnet_lr_schedule(a.batch) if a.lr == "sched" else constant_lr(0.02)
    t = Trainer(m, a.batch, lr, reducer=red, world_size=1, use_graph=True, graph_warmup=a.graph_warmup,
                force_overlap=not a.single)
    trace = torch.zeros(a.warmup + a.steps, device=dev)
    clones = []
    for i in range(a.warmup + a.steps):
        t.step(img, lab)
        if a.trace:
            trace[i:i + 1].copy_(t.loss)
        if a.clone:
            clones.append(t.loss.clone())
        if a.sync_each:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    final = float(t.loss.item())
    losses = [round(float(v), 4) for v in trace.tolist()] if a.trace else (
        [round(float(c.item()), 4) for c in clones] if a.clone else [])
    ok = math.isfinite(final) and final < 20 and all(math.isfinite(v) and v < 20 for v in losses)
    print(json.dumps({"args": vars(a), "final_loss": final, "finite": ok, "losses": losses[-6:],
                      "pc": os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE")}), flush=True)
    if red is not None:
        red.close()


if __name__ == "__main__":
    main()
