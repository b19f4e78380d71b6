#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 synchronous data-parallel training throughput,
images/sec for the whole node, bs=64 per GPU, synthetic ImageNet, random-init weights
(BASELINE.json metric; the reference's tf_cnn_benchmarks run of
/root/reference/benchmark-scripts/run-tf-sing-ucx-openmpi.sh:62-113, ``-np TOTAL_WORKERS``
at :99-109).

    python bench.py --gpus N --steps K --warmup W
        N=1: this process trains on cuda:0.
        N>1 without WORLD_SIZE in the environment: this process is only the launcher -- it
             starts N worker CHILD processes (one per MI355X, launch/launcher.py: rank env,
             NUMA pinning, fail-fast) before anything touches the GPU, waits for them and
             exits non-zero if any of them fails.
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
        each process is one rank (RANK / LOCAL_RANK / WORLD_SIZE from the environment);
        WORLD_SIZE must equal --gpus.

One process per MI355X; gradients averaged with RCCL over xGMI. The headline ``value`` is the
reference's precision, fp32 (tf_cnn_benchmarks with MKL-DNN trains fp32: no --use_fp16 in
run-tf-sing-ucx-openmpi.sh:62-81), on the hand-written HIP kernels; the same invocation then
times the bf16 step and reports it as ``bf16_value`` / ``bf16_ms_per_step``. Per dtype: W
untimed warmup steps (the first ones also capture the HIP graph), then EXACTLY K timed steps
bracketed by barrier + device sync; the max time over ranks is used; rank 0 prints one JSON line
that also carries ``world`` (torch.distributed) and ``rccl_nranks`` (read back from the native
RCCL communicator), and every rank prints its own ``total images/sec`` lines on stderr. A native
engine that fails its self-test at N>1 ends the run with exit code 5 (unless --engine torch).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import azure_hc_intel_tf_amd  # noqa: E402,F401  (HIP runtime defaults, before torch touches the GPU)

BASELINE_VALUE = None  # the reference publishes no number
METRIC = "images/sec (whole node) ResNet-50 bs=64/worker at 1/2/4/8 MI355X"


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch_size", type=int, default=64, help="per-GPU batch")
    ap.add_argument("--no_graph", action="store_true")
    ap.add_argument("--no_tune", action="store_true", help="skip per-shape kernel autotuning")
    ap.add_argument("--compression", default=None, choices=[None, "fp16", "bf16"])
    ap.add_argument("--engine", default="native", choices=["native", "torch"])
    ap.add_argument("--force_dp_path", action="store_true",
                    help="N=1 only: run the multi-GPU step (one graph with the collectives on a forked comm "
                         "stream, async RCCL engine on a 1-rank communicator) to time its overhead on one GPU")
    ap.add_argument("--use_fp16", action="store_true",
                    help="tf_cnn_benchmarks --use_fp16: IEEE fp16 compute on the fp16 build of the HIP kernels with "
                         "automatic loss scaling")
    ap.add_argument("--compute_dtype", default=None, choices=[None, "bf16", "fp16", "fp32"],
                    help="activation / GEMM precision of the reported value (default fp32 = the reference's "
                         "precision, with bf16 timed as a secondary figure in the same run)")
    ap.add_argument("--secondary", default="auto", choices=["auto", "none", "bf16", "fp16", "fp32"],
                    help="a second compute dtype timed in the same run and reported as <dtype>_value "
                         "(auto: bf16 when the primary is the default fp32, else none)")
    ap.add_argument("--backward_segments", default="stage", choices=["stage", "block"],
                    help="gradient-reduction granularity of the overlapped multi-GPU step (ResNet): one segment "
                         "per stage, or per block in stages 3-4 with stage 1 split from the stem")
    ap.add_argument("--rccl_channels", type=int, default=None, help="NCCL_MIN/MAX_NCHANNELS for the workers")
    ap.add_argument("--rccl_algo", default=None, help="NCCL_ALGO for the workers (Ring, Tree)")
    ap.add_argument("--rccl_proto", default=None, help="NCCL_PROTO for the workers (Simple, LL, LL128)")
    return ap.parse_args(argv)


def _rccl(args):
    from azure_hc_intel_tf_amd.launch.launcher import rccl_env

    return rccl_env(args.rccl_channels, args.rccl_algo, args.rccl_proto)


def spawn_workers(args, argv) -> int:
    """--gpus N with no rank environment: start N worker children (never exec: nothing here
    has touched the GPU yet, and the children are separate processes)."""
    from azure_hc_intel_tf_amd.launch.launcher import launch, visible_gpu_count

    one_device = os.environ.get("HCB_BENCH_ONE_DEVICE") == "1"
    # the parent never loads torch / HIP (tests/test_bench_spawn.py checks this line)
    print(f"[bench] launcher parent: torch loaded = {'torch' in sys.modules}", file=sys.stderr, flush=True)
    if not one_device:
        visible = visible_gpu_count()  # KFD topology: no torch, no HIP runtime in this process
        if visible < args.gpus:
            print(f"[bench] --gpus {args.gpus} but only {visible} GPU(s) visible; refusing to report a "
                  f"{visible}-GPU run as a {args.gpus}-GPU one", file=sys.stderr)
            return 3
    cmd = [sys.executable, os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    env["HCB_BENCH_SPAWNED"] = "1"
    return launch(cmd, nproc_per_node=args.gpus, master_addr="127.0.0.1", env=env, rccl=_rccl(args))


def setup_native_reducer(args, world, rank, dev, make_reducer, all_min):
    """The native C++ RCCL engine for a multi-rank run, self-tested against the known sum before
    it is trusted. Returns (reducer, rccl_nranks). A failing engine is an ERROR (exit non-zero via
    EngineUnavailable) unless --engine torch was asked for: a scaling run must never silently
    measure a different engine than the one it reports (``all_min``: the cross-rank MIN of an int,
    so every rank takes the same branch)."""
    import torch

    ok = 1
    reducer, err = None, None
    try:
        reducer = make_reducer("native", compression=args.compression)
        t = torch.full((4096,), float(rank + 1), device=dev)
        reducer.comm.allreduce_(t)
        torch.cuda.synchronize()
        ok = 1 if torch.allclose(t, torch.full_like(t, world * (world + 1) / 2)) else 0
        if not ok:
            err = "self-test sum mismatch"
    except Exception as e:  # noqa: BLE001
        ok, err = 0, f"{type(e).__name__}: {e}"
    if all_min(ok) != 1:
        raise EngineUnavailable(err or "another rank's native engine failed its self-test")
    return reducer, reducer.comm.size()


class EngineUnavailable(RuntimeError):
    pass


def init_comm(args, world, rank, dev, all_min, make_reducer=None, init_pg=True):
    """Process group + gradient reducer of a multi-rank run. Returns (exit code, reducer, backend,
    rccl_nranks); a non-zero code ends the run (5: the native engine failed its self-test)."""
    if world <= 1:
        return 0, None, None, None
    import torch.distributed as dist

    os.environ.update(_rccl(args))  # before the communicators exist (torchrun-launched workers)
    backend = os.environ.get("HCB_BENCH_BACKEND", "nccl")
    if init_pg:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    if backend != "nccl":
        args.engine = "torch"
    if make_reducer is None:
        from azure_hc_intel_tf_amd.parallel import make_reducer
    reducer, rccl_nranks = None, None
    if args.engine == "native":
        try:
            reducer, rccl_nranks = setup_native_reducer(args, world, rank, dev, make_reducer, all_min)
        except EngineUnavailable as e:
            print(f"[rank {rank}] native RCCL engine failed its self-test ({e}); refusing to report a "
                  f"torch.distributed run as the native engine (pass --engine torch for that)", file=sys.stderr)
            if init_pg:
                dist.destroy_process_group()
            return 5, None, backend, None
    else:
        reducer = make_reducer("torch", compression=args.compression)
    if rccl_nranks is None and backend == "nccl" and init_pg:
        rccl_nranks = dist.get_world_size()
    if rccl_nranks is not None and rccl_nranks != world:
        print(f"[bench] RCCL communicator has {rccl_nranks} ranks, expected {world}", file=sys.stderr)
        return 4, None, backend, None
    return 0, reducer, backend, rccl_nranks


def _all_min_fn(world, dev):
    import torch
    import torch.distributed as dist

    def all_min(v: int) -> int:
        if world <= 1:
            return int(v)
        t = torch.tensor([int(v)], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return int(t.item())

    return all_min


def run_model(args, dtype, world, rank, dev, reducer, all_min):
    """Build, tune, warm up and time one model at one compute dtype; returns its result dict."""
    import torch
    import torch.distributed as dist

    from azure_hc_intel_tf_amd.models import create_model
    from azure_hc_intel_tf_amd.ops import autotune
    from azure_hc_intel_tf_amd.trainer import Trainer, resnet_lr_schedule, synthetic_batch
    from azure_hc_intel_tf_amd.utils import tracing

    model = create_model(args.model, device=dev, compute_dtype=dtype)
    if hasattr(model, "segments"):
        model.segments = args.backward_segments
    B = args.batch_size
    autotune.load_cache()
    if not args.no_tune and model.native:
        n = autotune.tune_model(model, B, save=(rank == 0))
        if n and rank == 0:
            print(f"[bench] {dtype}: autotuned {n} conv problems", file=sys.stderr)
    if reducer is not None:
        reducer.broadcast_(model.ps.master, 0)
        reducer.broadcast_(model.ps.buf, 0)
    images, labels = synthetic_batch(model, B, seed=rank)
    fp16 = args.use_fp16 or dtype == "fp16"
    trainer = Trainer(model, B, resnet_lr_schedule(B * world), reducer=reducer, world_size=world,
                      use_graph=not args.no_graph, dynamic_loss_scale=fp16, force_overlap=args.force_dp_path)

    def barrier():
        if world > 1:
            dist.barrier()

    warmup = max(args.warmup, 0)
    with tracing.range_(f"bench.warmup.{dtype}"):
        for _ in range(warmup):
            trainer.step(images, labels)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    trace = torch.zeros(args.steps, device=dev) if os.environ.get("HCB_BENCH_LOSS_TRACE") == "1" else None
    t0 = time.perf_counter()
    with tracing.range_(f"bench.timed.{dtype}"):
        for i in range(args.steps):
            trainer.step(images, labels)
            if trace is not None:  # device-side copy, no host sync (debug only)
                trace[i:i + 1].copy_(trainer.loss)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    elapsed = own = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    loss = float(trainer.loss.item())
    comm = None
    if reducer is not None:
        if hasattr(reducer, "check_errors"):
            reducer.check_errors()
        if os.environ.get("HCB_BENCH_COMM_PROFILE", "1") == "1":  # after the timed region
            failed = 0
            try:  # restores the training state itself
                comm = trainer.comm_profile(images, labels)
            except RuntimeError as e:
                if "comm check" in str(e):  # the race detector's verdict is never swallowed
                    raise
                comm, failed = {"error": f"{type(e).__name__}: {e}"}, 1
            except Exception as e:  # noqa: BLE001
                comm, failed = {"error": f"{type(e).__name__}: {e}"}, 1
            # a rank that failed here must not leave the others blocked in the profile's
            # collectives, nor turn a correctness error into a field of a valid result line
            if all_min(1 - failed) != 1:
                raise RuntimeError(f"comm profile failed on at least one rank ({comm})")
    # tf_cnn_benchmarks prints "total images/sec" on every rank (run-tf-sing-ucx-openmpi.sh:99-113
    # runs it under mpirun); stderr keeps stdout to the one JSON line
    print(f"[rank {rank}] {dtype} total images/sec: {world * B * args.steps / own:.2f} "
          f"(own {1000.0 * own / args.steps:.3f} ms/step)", file=sys.stderr, flush=True)
    if trace is not None and rank == 0:
        print(f"[bench] {dtype} losses " + " ".join(f"{v:.4f}" for v in trace.tolist()), file=sys.stderr)
    res = {"dtype": dtype, "ips": world * B * args.steps / elapsed, "ms": 1000.0 * elapsed / args.steps,
           "loss": loss, "comm": comm, "graph": trainer.use_graph, "native": model.native,
           "image_size": model.image_size}
    del trainer, model
    torch.cuda.synchronize()
    return res


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    if args.gpus < 1:
        print("[bench] --gpus must be >= 1", file=sys.stderr)
        return 2
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_workers(args, argv)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"[bench] WORLD_SIZE={world} but --gpus {args.gpus}: refusing to run", file=sys.stderr)
        return 3
    # stdout carries exactly ONE line, the result JSON: libraries that print banners on stdout
    # (RCCL announces its version when a communicator is created) write to stderr instead
    sys.stdout.flush()
    result_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    if os.environ.get("HCB_BENCH_STUB_WORKER") == "1":  # CPU test of the spawn path: report the rank env
        print(json.dumps({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE",
                                                         "MASTER_ADDR", "MASTER_PORT", "HCB_BENCH_SPAWNED")}),
              file=result_out, flush=True)
        return 0

    import torch
    import torch.distributed as dist

    if not torch.cuda.is_available():
        print("bench.py needs a GPU", file=sys.stderr)
        return 2
    # rehearsal knobs for a one-GPU box (never used by the driver): every rank on device 0
    # and gloo instead of RCCL, which refuses two ranks on one device
    if os.environ.get("HCB_BENCH_ONE_DEVICE") == "1":
        local_rank = 0
    if local_rank >= torch.cuda.device_count():
        print(f"[rank {rank}] LOCAL_RANK {local_rank} but {torch.cuda.device_count()} GPU(s) visible",
              file=sys.stderr)
        return 3
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)

    from azure_hc_intel_tf_amd.ops import _ext

    _ext.load()
    # the headline is measured at the reference's precision: tf_cnn_benchmarks trains fp32
    # (MKL-DNN, run-tf-sing-ucx-openmpi.sh:62-81, no --use_fp16); the same invocation also times
    # the bf16 step as a secondary figure
    primary = args.compute_dtype or ("fp16" if args.use_fp16 else "fp32")
    secondary = args.secondary if args.secondary != "auto" else (
        "bf16" if (args.compute_dtype is None and not args.use_fp16) else "none")
    all_min = _all_min_fn(world, dev)
    code, reducer, backend, rccl_nranks = init_comm(args, world, rank, dev, all_min)
    if code:
        return code

    if world == 1 and args.force_dp_path:
        from azure_hc_intel_tf_amd.parallel.native import NativeReducer

        reducer = NativeReducer(compression=args.compression, force=True)
        rccl_nranks = reducer.comm.size()
    results = [run_model(args, primary, world, rank, dev, reducer, all_min)]
    if secondary not in ("none", primary):
        results.append(run_model(args, secondary, world, rank, dev, reducer, all_min))
    main_r = results[0]
    B = args.batch_size
    if rank == 0:
        res = {
            "metric": METRIC if (args.model == "resnet50" and B == 64)
            else f"images/sec (whole node) {args.model} bs={B}/worker",
            "value": round(main_r["ips"], 2),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": max(args.warmup, 0),
            "ms_per_step": round(main_r["ms"], 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (main_r["ips"] / BASELINE_VALUE) if BASELINE_VALUE else None,
            "dtype": primary,
            "data": f"synthetic (truncated-normal ImageNet {main_r['image_size']}x{main_r['image_size']}, "
                    "random-init weights)",
            "world": world,
            "rccl_nranks": rccl_nranks,
            "comm": main_r["comm"],
            # one-shot xGMI allreduce (HCB_XGMI_BYTES): "off" | "on" (passed the startup cross-check
            # against RCCL) | "disabled(reason)"
            "xgmi": getattr(reducer, "xgmi_status", "off"),
        }
        for r in results[1:]:
            d = r["dtype"]
            res[f"{d}_value"] = round(r["ips"], 2)
            res[f"{d}_ms_per_step"] = round(r["ms"], 3)
            res[f"{d}_final_loss"] = round(r["loss"], 4)
            res[f"{d}_comm"] = r["comm"]
        res["config"] = {"model": args.model, "global_batch": B * world, "per_gpu_batch": B, "seq_len": None,
                         "image_size": main_r["image_size"], "parallelism": f"dp{world}",
                         "optimizer": "momentum(0.9)+wd4e-5, fp32 master", "graph": main_r["graph"],
                         "engine": args.engine if (world > 1 or args.force_dp_path) else None,
                         "backend": backend, "compression": args.compression,
                         "backward_segments": args.backward_segments,
                         "loss_scaling": "dynamic" if primary == "fp16" else None,
                         "precision": {"fp32": "fp32 activations/accumulation; every GEMM operand as bf16 "
                                                "hi+mid+lo planes, six MFMA products (bf16x6, ~2^-24 per product)",
                                       "bf16": "bf16 activations, fp32 accumulation/statistics/masters",
                                       "fp16": "IEEE fp16 activations, fp32 accumulation, loss scaling"}.get(primary),
                         "kernels": "hip" if main_r["native"] else "pytorch-reference (MIOpen/rocBLAS)",
                         "final_loss": round(main_r["loss"], 4)}
        print(json.dumps(res), file=result_out, flush=True)
    if reducer is not None and hasattr(reducer, "close"):
        reducer.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
