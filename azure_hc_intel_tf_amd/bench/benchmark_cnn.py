"""BenchmarkCNN: the tf_cnn_benchmarks driver loop on the MI355X engine.

Reproduces the behaviour the reference harness relies on (SURVEY.md §2.2 "benchmark_cnn.py",
§3.3): parse flags -> setup (threads / KMP env on the CPU path) -> hvd.init -> build model +
synthetic ImageNet -> broadcast variables from rank 0 -> ``num_warmup_batches`` untimed steps
-> ``num_batches`` timed steps logging ``Step / Img/sec / total_loss`` every
``display_every`` steps in the tf_cnn_benchmarks format -> ``total images/sec``.
Plus: machine-readable JSON summary, checkpoint/resume (``--train_dir``), ``--trace_file``,
fault injection and the HOROVOD_* environment knobs.
"""
from __future__ import annotations

import json
import math
import os
import platform
import sys
import time
from typing import List, Optional

import numpy as np
import torch

from .flags import Params, compute_dtype_of, noop_flags_set, parse_flags

MODEL_DEFAULT_BATCH = {"inception3": 32, "trivial": 32, "alexnet": 512, "googlenet": 32, "overfeat": 32,
                       "lenet": 32, "vgg11": 32, "vgg16": 32, "vgg19": 32}


def log_fn(msg: str = ""):
    print(msg, flush=True)


def get_perf_timing_str(batch_size: int, step_train_times: List[float], scale: int = 1) -> str:
    """tf_cnn_benchmarks' per-step throughput line."""
    times = np.array(step_train_times, dtype=np.float64)
    speeds = batch_size / times
    speed_mean = scale * batch_size / np.mean(times)
    speed_uncertainty = np.std(speeds) / np.sqrt(float(len(speeds)))
    speed_jitter = 1.4826 * np.median(np.abs(speeds - np.median(speeds)))
    return "images/sec: %.1f +/- %.1f (jitter = %.1f)" % (speed_mean, speed_uncertainty, speed_jitter)


def setup(params: Params):
    """benchmark_cnn.setup(): host threading env (the reference's --num_intra_threads /
    --num_inter_threads / --kmp_* flags, run-tf-sing-ucx-openmpi.sh:67-70)."""
    if params.device == "cpu":
        if params.kmp_blocktime is not None:
            os.environ.setdefault("KMP_BLOCKTIME", str(params.kmp_blocktime))
        if params.kmp_affinity:
            os.environ.setdefault("KMP_AFFINITY", str(params.kmp_affinity))
        if params.num_intra_threads:
            torch.set_num_threads(int(params.num_intra_threads))
        if params.num_inter_threads:
            try:
                torch.set_num_interop_threads(int(params.num_inter_threads))
            except RuntimeError:
                pass
    return params


class BenchmarkCNN:
    def __init__(self, params: Params):
        from ..parallel import hvd

        self.params = params
        self.hvd = hvd
        p = params
        if p.variable_update in ("parameter_server", "distributed_replicated"):
            raise ValueError(f"--variable_update={p.variable_update} is not supported; use horovod")
        if p.num_gpus != 1:
            raise ValueError("one process per MI355X: use --num_gpus=1 and launch one worker per GPU")
        if not 0.0 <= p.label_smoothing <= 1.0:
            raise ValueError("--label_smoothing must be in [0, 1]")
        self.on_gpu = p.device == "gpu"
        if self.on_gpu and not torch.cuda.is_available():
            raise RuntimeError("--device=gpu but no GPU is visible (use --device=cpu for the CPU path)")
        backend = None
        if p.horovod_device == "cpu" or not self.on_gpu:
            backend = "gloo"
        hvd.init(backend=backend)
        self.rank, self.size, self.local_rank = hvd.rank(), hvd.size(), hvd.local_rank()
        if self.on_gpu:
            torch.cuda.set_device(self.local_rank)
            self.device = torch.device("cuda", self.local_rank)
            from ..ops import _ext

            _ext.load()
        else:
            self.device = torch.device("cpu")
        self.model_name = p.model
        self.batch_size = p.batch_size or MODEL_DEFAULT_BATCH.get(p.model, 64)
        self.num_batches = p.num_batches
        if p.num_warmup_batches is None:
            self.num_warmup_batches = 10 if self.on_gpu else 2
        else:
            self.num_warmup_batches = p.num_warmup_batches
        from ..models import create_model

        kw = {"device": self.device, "seed": p.tf_random_seed}
        if self.on_gpu:
            # tf_cnn_benchmarks trains fp32 unless --use_fp16, and the reference runs it without
            # (run-tf-sing-ucx-openmpi.sh:62-81): fp32 is the default here too, on the HIP plane
            # GEMMs (bf16x6) for the models that have them; --compute_dtype bf16 / --use_fp16 opt out
            self.compute_dtype = compute_dtype_of(p)
            kw["compute_dtype"] = self.compute_dtype
        else:
            self.compute_dtype = "fp32"
        if p.image_size:
            kw["image_size"] = p.image_size
        self.model = create_model(p.model, **kw)
        if p.num_epochs:
            self.num_batches = int(math.ceil(p.num_epochs * 1281167 / (self.batch_size * self.size)))
        self.step_offset = 0
        if self.on_gpu and p.autotune and self.model.native:
            # per-shape kernel configs (cached in tuned/mi355x.json; new shapes timed once here)
            from ..ops import autotune

            autotune.load_cache()
            n = autotune.tune_model(self.model, self.batch_size, save=(self.rank == 0))
            if n and self.rank == 0:
                log_fn(f"Autotuned {n} conv problems")
        self._build_trainer()

    # ------------------------------------------------------------------ setup pieces
    def _lr_fn(self):
        from ..trainer import constant_lr, resnet_lr_schedule

        p = self.params
        if p.init_learning_rate is not None:
            return constant_lr(p.init_learning_rate)
        gb = self.batch_size * self.size
        if self.model_name.startswith("resnet"):
            return resnet_lr_schedule(gb)
        # tf_cnn_benchmarks Model defaults: a constant rate scaled by global batch / the
        # model's default batch size
        m = self.model
        return constant_lr(getattr(m, "default_lr", 0.005) * gb / float(getattr(m, "default_batch_size", 32)))

    def _build_trainer(self):
        from ..parallel import make_reducer
        from ..trainer import Trainer

        p = self.params
        reducer = None
        comp = None if p.gradient_compression == "none" else p.gradient_compression
        if self.size > 1:
            engine = p.comm_engine if self.on_gpu and p.horovod_device != "cpu" else "torch"
            reducer = make_reducer(engine, compression=comp)
        self.reducer = reducer
        mom = p.momentum if p.optimizer == "momentum" else 0.0
        self.trainer = Trainer(self.model, self.batch_size, self._lr_fn(), momentum=mom,
                               weight_decay=p.weight_decay, reducer=reducer, world_size=self.size,
                               use_graph=bool(p.use_hip_graph) and self.on_gpu and p.horovod_device != "cpu",
                               forward_only=bool(p.forward_only), label_smoothing=p.label_smoothing,
                               # --use_fp16: loss scaling as in the reference flags (static scale or
                               # automatic scaling), whichever 16-bit type computes
                               loss_scale=p.fp16_loss_scale if p.use_fp16 else None,
                               dynamic_loss_scale=bool(p.use_fp16 and p.fp16_enable_auto_loss_scale),
                               loss_scale_interval=p.fp16_inc_loss_scale_every_n,
                               comm_check=True if p.comm_check else None)
        if p.horovod_device == "cpu" and self.size > 1 and self.on_gpu:
            self.trainer.reducer = _HostStagedReducer(reducer)

    # ------------------------------------------------------------------ info
    def print_info(self):
        p = self.params
        if self.rank != 0:
            return
        dev = [f"/gpu:{self.local_rank}"] if self.on_gpu else ["/cpu:0"]
        log_fn(f"Framework:   azure_hc_intel_tf_amd (PyTorch {torch.__version__}, HIP {torch.version.hip})")
        log_fn(f"Model:       {self.model_name}")
        log_fn(f"Dataset:     imagenet ({'TFRecords ' + p.data_dir if p.data_dir else 'synthetic'})")
        log_fn(f"Mode:        {'forward-only' if p.forward_only else 'training'}")
        log_fn(f"SingleSess:  False")
        log_fn(f"Batch size:  {self.batch_size * self.size} global")
        log_fn(f"             {self.batch_size} per device")
        log_fn(f"Num batches: {self.num_batches}")
        log_fn(f"Num epochs:  {self.num_batches * self.batch_size * self.size / 1281167:.2f}")
        log_fn(f"Devices:     {dev}")
        log_fn(f"NUMA bind:   False")
        log_fn(f"Data format: {p.data_format} (logical; NHWC kernels)")
        log_fn(f"Precision:   {self.compute_dtype}" + (" (HIP kernels)" if self.model.native else
                                                       " (PyTorch/MIOpen path)" if self.on_gpu else " (CPU)"))
        log_fn(f"Optimizer:   {p.optimizer}")
        log_fn(f"Variables:   {p.variable_update}")
        log_fn(f"Workers:     {self.size} (one process per {'MI355X' if self.on_gpu else 'CPU worker'})")
        log_fn(f"Params:      {self.model.num_params():,} in {self.model.ps.num_tensors()} tensors")
        noop = noop_flags_set(p)
        if noop and self.on_gpu:
            log_fn(f"Ignored on GPU (TF-runtime flags): {noop}")
        if p._unknown:
            log_fn(f"Unrecognized flags (ignored): {p._unknown}")
        log_fn("==========")

    # ------------------------------------------------------------------ run
    def run(self):
        from ..trainer import synthetic_batch
        from ..utils import checkpoint

        p = self.params
        hvd = self.hvd
        images, labels = synthetic_batch(self.model, self.batch_size, seed=p.tf_random_seed + self.rank)
        loader = None
        if p.data_dir:
            # real ImageNet TFRecords: each step's batch is written in place into the static
            # (graph-captured) input buffers by the native prefetch + GPU preprocess pipeline
            from ..data.imagenet import ImageNetLoader

            loader = ImageNetLoader(p.data_dir, self.batch_size, self.model.image_size, self.model.image_channels,
                                    self.device, rank=self.rank, world=self.size, train=not p.forward_only,
                                    seed=p.tf_random_seed, reader_threads=p.datasets_num_private_threads or 4,
                                    decode_threads=p.num_decode_threads or 8)
            if self.rank == 0:
                log_fn(f"Reading {len(loader.files)} TFRecord shards from {p.data_dir}")
        self.loader = loader
        # restore (rank 0) then broadcast_global_variables(0)
        if p.train_dir:
            step = checkpoint.restore_latest(p.train_dir, self.model.ps) if self.rank == 0 else 0
            self.step_offset = int(hvd.broadcast_object(step, 0)) if self.size > 1 else step
            if self.step_offset and self.rank == 0:
                log_fn(f"Restored checkpoint at step {self.step_offset} from {p.train_dir}")
        self.trainer.steps_done = self.step_offset
        if self.size > 1:
            hvd.broadcast_global_variables(self.model, 0)
        sync = torch.cuda.synchronize if self.on_gpu else (lambda: None)

        log_fn("Running warm up") if self.rank == 0 else None
        for i in range(self.num_warmup_batches):
            self._maybe_fault(i - self.num_warmup_batches)
            if loader is not None:
                loader.next_into(images, labels)
            self.trainer.step(images, labels)
        sync()
        hvd.barrier()
        log_fn("Done warm up") if self.rank == 0 else None
        if p.trace_file:
            self._trace_one_step(images, labels, p.trace_file)

        acc = bool(p.print_training_accuracy)
        if self.rank == 0:  # tf_cnn_benchmarks header (+ accuracy columns with --print_training_accuracy)
            log_fn("Step\tImg/sec\ttotal_loss" + ("\ttop_1_accuracy\ttop_5_accuracy" if acc else ""))
        step_times: List[float] = []
        use_events = self.on_gpu
        evs = []
        last_save = time.time()
        sync()
        t_start = time.perf_counter()
        t_prev = t_start
        if use_events:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
            evs.append(e0)
        for i in range(self.num_batches):
            self._maybe_fault(i)
            if loader is not None:
                loader.next_into(images, labels)
            loss_t = self.trainer.step(images, labels)
            if use_events:
                e = torch.cuda.Event(enable_timing=True)
                e.record()
                evs.append(e)
            step = i + 1
            display = step == 1 or step % p.display_every == 0 or step == self.num_batches
            if not use_events:
                now = time.perf_counter()
                step_times.append(now - t_prev)
                t_prev = now
            if display:
                loss = float(loss_t.item())
                if use_events:
                    evs[-1].synchronize()
                    while len(step_times) < len(evs) - 1:
                        k = len(step_times)
                        step_times.append(evs[k].elapsed_time(evs[k + 1]) / 1000.0)
                if self.rank == 0:
                    line = "%i\t%s\t%.3f" % (step, get_perf_timing_str(self.batch_size, step_times), loss)
                    if acc:
                        t1, t5 = self.trainer.accuracy(labels)
                        line += "\t%.3f\t%.3f" % (float(t1), float(t5))
                    log_fn(line)
                if not math.isfinite(loss):
                    raise RuntimeError(f"non-finite loss at step {step}")
            if p.train_dir and self.rank == 0:
                gstep = self.step_offset + self.num_warmup_batches + step
                due = (p.save_model_steps and gstep % p.save_model_steps == 0) or \
                      (p.save_model_secs and time.time() - last_save >= p.save_model_secs)
                if due:
                    checkpoint.save(p.train_dir, gstep, self.model.ps)
                    last_save = time.time()
        sync()
        elapsed = time.perf_counter() - t_start
        if use_events:
            while len(step_times) < len(evs) - 1:
                k = len(step_times)
                step_times.append(evs[k].elapsed_time(evs[k + 1]) / 1000.0)
        elapsed_max = elapsed
        if self.size > 1:
            t = torch.tensor([elapsed], dtype=torch.float64, device=self.device if self.on_gpu else "cpu")
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            elapsed_max = float(t.item())
        images_per_sec = self.size * self.batch_size * self.num_batches / elapsed_max
        own_images_per_sec = self.size * self.batch_size * self.num_batches / elapsed
        final_loss = float(self.trainer.loss.item())
        if self.reducer is not None and hasattr(self.reducer, "check_errors"):
            self.reducer.check_errors()
        if loader is not None:
            loader.close()
        # final state first (checkpoint, accuracy of the last timed step), THEN the comm profile,
        # which runs extra steps (it restores the training state afterwards, and a failure in it
        # cannot lose the measured result)
        if p.train_dir and self.rank == 0:
            checkpoint.save(p.train_dir, self.step_offset + self.num_warmup_batches + self.num_batches,
                            self.model.ps)
        accs = self.trainer.accuracy(labels) if acc else None
        comm = None
        if self.size > 1 and self.on_gpu and p.comm_profile:
            try:
                comm = self.trainer.comm_profile(images, labels)
            except Exception as e:  # noqa: BLE001 -- a profile failure must not lose the timed result
                comm = {"error": f"{type(e).__name__}: {e}"}
                log_fn(f"[rank {self.rank}] comm profile failed: {e}")
        # every worker prints its own total, as tf_cnn_benchmarks does under mpirun
        # (run-tf-sing-ucx-openmpi.sh:99-113); rank 0 reports the job figure (slowest rank)
        if self.rank == 0:
            log_fn("-" * 64)
            log_fn("total images/sec: %.2f" % images_per_sec)
            log_fn("-" * 64)
        else:
            log_fn("[rank %d] total images/sec: %.2f" % (self.rank, own_images_per_sec))
        summary = {
            "model": self.model_name, "device": "MI355X" if self.on_gpu else platform.processor() or "cpu",
            "workers": self.size, "batch_size_per_worker": self.batch_size,
            "global_batch": self.batch_size * self.size, "num_batches": self.num_batches,
            "num_warmup_batches": self.num_warmup_batches, "total_images_per_sec": images_per_sec,
            "elapsed_s": elapsed_max, "final_loss": final_loss,
            "step_time_ms": {"mean": 1000 * float(np.mean(step_times)) if step_times else None,
                             "p50": 1000 * float(np.percentile(step_times, 50)) if step_times else None,
                             "p90": 1000 * float(np.percentile(step_times, 90)) if step_times else None},
            "dtype": self.compute_dtype, "data": "imagenet-tfrecord" if loader else "synthetic",
            "input_decode_s": loader.decode_s if loader else None,
            "variable_update": p.variable_update, "comm_engine": p.comm_engine if self.size > 1 else None,
            "gradient_compression": p.gradient_compression, "hip_graph": self.trainer.use_graph,
            "fusion_threshold_bytes": getattr(self.reducer, "bucket_bytes", None),
            "comm": comm,
        }
        if self.size > 1:
            per_rank = torch.tensor([own_images_per_sec], dtype=torch.float64,
                                    device=self.device if self.on_gpu else "cpu")
            allr = [torch.zeros_like(per_rank) for _ in range(self.size)]
            torch.distributed.all_gather(allr, per_rank)
            summary["per_rank_images_per_sec"] = [round(float(x.item()), 2) for x in allr]
        if accs is not None:
            t1, t5 = accs
            summary["top_1_accuracy"], summary["top_5_accuracy"] = float(t1), float(t5)
        self.summary = summary
        if self.rank == 0:
            out = p.json_summary
            if not out and p.benchmark_log_dir:
                os.makedirs(p.benchmark_log_dir, exist_ok=True)
                out = os.path.join(p.benchmark_log_dir, "summary.json")
            if out:
                os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
                with open(out, "w") as f:
                    json.dump(summary, f, indent=1)
        return summary

    def _maybe_fault(self, step: int):
        p = self.params
        if p.fault_rank >= 0 and p.fault_rank == self.rank and p.fault_step == step:
            log_fn(f"[fault injection] rank {self.rank} aborting at step {step}")
            sys.stdout.flush()
            os._exit(17)

    def _trace_one_step(self, images, labels, path):
        from ..utils.tracing import trace_step

        trace_step(lambda: self.trainer._eager_step(images, labels), path, on_gpu=self.on_gpu)
        if self.rank == 0:
            log_fn(f"Wrote trace of one step to {path}")


class _HostStagedReducer:
    """--horovod_device=cpu: gradients staged to host memory and reduced over gloo (the
    reference's CPU-side Horovod allreduce, run-tf-sing-ucx-openmpi.sh:78)."""

    graph_safe = False

    def __init__(self, inner):
        self.inner = inner
        self._host = None

    def allreduce_(self, flat):
        if self._host is None:
            self._host = torch.empty(flat.numel(), dtype=flat.dtype, pin_memory=True)
        self._host.copy_(flat)
        from ..parallel import hvd

        hvd.allreduce_(self._host, average=False)
        flat.copy_(self._host, non_blocking=True)
        return flat

    def broadcast_(self, t, root=0):
        from ..parallel import hvd

        return hvd.broadcast_(t, root)


def main(argv: Optional[List[str]] = None) -> int:
    params = parse_flags(argv)
    setup(params)
    bench = BenchmarkCNN(params)
    bench.print_info()
    bench.run()
    bench.hvd.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
