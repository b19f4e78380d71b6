"""tf_cnn_benchmarks-compatible flag surface.

Accepts every flag the reference passes (/root/reference/benchmark-scripts/
run-tf-sing-ucx-openmpi.sh:62-81 and run-tf-sing-libfabric-intelmpi.sh:63-82)
in absl style (``--flag=value``, ``--flag value``, ``--flag`` / ``--noflag`` for booleans,
``TRUE/False/1/0`` values) plus the tf_cnn_benchmarks flags the BASELINE configs need.
TensorFlow-runtime-only flags (``--mkl``, ``--kmp_*``, ``--local_parameter_device``,
``--xla`` ...) are accepted; on the GPU they are no-ops and are reported as such.
"""
from __future__ import annotations

import argparse
from dataclasses import dataclass
from typing import Any, Dict, List, Optional

_TRUE = {"true", "1", "yes", "y", "t", "on"}
_FALSE = {"false", "0", "no", "n", "f", "off"}


def parse_bool(v) -> bool:
    if isinstance(v, bool):
        return v
    s = str(v).strip().lower()
    if s in _TRUE:
        return True
    if s in _FALSE:
        return False
    raise argparse.ArgumentTypeError(f"not a boolean: {v!r}")


@dataclass
class Flag:
    name: str
    default: Any
    type: Any
    help: str
    noop_on_gpu: bool = False
    choices: Optional[List[Any]] = None


FLAGS: List[Flag] = [
    # --- the reference's flag set (run-tf-sing-ucx-openmpi.sh:62-81)
    Flag("batch_size", 0, int, "per-device (per-worker) batch size; 0 = model default"),
    Flag("num_warmup_batches", None, int, "untimed warmup steps (default: model/device dependent)"),
    Flag("num_batches", 100, int, "timed steps"),
    Flag("model", "trivial", str, "model name: resnet50|101|152[_v1.5], inception3, vgg11|16|19, alexnet, googlenet, "
         "overfeat, lenet, trivial"),
    Flag("num_intra_threads", 0, int, "host intra-op threads (CPU path: torch.set_num_threads)"),
    Flag("num_inter_threads", 0, int, "host inter-op threads (CPU path)"),
    Flag("kmp_blocktime", 0, int, "KMP_BLOCKTIME for the CPU path", noop_on_gpu=True),
    Flag("kmp_affinity", "granularity=fine,verbose,compact,1,0", str, "KMP_AFFINITY for the CPU path",
         noop_on_gpu=True),
    Flag("kmp_settings", 1, int, "KMP_SETTINGS", noop_on_gpu=True),
    Flag("display_every", 10, int, "log cadence (steps)"),
    Flag("data_format", "NCHW", str, "logical layout (kernels run NHWC internally)", choices=["NCHW", "NHWC"]),
    Flag("optimizer", "sgd", str, "sgd | momentum", choices=["sgd", "momentum"]),
    Flag("forward_only", False, parse_bool, "inference-only benchmark"),
    Flag("device", "gpu", str, "gpu (MI355X) or cpu", choices=["gpu", "cpu"]),
    Flag("mkl", False, parse_bool, "TF-MKL switch", noop_on_gpu=True),
    Flag("variable_update", "horovod", str, "horovod (RCCL data parallel) | replicated (single process)",
         choices=["horovod", "replicated", "parameter_server", "distributed_replicated", "independent"]),
    Flag("horovod_device", "", str, "where gradients are reduced: gpu (RCCL, default) | cpu (gloo)"),
    Flag("local_parameter_device", "gpu", str, "accepted for compatibility", noop_on_gpu=True),
    Flag("data_dir", None, str, "real-data directory; absent = synthetic ImageNet"),
    Flag("data_name", None, str, "dataset name (imagenet)"),
    Flag("datasets_num_private_threads", None, int, "TFRecord reader threads per worker (real data)"),
    Flag("num_decode_threads", None, int, "JPEG decode threads per worker (real data)"),
    # --- tf_cnn_benchmarks flags used by the BASELINE configs / common runs
    Flag("num_gpus", 1, int, "GPUs per process (horovod: 1)"),
    Flag("use_fp16", False, parse_bool, "16-bit compute with loss scaling on the HIP kernels: IEEE fp16 "
         "(--half_dtype=fp16, the -DHCB_F16 kernel build) or bf16 (--half_dtype=bf16)"),
    Flag("half_dtype", "fp16", str, "the 16-bit type --use_fp16 selects", choices=["fp16", "bf16"]),
    Flag("compute_dtype", None, str, "activation / GEMM precision on the GPU: fp32 (default: the reference's "
         "precision, tf_cnn_benchmarks without --use_fp16) | bf16 | fp16; overrides --use_fp16's choice",
         choices=["bf16", "fp32", "fp16"]),
    Flag("fp16_loss_scale", 128.0, float, "static loss scale for --use_fp16"),
    Flag("fp16_enable_auto_loss_scale", False, parse_bool, "dynamic loss scaling for --use_fp16"),
    Flag("fp16_inc_loss_scale_every_n", 1000, int, "double the auto loss scale after N clean steps"),
    Flag("init_learning_rate", None, float, "constant learning rate (overrides the model schedule)"),
    Flag("momentum", 0.9, float, "momentum for --optimizer=momentum"),
    Flag("weight_decay", 0.00004, float, "L2 weight decay (coupled, tf_cnn_benchmarks semantics)"),
    Flag("num_epochs", None, float, "alternative to --num_batches"),
    Flag("train_dir", None, str, "checkpoint directory"),
    Flag("save_model_steps", None, int, "checkpoint every N steps"),
    Flag("save_model_secs", 0, int, "checkpoint every N seconds"),
    Flag("trace_file", "", str, "Chrome trace of one profiled step (torch.profiler / roctracer)"),
    Flag("comm_check", False, parse_bool, "race detector: re-do every overlapped gradient reduction with a blocking "
         "reference allreduce and fail on a mismatch (eager steps; HCB_COMM_CHECK=1)"),
    Flag("benchmark_log_dir", None, str, "directory for the machine-readable JSON summary"),
    Flag("tf_random_seed", 1234, int, "random seed"),
    Flag("print_training_accuracy", False, parse_bool, "log top-1/top-5 of the training batch"),
    Flag("summary_verbosity", 0, int, "accepted"),
    Flag("xla", False, parse_bool, "accepted", noop_on_gpu=True),
    Flag("xla_compile", False, parse_bool, "accepted", noop_on_gpu=True),
    Flag("allow_growth", None, parse_bool, "accepted", noop_on_gpu=True),
    Flag("gradient_repacking", 0, int, "accepted", noop_on_gpu=True),
    Flag("all_reduce_spec", None, str, "accepted", noop_on_gpu=True),
    Flag("label_smoothing", 0.0, float, "label smoothing of the softmax cross-entropy targets: (1-ls)*onehot + ls/num_classes"),
    Flag("image_size", 0, int, "override the model's input resolution (0 = model default)"),
    # --- MI355X engine knobs
    Flag("use_hip_graph", True, parse_bool, "capture the training step in a HIP graph"),
    Flag("autotune", True, parse_bool, "time the conv kernel configs of untuned shapes before the run"),
    Flag("comm_engine", "native", str, "gradient allreduce engine: native (C++ RCCL bucket engine, the one "
         "bench.py measures) | torch (torch.distributed)",
         choices=["native", "torch"]),
    Flag("gradient_compression", "none", str, "none | fp16 | bf16 (Horovod Compression)",
         choices=["none", "fp16", "bf16"]),
    Flag("json_summary", None, str, "write the run summary JSON to this path"),
    Flag("comm_profile", True, parse_bool, "after the timed run (N>1, GPU): measure allreduce time, exposed "
         "communication and overlap % for the JSON summary"),
    Flag("fault_rank", -1, int, "fault injection: rank that aborts (testing)"),
    Flag("fault_step", -1, int, "fault injection: step at which --fault_rank aborts"),
]

_BY_NAME = {f.name: f for f in FLAGS}


class Params(dict):
    __getattr__ = dict.get

    def __setattr__(self, k, v):
        self[k] = v


def _normalise(argv: List[str]) -> List[str]:
    out = []
    for a in argv:
        if a.startswith("--no") and "=" not in a:
            name = a[4:]
            if name in _BY_NAME and _BY_NAME[name].type is parse_bool:
                out.append(f"--{name}=false")
                continue
        if a.startswith("--") and "=" not in a:
            name = a[2:]
            if name in _BY_NAME and _BY_NAME[name].type is parse_bool:
                out.append(f"--{name}=true")
                continue
        out.append(a)
    return out


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="tf_cnn_benchmarks.py",
                                 description="MI355X-native tf_cnn_benchmarks-compatible CNN training benchmark")
    for f in FLAGS:
        kw = dict(default=f.default, help=f.help)
        kw["type"] = f.type
        if f.choices:
            kw["choices"] = f.choices
        ap.add_argument(f"--{f.name}", **kw)
    return ap


def parse_flags(argv: Optional[List[str]] = None, allow_unknown: bool = True) -> Params:
    import sys

    argv = list(sys.argv[1:] if argv is None else argv)
    ap = build_parser()
    ns, unknown = ap.parse_known_args(_normalise(argv))
    p = Params(vars(ns))
    p["_unknown"] = unknown
    if unknown and not allow_unknown:
        ap.error(f"unrecognized flags: {unknown}")
    return p


def noop_flags_set(p: Params) -> Dict[str, Any]:
    """TF-only flags explicitly given a non-default value (reported as no-ops on the GPU)."""
    return {f.name: p[f.name] for f in FLAGS if f.noop_on_gpu and p.get(f.name) != f.default}


# Models whose fp32 step (--compute_dtype fp32, the default) runs on the hand-written HIP kernels
# (bf16x6 plane GEMMs, fp32 BN / pool / loss): their classes set F32_NATIVE_OK. Kept here, torch-free,
# for the launcher's config echo; tests/test_cli.py checks it against the model classes.
FP32_NATIVE_MODELS = frozenset({"resnet50", "resnet50_v1.5", "resnet101", "resnet101_v1.5", "resnet152",
                                "resnet152_v1.5", "resnet50_v2", "resnet101_v2", "resnet152_v2", "inception3", "vgg11", "vgg16", "vgg19", "alexnet", "overfeat",
                                "lenet", "googlenet", "trivial"})


def compute_dtype_of(p: Params) -> str:
    """GPU compute precision of a run: --compute_dtype, else the 16-bit type of --use_fp16, else
    fp32 -- tf_cnn_benchmarks' own default, and what the reference runs
    (/root/reference/benchmark-scripts/run-tf-sing-ucx-openmpi.sh:62-81 passes no --use_fp16)."""
    return p.compute_dtype or (p.half_dtype if p.use_fp16 else "fp32")


def precision_label(p: Params) -> str:
    """'fp32 (HIP kernels)' etc.: the precision and the code path a run of these flags takes."""
    if p.device != "gpu":
        return "fp32 (CPU)"
    dt = compute_dtype_of(p)
    native = dt != "fp32" or p.model in FP32_NATIVE_MODELS
    return f"{dt} ({'HIP kernels' if native else 'PyTorch/MIOpen path'})"
