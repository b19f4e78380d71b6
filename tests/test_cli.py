"""CLI / flag / launcher-math parity with the reference runners (no GPU)."""
import json
import os
import subprocess
import sys

import pytest

from azure_hc_intel_tf_amd.bench.benchmark_cnn import get_perf_timing_str
from azure_hc_intel_tf_amd.bench.flags import noop_flags_set, parse_flags
from azure_hc_intel_tf_amd.launch.launcher import cpu_shares, fabric_env, worker_env
from azure_hc_intel_tf_amd.launch.run_tf_sing import tf_args, worker_math

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

REFERENCE_FLAGS = [  # /root/reference/benchmark-scripts/run-tf-sing-ucx-openmpi.sh:62-81
    "--batch_size=64", "--num_warmup_batches=50", "--num_batches=100", "--model=resnet50",
    "--num_intra_threads=11", "--num_inter_threads=2", "--kmp_blocktime=1",
    "--kmp_affinity=granularity=fine,noverbose,compact,1,0", "--display_every=10", "--data_format=NCHW",
    "--optimizer=momentum", "--forward_only=False", "--device=cpu", "--mkl=TRUE", "--variable_update=horovod",
    "--horovod_device=cpu", "--local_parameter_device=cpu", "--data_dir=/mnt/shared/imagenet-data/tfrecords-20",
    "--data_name=imagenet",
]


def test_reference_flag_set_parses():
    p = parse_flags(REFERENCE_FLAGS)
    assert p.batch_size == 64 and p.num_warmup_batches == 50 and p.num_batches == 100
    assert p.model == "resnet50" and p.optimizer == "momentum" and p.mkl is True and p.forward_only is False
    assert p.variable_update == "horovod" and p.horovod_device == "cpu" and p.data_format == "NCHW"
    assert not p._unknown
    assert "mkl" in noop_flags_set(p) and "kmp_blocktime" in noop_flags_set(p)


def test_bool_flag_forms():
    assert parse_flags(["--use_fp16"]).use_fp16 is True
    assert parse_flags(["--nouse_hip_graph"]).use_hip_graph is False
    assert parse_flags(["--forward_only=1"]).forward_only is True
    p = parse_flags(["--some_future_tf_flag=3"])
    assert p._unknown == ["--some_future_tf_flag=3"]


@pytest.mark.parametrize("wps,sockets,cps,gpus,exp_wpn,exp_total", [
    (0, 2, 22, 8, 1, 4),      # reference quirk fixed: WPS=0 -> 1 worker per node
    (1, 2, 22, 8, 2, 8),
    (4, 2, 22, 8, 8, 16),
    (8, 2, 22, 8, 8, 16),     # capped at one worker per GPU
])
def test_worker_math_gpu(wps, sockets, cps, gpus, exp_wpn, exp_total):
    p = worker_math(2 if exp_total > exp_wpn else 4, wps, sockets, cps, "gpu", gpus)
    assert p.workers_per_node == exp_wpn


def test_worker_math_cpu_matches_reference():
    # run-tf-sing-ucx-openmpi.sh:40-50 on a 2-socket 22-core node (HC44rs)
    p = worker_math(4, 1, 2, 22, "cpu")
    assert (p.workers_per_node, p.cores_per_worker, p.intra_t, p.inter_t, p.total_workers) == (2, 22, 11, 2, 8)
    p = worker_math(2, 2, 2, 22, "cpu")
    assert (p.workers_per_node, p.cores_per_worker, p.intra_t, p.total_workers) == (4, 11, 5, 8)
    p = worker_math(1, 0, 2, 22, "cpu")
    assert (p.workers_per_node, p.cores_per_worker, p.intra_t) == (1, 44, 22)


def test_tf_args_are_reference_flags(monkeypatch):
    monkeypatch.delenv("EXTRA_ARGS", raising=False)
    p = worker_math(1, 1, 2, 22, "cpu", batch_size=64)
    args = tf_args(p, env={})
    parsed = parse_flags(args)
    assert parsed.model == "resnet50" and parsed.num_warmup_batches == 50 and parsed.num_batches == 100
    assert parsed.num_intra_threads == 11 and parsed.variable_update == "horovod"


def test_fabric_env_and_worker_env():
    assert fabric_env("ib") == {}
    e = fabric_env("sock")
    assert e["NCCL_P2P_DISABLE"] == "1" and e["NCCL_SHM_DISABLE"] == "1"
    w = worker_env({}, 5, 1, 8, 4, 1, "10.0.0.1", 1234, "ib", 11)
    assert w["RANK"] == "5" and w["LOCAL_RANK"] == "1" and w["WORLD_SIZE"] == "8" and w["GROUP_RANK"] == "1"
    assert w["OMP_NUM_THREADS"] == "11" and w["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    shares = cpu_shares(4, list(range(16)))
    assert shares == [[0, 1, 2, 3], [4, 5, 6, 7], [8, 9, 10, 11], [12, 13, 14, 15]]


def test_perf_timing_string_format():
    s = get_perf_timing_str(64, [0.1, 0.1, 0.1])
    assert s == "images/sec: 640.0 +/- 0.0 (jitter = 0.0)"


def test_run_script_dry_run():
    env = dict(os.environ, DRY_RUN="1", DEVICE="cpu")
    out = subprocess.run([os.path.join(ROOT, "benchmark-scripts", "run-tf-sing-ucx-openmpi.sh"), "2", "1", "64",
                          "sock"], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "TOTAL_WORKERS" in out.stdout and "tf_cnn_benchmarks.py" in out.stdout
    bad = subprocess.run([os.path.join(ROOT, "benchmark-scripts", "run-tf-sing-libfabric-intelmpi.sh"), "1"],
                         env=env, capture_output=True, text=True, timeout=60)
    assert bad.returncode != 0 and "usage" in bad.stderr


def test_default_gpu_precision_is_fp32_on_hip_kernels():
    """tf_cnn_benchmarks without --use_fp16 trains fp32 -- the reference's precision
    (run-tf-sing-ucx-openmpi.sh:62-81) -- so the GPU default is fp32, on the HIP kernels for the
    ResNets; --compute_dtype bf16 / --use_fp16 opt out."""
    from azure_hc_intel_tf_amd.bench.flags import compute_dtype_of, precision_label

    p = parse_flags(REFERENCE_FLAGS[:-2] + ["--device=gpu"])
    assert compute_dtype_of(p) == "fp32"
    assert precision_label(p) == "fp32 (HIP kernels)"
    assert compute_dtype_of(parse_flags(["--use_fp16"])) == "fp16"
    assert compute_dtype_of(parse_flags(["--use_fp16", "--half_dtype=bf16"])) == "bf16"
    assert precision_label(parse_flags(["--compute_dtype=bf16"])) == "bf16 (HIP kernels)"


def test_fp32_native_model_list_matches_model_classes():
    from azure_hc_intel_tf_amd.bench.flags import FP32_NATIVE_MODELS
    from azure_hc_intel_tf_amd.models import _MODELS, model_names
    from azure_hc_intel_tf_amd.models import base

    seen = {}
    orig = base.CNNModel.__init__

    def grab(self, *a, **kw):  # the class attribute, without building the model
        seen["ok"] = type(self).F32_NATIVE_OK
        raise StopIteration

    base.CNNModel.__init__ = grab
    try:
        for name in model_names():
            seen.clear()
            try:
                _MODELS[name](device="cpu")
            except StopIteration:
                pass
            assert seen["ok"] == (name in FP32_NATIVE_MODELS), name
    finally:
        base.CNNModel.__init__ = orig


def test_run_script_dry_run_logs_fp32_hip_precision():
    env = dict(os.environ, DRY_RUN="1", GPUS_PER_NODE="8")
    env.pop("DEVICE", None)
    out = subprocess.run([os.path.join(ROOT, "benchmark-scripts", "run-tf-sing-ucx-openmpi.sh"), "1", "4", "64",
                          "ib"], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "Precision: fp32 (HIP kernels)" in out.stdout


def test_cpu_benchmark_end_to_end(tmp_path):
    js = tmp_path / "s.json"
    cmd = [sys.executable, os.path.join(ROOT, "tf_cnn_benchmarks.py"), "--device=cpu", "--model=resnet50",
           "--batch_size=2", "--image_size=32", "--num_batches=3", "--num_warmup_batches=1", "--display_every=1",
           "--optimizer=momentum", f"--json_summary={js}", f"--train_dir={tmp_path / 'ckpt'}",
           "--print_training_accuracy"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "Step\tImg/sec\ttotal_loss\ttop_1_accuracy\ttop_5_accuracy" in out.stdout
    assert "total images/sec:" in out.stdout
    s = json.loads(js.read_text())
    assert 0.0 <= s["top_1_accuracy"] <= s["top_5_accuracy"] <= 1.0
    assert s["workers"] == 1 and s["num_batches"] == 3 and s["total_images_per_sec"] > 0
    assert (tmp_path / "ckpt" / "model.ckpt-4.pt").exists()
    # resume continues from the saved step
    out2 = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert out2.returncode == 0 and "Restored checkpoint at step 4" in out2.stdout


def test_launcher_propagates_rank_failure(tmp_path):
    """Fault injection (--fault_rank/--fault_step) under the per-GPU launcher: rank 1 dies at step 2
    while rank 0 waits in the next allreduce; the launcher must tear rank 0 down and exit with the
    failing rank's code instead of hanging (MPI_Abort semantics, SURVEY.md §5 failure detection)."""
    import time
    cmd = [sys.executable, "-m", "azure_hc_intel_tf_amd.launch.launcher", "--nproc_per_node", "2", "--no_pin",
           "--", sys.executable, os.path.join(ROOT, "tf_cnn_benchmarks.py"), "--device=cpu", "--model=trivial",
           "--batch_size=2", "--image_size=32", "--num_batches=50", "--num_warmup_batches=1",
           "--variable_update=horovod", "--horovod_device=cpu", "--fault_rank=1", "--fault_step=2"]
    t0 = time.time()
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT,
                         env=dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1"))
    assert out.returncode == 17, out.stdout[-2000:] + out.stderr[-2000:]
    assert "[fault injection] rank 1 aborting at step 2" in out.stdout
    assert time.time() - t0 < 200


def test_cpu_shares_follow_gpu_numa_nodes(tmp_path):
    """Each worker is pinned to the cores of its GPU's NUMA node (fake sysfs: 4 GPUs, two per
    socket, behind two CPU agents)."""
    sysfs = tmp_path
    topo = sysfs / "class/kfd/kfd/topology/nodes"
    cpu_props = "cpu_cores_count 64\nsimd_count 0\nlocation_id 0\ndomain 0\n"
    gpus = [(0x1100, 0), (0x2100, 0), (0x9100, 1), (0xa100, 1)]
    (topo / "0").mkdir(parents=True)
    (topo / "0" / "properties").write_text(cpu_props)
    (topo / "1").mkdir()
    (topo / "1" / "properties").write_text(cpu_props)
    for i, (loc, node) in enumerate(gpus):
        d = topo / str(i + 2)
        d.mkdir()
        d.joinpath("properties").write_text(f"cpu_cores_count 0\nsimd_count 1024\nlocation_id {loc}\ndomain 0\n")
        bdf = f"0000:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7:x}"
        (sysfs / "bus/pci/devices" / bdf).mkdir(parents=True)
        (sysfs / "bus/pci/devices" / bdf / "numa_node").write_text(f"{node}\n")
    for node, cl in ((0, "0-7,16-23"), (1, "8-15,24-31")):
        (sysfs / f"devices/system/node/node{node}").mkdir(parents=True)
        (sysfs / f"devices/system/node/node{node}/cpulist").write_text(cl + "\n")
    from azure_hc_intel_tf_amd.launch.launcher import gpu_numa_nodes

    assert gpu_numa_nodes(str(sysfs)) == [0, 0, 1, 1]
    sh = cpu_shares(4, list(range(32)), sysfs=str(sysfs))
    assert sh[0] == [0, 1, 2, 3, 4, 5, 6, 7] and sh[1] == [16, 17, 18, 19, 20, 21, 22, 23]
    assert sh[2] == list(range(8, 16)) and sh[3] == list(range(24, 32))
    # unknown topology: contiguous equal shares
    assert cpu_shares(2, list(range(8)), sysfs=str(tmp_path / "none")) == [[0, 1, 2, 3], [4, 5, 6, 7]]


def test_flavors_differ_like_the_reference_runners():
    """IMPI runner: no core pinning, transport debug on, no HOROVOD_MPI_THREADS_DISABLE
    (run-tf-sing-libfabric-intelmpi.sh:94-105); OpenMPI runner: pinning + threads-disable."""
    from azure_hc_intel_tf_amd.launch.run_tf_sing import flavor_settings

    u, i = flavor_settings("ucx-openmpi"), flavor_settings("libfabric-intelmpi")
    assert u["pin"] and not i["pin"]
    assert u["env"]["HOROVOD_MPI_THREADS_DISABLE"] == "1" and "HOROVOD_MPI_THREADS_DISABLE" in i["unset"]
    assert i["env"]["NCCL_DEBUG"] == "INFO" and "NCCL_DEBUG" not in u["env"]
    env = dict(os.environ, DRY_RUN="1", DEVICE="cpu")
    out = subprocess.run([os.path.join(ROOT, "benchmark-scripts", "run-tf-sing-libfabric-intelmpi.sh"), "1", "1", "32",
                          "ib"], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "--no_pin" in out.stdout and "NCCL_DEBUG=INFO" in out.stdout
    out = subprocess.run([os.path.join(ROOT, "benchmark-scripts", "run-tf-sing-ucx-openmpi.sh"), "1", "1", "32",
                          "ib"], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and "--no_pin" not in out.stdout and "HOROVOD_MPI_THREADS_DISABLE=1" in out.stdout


def test_api_default_gpu_precision_is_fp32():
    """create_model(..., device="cuda") trains at the reference's precision, fp32, like the CLI,
    the runners and bench.py; bf16 / fp16 are opt-in. Checked on the CPU
    through the dtype resolution itself (no GPU needed)."""
    from azure_hc_intel_tf_amd.models.base import check_compute_dtype

    assert check_compute_dtype(None, "cuda") == "fp32"
    assert check_compute_dtype(None, "cuda:0") == "fp32"
    assert check_compute_dtype("bf16", "cuda") == "bf16"
    assert check_compute_dtype(None, "cpu") == "fp32"


def test_resnet_v2_is_fp32_native():
    from azure_hc_intel_tf_amd.bench.flags import FP32_NATIVE_MODELS, parse_flags, precision_label
    from azure_hc_intel_tf_amd.models.resnet import ResNetV2

    assert ResNetV2.F32_NATIVE_OK
    for n in ("resnet50_v2", "resnet101_v2", "resnet152_v2"):
        assert n in FP32_NATIVE_MODELS
        assert precision_label(parse_flags([f"--model={n}"])) == "fp32 (HIP kernels)"


def test_multi_node_fanout_from_one_shell(tmp_path, capsys, monkeypatch):
    """FANOUT=1 on the hostfile's first node (the reference's mpirun -hostfile): one ssh command per
    other host, starting the same runner with the overrides and HCB_* / NCCL_* variables forwarded,
    marked as a child (no second fan-out); the child itself plans no fan-out."""
    from azure_hc_intel_tf_amd.launch import run_tf_sing as R

    hf = tmp_path / "nodeips.txt"
    hf.write_text("127.0.0.1\nnode-b\nnode-c\n")
    for k, v in {"HOSTFILE": str(hf), "FANOUT": "1", "DRY_RUN": "1", "DEVICE": "cpu", "MODEL": "resnet101",
                 "HCB_X": "7", "NCCL_DEBUG": "WARN", "SSH": "fakessh -p 22"}.items():
        monkeypatch.setenv(k, v)
    monkeypatch.delenv("HCB_FANOUT_CHILD", raising=False)
    assert R.main(["3", "1", "64", "ib"]) == 0
    out = capsys.readouterr().out
    fan = [l for l in out.splitlines() if l.startswith("FANOUT: ")]
    assert len(fan) == 2 and "node-b" in fan[0] and "node-c" in fan[1], out
    for l in fan:
        assert l.startswith("FANOUT: fakessh -p 22 node-")
        for tok in ("HCB_FANOUT_CHILD=1", "MODEL=resnet101", "HCB_X=7", "NCCL_DEBUG=WARN",
                    "azure_hc_intel_tf_amd.launch.run_tf_sing 3 1 64 ib"):
            assert tok in l, (tok, l)
        assert "DRY_RUN" not in l and "FANOUT=1" not in l
    monkeypatch.setenv("HCB_FANOUT_CHILD", "1")
    assert R.main(["3", "1", "64", "ib"]) == 0
    assert "FANOUT: " not in capsys.readouterr().out
