"""bench.py --gpus N scaling entry: without a rank environment the process only launches N
worker children (one per GPU) and fails loudly when the node cannot give it N GPUs
(the reference's ``mpirun -np TOTAL_WORKERS``, run-tf-sing-ucx-openmpi.sh:99-109)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    e = {k: v for k, v in os.environ.items()
         if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_PORT")}
    e.update(kw)
    return e


def test_gpus4_spawns_four_ranks_with_rank_env():
    out = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--steps", "1", "--warmup", "0"],
                         env=_env(HCB_BENCH_ONE_DEVICE="1", HCB_BENCH_STUB_WORKER="1"),
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    recs = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(recs) == 4
    assert sorted(int(r["RANK"]) for r in recs) == [0, 1, 2, 3]
    assert sorted(int(r["LOCAL_RANK"]) for r in recs) == [0, 1, 2, 3]
    assert {r["WORLD_SIZE"] for r in recs} == {"4"} and {r["LOCAL_WORLD_SIZE"] for r in recs} == {"4"}
    assert {r["MASTER_ADDR"] for r in recs} == {"127.0.0.1"} and len({r["MASTER_PORT"] for r in recs}) == 1
    assert {r["HCB_BENCH_SPAWNED"] for r in recs} == {"1"}


def test_more_gpus_than_visible_fails_loudly():
    out = subprocess.run([sys.executable, BENCH, "--gpus", "8"], env=_env(HIP_VISIBLE_DEVICES=""),
                         capture_output=True, text=True, timeout=300)
    assert out.returncode != 0
    assert "GPU(s) visible" in out.stderr
    assert '"n_gpus"' not in out.stdout


def test_world_size_must_match_gpus():
    out = subprocess.run([sys.executable, BENCH, "--gpus", "2"],
                         env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"),
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 3 and "refusing" in out.stderr


def test_spawned_worker_failure_propagates():
    # no stub: the children find no GPU and exit 2; the parent must exit non-zero too
    out = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1", "--warmup", "0"],
                         env=_env(HCB_BENCH_ONE_DEVICE="1", HIP_VISIBLE_DEVICES=""),
                         capture_output=True, text=True, timeout=300)
    assert out.returncode != 0


def test_launcher_parent_never_loads_torch():
    """The process that forks the workers counts GPUs from the KFD topology: torch (and with it
    the HIP runtime) must not be loaded there, on the spawn path and on the refusal path."""
    for extra in ({"HCB_BENCH_ONE_DEVICE": "1", "HCB_BENCH_STUB_WORKER": "1"}, {}):
        out = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--steps", "1", "--warmup", "0"],
                             env=_env(**extra), capture_output=True, text=True,
                             timeout=300)
        assert "[bench] launcher parent: torch loaded = False" in out.stderr, out.stderr


def test_visible_gpu_count_from_kfd_topology(tmp_path, monkeypatch):
    from azure_hc_intel_tf_amd.launch import launcher

    root = tmp_path / "class/kfd/kfd/topology/nodes"
    for n, simd in enumerate([0, 256, 256, 256]):  # one CPU agent, three GPUs
        d = root / str(n)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"simd_count {simd}\nlocation_id {n * 8}\ndomain 0\n")
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    assert launcher.visible_gpu_count(str(tmp_path)) == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,2")
    assert launcher.visible_gpu_count(str(tmp_path)) == 2
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert launcher.visible_gpu_count(str(tmp_path)) == 0


def _bench_module():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_under_test", BENCH)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_native_engine_failure_is_a_nonzero_exit(monkeypatch):
    """A native RCCL engine that fails its self-test at N>1 must end the run with a non-zero code
    (never a silent torch.distributed fallback reported as the native engine)."""
    bench = _bench_module()
    monkeypatch.delenv("HCB_BENCH_BACKEND", raising=False)
    args = bench.parse_args(["--gpus", "2"])
    assert args.engine == "native"

    def broken(kind, compression=None):
        raise RuntimeError("ncclCommInitRank failed")

    code, reducer, backend, n = bench.init_comm(args, 2, 0, "cpu", lambda v: v, make_reducer=broken,
                                                init_pg=False)
    assert code == 5 and reducer is None and backend == "nccl"
    # the same failure on ANOTHER rank (this one healthy) must end this rank too
    with __import__("pytest").raises(bench.EngineUnavailable):
        bench.setup_native_reducer(args, 2, 1, "cpu", broken, lambda v: 0)
    # --engine torch is the explicit opt-in to the torch.distributed reducer
    args_t = bench.parse_args(["--gpus", "2", "--engine", "torch"])
    made = []
    code, reducer, _, _ = bench.init_comm(args_t, 2, 0, "cpu", lambda v: v,
                                          make_reducer=lambda k, compression=None: made.append(k) or object(),
                                          init_pg=False)
    assert code == 0 and made == ["torch"]


def test_default_headline_is_reference_precision():
    """bench.py reports fp32 (the reference's MKL-DNN precision) as the headline value and times bf16
    as the secondary figure in the same invocation."""
    bench = _bench_module()
    a = bench.parse_args([])
    assert a.compute_dtype is None and a.secondary == "auto" and not a.use_fp16
    src = open(BENCH).read()
    assert 'primary = args.compute_dtype or ("fp16" if args.use_fp16 else "fp32")' in src
    assert 'res[f"{d}_value"]' in src
