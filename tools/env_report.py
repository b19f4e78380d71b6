#!/usr/bin/env python3
"""Software / hardware environment report -- the role of the reference container's
``%runscript`` (prints OS, GCC, TF version, MKL libs, IsMklEnabled, Horovod, MPI/UCX, OFED:
/root/reference/install-scripts/tf-hvd-gcc-ompi-ucx-mlnx.def:45-55,
tf-hvd-gcc-ompi-ucx-mlnx-osu.def:48-62), for the MI355X stack: OS, compilers, ROCm, PyTorch
HIP build, RCCL, GPUs (arch / CUs / HBM), the xGMI link topology, NUMA layout, the relevant
environment variables, and whether this framework's native libraries are built and load.

    python tools/env_report.py [--json out.json]

External commands run BEFORE anything touches the GPU (children are started, nothing is
exec'd from a GPU-initialised process).
"""
import argparse
import json
import os
import platform
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def sh(cmd, timeout=20):
    exe = shutil.which(cmd[0]) or (cmd[0] if os.path.exists(cmd[0]) else None)
    if exe is None:
        return None
    try:
        r = subprocess.run([exe] + cmd[1:], capture_output=True, text=True, timeout=timeout)
        return (r.stdout or r.stderr).strip()
    except Exception as e:  # pragma: no cover - diagnostic tool
        return f"<{type(e).__name__}: {e}>"


def first_line(s):
    return None if not s else s.splitlines()[0]


def rocm_version():
    for p in ("/opt/rocm/.info/version", "/opt/rocm/.info/version-dev"):
        if os.path.exists(p):
            return open(p).read().strip()
    return None


def collect():
    rep = {}
    # ---- host side (no GPU touched yet)
    rep["os"] = {"platform": platform.platform(), "python": sys.version.split()[0]}
    if os.path.exists("/etc/os-release"):
        kv = dict(l.strip().split("=", 1) for l in open("/etc/os-release") if "=" in l)
        rep["os"]["distro"] = kv.get("PRETTY_NAME", "").strip('"')
    rep["compilers"] = {"gcc": first_line(sh(["gcc", "--version"])),
                        "hipcc": first_line(sh(["/opt/rocm/bin/hipcc", "--version"])),
                        "cmake": first_line(sh(["cmake", "--version"]))}
    rep["rocm"] = {"version": rocm_version()}
    topo = sh(["rocm-smi", "--showtopo"], timeout=30)
    rep["xgmi_topology"] = topo
    rep["numa"] = sh(["lscpu"])
    if rep["numa"]:
        keep = ("Model name", "Socket(s)", "Core(s) per socket", "Thread(s) per core", "NUMA node")
        rep["numa"] = "\n".join(l for l in rep["numa"].splitlines() if l.startswith(keep))
    rep["env"] = {k: v for k, v in sorted(os.environ.items())
                  if k.startswith(("HSA_", "HIP_", "ROCR_", "NCCL_", "RCCL_", "HOROVOD_", "HCB_", "OMP_",
                                   "GPU_MAX_HW_QUEUES", "PYTORCH_ROCM_ARCH"))}
    # ---- python / torch / GPU
    import torch

    rep["torch"] = {"version": torch.__version__, "hip": getattr(torch.version, "hip", None),
                    "cxx11_abi": bool(torch._C._GLIBCXX_USE_CXX11_ABI)}
    try:
        v = torch.cuda.nccl.version()
        rep["torch"]["rccl"] = ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
    except Exception as e:  # pragma: no cover
        rep["torch"]["rccl"] = f"<{e}>"
    gpus = []
    n = torch.cuda.device_count()
    if n and torch.cuda.is_available():
        for i in range(n):
            p = torch.cuda.get_device_properties(i)
            gpus.append({"index": i, "name": p.name, "arch": getattr(p, "gcnArchName", None),
                         "cus": p.multi_processor_count, "hbm_GiB": round(p.total_memory / 2 ** 30, 1)})
    rep["gpus"] = gpus
    # ---- this framework's native libraries
    from azure_hc_intel_tf_amd import _build

    nat = {"kernels_so": os.path.exists(_build.KERNELS_SO), "comm_so": os.path.exists(_build.COMM_SO),
           "rccl_bench": os.path.exists(_build.RCCL_BENCH), "offload_arch": _build.ARCH}
    if nat["kernels_so"] and gpus:
        try:
            from azure_hc_intel_tf_amd.ops import _ext

            _ext.load(build_if_missing=False)
            nat["kernels_loaded"] = True
        except Exception as e:  # pragma: no cover
            nat["kernels_loaded"] = f"<{e}>"
    rep["native"] = nat
    return rep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    rep = collect()
    print("=" * 72)
    print(f"OS            : {rep['os'].get('distro', '')} ({rep['os']['platform']}), Python {rep['os']['python']}")
    for k, v in rep["compilers"].items():
        print(f"{k:14s}: {v}")
    print(f"ROCm          : {rep['rocm']['version']}")
    t = rep["torch"]
    print(f"PyTorch       : {t['version']} (HIP {t['hip']}), RCCL {t['rccl']}")
    for g in rep["gpus"]:
        print(f"GPU {g['index']}         : {g['name']} {g['arch']} {g['cus']} CUs {g['hbm_GiB']} GiB")
    if not rep["gpus"]:
        print("GPU           : none visible")
    nat = rep["native"]
    print(f"native libs   : kernels={nat['kernels_so']} comm={nat['comm_so']} rccl_bench={nat['rccl_bench']} "
          f"arch={nat['offload_arch']} loaded={nat.get('kernels_loaded', 'n/a')}")
    if rep["numa"]:
        print(rep["numa"])
    if rep["xgmi_topology"]:
        print("-- xGMI / PCIe topology (rocm-smi --showtopo) --")
        print(rep["xgmi_topology"])
    if rep["env"]:
        print("-- environment --")
        for k, v in rep["env"].items():
            print(f"  {k}={v}")
    print("=" * 72)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rep, f, indent=1)


if __name__ == "__main__":
    main()
