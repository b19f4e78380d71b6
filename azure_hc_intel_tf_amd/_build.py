"""In-tree native build for the gfx950 HIP kernels and the C++ runtime.

Produces two shared objects next to this file (git-ignored, but they travel to the GPU
box with the repo snapshot):

* ``_hcb_kernels.so`` -- the hand-written CDNA4 kernels (``csrc/kernels/*.hip``, compiled
  with ``hipcc --offload-arch=gfx950``) plus their ``torch.library`` registrations
  (``csrc/bindings.cpp``), loaded with ``torch.ops.load_library``.
* ``_hcb_kernels_f16.so`` -- the same kernel sources built for IEEE-fp16 activations
  (``-DHCB_F16``, C++ and torch.library namespace ``hcb16``): the native ``--use_fp16`` path.
* ``_hcb_data*.so`` -- the native real-data pipeline core (TFRecord / tf.Example / crop
  windows / prefetch threads; ``csrc/data/*.cpp``).
* ``_hcb_engine_cpu*.so`` -- the bucket engine core on an in-process fake fabric (CPU tests).
* ``_hcb_comm.so`` -- the C++ communication runtime (RCCL communicator, bucketed
  allreduce engine, Chrome-trace timeline, stall watchdog; ``csrc/comm/*.cpp``).

The kernels' translation units include no torch headers, so a kernel edit recompiles in
seconds; objects are rebuilt only when a source or header is newer than the object.
This is the MI355X replacement for the reference's container build step
(/root/reference/install-scripts/build-container.sh:23-30).
"""
from __future__ import annotations

import concurrent.futures as _cf
import glob
import os
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
CSRC = os.path.join(REPO, "csrc")
BUILD = os.path.join(REPO, "build", "obj")
ARCH = os.environ.get("HCB_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
KERNELS_SO = os.path.join(PKG_DIR, "_hcb_kernels.so")
KERNELS_F16_SO = os.path.join(PKG_DIR, "_hcb_kernels_f16.so")
# IEEE-fp16 build: the activation-type switch of csrc/kernels/common.h plus a renamed namespace
# (C++ symbols and torch.library ops), so both libraries load into one process side by side
F16_FLAGS = ["-DHCB_F16", "-Dhcb=hcb16"]
COMM_SO = os.path.join(PKG_DIR, "_hcb_comm.so")


def _torch_paths():
    import torch

    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    lib = os.path.join(tdir, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("native build failed:\n" + " ".join(cmd) + "\n" + r.stdout + r.stderr)
    return r


def _headers():
    return glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)


# No packed-fp32 VALU code (v_pk_{add,mul,fma,mov}_f32): with it, the BN-statistics epilogue of
# the 64x64 conv tile summed its squares non-deterministically wrong on MI355X (relative errors
# up to 3x the variance, other sums exact; tools/diag_bn_stats.py, profiles/r2e_bn_shift_and_pkf32.txt)
# while the same source built without it is exact -- and the whole step is ~1.7% faster without.
NO_PACKED_FP32 = ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]


def build_kernels(verbose: bool = False, jobs: int = 8, f16: bool = False) -> str:
    build = os.path.join(BUILD, "f16") if f16 else BUILD
    so = KERNELS_F16_SO if f16 else KERNELS_SO
    extra = F16_FLAGS if f16 else []
    os.makedirs(build, exist_ok=True)
    hdrs = _headers()
    hips = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    inc, tlib, abi = _torch_paths()
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    objs, jobs_list = [], []
    for src in hips:
        obj = os.path.join(build, os.path.basename(src) + ".o")
        objs.append(obj)
        if _newer(obj, [src] + hdrs):
            jobs_list.append([hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
                              "-munsafe-fp-atomics", "-Wno-unused-result", *NO_PACKED_FP32, *extra,
                              "-I" + os.path.join(CSRC, "kernels"), "-c", src, "-o", obj])
    bsrc = os.path.join(CSRC, "bindings.cpp")
    bobj = os.path.join(build, "bindings.o")
    objs.append(bobj)
    if _newer(bobj, [bsrc] + hdrs):
        jobs_list.append(["g++", "-std=c++17", "-O2", "-fPIC", "-D__HIP_PLATFORM_AMD__", "-DUSE_ROCM", *extra,
                          f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-I" + os.path.join(ROCM, "include"),
                          *["-I" + i for i in inc], "-I" + CSRC, "-c", bsrc, "-o", bobj])
    if jobs_list:
        with _cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            list(ex.map(lambda c: _run(c, verbose), jobs_list))
    if _newer(so, objs):
        _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", so, *objs,
              "-Wl,-soname," + os.path.basename(so),
              "-L" + tlib, "-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch_hip",
              "-Wl,-rpath," + tlib], verbose)
    return so


def build_comm(verbose: bool = False, jobs: int = 8) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "comm", "*.cpp")))
    if not srcs:
        return ""
    os.makedirs(BUILD, exist_ok=True)
    hdrs = _headers()
    inc, tlib, abi = _torch_paths()
    objs, jobs_list = [], []
    for src in srcs:
        obj = os.path.join(BUILD, "comm_" + os.path.basename(src) + ".o")
        objs.append(obj)
        if _newer(obj, [src] + hdrs):
            jobs_list.append(["g++", "-std=c++17", "-O2", "-fPIC", "-D__HIP_PLATFORM_AMD__", "-DUSE_ROCM",
                              f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-I" + os.path.join(ROCM, "include"),
                              *["-I" + i for i in inc], "-I" + CSRC, "-c", src, "-o", obj])
    if jobs_list:
        with _cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            list(ex.map(lambda c: _run(c, verbose), jobs_list))
    if _newer(COMM_SO, objs + [KERNELS_SO]):
        # link RCCL from torch's lib dir: the process already has torch's librccl loaded,
        # so both resolve to ONE RCCL instance. The bucket pack/unpack kernels come from
        # _hcb_kernels.so (found next to this library through $ORIGIN).
        _run(["g++", "-shared", "-fPIC", "-o", COMM_SO, *objs, "-L" + PKG_DIR, "-l:_hcb_kernels.so",
              "-L" + tlib, "-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch_hip", "-lrccl",
              "-L" + os.path.join(ROCM, "lib"), "-lamdhip64",
              "-Wl,-rpath,$ORIGIN", "-Wl,-rpath," + tlib], verbose)
    return COMM_SO


def _data_so() -> str:
    import sysconfig

    return os.path.join(PKG_DIR, "_hcb_data" + sysconfig.get_config_var("EXT_SUFFIX"))


def build_data(verbose: bool = False) -> str:
    """``_hcb_data`` -- the native half of the real-data input pipeline (TFRecord reader /
    writer with CRC-32C, tf.Example parsing, crop-window sampling, prefetch threads;
    ``csrc/data/*.cpp``), a plain CPython extension (pybind11, no torch dependency)."""
    import sysconfig

    import pybind11

    srcs = sorted(glob.glob(os.path.join(CSRC, "data", "*.cpp")))
    if not srcs:
        return ""
    so = _data_so()
    if _newer(so, srcs + _headers()):
        _run(["g++", "-std=c++17", "-O2", "-fPIC", "-shared", "-Wall", "-I" + pybind11.get_include(),
              "-I" + sysconfig.get_paths()["include"], *srcs, "-o", so, "-lpthread"], verbose)
    return so


def _engine_cpu_so() -> str:
    import sysconfig

    return os.path.join(PKG_DIR, "_hcb_engine_cpu" + sysconfig.get_config_var("EXT_SUFFIX"))


def build_engine_cpu(verbose: bool = False) -> str:
    """``_hcb_engine_cpu`` -- the gradient bucket engine core (``csrc/comm/engine.h``, the same
    code the RCCL library runs) on an in-process fake fabric of emulated ranks
    (``csrc/engine_cpu/*.cpp``): the CPU test suite's fake backend (pybind11, no torch/HIP)."""
    import sysconfig

    import pybind11

    srcs = sorted(glob.glob(os.path.join(CSRC, "engine_cpu", "*.cpp")))
    if not srcs:
        return ""
    so = _engine_cpu_so()
    if _newer(so, srcs + _headers()):
        _run(["g++", "-std=c++17", "-O2", "-fPIC", "-shared", "-Wall", "-I" + CSRC, "-I" + pybind11.get_include(),
              "-I" + sysconfig.get_paths()["include"], *srcs, "-o", so, "-lpthread"], verbose)
    return so


RCCL_BENCH = os.path.join(REPO, "tools", "rccl_bench", "rccl_allreduce_bench")


def build_tools(verbose: bool = False) -> str:
    """tools/rccl_bench: the OSU-style RCCL collective benchmark (standalone executable)."""
    src = RCCL_BENCH + ".hip"
    if not os.path.exists(src):
        return ""
    if _newer(RCCL_BENCH, [src]):
        _run([os.path.join(ROCM, "bin", "hipcc"), f"--offload-arch={ARCH}", "-O2", "-std=c++17", src, "-o",
              RCCL_BENCH, "-L" + os.path.join(ROCM, "lib"), "-lrccl", "-Wl,-rpath," + os.path.join(ROCM, "lib")],
             verbose)
    return RCCL_BENCH


def build_all(verbose: bool = False) -> None:
    build_kernels(verbose)
    build_kernels(verbose, f16=True)
    build_comm(verbose)
    build_data(verbose)
    build_engine_cpu(verbose)
    build_tools(verbose)


if __name__ == "__main__":
    build_all(verbose="-v" in sys.argv)
    print("built", KERNELS_SO, COMM_SO)
