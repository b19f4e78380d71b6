#!/usr/bin/env python3
"""Build a variant of the kernel library for an A/B run on the GPU box:

    python tools/build_variant.py abvar/epi1 -DHCB_EPI_VARIANT=1
    HCB_KERNELS_SO=abvar/epi1/_hcb_kernels.so python bench.py ...

Extra arguments go to every hipcc line (defines, -Xclang target features); --packed-fp32 builds
with the packed-fp32 VALU code the in-tree build disables. The output directory
must not be gpurun-ignored (abvar/ is git-ignored only)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from azure_hc_intel_tf_amd import _build  # noqa: E402


def main():
    out, extra = os.path.abspath(sys.argv[1]), sys.argv[2:]
    if "--packed-fp32" in extra:  # the toolchain default the in-tree build turns off
        extra.remove("--packed-fp32")
        _build.NO_PACKED_FP32.clear()
    os.makedirs(out, exist_ok=True)
    real_run = _build._run

    def run(cmd, verbose=False):
        if os.path.basename(cmd[0]) == "hipcc" and "-c" in cmd:
            cmd = cmd[:1] + extra + cmd[1:]
        return real_run(cmd, verbose)

    _build._run = run
    _build.BUILD = out
    _build.KERNELS_SO = os.path.join(out, "_hcb_kernels.so")
    print(_build.build_kernels())


if __name__ == "__main__":
    main()
