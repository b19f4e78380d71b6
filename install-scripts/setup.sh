#!/bin/bash
# Install dispatcher: setup.sh <native|torch> <host|container>
#   host      : verify the ROCm driver/runtime, host limits, container runtime
#   container : build the native HIP/C++ libraries for gfx950 in-tree and verify they load
# (MI355X counterpart of the reference's install-scripts/setup.sh dispatcher; there is no
# MPI / OFED / compiler build here: ROCm ships hipcc, RCCL and the xGMI fabric driver.)
set -e
if [ "$#" -ne 2 ]; then
  echo "usage: $0 <native|torch> <host|container>" >&2
  exit 1
fi
ENGINE=$1
TARGET=$2
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
case "$ENGINE" in native|torch) ;; *) echo "unknown engine $ENGINE" >&2; exit 1 ;; esac

common() {
  bash "$HERE/check_rocm.sh"
  bash "$HERE/update_config.sh"
}
case "$TARGET" in
  host)
    common
    if command -v apptainer >/dev/null 2>&1 || command -v singularity >/dev/null 2>&1; then
      echo "[setup] container runtime: $(command -v apptainer || command -v singularity)"
    elif command -v docker >/dev/null 2>&1; then
      echo "[setup] container runtime: docker"
    else
      echo "[setup] no container runtime found: run natively (install-scripts/build_native.sh)"
    fi
    ;;
  container)
    common
    bash "$HERE/build_native.sh"
    bash "$HERE/build_rccl_bench.sh"
    ;;
  *)
    echo "unknown target $TARGET (host|container)" >&2
    exit 1
    ;;
esac
