#!/bin/bash
# Build the framework image (role of the reference's build-container.sh): an Apptainer SIF
# from hcb-rocm[-rcclbench].def when apptainer/singularity exists, else a docker image from
# the Dockerfile, then a sanity run of the image's runscript (tools/env_report.py).
# usage: build-container.sh <native|torch> [rcclbench]
set -e
ENGINE=${1:-native}
VARIANT=${2:-}
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
REPO="$(dirname "$HERE")"
OUT=${HCB_IMAGE_DIR:-${HCB_SHARED:-$HOME/hcb-shared}/images}
mkdir -p "$OUT"
DEF="$HERE/hcb-rocm.def"
[ "$VARIANT" = rcclbench ] && DEF="$HERE/hcb-rocm-rcclbench.def"
NAME=$(basename "$DEF" .def)
if command -v apptainer >/dev/null 2>&1 || command -v singularity >/dev/null 2>&1; then
  RT=$(command -v apptainer || command -v singularity)
  (cd "$REPO" && "$RT" build --force "$OUT/$NAME.sif" "$DEF")
  HCB_ENGINE=$ENGINE "$RT" run --rocm "$OUT/$NAME.sif"
elif command -v docker >/dev/null 2>&1; then
  docker build -t "hcb/$NAME" -f "$HERE/Dockerfile" "$REPO"
  docker run --rm --device=/dev/kfd --device=/dev/dri --group-add video -e HCB_ENGINE=$ENGINE "hcb/$NAME"
else
  echo "[build-container] no apptainer/singularity/docker: building natively instead"
  bash "$HERE/build_native.sh"
fi
