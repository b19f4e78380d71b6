#!/bin/bash
# Top-level installer for an MI355X node (role of the reference's
# 2-setup-host-and-build-container.sh): checks the ROCm host stack, prepares the shared
# env directory, then builds the container image with this framework's native libraries.
#
# usage: ./2-setup-host-and-build-container.sh <native|torch>
#   native : gradients reduced by the C++ RCCL engine (default runtime)
#   torch  : gradients reduced through torch.distributed (RCCL backend)
# No network access is assumed: nothing is downloaded; the ROCm + PyTorch-ROCm base must exist.
set -e
if [ "$#" -ne 1 ] || { [ "$1" != "native" ] && [ "$1" != "torch" ]; }; then
  echo "usage: $0 <native|torch>" >&2
  exit 1
fi
ENGINE=$1
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
SHARED=${HCB_SHARED:-$HOME/hcb-shared}
mkdir -p "$SHARED"
echo "export HCB_ENGINE=$ENGINE" > "$SHARED/setenv"
echo "[setup] shared env file: $SHARED/setenv"
bash "$HERE/install-scripts/setup.sh" "$ENGINE" host
bash "$HERE/install-scripts/build-container.sh" "$ENGINE"
