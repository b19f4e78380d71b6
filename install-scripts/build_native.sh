#!/bin/bash
# Build the framework's native libraries for gfx950 in-tree and verify the package imports
# (role of the reference's install_conda_tf_hvd.sh: there the engine was pip/conda installed;
# here the engine IS this repository's HIP + C++ code).
set -e
REPO="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
cd "$REPO"
PYTORCH_ROCM_ARCH=${PYTORCH_ROCM_ARCH:-gfx950} python3 __graft_entry__.py
python3 -c "import azure_hc_intel_tf_amd as h; print('[build_native] package', h.__file__)"
