#!/bin/bash
# Build tools/rccl_bench/rccl_allreduce_bench (role of the reference's install_osu_bench.sh).
set -e
REPO="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
cd "$REPO"
python3 -c "from azure_hc_intel_tf_amd import _build; print('[build_rccl_bench]', _build.build_tools())"
