#!/bin/bash
# Host-side sanitizer run of the native data library: build it with ASan + UBSan into a
# scratch dir and drive it with tools/sanitize_data.py (no torch, no GPU). GPU sanitizers are
# not available on the MI355X pool; this covers the C++ host code.
set -eo pipefail
OUT=${1:-/tmp/hcb_asan}
mkdir -p "$OUT"
read -r PYBIND PYINC <<< "$(python -c "import pybind11,sysconfig; print(pybind11.get_include(), sysconfig.get_paths()['include'])")"
EXT=$(python -c "import sysconfig; print(sysconfig.get_config_var('EXT_SUFFIX'))")
g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined \
    -fPIC -shared -I"$PYBIND" -I"$PYINC" csrc/data/tfrecord.cpp -o "$OUT/_hcb_data$EXT" -lpthread
LD_PRELOAD="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)" \
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 HCB_DATA_LIB_DIR="$OUT" python tools/sanitize_data.py
