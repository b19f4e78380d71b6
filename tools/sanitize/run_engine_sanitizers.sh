#!/usr/bin/env bash
# Build the bucket-engine core + its fake backend, and the HIP-free host bookkeeping of the RCCL
# runtime (csrc/comm/host.h: handle tables, event pool / timeline, watch state, xGMI checks --
# the same header comm.cpp compiles), with AddressSanitizer/UBSan and with ThreadSanitizer (host
# code only, CPU; SURVEY.md §5 "Race detection / sanitizers") and run both stress drivers under
# each. Exit non-zero on any sanitizer report or check failure.
set -euo pipefail
cd "$(dirname "$0")/../.."
OUT=${OUT:-build/sanitize}
mkdir -p "$OUT"
SRC="tools/sanitize/engine_stress.cpp csrc/engine_cpu/fake_engine.cpp"
INC="-Icsrc"
g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all \
    $INC $SRC -o "$OUT/engine_stress_asan" -lpthread
g++ -std=c++17 -O1 -g -fsanitize=thread $INC $SRC -o "$OUT/engine_stress_tsan" -lpthread
HSRC=tools/sanitize/comm_host_stress.cpp
g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all \
    $INC $HSRC -o "$OUT/comm_host_asan" -lpthread
g++ -std=c++17 -O1 -g -fsanitize=thread $INC $HSRC -o "$OUT/comm_host_tsan" -lpthread
echo "== ASan + UBSan"
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
    "$OUT/engine_stress_asan"
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
    "$OUT/comm_host_asan"
echo "== TSan"
TSAN_OPTIONS=halt_on_error=1:second_deadlock_stack=1 "$OUT/engine_stress_tsan"
TSAN_OPTIONS=halt_on_error=1:second_deadlock_stack=1 "$OUT/comm_host_tsan"
