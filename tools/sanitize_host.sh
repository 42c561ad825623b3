#!/bin/bash
# ASan + UBSan build of the host (CPU) half of libdmlp plus a driver that exercises it.
# GPU sanitizers / xnack are unavailable on the MI355X pool, so device code is covered by the
# numerics tests instead.  A second build runs the same driver under ThreadSanitizer (the parser
# and the brute force are multi-threaded).  Then csrc/host_prep.cpp — the persistent worker pool
# and the host-side screen-operand conversions of every bench step — under ASan+UBSan and under
# TSan (tests/native/host_prep_driver.cpp; the HIP copies of the pipeline stubbed by memcpy),
# with a pool that fits the CPUs (spin path) and an oversubscribed one (condvar path).
#   usage: tools/sanitize_host.sh [outdir]
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="${1:-/tmp/dmlp_asan}"
mkdir -p "$OUT"
SRC="$ROOT/distributed_machine_learning_project_amd/csrc"
g++ -O1 -g -std=c++17 -ffp-contract=off -fno-omit-frame-pointer -fsanitize=address,undefined \
    -fno-sanitize-recover=undefined -I"$SRC" "$SRC/cpu.cpp" "$SRC/host_prep.cpp" \
    "$ROOT/tests/native/host_driver.cpp" \
    -pthread -o "$OUT/host_driver"
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 "$OUT/host_driver"
g++ -O1 -g -std=c++17 -ffp-contract=off -fsanitize=thread -I"$SRC" "$SRC/cpu.cpp" \
    "$SRC/host_prep.cpp" "$ROOT/tests/native/host_driver.cpp" -pthread -o "$OUT/host_driver_tsan"
TSAN_OPTIONS=halt_on_error=1 "$OUT/host_driver_tsan"
g++ -O1 -g -std=c++17 -ffp-contract=off -fno-omit-frame-pointer -fsanitize=address,undefined \
    -fno-sanitize-recover=undefined -I"$SRC" "$SRC/host_prep.cpp" \
    "$ROOT/tests/native/host_prep_driver.cpp" -pthread -o "$OUT/host_prep_asan"
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 DMLP_HOST_THREADS=4 "$OUT/host_prep_asan"
g++ -O1 -g -std=c++17 -ffp-contract=off -fsanitize=thread -I"$SRC" "$SRC/host_prep.cpp" \
    "$ROOT/tests/native/host_prep_driver.cpp" -pthread -o "$OUT/host_prep_tsan"
TSAN_OPTIONS=halt_on_error=1 DMLP_HOST_THREADS=4 "$OUT/host_prep_tsan"
TSAN_OPTIONS=halt_on_error=1 DMLP_HOST_THREADS=16 "$OUT/host_prep_tsan"
