#!/bin/bash
# One measuring session (after the GPU tier): headline bench, the reference-harness drop-in,
# the k sweep at N 1e5 / 1e6 x A 32 / 128 / 256, each step under its own time limit.
#   gpurun --timeout 1200 -- bash tools/gpu_measure.sh <tag>
set -u
TAG=${1:?tag}
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
bash tools/gpu_session.sh "$TAG" bench prof dropin || exit $?
timeout -k 10 600 python3 -u tools/bench_sweep.py --out "$OUT/sweep.jsonl" --timeout 120 \
    --ns 100000,1000000 --attrs 32,128,256 --ks 16,1-64,200 > "$OUT/sweep.log" 2>&1
