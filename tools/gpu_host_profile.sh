#!/bin/bash
# Host-side (Python) profile of the bench step: cProfile over 300 steps, top functions by own time.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/hprof
timeout -k 10 300 python -m cProfile -o gpurun_out/hprof/bench.pstats bench.py --steps 300 --warmup 5 \
    > gpurun_out/hprof/bench.json 2> gpurun_out/hprof/bench.err || exit $?
python - <<'PY' > gpurun_out/hprof/top.txt
import pstats
p = pstats.Stats("gpurun_out/hprof/bench.pstats")
p.sort_stats("tottime").print_stats(45)
p.sort_stats("cumulative").print_stats(60)
PY
cat gpurun_out/hprof/bench.json
