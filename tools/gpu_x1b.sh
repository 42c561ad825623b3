#!/bin/bash
# x1 A/B: ring depth 4 vs 8, kernel stats of the pipeline.
set -u
TAG=${1:-x1b}
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > gpurun_out/$TAG/pytest_kernels.log 2>&1; rc=$?
tail -3 gpurun_out/$TAG/pytest_kernels.log; [ $rc -eq 0 ] || exit $rc
for d in 4 8; do
  DMLP_X1_DEPTH=$d timeout -k 10 200 python tools/quick_gpu_bench.py --q 131072 --modes 0,1 > gpurun_out/$TAG/ab_d$d.log 2>&1; rc=$?
  echo "depth $d"; grep mode gpurun_out/$TAG/ab_d$d.log; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o run --output-format csv \
    -- python3 tools/quick_gpu_bench.py --q 131072 --iters 3 > gpurun_out/$TAG/prof.log 2>&1; rc=$?
[ $rc -eq 0 ] || { tail -5 gpurun_out/$TAG/prof.log; exit $rc; }
cut -d, -f1-4 gpurun_out/$TAG/prof/run_kernel_stats.csv | head -5 | cut -c1-50,140-
timeout -k 10 300 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err; rc=$?
cat gpurun_out/$TAG/bench.json; [ $rc -eq 0 ] || { tail gpurun_out/$TAG/bench.err; exit $rc; }
