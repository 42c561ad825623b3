#!/bin/bash
# Kernel stats of the local pipeline (quick bench) + numerics tests.
set -u
TAG=${1:-qp}
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > gpurun_out/$TAG/pytest_kernels.log 2>&1; rc=$?
tail -2 gpurun_out/$TAG/pytest_kernels.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o run --output-format csv \
    -- python3 tools/quick_gpu_bench.py --q 131072 --iters 5 > gpurun_out/$TAG/prof.log 2>&1; rc=$?
grep -v amdgpu gpurun_out/$TAG/prof.log | tail -2; [ $rc -eq 0 ] || exit $rc
python3 - "$TAG" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(f"gpurun_out/{sys.argv[1]}/prof/run_kernel_stats.csv")))[:8]:
    print(f"{float(r['AverageNs'])/1e3:9.1f} us  x{r['Calls']:>3}  {r['Name'][:90]}")
PY
