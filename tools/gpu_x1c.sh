#!/bin/bash
# x1 session: kernel numerics, fill-check period A/B (quick pipeline bench, verified), bench.
set -u
TAG=${1:-x1c}
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > gpurun_out/$TAG/pytest_kernels.log 2>&1; rc=$?
tail -3 gpurun_out/$TAG/pytest_kernels.log; [ $rc -eq 0 ] || exit $rc
for c in 1 2 4; do
  DMLP_X1_CHECK=$c timeout -k 10 100 python tools/quick_gpu_bench.py --q 131072 --iters 5 > gpurun_out/$TAG/c$c.log 2>&1; rc=$?
  echo "check $c: $(grep -v amdgpu gpurun_out/$TAG/c$c.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o run --output-format csv \
    -- python3 tools/quick_gpu_bench.py --q 131072 --iters 3 > gpurun_out/$TAG/prof.log 2>&1; rc=$?
[ $rc -eq 0 ] || { tail -5 gpurun_out/$TAG/prof.log; exit $rc; }
timeout -k 10 300 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err; rc=$?
cat gpurun_out/$TAG/bench.json; [ $rc -eq 0 ] || { tail gpurun_out/$TAG/bench.err; exit $rc; }
