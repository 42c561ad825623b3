#!/bin/bash
# Screen-kernel ablation + PMC counters.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/quick_gpu_bench.py --n 100000 --q 100000 --modes 0,1,2,3,4,5,6,7 > gpurun_out/ablate.log 2>&1; rc=$?
cat gpurun_out/ablate.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc1 -o run --output-format csv -- python3 tools/quick_gpu_bench.py --n 100000 --q 100000 --iters 1 --check 0 > gpurun_out/pmc1.log 2>&1; rc=$?
echo "pmc rc=$rc"; tail -3 gpurun_out/pmc1.log
exit $rc
