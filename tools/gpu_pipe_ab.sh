#!/bin/bash
# A/B of the chunked query-H2D pipeline on the bench step (KNN_PIPELINE=0/1), plus the tests
# that cover the pipelined path.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/pipeab
mkdir -p $OUT
for t in 1 4 8 16; do DMLP_HOST_THREADS=$t timeout -k 10 60 python3 tools/bench_host_prep.py || exit 1; done
for p in 0 1 0 1; do
  KNN_PIPELINE=$p timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 > $OUT/bench_p$p.json 2> $OUT/bench_p$p.err || { tail -20 $OUT/bench_p$p.err; exit 1; }
  echo "pipeline=$p $(python3 -c "import json,sys; d=json.load(open('$OUT/bench_p$p.json')); print(d['ms_per_step'], d['value'])")"
done
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_engine_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "pipelin or strateg or shared or host_prep" > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log; exit $rc
