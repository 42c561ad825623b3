#!/bin/bash
# GPU: default bench (shm ingress), root-ingress bench, traced bench, screen ablation + counters,
# rocprof kernel stats of the bench step, native engine timing on a bench-shaped input.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err; rc=$?
cat gpurun_out/bench_default.json; [ $rc -eq 0 ] || { tail gpurun_out/bench_default.err; exit $rc; }
timeout -k 10 300 python bench.py --ingress root > gpurun_out/bench_root.json 2>&1; rc=$?
tail -1 gpurun_out/bench_root.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --verify > gpurun_out/bench_verify.json 2>&1; rc=$?
tail -1 gpurun_out/bench_verify.json; [ $rc -eq 0 ] || exit $rc
KNN_TRACE=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 > gpurun_out/bench_trace.log 2>&1; rc=$?
grep "dmlp-trace" gpurun_out/bench_trace.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/quick_gpu_bench.py --q 131072 --modes 0,1,3,8 > gpurun_out/ablate.log 2>&1; rc=$?
cat gpurun_out/ablate.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 > gpurun_out/prof_bench.log 2>&1; rc=$?
echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/generate_input.py --fast --num_data 100000 --num_queries 131072 --num_attrs 32 --min 0 --max 1000 --minK 16 --maxK 16 --num_labels 10 --output /tmp/bench4.in > /dev/null && \
KNN_TRACE=1 KNN_METRICS=gpurun_out/engine_metrics.json timeout -k 10 300 distributed_machine_learning_project_amd/knn_engine --strategy farm --input /tmp/bench4.in > /tmp/bench4.out 2> gpurun_out/engine_bench.err; rc=$?
cat gpurun_out/engine_bench.err; cat gpurun_out/engine_metrics.json
exit $rc
