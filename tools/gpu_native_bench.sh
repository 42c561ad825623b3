#!/bin/bash
# Native knn_engine (reference harness contract) on the bench shape: "Time taken" + metrics
# sidecar, output cross-checked against the Python harness on the same GPU.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/native
mkdir -p $OUT
python3 tools/generate_input.py --fast --num_data 100000 --num_queries 131072 --num_attrs 32 \
    --min 0 --max 1000 --minK 16 --maxK 16 --num_labels 10 --output /tmp/bench4.in > /dev/null || exit 1
for s in farm shard_gather; do
  KNN_TRACE=1 KNN_METRICS=$OUT/metrics_$s.json timeout -k 10 200 distributed_machine_learning_project_amd/knn_engine \
      --strategy $s < /tmp/bench4.in > $OUT/$s.out 2> $OUT/$s.err; rc=$?
  echo "native $s rc=$rc: $(grep 'Time taken' $OUT/$s.err)"; [ $rc -eq 0 ] || { tail -5 $OUT/$s.err; exit $rc; }
done
timeout -k 10 200 python3 -m distributed_machine_learning_project_amd.harness --strategy farm \
    --input /tmp/bench4.in > $OUT/py_farm.out 2> $OUT/py_farm.err; rc=$?
echo "python farm rc=$rc: $(grep 'Time taken' $OUT/py_farm.err)"; [ $rc -eq 0 ] || exit $rc
cmp -s $OUT/farm.out $OUT/py_farm.out && echo "native == python output" || { echo "OUTPUT MISMATCH"; exit 1; }
cmp -s $OUT/farm.out $OUT/shard_gather.out && echo "farm == shard_gather output" || { echo "OUTPUT MISMATCH sg"; exit 1; }
grep "dmlp-trace" $OUT/farm.err | head -20
cat $OUT/metrics_farm.json
