set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r7g; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "escalates_per_query or step_front or mixed_k or native_step" > $OUT/kt.log 2>&1; rc=$?; echo "ktests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/kt.log | tail -8
[ $rc -le 1 ] || exit $rc
for T in 14 4 2; do
  for H in 1 0; do
    DMLP_HOST_THREADS=$T DMLP_HOST_OPS=$H timeout -k 10 200 python bench.py --steps 100 > $OUT/b_t${T}_h${H}.log 2>&1 || exit 1
    echo "threads $T host_ops $H: $(grep -o '"ms_per_step": [0-9.]*' $OUT/b_t${T}_h${H}.log | head -1) $(grep -o '"step_timeline_ms": {[^}]*}' $OUT/b_t${T}_h${H}.log)"
  done
done
for T in 14 2; do
  DMLP_DATA_PLANE=host DMLP_HOST_THREADS=$T timeout -k 10 400 python bench.py --gpus 3 --steps 30 --warmup 3 --min-warmup-s 1 --no-busbw --verify > $OUT/p3_t$T.log 2>&1 || { tail -5 $OUT/p3_t$T.log; exit 1; }
  echo "P=3 threads $T: $(grep -o '"ms_per_step": [0-9.]*' $OUT/p3_t$T.log | head -1) verify $(grep -o '"verify_ok": [a-z]*' $OUT/p3_t$T.log)"
done
