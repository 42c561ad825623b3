set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r7e; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "x1_screen_shapes or native_step or mixed_k or single_term or pipelined or escalat or step_front or screen_impls" > $OUT/kt.log 2>&1; rc=$?; echo "ktests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/kt.log | tail -15
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1; echo "bench rc=$?"; grep -o '"ms_per_step": [0-9.]*\|"native_step": {[^}]*}\|"timed_step_ms": {[^}]*}' $OUT/bench.log
timeout -k 10 900 python3 -u tools/bench_sweep.py --out $OUT/sweep.jsonl --timeout 120 --ns 100000,1000000 --attrs 32,128 --ks 16,1-64,200 > $OUT/sweep.log 2>&1; echo "sweep rc=$?"; tail -15 $OUT/sweep.log
