set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r7j; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "exact or policy or early_start or native_step" > $OUT/kt.log 2>&1; rc=$?; echo "ktests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/kt.log | tail -12
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --exact --steps 5 --warmup 1 --min-warmup-s 0 --verify > $OUT/exact.log 2>&1 || { tail -5 $OUT/exact.log; exit 1; }
echo "exact: $(grep -o '"ms_per_step": [0-9.]*' $OUT/exact.log | head -1) $(grep -o '"verify_ok": [a-z]*' $OUT/exact.log)"
DMLP_EXACT_F64=0 timeout -k 10 300 python bench.py --exact --steps 3 --warmup 1 --min-warmup-s 0 > $OUT/exact_valu.log 2>&1 || { tail -5 $OUT/exact_valu.log; exit 1; }
echo "exact valu: $(grep -o '"ms_per_step": [0-9.]*' $OUT/exact_valu.log | head -1)"
R=$PWD
cd /tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof_exact -o prof -- python3 $R/bench.py --exact --steps 3 --warmup 1 --min-warmup-s 0 > $R/$OUT/prof_exact.log 2>&1 || { echo "prof failed"; tail -5 $R/$OUT/prof_exact.log; exit 1; }
echo "prof ok"
