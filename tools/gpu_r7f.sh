set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r7f; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/tests.log | tail -15
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -u tools/bench_sweep.py --out $OUT/sweep.jsonl --timeout 120 --ns 100000,1000000 --attrs 32,128 --ks 1-64 > $OUT/sweep.log 2>&1; echo "sweep rc=$?"; tail -6 $OUT/sweep.log
