set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r7c; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/tests.log | tail -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --min-warmup-s 1 --no-busbw --diag-steps 0 > $OUT/prof.log 2>&1; echo "prof rc=$?"
find $OUT/prof -name '*kernel_stats.csv' -exec sh -c 'head -14 "$1" | cut -c1-180' _ {} \;
