set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r7b; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; echo "smoke rc=$?"; tail -3 $OUT/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "native_step or step_front or pipelined or test_engine_gpu" > $OUT/ktests.log 2>&1; rc=$?; echo "ktests rc=$rc"; grep -E "PASSED|FAILED|ERROR" $OUT/ktests.log | sed 's/.*:://' | tail -60
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 200 > $OUT/bench.log 2>&1; echo "bench rc=$?"; tail -c 1500 $OUT/bench.log
