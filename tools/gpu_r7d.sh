set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r7d; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/screen_bench.py --modes 0,256,128,2,1 --rounds 3 --iters 20 > $OUT/screen.log 2>&1; echo "screen rc=$?"; cat $OUT/screen.log | grep -v amdgpu.ids
timeout -k 10 300 python -u -m pytest tests/test_engine_native.py -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "escalates" > $OUT/t.log 2>&1; echo "test rc=$?"; grep -E "PASSED|FAILED" $OUT/t.log
