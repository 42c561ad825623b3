# End-of-round validation on one MI355X: GPU tier, smoke(), the driver's bench line, --verify of the
# default and the exact path, the P = 3 host-plane rehearsal with --verify.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/final; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/gpu_tier.log 2>&1; rc=$?; echo "gpu tier rc=$rc"; tail -2 $OUT/gpu_tier.log
[ $rc -eq 0 ] || { grep FAILED $OUT/gpu_tier.log | head; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.log 2>&1 || { tail -5 $OUT/bench_driver.log; exit 1; }
echo "driver-style bench: $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_driver.log | head -1)"
timeout -k 10 300 python bench.py --steps 200 --verify > $OUT/verify.log 2>&1 || { tail -5 $OUT/verify.log; exit 1; }
echo "verify: $(grep -o '"ms_per_step": [0-9.]*' $OUT/verify.log | head -1) $(grep -o '"verify_ok": [a-z]*' $OUT/verify.log)"
timeout -k 10 300 python bench.py --exact --steps 5 --warmup 1 --min-warmup-s 0 --verify > $OUT/exact.log 2>&1 || { tail -5 $OUT/exact.log; exit 1; }
echo "exact: $(grep -o '"ms_per_step": [0-9.]*' $OUT/exact.log | head -1) $(grep -o '"verify_ok": [a-z]*' $OUT/exact.log)"
DMLP_DATA_PLANE=host timeout -k 10 400 python bench.py --gpus 3 --steps 30 --warmup 3 --min-warmup-s 1 --no-busbw --verify > $OUT/p3.log 2>&1 || { tail -5 $OUT/p3.log; exit 1; }
echo "P=3 host plane: $(grep -o '"ms_per_step": [0-9.]*' $OUT/p3.log | head -1) $(grep -o '"verify_ok": [a-z]*' $OUT/p3.log)"
