set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r7l; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --exact --steps 5 --warmup 1 --min-warmup-s 0 --verify > $OUT/exact.log 2>&1 || { tail -5 $OUT/exact.log; exit 1; }
echo "exact: $(grep -o '"ms_per_step": [0-9.]*' $OUT/exact.log | head -1) $(grep -o '"verify_ok": [a-z]*' $OUT/exact.log)"
R=$PWD; cd /tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof_exact -o prof --output-format csv -- python3 $R/bench.py --exact --steps 3 --warmup 1 --min-warmup-s 0 > $R/$OUT/prof_exact.log 2>&1 || { echo "prof failed"; exit 1; }
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/gpu_tier.log 2>&1; rc=$?; echo "gpu tier rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/gpu_tier.log | tail -15
