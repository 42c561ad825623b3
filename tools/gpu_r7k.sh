set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r7k; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/gpu_tier.log 2>&1; rc=$?; echo "gpu tier rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/gpu_tier.log | tail -15
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 100 --verify > $OUT/verify.log 2>&1 || { tail -5 $OUT/verify.log; exit 1; }
echo "verify: $(grep -o '"ms_per_step": [0-9.]*' $OUT/verify.log | head -1) $(grep -o '"verify_ok": [a-z]*' $OUT/verify.log)"
cp ab/libdmlp_old.so ab/libdmlp_new.so 2>/dev/null; cp distributed_machine_learning_project_amd/libdmlp.so ab/libdmlp_new.so
AB_ROUNDS=3 AB_STEPS=30 timeout -k 10 900 bash tools/kernel_ab.sh new old > $OUT/ab.log 2>&1; echo "ab rc=$?"; cat $OUT/ab.log | tail -8
python tools/ab_summary.py gpurun_out/ab > $OUT/ab_summary.txt 2>&1; head -30 $OUT/ab_summary.txt
