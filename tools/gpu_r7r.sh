set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r7r; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -k "escalates_per_query or early_start or x1 or screen" -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/gpu_tier.log 2>&1; rc=$?; echo "gpu tier rc=$rc"; tail -3 $OUT/gpu_tier.log
[ $rc -eq 0 ] || { grep -E "FAILED" $OUT/gpu_tier.log | head; exit 1; }
timeout -k 10 300 python bench.py --steps 100 --verify > $OUT/verify.log 2>&1 || { tail -5 $OUT/verify.log; exit 1; }
echo "verify: $(grep -o '"ms_per_step": [0-9.]*' $OUT/verify.log | head -1) $(grep -o '"verify_ok": [a-z]*' $OUT/verify.log)"
rm -rf gpurun_out/ab
AB_ROUNDS=3 AB_STEPS=30 timeout -k 10 900 bash tools/kernel_ab.sh new old > $OUT/ab.log 2>&1; echo "ab rc=$?"
python - <<'PY'
import csv, glob
for v in ("new", "old"):
    ts = []
    for f in sorted(glob.glob(f"gpurun_out/ab/{v}.*/run_kernel_stats.csv")):
        for r in csv.DictReader(open(f)):
            if "k_screen_x1ILi1ELi16ELi4ELi2ELi4ELi0ELb1E" in r["Name"]:
                ts.append(round(float(r["AverageNs"]) / 1e3, 1))
    print(v, "screen avg us", ts)
PY
grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/ab/*.log
timeout -k 10 200 python tools/screen_bench.py --modes 0 --rounds 3 --iters 20 --verify 0 > $OUT/sb_new.log 2>&1; tail -1 $OUT/sb_new.log
DMLP_LIB=ab/libdmlp_old.so timeout -k 10 200 python tools/screen_bench.py --modes 0 --rounds 3 --iters 20 --verify 0 > $OUT/sb_old.log 2>&1; tail -1 $OUT/sb_old.log
