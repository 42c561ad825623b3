set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r7n; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "early_start or native_step or mixed or pipelined or policy or step_front or screen_impls" > $OUT/kt.log 2>&1; rc=$?; echo "ktests rc=$rc"; tail -3 $OUT/kt.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 100 --verify > $OUT/verify.log 2>&1 || { tail -5 $OUT/verify.log; exit 1; }
echo "verify: $(grep -o '"ms_per_step": [0-9.]*' $OUT/verify.log | head -1) $(grep -o '"verify_ok": [a-z]*' $OUT/verify.log)"
rm -rf gpurun_out/ab
AB_ROUNDS=2 AB_STEPS=30 timeout -k 10 900 bash tools/kernel_ab.sh prev w6 w5 > $OUT/ab.log 2>&1; echo "ab rc=$?"
python - <<'PY'
import csv, glob, statistics
for v in ("prev", "w6", "w5"):
    ts = []
    for f in glob.glob(f"gpurun_out/ab/{v}.*/run_kernel_stats.csv"):
        for r in csv.DictReader(open(f)):
            if "k_refine" in r["Name"] and int(r["Calls"]) > 20:
                ts.append(float(r["AverageNs"]) / 1e3)
    print(v, "refine avg us", [round(t, 1) for t in ts])
PY
grep -h "ms_per_step" gpurun_out/ab/*.log | head -8
