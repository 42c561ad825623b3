# Where do the in-step screen's extra ~0.2 ms (vs screen_bench standalone) go?  Kernel trace of
# the bench step with the early start on / off, int32 rows on / off, and the standalone screen.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r7p; mkdir -p $OUT
export TMPDIR=/tmp
R=$PWD; cd /tmp
for cfg in "base:BASE=1" "noearly:DMLP_FAST_EARLY=0" "fp64rows:DMLP_ROWS_I32=0" "delay:DMLP_FAST_QCHUNKS=2"; do
  n=${cfg%%:*}; e=${cfg#*:}
  env $e timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $R/$OUT/$n -o p --output-format csv -- python3 $R/bench.py --steps 50 --warmup 3 > $R/$OUT/$n.log 2>&1 || { echo "$n failed"; tail -3 $R/$OUT/$n.log; exit 1; }
  python3 - "$R/$OUT/$n" "$n" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1] + "/p_kernel_stats.csv")):
    if "k_screen_x1ILi1ELi16ELi4ELi2ELi4ELi0ELb1E" in r["Name"] or "k_refine_pair" in r["Name"] or "rows_from" in r["Name"]:
        print(sys.argv[2], r["Name"][:36], r["Calls"], "avg %.1f us" % (float(r["AverageNs"]) / 1e3), "median-ish min %.1f" % (float(r["MinNs"]) / 1e3))
PY
  echo "$n: $(grep -o '"ms_per_step": [0-9.]*' $R/$OUT/$n.log | head -1) $(grep -o '"step_timeline_ms": {[^}]*}' $R/$OUT/$n.log)"
done
cd $R
timeout -k 10 200 python tools/screen_bench.py --modes 0 --rounds 3 --iters 20 --verify 0 > $OUT/screen_bench.log 2>&1; tail -2 $OUT/screen_bench.log
