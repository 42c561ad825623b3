#!/bin/bash
# Kernel stats of the local pipeline and of the bench step, plus PMC passes on the x1 screen.
#   gpurun --timeout 900 -- bash tools/gpu_prof_x1.sh [tag]
set -u
TAG=${1:-px1}
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/bench -o run --output-format csv \
    -- python3 bench.py --steps 5 --warmup 1 > $OUT/bench.log 2>&1; rc=$?
echo "bench stats rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/bench.log; exit $rc; }
S1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
S2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM"
S3="TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"
n=0
for C in "$S1" "$S2" "$S3"; do
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d $OUT/pmc$n -o run --output-format csv \
      -- python3 tools/quick_gpu_bench.py --q 131072 --modes 0 --iters 0 > $OUT/pmc$n.log 2>&1; rc=$?
  echo "pmc pass $n rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/pmc$n.log; exit $rc; }
done
python3 - "$OUT" <<'PY'
import csv, glob, collections, sys
out = sys.argv[1]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"{out}/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        key = ("screen_x1" if "k_screen_x1" in n else "screen_stream" if "k_screen_stream" in n
               else "refine" if "k_refine" in n else None)
        if key:
            tot[key][r["Counter_Name"]] += float(r["Counter_Value"])
with open(f"{out}/pmc_summary.txt", "w") as fo:
    for k, v in tot.items():
        line = k + " " + str({a: f"{b:.4g}" for a, b in sorted(v.items())})
        print(line)
        fo.write(line + "\n")
PY
find $OUT/bench -name '*kernel_stats.csv' -exec sh -c 'head -8 "$1" | cut -c1-150' _ {} \;
