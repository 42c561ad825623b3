#!/bin/bash
set -u
TAG=${1:-pmcx1b}
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 100 python3 tools/quick_gpu_bench.py --q 131072 --modes 8 --iters 1 > $OUT/mode8.log 2>&1; rc=$?
grep -v amdgpu $OUT/mode8.log; [ $rc -eq 0 ] || exit $rc
S1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
S2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM"
n=0
for C in "$S1" "$S2"; do
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d $OUT/p$n -o run --output-format csv \
      -- python3 tools/quick_gpu_bench.py --q 131072 --modes 0 --iters 0 > $OUT/p$n.log 2>&1; rc=$?
  echo "pass $n rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/p$n.log; exit $rc; }
done
python3 - "$OUT" <<'PY'
import csv, glob, collections, sys
out = sys.argv[1]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        key = "screen_x1" if "k_screen_x1" in n else "refine" if "k_refine" in n else None
        if key:
            tot[key][r["Counter_Name"]] += float(r["Counter_Value"])
with open(f"{out}/pmc_summary.txt", "w") as fo:
    for k, v in tot.items():
        line = f"{k} " + str({a: f"{b:.4g}" for a, b in sorted(v.items())})
        print(line); fo.write(line + "\n")
PY
