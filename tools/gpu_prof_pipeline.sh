#!/bin/bash
# Kernel-level stats + PMC counters of the local pipeline (quick bench, default screen).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/pp
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pp/stats -o run --output-format csv -- python3 tools/quick_gpu_bench.py --q 131072 --modes 0 --iters 3 > gpurun_out/pp/stats.log 2>&1; rc=$?
echo "stats rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pp/stats.log; exit $rc; }
head -8 gpurun_out/pp/stats/run_kernel_stats.csv | cut -c1-200
S1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
S2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA"
for set in 1 2; do
  if [ $set -eq 1 ]; then C=$S1; else C=$S2; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/pp/pmc$set -o run --output-format csv -- python3 tools/quick_gpu_bench.py --q 131072 --modes 0 --iters 0 > gpurun_out/pp/pmc$set.log 2>&1; rc=$?
  echo "pmc set $set rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pp/pmc$set.log; exit $rc; }
done
python3 - <<'PY'
import csv, glob, collections
tot = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob("gpurun_out/pp/pmc*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        key = "screen_stream" if "k_screen_stream" in n else ("refine" if "k_refine" in n else None)
        if key:
            tot[key][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in tot.items():
    print(k, {a: f"{b:.4g}" for a, b in sorted(v.items())})
PY
