#!/bin/bash
# PMC counters of the streaming screen kernel, full (mode 0) vs no-candidate (mode 1) variant.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/pmc_stream
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
S1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
S2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA"
for m in 0 1; do
  for set in 1 2; do
    if [ $set -eq 1 ]; then C=$S1; else C=$S2; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/pmc_stream/m${m}_s${set} -o run --output-format csv -- python3 tools/quick_gpu_bench.py --q 131072 --modes $m --iters 1 > gpurun_out/pmc_stream/m${m}_s${set}.log 2>&1; rc=$?
    echo "mode $m set $set rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pmc_stream/m${m}_s${set}.log; exit $rc; }
  done
done
python3 - <<'PY'
import csv, glob, collections
for m in (0, 1):
    tot = collections.defaultdict(float)
    for f in glob.glob(f"gpurun_out/pmc_stream/m{m}_s*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "k_screen_stream" in r["Kernel_Name"]:
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
    print(f"mode {m}:", {k: f"{v:.4g}" for k, v in sorted(tot.items())})
PY
