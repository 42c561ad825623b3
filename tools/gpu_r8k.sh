# Final tree: kernel-trace stats of the headline bench + 4 PMC passes over the screen and the
# pair refine (tools/pmc_summary.py reads them)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
OUT=gpurun_out/r8k; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof -o prof --output-format csv -- python3 $R/bench.py --steps 50 --warmup 3 --min-warmup-s 0 --no-busbw > $R/$OUT/prof.log 2>&1 || { echo "prof failed"; tail -5 $R/$OUT/prof.log; exit 1; }
echo "prof ok"
n=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU" \
         "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
         "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_IFETCH SQ_INSTS_SMEM GRBM_COUNT" \
         "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE"; do
  n=$((n+1))
  timeout -s KILL 150 rocprofv3 --pmc $P --kernel-include-regex "k_refine|k_screen_x1|k_x1_rowmajor" -d $R/$OUT/pmc$n -o pmc -- python3 $R/bench.py --steps 3 --warmup 1 --min-warmup-s 0 --no-busbw > $R/$OUT/pmc$n.log 2>&1 || { echo "pmc $n failed"; tail -5 $R/$OUT/pmc$n.log; exit 1; }
  echo "pmc pass $n ok"
done
cd $R
python tools/pmc_summary.py $OUT/pmc1 $OUT/pmc2 $OUT/pmc3 $OUT/pmc4 > $OUT/pmc_summary.txt 2>&1
grep -A3 "k_refine_pair\|k_x1_rowmajor" $OUT/pmc_summary.txt | head -12
