set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r7i; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "policy or early_start" > $OUT/kt.log 2>&1; rc=$?; echo "ktests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/kt.log | tail -8
[ $rc -le 1 ] || exit $rc
# PMC passes over the bench step (screen + refine), counters in their own runs
R=$PWD
timeout -k 10 600 python bench.py --harness dropin --steps 20 --warmup 2 > $OUT/dropin.log 2>&1 || { tail -5 $OUT/dropin.log; exit 1; }
echo "dropin: $(grep -o '"time_ms_median": [0-9.]*' $OUT/dropin.log | tr '\n' ' ')"
timeout -k 10 600 python bench.py --harness native --steps 20 --warmup 2 > $OUT/native.log 2>&1 || { tail -5 $OUT/native.log; exit 1; }
echo "native: $(grep -o '"time_ms_median": [0-9.]*' $OUT/native.log | tr '\n' ' ')"
cd /tmp
n=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU" \
         "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
         "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_IFETCH SQ_INSTS_SMEM GRBM_COUNT"; do
  n=$((n+1))
  timeout -s KILL 150 rocprofv3 --pmc $P --kernel-include-regex "k_refine|k_screen_x1" -d $R/$OUT/pmc$n -o pmc -- python3 $R/bench.py --steps 3 --warmup 1 --min-warmup-s 0 > $R/$OUT/pmc$n.log 2>&1 || { echo "pmc $n failed"; tail -5 $R/$OUT/pmc$n.log; exit 1; }
  echo "pmc pass $n ok"
done
