set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r7j; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "exact or policy or early_start or native_step" > $OUT/kt.log 2>&1; rc=$?; echo "ktests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/kt.log | tail -12
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --exact --steps 5 --warmup 1 --min-warmup-s 0 --verify > $OUT/exact.log 2>&1 || { tail -5 $OUT/exact.log; exit 1; }
echo "exact: $(grep -o '"ms_per_step": [0-9.]*' $OUT/exact.log | head -1) $(grep -o '"verify_ok": [a-z]*' $OUT/exact.log)"
DMLP_EXACT_F64=0 timeout -k 10 300 python bench.py --exact --steps 3 --warmup 1 --min-warmup-s 0 > $OUT/exact_valu.log 2>&1 || { tail -5 $OUT/exact_valu.log; exit 1; }
echo "exact valu: $(grep -o '"ms_per_step": [0-9.]*' $OUT/exact_valu.log | head -1)"
R=$PWD
cd /tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof_exact -o prof -- python3 $R/bench.py --exact --steps 3 --warmup 1 --min-warmup-s 0 > $R/$OUT/prof_exact.log 2>&1 || { echo "prof failed"; tail -5 $R/$OUT/prof_exact.log; exit 1; }
echo "prof ok"
n=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU" \
         "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
         "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_IFETCH SQ_INSTS_SMEM GRBM_COUNT" \
         "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE"; do
  n=$((n+1))
  timeout -s KILL 150 rocprofv3 --pmc $P --kernel-include-regex "k_refine|k_screen_x1" -d $R/$OUT/pmc$n -o pmc -- python3 $R/bench.py --steps 3 --warmup 1 --min-warmup-s 0 > $R/$OUT/pmc$n.log 2>&1 || { echo "pmc $n failed"; tail -5 $R/$OUT/pmc$n.log; exit 1; }
  echo "pmc pass $n ok"
done
cd $R
timeout -k 10 600 python bench.py --harness dropin --steps 20 --warmup 2 > $OUT/dropin.log 2>&1 || { tail -5 $OUT/dropin.log; exit 1; }
echo "dropin: $(grep -o '"time_ms_median": [0-9.]*' $OUT/dropin.log | tr '\n' ' ')"
timeout -k 10 600 python bench.py --harness native --steps 20 --warmup 2 > $OUT/native.log 2>&1 || { tail -5 $OUT/native.log; exit 1; }
echo "native: $(grep -o '"time_ms_median": [0-9.]*' $OUT/native.log | tr '\n' ' ')"
# copy engine A/B: the step's H2D/D2H run as __amd_rocclr_copyBuffer blit kernels by default
for E in "BASE=1" "DMLP_REFINE_PAIR=0" "HSA_ENABLE_SDMA=1" "GPU_FORCE_BLIT_COPY_SIZE=0" "HSA_ENABLE_SDMA=0" "BASE=2" "DMLP_REFINE_PAIR=0"; do
  T=$(echo $E | tr '=' '_')
  env $E timeout -k 10 200 python bench.py --steps 100 > $OUT/ab_$T.log 2>&1 || { tail -5 $OUT/ab_$T.log; exit 1; }
  echo "ab $E: $(grep -o '"ms_per_step": [0-9.]*' $OUT/ab_$T.log | head -1) $(grep -o '"step_timeline_ms": {[^}]*}' $OUT/ab_$T.log)"
done
cd /tmp
HSA_ENABLE_SDMA=1 timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof_sdma -o prof -- python3 $R/bench.py --steps 20 --warmup 2 --min-warmup-s 0 > $R/$OUT/prof_sdma.log 2>&1 || { echo "prof sdma failed"; exit 1; }
echo "prof sdma ok"
