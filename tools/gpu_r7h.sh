set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r7h; mkdir -p $OUT
export TMPDIR=/tmp
for H in 1 0; do
  DMLP_HOST_THREADS=1 DMLP_HOST_OPS=$H timeout -k 10 200 python bench.py --steps 100 > $OUT/b_t1_h${H}.log 2>&1 || exit 1
  echo "threads 1 host_ops $H: $(grep -o '"ms_per_step": [0-9.]*' $OUT/b_t1_h${H}.log | head -1) $(grep -o '"step_timeline_ms": {[^}]*}' $OUT/b_t1_h${H}.log)"
done
for cfg in "4 1" "14 0" "2 0"; do
  set -- $cfg
  DMLP_FAST_EARLY=$2 DMLP_DATA_PLANE=host DMLP_HOST_THREADS=$1 timeout -k 10 300 python bench.py --gpus 3 --steps 30 --warmup 3 --min-warmup-s 1 --no-busbw > $OUT/p3_t$1_e$2.log 2>&1 || { tail -5 $OUT/p3_t$1_e$2.log; exit 1; }
  echo "P=3 threads $1 early $2: $(grep -o '"ms_per_step": [0-9.]*' $OUT/p3_t$1_e$2.log | head -1)"
done
# PMC passes over the bench step (screen + refine), counters in their own runs
cd /tmp
R=$GRAFT_REPO_ROOT
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU" \
         "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE" ; do
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "k_refine|k_screen_x1" -d $R/$OUT/pmc$n -o pmc -- python3 $R/bench.py --steps 3 --warmup 1 --min-warmup-s 0 > $R/$OUT/pmc$n.log 2>&1 || { echo "pmc $n failed"; tail -5 $R/$OUT/pmc$n.log; exit 1; }
  echo "pmc pass $n ok"
done
