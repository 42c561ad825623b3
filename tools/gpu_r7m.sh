set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r7m; mkdir -p $OUT
export TMPDIR=/tmp
R=$PWD; cd /tmp
for A in 0 1 2 3; do
  DMLP_REFINE_ABL=$A timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $R/$OUT/abl$A -o p --output-format csv -- python3 $R/bench.py --steps 30 --warmup 2 --min-warmup-s 0 > $R/$OUT/abl$A.log 2>&1 || { echo "abl $A failed"; tail -3 $R/$OUT/abl$A.log; exit 1; }
  echo "abl $A: $(grep -h 'k_refine_pair' $R/$OUT/abl$A/p_kernel_stats.csv | cut -d, -f2-4)"
done
