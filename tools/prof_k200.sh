set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r5h; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/k200 -o run --output-format csv -- python3 bench.py --n-data 100000 --attrs 32 --k 200 --kmin 200 --kmax 200 --q-per-gpu 16384 --steps 10 --warmup 2 --no-busbw --diag-steps 3 > $OUT/k200.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/k16 -o run --output-format csv -- python3 bench.py --n-data 100000 --attrs 32 --k 16 --kmin 16 --kmax 16 --q-per-gpu 16384 --steps 10 --warmup 2 --no-busbw --diag-steps 3 > $OUT/k16.log 2>&1 || exit 1
