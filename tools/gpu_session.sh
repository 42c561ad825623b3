#!/bin/bash
# Maintained GPU entry point (one gpurun call = one session).  Every GPU step runs under its own
# time limit and the session stops at the first failing step.
#
#   gpurun --timeout 900 -- bash tools/gpu_session.sh <tag> <task> [<task> ...]
#
# tasks:
#   tests      pytest -m gpu (the round-end GPU tier)
#   ktests     the GPU tests selected by KTESTS (a pytest -k expression)
#   bench      python bench.py (defaults: 1 GPU, headline config)
#   verify     python bench.py --verify (every report line vs the exact CPU path)
#   prof       rocprofv3 --kernel-trace --stats over a short bench run (kernel split)
#   timeline   rocprofv3 kernel + memory-copy trace of the last steps (tools/timeline.py)
#   pmc        one --pmc pass per counter group over the screen + refine (tools/pmc_summary.py)
#   exactprof  the fused exact kernel (bench.py --exact): kernel split + one PMC pass
#   engine     native knn_engine: every strategy vs the CPU oracle bytes (tools/engine_check.sh)
#   sweep      bench sweep over N / A / k (profiles/ sweep table)
#   sweepa     the sweep at N 1e5 / 1e6 with A 32 / 128 / 256
#   exact      bench.py --exact (fp64-only path)
#   harness    bench.py --harness native (knn_engine through the reference contract)
#   dropin     bench.py --harness dropin (engine.h drop-in linked with the reference's common.cpp)
#   split      kernel split of the local pipeline at Q = 131072 / 65536 / 32768 (S = 1 / 2 / 4)
#   merge      K4 merge micro-benchmark (P=8, Q=131072, k=16/128) under rocprofv3 --stats
#   hostprof   cProfile of the step loop (tools/host_profile.py) + per-call host phase clocks
#   dr         device render A/B (DMLP_DEVICE_RENDER), step timelines
#   plane      node render plane rehearsal: bench.py --gpus 3 / 8 on the one GPU, plane on / off
#   rehearsal  8-GPU host budget on one GPU: GPU rank + 7 CPU phantoms (tools/host_rehearsal.py)
#   blits      copy-engine probe + every runtime kernel / SDMA copy of 6 native steps (step_driver)
#   dropin8    drop-in at P = 8, Q = 131072 per rank on the one GPU: CMA / fill / auto fronts
#   dropinp    drop-in at P = 4 / 8 through the node window, each front of FRONTS (cma fill)
#   lnr        large-N steps: host vs device render at N 1e6 / 1e7 (step_driver)
#   pyck       NoCU copies from Python with / without torch (tools/copy_kind_py.py)
#   h2dbw      H2D bandwidth over 1 / 2 / 4 streams (tests/native/h2d_bw.cpp)
#   rt70       torch's bundled HIP runtime vs /opt/rocm's: copy kinds, the step's copies, step time
#   final      end-of-round validation (GPU tier, smoke, driver bench line, verify, exact, P = 3)
#   dropin_p   the engine.h drop-in at P = 2 / 3 through the node window (one GPU)
#   exact64    the exact path at A = 48 / 64: fp64 MFMA screen vs VALU kernel, --verify
#   modes      h2d / xgmi dataset ingress at P = 3 / 4 (host plane) with --verify
#   prewarm    the drop-in contract at KNN_PREWARM_US 0 / 300 / 2000 / 5000
#   cmpab      pair refine over compacted group entries vs the previous tree (library A/B)
#   qcab       early start query-operand slices 4 / 6 / 8 (DMLP_FAST_QCHUNKS A/B, timelines)
#   rl4ab      pair refine at 4 vs 8 lanes per exact row (library A/B, --verify of the variant)
#   p32kt      pair epilogue on the 32-entry screen up to KT 8 / 2 / 1 (library A/B over the sweep rows)
#   p32q       the pair-epilogue KT limit A/B at Q = 131072 (A = 64 / 128, k 17-64)
#   kt2b       KT 2 at k = 32: 16- vs 32-entry screen (library A/B, after the pair limit)
#   rdab       report straight into pinned host memory vs staged + D2H (DMLP_REPORT_DIRECT A/B)
set -u
TAG=${1:?tag}
shift
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
# bench.py's reference-contract runs (fresh drop-in processes after the timed steps) only where a
# task wants the driver's line: bench, bench3, final
export DMLP_BENCH_CONTRACT_RUNS=0 DMLP_BENCH_LARGE_N=0
step() {  # name seconds cmd...  (stdout+stderr to $OUT/name.log)
  local name=$1 secs=$2
  shift 2
  echo "[session] $name: $*"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -n 25 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "[session] $name failed rc=$rc"; exit $rc; fi
}
for task in "$@"; do
  case "$task" in
    tests)
      step tests 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 \
          --timeout-method thread ;;
    ktests)  # a subset of the GPU tier: KTESTS='<pytest -k expression>'
      step ktests 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 \
          --timeout-method thread -k "${KTESTS:?KTESTS}" ;;
    bench)
      DMLP_BENCH_CONTRACT_RUNS=3 DMLP_BENCH_LARGE_N=1 step bench 300 python bench.py ;;
    bench3)  # three headline runs in a row (run-to-run spread: timed_step_ms, cgroup throttling)
      for r in 1 2 3; do DMLP_BENCH_CONTRACT_RUNS=3 DMLP_BENCH_LARGE_N=1 step bench_$r 300 python bench.py; done ;;
    verify)
      step verify 300 python bench.py --steps 20 --warmup 2 --verify ;;
    exact)
      step exact 300 python bench.py --exact --steps 5 --warmup 1 ;;
    early)  # native step early start (default) -- its tests, verify, interleaved step A/B against DMLP_FAST_EARLY=0
      step early_tests 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 \
          --timeout-method thread -k "native_step"
      step early_verify 300 python bench.py --steps 20 --warmup 2 --verify
      AB_PROF=0 AB_ROUNDS=3 AB_STEPS=200 step early_ab 900 bash tools/kernel_ab.sh base:DMLP_FAST_EARLY=0 \
          early:DMLP_FAST_EARLY=1 ;;
    qchunks)  # early start: query render slices 2 / 4 / 6 (DMLP_FAST_QCHUNKS), interleaved
      AB_PROF=0 AB_ROUNDS=4 AB_STEPS=200 step qchunks_ab 900 bash tools/kernel_ab.sh \
          q2:DMLP_FAST_QCHUNKS=2 q4:DMLP_FAST_QCHUNKS=4 q6:DMLP_FAST_QCHUNKS=6 ;;
    warm)  # the headline bench after a 3 s warm-up instead of 0.6 s (box-to-box host variance)
      step bench_warm3 300 python bench.py --min-warmup-s 3 ;;
    prof)
      step prof 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
          -- python3 bench.py --steps 10 --warmup 2 --no-busbw --diag-steps 0
      find "$OUT/prof" -name '*kernel_stats.csv' -exec sh -c 'head -12 "$1" | cut -c1-200' _ {} \; ;;
    timeline)
      step timeline 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT/tl" -o run \
          --output-format csv -- python3 bench.py --steps 4 --warmup 2 --no-busbw --diag-steps 0
      python3 tools/timeline.py "$OUT/tl" 7 > "$OUT/timeline.txt"; tail -40 "$OUT/timeline.txt" ;;
    pmc)
      n=0
      for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
               "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM" \
               "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
               "GRBM_GUI_ACTIVE GRBM_COUNT"; do
        n=$((n + 1))
        # counters only: no trace domains beside --pmc
        # (the headline step itself: the native step driver, early start, host operands)
        step pmc$n 120 rocprofv3 --kernel-trace --pmc $C -d "$OUT/pmc$n" -o run --output-format csv \
            -- tools/bin/step_driver --steps 3 --warmup 3
      done
      python3 tools/pmc_csv_summary.py "$OUT" pmc > "$OUT/pmc_summary.txt"; cat "$OUT/pmc_summary.txt" ;;
    exactprof)  # the fused exact kernel: kernel split + one counter pass
      step exact_stats 300 rocprofv3 --kernel-trace --stats -d "$OUT/exact_stats" -o run \
          --output-format csv -- python3 bench.py --exact --steps 3 --warmup 1 --no-busbw --diag-steps 0
      find "$OUT/exact_stats" -name '*kernel_stats.csv' -exec sh -c 'head -6 "$1" | cut -c1-160' _ {} \;
      step exact_pmc 180 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
          SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU \
          -d "$OUT/pmc_exact" -o run --output-format csv \
          -- python3 bench.py --exact --steps 1 --warmup 1 --no-busbw --diag-steps 0
      python3 tools/pmc_summary.py "$OUT" > "$OUT/pmc_summary.txt"; cat "$OUT/pmc_summary.txt" ;;
    engine)
      step engine 400 bash tools/engine_check.sh "$OUT/engine" ;;
    sweep)
      step sweep 1150 python3 -u tools/bench_sweep.py --out "$OUT/sweep.jsonl" --timeout 170 ;;
    sweepa)  # N 1e5 / 1e6 x A 32 / 128 / 256 x k 16 / 1-64 / 200
      step sweepa 1100 python3 -u tools/bench_sweep.py --out "$OUT/sweep.jsonl" --timeout 150 \
          --ns 100000,1000000 --attrs 32,128,256 ;;
    harness)
      step harness 600 python bench.py --harness native ;;
    dropin)
      step dropin 600 python bench.py --harness dropin --steps 20 --warmup 1
      python -m distributed_machine_learning_project_amd.build --dropin \
          distributed_machine_learning_project_amd/_refharness/common.cpp --dropin-out /tmp/eng_dropin
      python tools/generate_input.py --num_data 100000 --num_queries 131072 --num_attrs 32 --min 0 \
          --max 1000 --minK 16 --maxK 16 --num_labels 10 --output /tmp/dropin_bench.in > /dev/null
      for i in 1 2 3; do
        KNN_TRACE=1 timeout -k 10 120 /tmp/eng_dropin < /tmp/dropin_bench.in > /tmp/dropin.out \
            2> "$OUT/dropin_trace_$i.txt" || exit 1
      done
      KNN_ROWS_I32=0 KNN_TRACE=1 timeout -k 10 120 /tmp/eng_dropin < /tmp/dropin_bench.in \
          > /tmp/dropin.out 2> "$OUT/dropin_trace_fp64rows.txt" || exit 1
      for i in 1 2; do  # the same input through knn_engine (row-major arrays, its own parser)
        KNN_TRACE=1 timeout -k 10 120 distributed_machine_learning_project_amd/knn_engine \
            --input /tmp/dropin_bench.in > /tmp/native.out 2> "$OUT/native_trace_$i.txt" || exit 1
      done
      cmp /tmp/dropin.out /tmp/native.out && echo "dropin == native report bytes"
      tail -n 12 "$OUT/dropin_trace_3.txt" "$OUT/dropin_trace_fp64rows.txt" "$OUT/native_trace_2.txt" ;;
    split)
      for q in 131072 65536 32768; do
        step split_$q 240 rocprofv3 --kernel-trace --stats -d "$OUT/split_$q" -o run --output-format csv \
            -- python3 tools/quick_gpu_bench.py --q $q --iters 6 --check 200
        find "$OUT/split_$q" -name '*kernel_stats.csv' -exec sh -c 'head -6 "$1" | cut -c1-150' _ {} \;
      done ;;
    merge)
      step merge 300 rocprofv3 --kernel-trace --stats -d "$OUT/merge" -o run --output-format csv \
          -- python3 tools/merge_bench.py --p 8 --q 131072 --ks 16,128
      DMLP_MERGE_WIN=0 step merge_seq 120 python3 tools/merge_bench.py --p 8 --q 131072 --ks 16,128
      find "$OUT/merge" -name '*kernel_stats.csv' -exec sh -c 'head -8 "$1" | cut -c1-160' _ {} \; ;;
    hostprof)
      step hostprof 300 python tools/host_profile.py --steps 100
      DMLP_PIPE_DEBUG=1 step pipedebug 120 python bench.py --steps 5 --warmup 2 --no-busbw ;;
    dr)  # device render of the screen operands: host render / device render, +/- query blocks
      # (the early-start bench shape renders on the host either way: Q = 32768 per step, no early
      # start, and the bench shape with the early start off)
      AB_PROF=0 AB_ROUNDS=3 AB_STEPS=200 AB_ARGS="--q-per-gpu 32768" step dr_ab 900 bash tools/kernel_ab.sh \
          hr:DMLP_DEVICE_RENDER=0 dr:DMLP_DEVICE_RENDER=1
      python3 tools/ab_timeline.py gpurun_out/ab > "$OUT/dr_q32k.txt"; rm -rf gpurun_out/ab
      AB_PROF=0 AB_ROUNDS=3 AB_STEPS=200 step dr_ab2 900 bash tools/kernel_ab.sh \
          early_hr:DMLP_DEVICE_RENDER=0 noearly_hr:DMLP_DEVICE_RENDER=0,DMLP_FAST_EARLY=0 \
          noearly_dr:DMLP_DEVICE_RENDER=1,DMLP_FAST_EARLY=0
      python3 tools/ab_timeline.py gpurun_out/ab > "$OUT/dr_bench.txt"
      cat "$OUT/dr_q32k.txt" "$OUT/dr_bench.txt" ;;
    plane)  # node render plane: P = 3 / 8 ranks sharing the one GPU (host-staged plane), --verify,
            # plane on / off: per-rank ms, the cgroup's CPU time in the timed region
      for P in 3 8; do
        Qp=$([ $P = 3 ] && echo 65536 || echo 16384)
        for pl in 1 0; do
          DMLP_DATA_PLANE=host KNN_PLANE=$pl step plane_p${P}_$pl 400 python bench.py --gpus $P \
              --steps 10 --warmup 2 --min-warmup-s 1 --q-per-gpu $Qp --verify --no-busbw
        done
      done ;;
    rehearsal)  # host budget of an 8-GPU node: the GPU rank + 7 CPU phantom ranks, 2 threads each
      step reh_solo2 300 python tools/host_rehearsal.py --ranks 1 --threads 2
      step reh_solo14 300 python tools/host_rehearsal.py --ranks 1 --threads 14
      for PL in 1 0; do
        step reh_p$PL 300 python tools/host_rehearsal.py --ranks 8 --threads 2 --plane $PL
      done
      grep -h '^{' "$OUT"/reh_*.log ;;
    dropin_p)  # the drop-in at P = 2 / 3 through the node window on the one GPU (host-staged plane):
               # bench.py --harness dropin (per-rank step times), knn_engine's shm farm beside it
      for P in 2 3; do
        KNN_DATA_PLANE=host step dropin_p$P 600 python bench.py --harness dropin --gpus $P --steps 5 \
            --warmup 1 --q-per-gpu 65536
        KNN_DATA_PLANE=host step native_p$P 600 python bench.py --harness native --gpus $P --steps 5 \
            --warmup 1 --q-per-gpu 65536 --ingress shm
      done ;;
    exact64)  # the exact path at A = 48 / 64 on the fp64 MFMA screen vs the VALU kernel, --verify
      for A in 48 64; do
        step exact_a${A}_f64 300 python bench.py --exact --attrs $A --steps 3 --warmup 1 \
            --min-warmup-s 0 --verify --no-busbw
        DMLP_EXACT_F64=0 step exact_a${A}_valu 300 python bench.py --exact --attrs $A --steps 3 \
            --warmup 1 --min-warmup-s 0 --verify --no-busbw
      done
      grep -ho '"ms_per_step": [0-9.]*\|"verify_ok": [a-z]*' "$OUT"/exact_a*.log ;;
    modes)  # the replicated dataset's two ingress modes at P = 3 / 4 on the one GPU (host plane),
            # --verify, collective bytes per step in the JSON
      for P in 3 4; do
        for M in h2d xgmi; do
          DMLP_DATA_PLANE=host KNN_DATA_INGRESS=$M step modes_p${P}_$M 400 python bench.py --gpus $P \
              --steps 10 --warmup 2 --min-warmup-s 1 --q-per-gpu 32768 --verify --no-busbw
        done
      done
      grep -ho '"ms_per_step": [0-9.]*\|"verify_ok": [a-z]*\|"collective_bytes_per_step": {[^}]*}' \
          "$OUT"/modes_*.log ;;
    prewarm)  # the drop-in contract at KNN_PREWARM_US 0 / 300 / 2000 / 5000 (GPU busy before the call)
      for US in 0 300 2000 5000; do
        KNN_PREWARM_US=$US step prewarm_$US 300 python bench.py --harness dropin --steps 10 --warmup 1
      done
      grep -ho '"knn_ms_median": [0-9.]*' "$OUT"/prewarm_*.log ;;
    blits)  # which copies / memsets the runtime runs as kernels (tests/native/copy_kind_probe.cpp,
            # built to tools/bin), then every runtime kernel and SDMA copy of 4 bench steps
      step copykind 120 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT/ck" -o run \
          --output-format csv -- tools/bin/copy_kind_probe
      python3 tools/copy_kind.py probe "$OUT/ck" > "$OUT/copy_kind.txt"; cat "$OUT/copy_kind.txt"
      step blits 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT/bl" -o run \
          --output-format csv -- tools/bin/step_driver --steps 6 --warmup 30 --timeline
      python3 tools/copy_kind.py step "$OUT/bl" > "$OUT/step_copies.txt"; tail -80 "$OUT/step_copies.txt" ;;
    rt70)  # the HIP runtime torch bundles (torch/lib, ROCm 7.0: what libdmlp runs on inside a
           # Python process) vs /opt/rocm's: the copy-kind probe and the native step's copies
           # under it, then bench-shape step time on each runtime
      TL=$(python3 -c "import os, torch; print(os.path.dirname(torch.__file__) + '/lib')")
      LD_LIBRARY_PATH=$TL step copykind70 120 rocprofv3 --kernel-trace --memory-copy-trace \
          -d "$OUT/ck70" -o run --output-format csv -- tools/bin/copy_kind_probe
      python3 tools/copy_kind.py probe "$OUT/ck70" > "$OUT/copy_kind70.txt"; cat "$OUT/copy_kind70.txt"
      LD_LIBRARY_PATH=$TL step blits70 300 rocprofv3 --kernel-trace --memory-copy-trace \
          -d "$OUT/bl70" -o run --output-format csv -- tools/bin/step_driver --steps 6 --warmup 30 \
          --timeline
      python3 tools/copy_kind.py step "$OUT/bl70" > "$OUT/step_copies70.txt"
      tail -60 "$OUT/step_copies70.txt"
      for R in 1 2; do
        step sd72_$R 120 tools/bin/step_driver --steps 300 --warmup 200
        LD_LIBRARY_PATH=$TL step sd70_$R 120 tools/bin/step_driver --steps 300 --warmup 200
      done
      grep -H '"ms_per_step"' "$OUT"/sd7*.log | cut -c1-200 ;;
    cklog)  # which engine runs each copy WITHOUT a profiler attached: the runtime's own log
            # (AMD_LOG_LEVEL=4: "HSA Copy ... forceSDMA=" per SDMA copy, a launch per blit kernel),
            # native probe and Python probe; then the native probe under --kernel-trace alone
      AMD_LOG_LEVEL=4 step cklog_native 120 tools/bin/copy_kind_probe
      AMD_LOG_LEVEL=4 step cklog_py 120 python3 tools/copy_kind_py.py 0 hostmalloc
      step ck_kt 120 rocprofv3 --kernel-trace --stats -d "$OUT/ck_kt" -o run --output-format csv \
          -- tools/bin/copy_kind_probe
      for f in cklog_native cklog_py; do
        echo "$f: HSA Copy $(grep -c 'HSA Copy' "$OUT/$f.log" || true)," \
             "forceSDMA=1 $(grep -c 'forceSDMA=1' "$OUT/$f.log" || true)," \
             "copyBuffer $(grep -c 'copyBuffer' "$OUT/$f.log" || true)"
      done
      echo "native probe, kernel trace only: copyBuffer $(grep -c copyBuffer \
          "$OUT/ck_kt/run_kernel_trace.csv" || true)" ;;
    kverify2)  # --verify at A = 48 / 64 (KT 2) across the k classes
      for AK in "48 32 32" "64 1 32" "64 17 64" "48 1 16"; do
        set -- $AK
        step kv2_$1_$2_$3 300 python bench.py --attrs $1 --k $3 --kmin $2 --kmax $3 --steps 20 \
            --warmup 2 --min-warmup-s 1 --no-busbw --diag-steps 0 --verify
      done
      grep -Ho '"ms_per_step": [0-9.]*\|"verify_ok": [a-z]*\|"escalated_queries": [0-9]*\|"early_start_calls": [0-9]*' \
          "$OUT"/kv2_*.log ;;
    cmpab)  # pair refine over the compacted passing group entries (ab/libdmlp_cmp.so) vs the
            # previous tree (ab/libdmlp_base.so), interleaved under the kernel tracer
      rm -rf gpurun_out/ab
      AB_ROUNDS=3 AB_STEPS=30 step cmpab 900 bash tools/kernel_ab.sh base cmp
      python tools/ab_summary.py gpurun_out/ab | tee "$OUT/cmpab_kernels.txt" ;;
    qcab)  # early start: the query operands rendered + copied in 4 / 6 / 8 slices, interleaved,
           # with step timelines (operands_landed)
      rm -rf gpurun_out/ab
      AB_PROF=0 AB_ROUNDS=3 AB_STEPS=100 AB_ARGS="--diag-steps 30" \
          step qcab 900 bash tools/kernel_ab.sh qc4:DMLP_FAST_QCHUNKS=4 qc6:DMLP_FAST_QCHUNKS=6 qc8:DMLP_FAST_QCHUNKS=8
      for f in gpurun_out/ab/*.log; do
        echo "$f $(grep -o '"p50": [0-9.]*' "$f" | head -1) $(grep -o '"operands_landed": [0-9.]*' "$f")"
      done | tee "$OUT/qcab_summary.txt" ;;
    rl4ab)  # pair refine exact rows at 4 lanes per row (ab/libdmlp_rl4.so) vs 8 (ab/libdmlp_base.so):
            # --verify of the variant, then interleaved under the kernel tracer
      DMLP_LIB=ab/libdmlp_rl4.so step rl4_verify 300 python bench.py --steps 20 --warmup 2 --verify
      grep -o '"verify_ok": [a-z]*' "$OUT/rl4_verify.log"
      rm -rf gpurun_out/ab
      AB_ROUNDS=3 AB_STEPS=30 step rl4ab 900 bash tools/kernel_ab.sh base rl4
      python tools/ab_summary.py gpurun_out/ab | tee "$OUT/rl4ab_kernels.txt" ;;
    p32kt)  # the pair epilogue on the 32-entry screen (k in (32, 64]) up to KT = 8 / 2 / 1
            # (ab/libdmlp_k{8,2,1}.so): --verify of each variant at A = 64 / 128, then the sweep's
            # k 1-64 / 33-64 rows at A = 64 / 128 / 256 alternating over the variants, two rounds
      for V in 2 1; do
        DMLP_LIB=ab/libdmlp_k$V.so step p32kt_verify_k$V 300 python bench.py --attrs $((64 * V)) \
            --k 48 --kmin 33 --kmax 64 --q-per-gpu 16384 --steps 5 --warmup 1 --min-warmup-s 0 \
            --no-busbw --diag-steps 0 --verify
      done
      grep -Ho '"verify_ok": [a-z]*' "$OUT"/p32kt_verify_*.log
      for R in 1 2; do
        for V in 8 2 1; do
          DMLP_LIB=ab/libdmlp_k$V.so step p32kt_k${V}_$R 400 python3 -u tools/bench_sweep.py \
              --out "$OUT/p32kt_k${V}_$R.jsonl" --timeout 120 --ns 100000 --attrs 64,128,256 \
              --ks 1-64,33-64
        done
      done ;;
    p32q)  # the same A/B at the headline's Q = 131072: A = 64 / 128 at k 17-64, interleaved
      for A in 64 128; do
        AB_PROF=0 AB_ROUNDS=3 AB_STEPS=60 AB_ARGS="--attrs $A --k 40 --kmin 17 --kmax 64 --diag-steps 0" \
            step p32q_a$A 600 bash tools/kernel_ab.sh k8 k1
      done ;;
    kt2b)  # A = 48 / 64 at k = 32 with the pair epilogue off on the 32-entry screen: the 16-entry
           # screen (ab/libdmlp_s16.so, no early start) vs the 32-entry one (ab/libdmlp_s32.so)
      for A in 48 64; do
        AB_PROF=0 AB_ROUNDS=3 AB_STEPS=60 AB_ARGS="--attrs $A --k 32 --diag-steps 0" \
            step kt2b_a$A 600 bash tools/kernel_ab.sh s16 s32
      done ;;
    rdab)  # the report written straight into the caller's pinned buffer vs staged + one D2H copy,
           # interleaved (AB_ROUNDS x 100 steps), then the contract (drop-in, mpiexec) both ways
      AB_PROF=0 AB_ROUNDS=${AB_ROUNDS:-3} AB_STEPS=100 AB_ARGS="--diag-steps 30" \
          step rdab 900 bash tools/kernel_ab.sh direct:DMLP_REPORT_DIRECT=1 staged:DMLP_REPORT_DIRECT=0 ;;
    kt2)  # A = 48 / 64 (KT 2) at k = 32: the 16-entry screen (no early start there) vs the 32-entry
          # screen with the early start, interleaved
      for A in 48 64; do
        AB_PROF=0 AB_ROUNDS=2 AB_STEPS=100 AB_ARGS="--attrs $A --k 32 --diag-steps 0" \
            step kt2_a$A 600 bash tools/kernel_ab.sh s16:DMLP_X1_SUB16_KMAX=32 s32:DMLP_X1_SUB16_KMAX=16
      done ;;
    pair32)  # the pair epilogue on the 32-entry screen too (k in (32, 64]): library builds
             # ab/libdmlp_base.so vs ab/libdmlp_pair32.so, interleaved, at k 17-64 and 33-64
      AB_PROF=0 AB_ROUNDS=2 AB_STEPS=100 AB_ARGS="--k 40 --kmin 17 --kmax 64 --diag-steps 0" \
          step pair32_a 600 bash tools/kernel_ab.sh base pair32
      AB_PROF=0 AB_ROUNDS=2 AB_STEPS=100 AB_ARGS="--k 48 --kmin 33 --kmax 64 --diag-steps 0" \
          step pair32_b 600 bash tools/kernel_ab.sh base pair32 ;;
    sub16)  # k in (16, 32] on the SUB = 16 screen (pair epilogue, two waves per SIMD) vs SUB = 32,
            # interleaved, bench shape at k = 32 and k 1-32 (escalations in the JSON)
      for R in 1 2; do
        for V in 16 32; do
          DMLP_X1_SUB16_KMAX=$V step sub16_k32_${V}_$R 300 python bench.py --k 32 --steps 100 \
              --min-warmup-s 1 --no-busbw --diag-steps 0
          DMLP_X1_SUB16_KMAX=$V step sub16_k1_32_${V}_$R 300 python bench.py --k 32 --kmin 1 \
              --kmax 32 --steps 100 --min-warmup-s 1 --no-busbw --diag-steps 0
        done
      done
      for f in "$OUT"/sub16_*.log; do
        echo "$f $(grep -o '"ms_per_step": [0-9.]*' "$f" | head -1) $(grep -o '"escalated_queries": [0-9]*' "$f" | head -1)"
      done ;;
    kverify)  # --verify at k = 24 / 32 / 1-32 / 17-64 (the k classes around the SUB 16 / 32 line)
      for KS in "24 24 24" "32 32 32" "32 1 32" "40 17 64"; do
        set -- $KS
        step kv_$1_$2_$3 300 python bench.py --k $1 --kmin $2 --kmax $3 --steps 20 --warmup 2 \
            --min-warmup-s 1 --no-busbw --diag-steps 0 --verify
      done
      grep -Ho '"ms_per_step": [0-9.]*\|"verify_ok": [a-z]*\|"escalated_queries": [0-9]*' \
          "$OUT"/kv_*.log ;;
    p3c)  # the P = 3 host-plane rehearsal with the node contract after the timed steps (rank 0
          # runs the drop-in through mpiexec -n 3, the other ranks wait on the segment)
      DMLP_BENCH_CONTRACT_RUNS=2 KNN_DATA_PLANE=host DMLP_DATA_PLANE=host step p3c 600 python bench.py \
          --gpus 3 --steps 20 --warmup 2 --min-warmup-s 1 --no-busbw
      grep -o '"reference_contract_node": {[^}]*' "$OUT/p3c.log" | head -c 600; echo ;;
    k200)  # the two-pass class (k = 200) at N = 1e7: device vs host render, alternating
      for R in 1 2; do
        for DR in 1 0; do
          DMLP_DEVICE_RENDER=$DR step k200_dr${DR}_$R 300 tools/bin/step_driver --n 10000000 --a 32 \
              --q 16384 --k 200 --steps 3 --warmup 1 --timeline
        done
      done
      grep -H '^{' "$OUT"/k200_*.log | sed 's/"timeline.*//' ;;
    sweep7)  # the sweep's N = 1e7 rows (A 32 / 128 x k 16 / 1-64 / 200)
      step sweep7 1150 python3 -u tools/bench_sweep.py --out "$OUT/sweep7.jsonl" --timeout 240 \
          --ns 10000000 --attrs 32,128 ;;
    drab)  # the render choice per k class at N 1e5 / 1e6 x A 32 / 128: the host render forced
           # (DMLP_DEVICE_RENDER=0) against the cost model's choice, alternating on one box
      for R in 1 2; do
        DMLP_DEVICE_RENDER=0 step drab_host_$R 500 python3 -u tools/bench_sweep.py \
            --out "$OUT/drab_host_$R.jsonl" --timeout 120 --ns 100000,1000000 --attrs 32,128
        step drab_auto_$R 500 python3 -u tools/bench_sweep.py --out "$OUT/drab_auto_$R.jsonl" \
            --timeout 120 --ns 100000,1000000 --attrs 32,128
      done ;;
    prio)  # the copies' stream at the high priority vs the default, interleaved (bench shape)
      AB_PROF=0 AB_ROUNDS=4 AB_STEPS=200 step prio_ab 900 bash tools/kernel_ab.sh \
          p0:DMLP_SIDE_PRIORITY=0 p1:DMLP_SIDE_PRIORITY=1
      grep -Ho '"ms_per_step": [0-9.]*' gpurun_out/ab/p*.log | tee "$OUT/prio_ab.txt" ;;
    refabl)  # the pair refine's time with its exact-row gathers / member loads ablated
             # (DMLP_REFINE_ABL 1 / 2 / 3: wrong results, timing only), native step driver
      for AB in 0 1 2 3; do
        DMLP_REFINE_ABL=$AB step refabl_$AB 120 rocprofv3 --kernel-trace --stats -d "$OUT/refabl_$AB" \
            -o run --output-format csv -- tools/bin/step_driver --steps 20 --warmup 5
        echo "abl=$AB: $(grep -h k_refine_pair "$OUT/refabl_$AB/run_kernel_stats.csv" | cut -d, -f2-4)"
      done ;;
    h2dbw)  # H2D bandwidth from page-locked memory over 1 / 2 / 4 concurrent streams
      step h2dbw 120 tools/bin/h2d_bw ;;
    pyck)  # the NoCU copies from a Python process, with / without torch initialised first
      for T in 0 1; do
        for M in hostmalloc registered; do
          step pyck_${T}_$M 120 rocprofv3 --kernel-trace --stats -d "$OUT/pyck_${T}_$M" -o run \
              --output-format csv -- python3 tools/copy_kind_py.py $T $M
          echo "torch=$T mem=$M copyBuffer kernels: $(grep -c copyBuffer \
              "$OUT/pyck_${T}_$M/run_kernel_trace.csv" || true)"
        done
      done ;;
    dropin8)  # the engine.h drop-in at P = 8 through the node window on the one GPU, Q = 131072 per
              # rank (KNN_DATA_PLANE=host), each front (CMA / rank-0 fill), plus the CMA probe
      step cmaprobe 120 tools/bin/cma_probe
      for F in cma fill auto; do
        KNN_WINDOW_FRONT=$F KNN_DATA_PLANE=host step dropin8_$F 900 python bench.py --harness dropin \
            --gpus 8 --q-per-gpu 131072 --steps 2 --warmup 1
      done
      grep -h -o '"window": {[^}]*}' "$OUT"/dropin8_*.log | tee "$OUT/dropin8_window.txt" ;;
    lnr)  # large-N steps (native step driver): the default (device render by the cost model, the
          # chunked screen pipeline) vs the host render forced, alternating, step timelines
      for SH in "1000000 32 10" "1000000 128 6" "10000000 32 4"; do
        set -- $SH
        for R in 1 2; do
          step lnr_n$1_a$2_auto_$R 300 tools/bin/step_driver --n $1 --a $2 --q 16384 --steps $3 \
              --warmup 2 --timeline
          DMLP_DEVICE_RENDER=0 step lnr_n$1_a$2_host_$R 300 tools/bin/step_driver --n $1 --a $2 \
              --q 16384 --steps $3 --warmup 2 --timeline
        done
      done
      grep -H '^{' "$OUT"/lnr_*.log | tee "$OUT/lnr_summary.txt" ;;
    dropinp)  # the drop-in at P = 4 / 8 through the node window on the one GPU, each front, with
              # every rank's fetch phases (KNN_METRICS)
      for P in 4 8; do
        for F in ${FRONTS:-cma fill}; do
          KNN_WINDOW_FRONT=$F KNN_DATA_PLANE=host step dropin${P}_$F 600 python bench.py \
              --harness dropin --gpus $P --q-per-gpu 131072 --steps 2 --warmup 1
        done
      done ;;
    final)  # end-of-round validation: GPU tier, smoke(), the driver's bench line, --verify of the
            # default and the exact path, the P = 3 host-plane rehearsal with --verify
      step tests 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 \
          --timeout-method thread
      step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
      DMLP_BENCH_CONTRACT_RUNS=3 DMLP_BENCH_LARGE_N=1 step bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5
      step verify 300 python bench.py --steps 200 --verify
      step exact 300 python bench.py --exact --steps 5 --warmup 1 --min-warmup-s 0 --verify
      DMLP_DATA_PLANE=host step p3 400 python bench.py --gpus 3 --steps 30 --warmup 3 \
          --min-warmup-s 1 --no-busbw --verify
      grep -ho '"ms_per_step": [0-9.]*\|"verify_ok": [a-z]*' "$OUT"/bench_driver.log \
          "$OUT"/verify.log "$OUT"/exact.log "$OUT"/p3.log ;;
    *)
      echo "unknown task $task"; exit 2 ;;
  esac
done
