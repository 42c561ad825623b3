cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/hp
{ nproc; lscpu | grep -E "Model name|Socket|L3|NUMA node|Core"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; 
for t in 4 8 12 16; do DMLP_HOST_THREADS=$t timeout 120 python tools/bench_host_prep.py; done; } > gpurun_out/hp/hp.txt 2>&1
cat gpurun_out/hp/hp.txt
