# Copy engines during the early-start step (a --memory-copy-trace run segfaulted in the tracer's exit: dropped):
# plain-bench A/B of the runtime's copy settings (blit kernels vs SDMA, blit workgroup limit).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r8b
AB_PROF=0 AB_ROUNDS=2 AB_STEPS=200 bash tools/kernel_ab.sh base: sdma:HSA_ENABLE_SDMA=1 \
    noblit:GPU_FORCE_BLIT_COPY_SIZE=0 wg4:DEBUG_CLR_LIMIT_BLIT_WG=4 wg64:DEBUG_CLR_LIMIT_BLIT_WG=64
