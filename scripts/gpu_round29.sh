# rmsnorm / GEMM next to SDMA H2D and D2H (no profiler)
set -o pipefail
mkdir -p gpurun_out/r29
cd "$GRAFT_REPO_ROOT"
CO_JSON=gpurun_out/r29/copy_overlap.json timeout -k 10 600 python scripts/copy_overlap.py default sdma_off > gpurun_out/r29/copy_overlap.log 2>&1
rc=$?; echo "rc=$rc"; cut -c1-600 gpurun_out/r29/copy_overlap.log
