# weight-stream (H2D blit) vs GEMM interference, per runtime copy setting
set -o pipefail
mkdir -p gpurun_out/r19
cd "$GRAFT_REPO_ROOT"
CO_JSON=gpurun_out/r19/copy_overlap.json timeout -k 10 900 python scripts/copy_overlap.py > gpurun_out/r19/copy_overlap.log 2>&1
rc=$?; echo "rc=$rc"; cat gpurun_out/r19/copy_overlap.log | cut -c1-400
