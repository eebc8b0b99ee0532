# epilogue cost per projection (EPI none vs fused epilogue), 70B and 7B shapes
set -o pipefail
mkdir -p gpurun_out/r64
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python scripts/gemm_epi_cost.py > gpurun_out/r64/epi.log 2>&1
rc=$?; echo "rc=$rc"; grep "^{" gpurun_out/r64/epi.log; tail -2 gpurun_out/r64/epi.log
exit $rc
