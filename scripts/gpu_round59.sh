# GEMM v10 tile-order sweep (TFLOP/s) on the 70B shapes
set -o pipefail
mkdir -p gpurun_out/r59
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python scripts/gemm_order.py > gpurun_out/r59/order.log 2>&1
rc=$?; echo "rc=$rc"; grep "^{" gpurun_out/r59/order.log
exit $rc
