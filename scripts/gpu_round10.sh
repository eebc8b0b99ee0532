# GEMM v4 (5-stage ring) correctness + A/B
set -o pipefail
mkdir -p gpurun_out/r10
FLS_GEMM_VARIANT=5 timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k gemm > gpurun_out/r10/pytest_v4.log 2>&1
rc=$?; echo "pytest v4 rc=$rc"; tail -3 gpurun_out/r10/pytest_v4.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/kernel_bench.py --json gpurun_out/r10/kernel_bench.json > gpurun_out/r10/kernel_bench.log 2>&1
rc=$?; echo "kbench rc=$rc"; grep -v amdgpu gpurun_out/r10/kernel_bench.log | head -5
