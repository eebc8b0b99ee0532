# GEMM v2 correctness + A/B microbench, then 70B bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu > gpurun_out/pytest_gpu5.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu5.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/kernel_bench.py --json gpurun_out/kernel_bench5.json > gpurun_out/kernel_bench5.log 2>&1
rc=$?; echo "kbench rc=$rc"; grep -v amdgpu gpurun_out/kernel_bench5.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 2 --warmup 1 > gpurun_out/bench70b_cpu5.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -E "step|metric" gpurun_out/bench70b_cpu5.log
