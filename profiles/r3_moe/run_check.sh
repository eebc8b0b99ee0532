set -o pipefail
O=gpurun_out/r3b_moe
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_moe_gpu.py -x -v --timeout 120 --timeout-method thread > $O/moe_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/kernel_tests.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --model mixtral-8x7b --steps 3 --warmup 1 > $O/bench_mixtral.log 2>&1 || exit 1
timeout -k 10 200 python scripts/gemm_k_scaling.py > $O/k_scaling.log 2>&1
