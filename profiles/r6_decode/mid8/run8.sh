# 64-column 8-wave blocks for two row tiles (M 65-128): bitwise kernel tests, GEMM A/B at M = 96 / 128,
# generation probe with 20 prompts (M = 100)
set -o pipefail
O=gpurun_out/${1:-r6_mid8_m96}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "small_m or mid or resid_gemm" > $O/kernel_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/decode_gemm_bench.py --rows 96,128 > $O/gemm_bench.log 2>&1 || exit 1
timeout -k 10 600 python -u scripts/gen_exact_probe.py --prompts 20 --gen 6 --fast --json $O/probe20.json > $O/probe20.log 2>&1 || exit 1
timeout -k 10 600 python -u scripts/gen_exact_probe.py --prompts 20 --gen 6 --only reuse --mid-waves 4 > $O/probe20_w4.log 2>&1 || exit 1
