# 32-column 8-wave mid blocks (O / down at M <= 64): bitwise kernel tests, decode GEMM A/B, probe 8
set -o pipefail
O=gpurun_out/${1:-r6_mid8_bn32}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "small_m or mid or resid_gemm or row_stat" > $O/kernel_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/decode_gemm_bench.py --rows 16,40,64 > $O/gemm_bench.log 2>&1 || exit 1
timeout -k 10 600 python -u scripts/gen_exact_probe.py --prompts 8 --gen 6 --fast --json $O/probe8.json > $O/probe8.log 2>&1 || exit 1
