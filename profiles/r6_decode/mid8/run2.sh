# 8-wave mid-M blocks with a 3- / 4- / 5-stage LDS ring: bitwise kernel tests, decode GEMM A/B
set -o pipefail
O=gpurun_out/${1:-r6_mid8_stages}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "small_m or mid or resid_gemm" > $O/kernel_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/decode_gemm_bench.py --rows 16,64,160,320 > $O/gemm_bench.log 2>&1 || exit 1
