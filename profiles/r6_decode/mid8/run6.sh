# 64-column mid blocks of 8 waves (4 x 2 waves of 16 x 32): bitwise kernel tests, decode GEMM A/B,
# generation probes 8 / 32 prompts
set -o pipefail
O=gpurun_out/${1:-r6_mid8_bn64}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "small_m or mid or resid_gemm or row_stat" > $O/kernel_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/decode_gemm_bench.py --rows 16,40,64,160,320 > $O/gemm_bench.log 2>&1 || exit 1
timeout -k 10 600 python -u scripts/gen_exact_probe.py --prompts 8 --gen 6 --only reuse > $O/probe8.log 2>&1 || exit 1
timeout -k 10 600 python -u scripts/gen_exact_probe.py --prompts 8 --gen 6 --only reuse --mid-waves 4 >> $O/probe8.log 2>&1 || exit 1
