# 8-wave mid-M blocks of 64 or 128 rows: bitwise kernel tests, decode GEMM A/B, generation probes
# (32 prompts: M = 160; 64 prompts: M = 320) with the auto choice against 4-wave blocks
set -o pipefail
O=gpurun_out/${1:-r6_mid8_rows}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "small_m or mid or resid_gemm" > $O/kernel_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/decode_gemm_bench.py --rows 16,64,160,256,320 > $O/gemm_bench.log 2>&1 || exit 1
for w in 0 4; do timeout -k 10 300 python -u scripts/gen_exact_probe.py --prompts 64 --gen 6 --only reuse --mid-waves $w >> $O/probe64.log 2>&1 || exit 1; done
timeout -k 10 300 python -u scripts/gen_exact_probe.py --prompts 32 --gen 6 --only reuse >> $O/probe32.log 2>&1 || exit 1
