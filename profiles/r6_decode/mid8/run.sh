# 8-wave 128-column mid-M blocks (two waves per SIMD) for one-round grids: bitwise kernel tests,
# decode GEMM A/B (4 vs 8 waves), generation probe 32 prompts with each, then auto
set -o pipefail
O=gpurun_out/${1:-r6_mid8}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "small_m or mid or resid_gemm or row_scale or row_ss" > $O/kernel_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/decode_gemm_bench.py --rows 16,64,160,320 > $O/gemm_bench.log 2>&1 || exit 1
for w in 4 8 0; do timeout -k 10 300 python -u scripts/gen_exact_probe.py --prompts 32 --gen 6 --only reuse --mid-waves $w >> $O/probe32.log 2>&1 || exit 1; done
for w in 4 8; do timeout -k 10 300 python -u scripts/gen_exact_probe.py --prompts 8 --gen 6 --only reuse --mid-waves $w >> $O/probe8.log 2>&1 || exit 1; done
