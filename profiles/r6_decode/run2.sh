# 6-stage mid-M kernel for one-round grids: bitwise tests, per-shape A/B at 70B, engine tests,
# generation probe (resident: exact reuse vs fast), headline bench check
set -o pipefail
O=gpurun_out/${1:-r6_decode2}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "panel or mid or bias_epilogues or main_all or row_scale" > $O/kernel_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/decode_gemm_bench.py --rows 16,64,160,320 > $O/gemm_bench.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 300 --timeout-method thread -k "suffix_reuse_bitwise_exact or decode_graphs or fast_reuse or speculative" > $O/engine_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u scripts/gen_exact_probe.py --prompts 32 --gen 6 --fast --json $O/probe32.json > $O/probe32.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > $O/bench.log 2>&1 || exit 1
