# canonical row statistic (fls_row_ss == the residual epilogue's partials), panel kernel removed:
# targeted kernel tests, the whole GPU suite, decode GEMM A/B, generation probe, smoke, headline bench
set -o pipefail
O=gpurun_out/${1:-r6_final_checks}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "row_ss or small_m or mid or resid_gemm or row_scale" > $O/kernel_tests.log 2>&1 || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/decode_gemm_bench.py --rows 16,64,160,320 > $O/gemm_bench.log 2>&1 || exit 1
timeout -k 10 600 python -u scripts/gen_exact_probe.py --prompts 32 --gen 6 --fast --json $O/probe32.json > $O/probe32.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > $O/bench.log 2>&1 || exit 1
