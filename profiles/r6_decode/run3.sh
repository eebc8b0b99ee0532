# mid-M kernel with 64-column blocks for one-round grids: GEMM A/B at 70B decode shapes, generation
# probe, then the whole GPU test suite and smoke()
set -o pipefail
O=gpurun_out/${1:-r6_decode3}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "panel or mid or bias_epilogues or main_all" > $O/kernel_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/decode_gemm_bench.py --rows 16,64,160,320 > $O/gemm_bench.log 2>&1 || exit 1
timeout -k 10 600 python -u scripts/gen_exact_probe.py --prompts 32 --gen 6 --fast --json $O/probe32.json > $O/probe32.log 2>&1 || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
