# fused row statistic (fls_row_stat): bitwise tests, engine / pipeline bitwise tests, decode probe
set -o pipefail
O=gpurun_out/${1:-r6_rowstat}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "row_ss or small_m or row_rstd" > $O/kernel_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_multigpu_gpu.py -x -v --timeout 300 --timeout-method thread > $O/engine_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u scripts/gen_exact_probe.py --prompts 32 --gen 6 --fast --json $O/probe32.json > $O/probe32.log 2>&1 || exit 1
