# row statistic one wave per row (lane = 128-column part): bitwise tests, engine tests, micro-bench
# (graph replay), generation probes 8 / 32 prompts
set -o pipefail
O=gpurun_out/${1:-r6_row_stat2}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "row_ss or row_stat or small_m or row_rstd or rmsnorm" > $O/kernel_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_multigpu_gpu.py -x -v --timeout 300 --timeout-method thread > $O/engine_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/row_stat_bench.py --rows 16,40,160,320,1024 > $O/row_stat_bench.log 2>&1 || exit 1
timeout -k 10 600 python -u scripts/gen_exact_probe.py --prompts 32 --gen 6 --fast --json $O/probe32.json > $O/probe32.log 2>&1 || exit 1
timeout -k 10 600 python -u scripts/gen_exact_probe.py --prompts 8 --gen 6 --fast --json $O/probe8.json > $O/probe8.log 2>&1 || exit 1
