# tie guard + row-exact + top-2 + persistent attention + setprio A/B: GPU tests, then attention A/B
set -o pipefail
O=gpurun_out/${1:-r6_gen_tests}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 120 python -u scripts/attn_head_bench.py > $O/attn_prio.log 2>&1 || exit 1
