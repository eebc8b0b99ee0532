# persistent attention: bitwise tests, then the headline-shape A/B (1k and 4k prefixes)
set -o pipefail
O=gpurun_out/${1:-r6_attn}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention" > $O/tests.log 2>&1 || exit 1
timeout -k 10 120 python -u scripts/attn_head_bench.py > $O/bench_1k.log 2>&1 || exit 1
timeout -k 10 120 python -u scripts/attn_head_bench.py --prefix 4096 --prompts 8 > $O/bench_4k.log 2>&1 || exit 1
