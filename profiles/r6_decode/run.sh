# row-exact panel GEMM: bitwise tests, per-shape A/B at 70B, engine bitwise tests (resident /
# streamed / capped host-mode K/V), generation probes (resident; --max_vram_gb 6)
set -o pipefail
O=gpurun_out/${1:-r6_decode}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "panel" > $O/kernel_tests.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 300 --timeout-method thread -k "suffix_reuse_bitwise_exact or decode_graphs or fast_reuse" > $O/engine_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u scripts/gen_exact_probe.py --prompts 32 --gen 6 --fast --json $O/probe32.json > $O/probe32.log 2>&1 || exit 1
timeout -k 10 900 python -u scripts/gen_exact_probe.py --prompts 32 --gen 6 --max-vram-gb 6 --json $O/cap32.json > $O/cap32.log 2>&1 || exit 1
