# grouped attention with the pruned last layer's Q / O projections over all scored rows: bits probe,
# the VRAM / engine / v11 GPU tests, then headline, 16k token budget (resident states, v11 by tile
# rounds) and 128 prompts on one box
set -o pipefail
O=gpurun_out/${1:-r5_bits2}
mkdir -p $O
timeout -k 10 200 python -u scripts/bits_probe.py > $O/bits.log 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest tests/test_vram_gpu.py tests/test_engine_gpu.py tests/test_kernels_gpu.py -q --timeout 280 --timeout-method thread -k "vram or v11 or engine or piece or grouped or prun or graph or spec" > $O/tests.log 2>&1
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
B="python -u bench.py --steps 3 --warmup 1"
timeout -k 10 300 $B > $O/head.log 2>&1 || exit 1
timeout -k 10 300 $B --token-budget 16384 > $O/tb16k.log 2>&1 || exit 1
timeout -k 10 400 $B --prompts-per-gpu 128 --steps 2 > $O/p128.log 2>&1 || exit 1
