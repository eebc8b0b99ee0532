# generation under --max_vram_gb 6: weights through the piece pool, prefix / suffix K/V caches in
# pinned host memory staged per layer (runtime/prefix_cache.py host mode); exact vs reuse
set -o pipefail
O=gpurun_out/${1:-r6_gen_cap}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 300 --timeout-method thread -k "suffix_reuse_bitwise_exact" > $O/tests.log 2>&1 || exit 1
timeout -k 10 900 python -u scripts/gen_exact_probe.py --prompts 32 --gen 6 --max-vram-gb 6 --json $O/cap32.json > $O/cap32.log 2>&1 || exit 1
