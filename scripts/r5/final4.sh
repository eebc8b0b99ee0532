# closing validation of the final tree (bounded streamed state buffers, 6-chunk ring): every GPU
# test, smoke, the headline (driver command) and the 16k-budget / 128-prompt runs on one box
set -o pipefail
O=gpurun_out/r5_final4
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 > $O/head.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --token-budget 16384 > $O/tb16k.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --prompts-per-gpu 128 > $O/p128.log 2>&1 || exit 1
