# landing the next micro-batch's state ahead of the current compute: GPU tests of the capped /
# spilling paths, then the spill regimes at two run-ahead bounds, the headline and the envelope
set -o pipefail
O=gpurun_out/${1:-r5_land}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_vram_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
B="python -u bench.py --warmup 1"
for n in 0 6; do
  FLS_RUNAHEAD_ITEMS=$n timeout -k 10 500 $B --steps 2 --prompts-per-gpu 128 > $O/p128_ra$n.log 2>&1 || exit 1
  FLS_RUNAHEAD_ITEMS=$n timeout -k 10 300 $B --steps 3 --token-budget 16384 > $O/tb16k_ra$n.log 2>&1 || exit 1
done
timeout -k 10 300 $B --steps 3 > $O/head.log 2>&1 || exit 1
