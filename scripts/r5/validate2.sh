# round-5 validation: GPU tests, then the headline and the spill regimes (capped and uncapped)
set -o pipefail
O=gpurun_out/${1:-r5_validate2}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 > $O/headline.log 2>&1 || exit 1
timeout -k 10 500 python -u bench.py --steps 2 --warmup 1 --prompts-per-gpu 128 > $O/p128.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --token-budget 16384 > $O/tb16k.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --token-budget 16384 --max-vram-gb 0 > $O/tb16k_uncapped.log 2>&1 || exit 1
