# after the packing change: the engine GPU tests, smoke, a short headline bench
set -o pipefail
O=gpurun_out/${1:-r6_final_checks2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_vram_gpu.py tests/test_multigpu_gpu.py -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > $O/bench.log 2>&1 || exit 1
