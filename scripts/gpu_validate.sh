# round-3 tree after the container re-creation: full GPU suite, smoke, driver bench command (short)
set -o pipefail
O=gpurun_out/${1:-r3_final}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --gpus 1 --steps 8 --warmup 2 > $O/bench.log 2>&1 || exit 1
