# Round 2: main.py end to end on the GPU vs the CPU backend (new GPU test), plus the engine GPU tests.
set -o pipefail
O=gpurun_out/r2_clitest
mkdir -p $O
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 300 --timeout-method thread > $O/engine_gpu.log 2>&1
rc=$?; echo "engine gpu tests rc=$rc $(tail -1 $O/engine_gpu.log)"; [ $rc -eq 0 ] || exit 1
