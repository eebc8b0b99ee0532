# final tree (FLOP-count fix on the graphed path): whole GPU suite, smoke
set -o pipefail
O=gpurun_out/${1:-r6_final4}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
