# full GPU test suite + smoke on the current tree
set -o pipefail
O=gpurun_out/r4_val
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
