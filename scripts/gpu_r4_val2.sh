# final round-4 validation: full GPU suite, smoke, default bench
set -o pipefail
O=gpurun_out/${1:-r4_val5}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > $O/bench.log 2>&1 || exit 1
