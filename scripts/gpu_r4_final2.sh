# Round-4 closing validation: full GPU suite, smoke, the default (headline) bench, and a Granite-3-8B
# bench row (synthetic weights, lnps 1, storage cpu).
set -o pipefail
O=gpurun_out/${1:-r4_final2}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > $O/bench.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --model granite-3-8b --steps 4 --warmup 2 > $O/bench_granite8b.log 2>&1 || exit 1
