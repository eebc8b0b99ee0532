# final tree (all mid-block variants): whole GPU suite, smoke, default bench, probes 8 / 32 / 64
set -o pipefail
O=gpurun_out/${1:-r6_final3}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || exit 1
for n in 8 32 64; do timeout -k 10 600 python -u scripts/gen_exact_probe.py --prompts $n --gen 6 --fast --json $O/probe$n.json > $O/probe$n.log 2>&1 || exit 1; done
