# final tree after the 8-wave mid blocks and the one-wave-per-row statistic: whole GPU suite, smoke,
# the driver's bench command, generation probes
set -o pipefail
O=gpurun_out/${1:-r6_final2}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit 1
timeout -k 10 600 python -u scripts/gen_exact_probe.py --prompts 32 --gen 6 --fast --json $O/probe32.json > $O/probe32.log 2>&1 || exit 1
timeout -k 10 600 python -u scripts/gen_exact_probe.py --prompts 8 --gen 6 --fast --json $O/probe8.json > $O/probe8.log 2>&1 || exit 1
