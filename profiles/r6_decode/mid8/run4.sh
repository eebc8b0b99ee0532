# 8-wave mid-M blocks (final dispatch): the whole GPU suite, smoke, decode GEMM A/B, generation probes
# (8 / 32 / 64 prompts, exact reuse and --exact_reuse false), headline bench
set -o pipefail
O=gpurun_out/${1:-r6_mid8_final}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/decode_gemm_bench.py --rows 16,64,160,320 > $O/gemm_bench.log 2>&1 || exit 1
timeout -k 10 600 python -u scripts/gen_exact_probe.py --prompts 32 --gen 6 --fast --json $O/probe32.json > $O/probe32.log 2>&1 || exit 1
timeout -k 10 600 python -u scripts/gen_exact_probe.py --prompts 8 --gen 6 --fast --json $O/probe8.json > $O/probe8.log 2>&1 || exit 1
timeout -k 10 600 python -u scripts/gen_exact_probe.py --prompts 64 --gen 6 --fast --json $O/probe64.json > $O/probe64.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > $O/bench.log 2>&1 || exit 1
