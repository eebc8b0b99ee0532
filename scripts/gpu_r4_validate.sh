# round-4 tree: full GPU suite, smoke, then headline bench A/B (v11 chunk alignment 768 vs 3072)
set -o pipefail
O=gpurun_out/${1:-r4_validate}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
FLS_CHUNK_ALIGN=768 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > $O/bench_a768.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > $O/bench_a3072.log 2>&1 || exit 1
