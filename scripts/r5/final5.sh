# last check of the final tree (kernel ABI 24, resident-ring guard): every GPU test and smoke
set -o pipefail
O=gpurun_out/r5_final5
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 > $O/head.log 2>&1 || exit 1
