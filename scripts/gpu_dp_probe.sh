set -o pipefail
O=gpurun_out/${1:-r3_dpprobe}
mkdir -p $O
timeout -k 10 200 python -u scripts/dp_loopback_probe.py 2 > $O/probe2.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_multigpu_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
