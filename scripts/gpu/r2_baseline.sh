# Round 2 baseline on the restored tree: GPU tests, then the driver's bench (70B lnps=1 storage=cpu).
set -o pipefail
mkdir -p gpurun_out/r2_base
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_base/gputest.log 2>&1
echo "gputest rc=$? $(tail -1 gpurun_out/r2_base/gputest.log)"
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > gpurun_out/r2_base/bench.log 2>&1
echo "bench rc=$? $(grep -o '"value": [0-9.]*' gpurun_out/r2_base/bench.log)"
free -g > gpurun_out/r2_base/free.txt; df -h /tmp . > gpurun_out/r2_base/df.txt; nproc >> gpurun_out/r2_base/free.txt
