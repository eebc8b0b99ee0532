# bias epilogues (Qwen2) + full GPU suite + headline bench sanity
set -o pipefail
mkdir -p gpurun_out/r31
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > gpurun_out/r31/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r31/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --steps 3 --warmup 1 > gpurun_out/r31/bench70b.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -E "metric" gpurun_out/r31/bench70b.log | cut -c1-200
