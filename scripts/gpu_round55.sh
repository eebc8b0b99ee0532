# DP all-gather weight path on real RCCL (one-rank nccl group)
set -o pipefail
mkdir -p gpurun_out/r55
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v -k "rccl" --timeout 180 --timeout-method thread > gpurun_out/r55/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/r55/pytest.log
exit $rc
