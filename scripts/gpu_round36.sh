# attention v2 (32 rows/wave, staged prefetch): numerics vs fp32 torch, v1/v2 timing
set -o pipefail
mkdir -p gpurun_out/r36
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "attention" --timeout 120 --timeout-method thread > gpurun_out/r36/pytest_attn.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r36/pytest_attn.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/kernel_bench.py --json gpurun_out/r36/kb.json > gpurun_out/r36/kb.log 2>&1
rc=$?; echo "kb rc=$rc"; grep attention gpurun_out/r36/kb.log
exit $rc
