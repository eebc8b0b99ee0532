# pipelined v10 epilogue: GEMM numerics tests, epilogue cost, 70B / 7B benches
set -o pipefail
mkdir -p gpurun_out/r65
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r65/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r65/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/gemm_epi_cost.py > gpurun_out/r65/epi.log 2>&1
rc=$?; echo "epi rc=$rc"; grep "^{" gpurun_out/r65/epi.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/r65/bench70b.log 2>&1
rc=$?; echo "bench70b rc=$rc"; grep -o '"value": [0-9.]*\|"scores_finite": [a-z]*' gpurun_out/r65/bench70b.log | tr '\n' ' '; echo
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model llama2-7b --lnps 8 --storage gpu --steps 5 --warmup 1 > gpurun_out/r65/bench7b.log 2>&1
rc=$?; echo "bench7b rc=$rc"; grep -o '"value": [0-9.]*' gpurun_out/r65/bench7b.log
exit $rc
