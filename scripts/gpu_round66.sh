# 128-row attention items for multi-head models: numerics, microbench, 7B bench
set -o pipefail
mkdir -p gpurun_out/r66
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/r66/pytest_attn.log 2>&1
rc=$?; echo "pytest attn rc=$rc"; tail -2 gpurun_out/r66/pytest_attn.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/attn_mha.py > gpurun_out/r66/attn_mha.log 2>&1
rc=$?; echo "mha rc=$rc"; grep "^{" gpurun_out/r66/attn_mha.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r66/pytest.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -2 gpurun_out/r66/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model llama2-7b --lnps 8 --storage gpu --steps 5 --warmup 1 > gpurun_out/r66/bench7b.log 2>&1
rc=$?; echo "bench7b rc=$rc"; grep -o '"value": [0-9.]*\|"scores_finite": [a-z]*' gpurun_out/r66/bench7b.log | tr '\n' ' '; echo
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/r66/bench70b.log 2>&1
rc=$?; echo "bench70b rc=$rc"; grep -o '"value": [0-9.]*\|"scores_finite": [a-z]*' gpurun_out/r66/bench70b.log | tr '\n' ' '; echo
exit $rc
