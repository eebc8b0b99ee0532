# shape-based v10 tile order: GEMM tests, then same-box A/B of the 70B / 7B benches (FLS_GEMM_ORDER=8 = old order)
set -o pipefail
mkdir -p gpurun_out/r60
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/r60/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r60/pytest.log
[ $rc -eq 0 ] || exit $rc
for o in 0 8 0 8; do
  FLS_GEMM_ORDER=$o timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/r60/bench70b_o$o.log 2>&1
  rc=$?; echo "70b order=$o rc=$rc"; grep -o '"value": [0-9.]*' gpurun_out/r60/bench70b_o$o.log
  [ $rc -eq 0 ] || exit $rc
done
for o in 0 8; do
  FLS_GEMM_ORDER=$o timeout -k 10 300 python bench.py --model llama2-7b --lnps 8 --storage gpu --steps 5 --warmup 1 > gpurun_out/r60/bench7b_o$o.log 2>&1
  rc=$?; echo "7b order=$o rc=$rc"; grep -o '"value": [0-9.]*' gpurun_out/r60/bench7b_o$o.log
  [ $rc -eq 0 ] || exit $rc
done
