# persistent GEMM v13: bitwise tests vs v10, microbench on 70B shapes, 70B bench A/B (v10 vs v13)
set -o pipefail
mkdir -p gpurun_out/r67
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/r67/pytest_gemm.log 2>&1
rc=$?; echo "pytest gemm rc=$rc"; tail -2 gpurun_out/r67/pytest_gemm.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/kernel_bench.py > gpurun_out/r67/kbench.log 2>&1
rc=$?; echo "kbench rc=$rc"; grep '"op"' gpurun_out/r67/kbench.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
FLS_GEMM_VARIANT=13 timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/r67/bench70b_v13.log 2>&1
rc=$?; echo "bench70b v13 rc=$rc"; grep -o '"value": [0-9.]*\|"scores_finite": [a-z]*' gpurun_out/r67/bench70b_v13.log | tr '\n' ' '; echo
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/r67/bench70b_v10.log 2>&1
rc=$?; echo "bench70b v10 rc=$rc"; grep -o '"value": [0-9.]*\|"scores_finite": [a-z]*' gpurun_out/r67/bench70b_v10.log | tr '\n' ' '; echo
exit $rc
