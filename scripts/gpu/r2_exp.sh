set -o pipefail
O=gpurun_out/r2_exp
mkdir -p $O
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u scripts/exp/gemm_diag.py 0,1,3,4,5 > $O/diag.log 2>&1
echo "diag rc=$?"; grep -v amdgpu.ids $O/diag.log
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_production_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/test.log)"; [ $rc -eq 0 ] || tail -30 $O/test.log
