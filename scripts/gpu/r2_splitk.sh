# Split-K tail: GEMM tests, then on/off A/B on the 70B shapes at the bench's micro-batch sizes.
set -o pipefail
O=gpurun_out/r2_splitk
mkdir -p $O
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_production_gpu.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/test.log)"; [ $rc -eq 0 ] || { tail -30 $O/test.log; exit 1; }
timeout -k 10 400 python -u scripts/gemm_splitk_ab.py --ms 16128,10752 --iters 10 > $O/ab.log 2>&1
echo "ab rc=$?"; grep -v amdgpu.ids $O/ab.log
