# v13 with counted vmcnt at the tile seam (buffer-store epilogues): GEMM tests, then v10 vs v13 A/B.
set -o pipefail
O=gpurun_out/r2_v13cnt
mkdir -p $O
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_production_gpu.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/test.log)"; [ $rc -eq 0 ] || { tail -30 $O/test.log; exit 1; }
timeout -k 10 300 python -u scripts/gemm_v13_ab.py --m 14336 --iters 10 > $O/ab.log 2>&1
echo "ab rc=$?"; grep -v amdgpu.ids $O/ab.log
