# runtime tile order + buffer-form LDS-DMA: GEMM tests, per-shape bench vs hipBLASLt
set -o pipefail
O=gpurun_out/r2_order
mkdir -p $O
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_production_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/test.log)"; [ $rc -eq 0 ] || { tail -30 $O/test.log; exit 1; }
timeout -k 10 300 python -u scripts/kernel_bench.py --m 14336 --iters 20 --json $O/kernel_bench.json > $O/kernel_bench.log 2>&1
echo "kernel_bench rc=$?"; grep -v amdgpu.ids $O/kernel_bench.log | cut -c1-330 | head -5
