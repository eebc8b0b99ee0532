# v7 GEMM (counted-vmcnt 4-phase pipeline): tests, kernel bench, 70B bench
set -o pipefail
mkdir -p gpurun_out/r13
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > gpurun_out/r13/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r13/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/kernel_bench.py --json gpurun_out/r13/kernel_bench.json > gpurun_out/r13/kernel_bench.log 2>&1
rc=$?; echo "kbench rc=$rc"; cut -c1-400 gpurun_out/r13/kernel_bench.log
[ $rc -eq 0 ] || exit $rc
FLS_GEMM_VARIANT=7 FLS_GEMM_BACKEND=hip timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/r13/bench70b_hip7.log 2>&1
rc=$?; echo "bench hip7 rc=$rc"; grep -E "metric" gpurun_out/r13/bench70b_hip7.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
FLS_GEMM_VARIANT=7 timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/r13/bench70b_auto7.log 2>&1
rc=$?; echo "bench auto7 rc=$rc"; grep -E "metric" gpurun_out/r13/bench70b_auto7.log | cut -c1-300
