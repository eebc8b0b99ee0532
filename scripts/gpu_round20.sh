# gemv + full GPU tests + kernel bench + copy/GEMM interference
set -o pipefail
mkdir -p gpurun_out/r20
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > gpurun_out/r20/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r20/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/kernel_bench.py --json gpurun_out/r20/kernel_bench.json > gpurun_out/r20/kernel_bench.log 2>&1
rc=$?; echo "kbench rc=$rc"; grep -E "gemv|attention" gpurun_out/r20/kernel_bench.log
[ $rc -eq 0 ] || exit $rc
CO_JSON=gpurun_out/r20/copy_overlap.json timeout -k 10 900 python scripts/copy_overlap.py > gpurun_out/r20/copy_overlap.log 2>&1
rc=$?; echo "overlap rc=$rc"; cut -c1-400 gpurun_out/r20/copy_overlap.log
