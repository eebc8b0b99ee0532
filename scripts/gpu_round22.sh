# v8 GEMM (read-ahead phases): variant tests + kernel bench
set -o pipefail
mkdir -p gpurun_out/r22
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "variants or plain or asym" > gpurun_out/r22/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r22/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/kernel_bench.py --json gpurun_out/r22/kernel_bench.json > gpurun_out/r22/kernel_bench.log 2>&1
rc=$?; echo "kbench rc=$rc"; grep -v amdgpu.ids gpurun_out/r22/kernel_bench.log | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print({k:(round(v,1) if isinstance(v,float) else v) for k,v in d.items() if 'tflops' in k or k in ('op',)})"
