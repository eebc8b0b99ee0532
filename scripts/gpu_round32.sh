# v12 (32x32x16 MFMA): variant tests, kernel bench, ablation vs v10
set -o pipefail
mkdir -p gpurun_out/r32
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "variants or plain or asym or resid or bias" > gpurun_out/r32/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r32/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/kernel_bench.py --json gpurun_out/r32/kernel_bench.json > gpurun_out/r32/kernel_bench.log 2>&1
rc=$?; echo "kbench rc=$rc"; grep -v amdgpu.ids gpurun_out/r32/kernel_bench.log | head -5 | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print({k:(round(v,1) if isinstance(v,float) else v) for k,v in d.items() if 'tflops' in k or k in ('op',)})"
[ $rc -eq 0 ] || exit $rc
ABL_ONLY=70 timeout -k 10 400 python scripts/gemm_ablate.py > gpurun_out/r32/ablate.json 2>&1
rc=$?; echo "abl rc=$rc"; grep -v amdgpu.ids gpurun_out/r32/ablate.json | python -c "
import json,sys; d=json.load(sys.stdin); print({k:v['tflops_equiv'] for k,v in d.items()})"
