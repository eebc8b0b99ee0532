# mid-M GEMM kernel: numerics, microbench vs main kernel / hipBLASLt, small 7B resident run (graphs on/off)
set -o pipefail
mkdir -p gpurun_out/r48
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/r48/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r48/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/gemm_mid_bench.py --json gpurun_out/r48/gemm_mid.json > gpurun_out/r48/gemm_mid.log 2>&1
rc=$?; echo "midbench rc=$rc"; grep -v amdgpu gpurun_out/r48/gemm_mid.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['shape'], d['M'], 'mid', d['mid_us'], 'main', d['main_us'], 'blt', d['hipblaslt_us'], 'TF', d['tflops_mid'])"
[ $rc -eq 0 ] || exit $rc
for g in "" "--hip-graphs"; do
timeout -k 10 300 python bench.py --model llama2-7b --resident --storage gpu --prompts-per-gpu 4 --prefix-len 64 --suffix-len 8 --steps 10 --warmup 2 $g > gpurun_out/r48/bench7b_small$g.log 2>&1
rc=$?; echo "bench7b small $g rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r48/bench7b_small$g.log | tr '\n' ' '; echo
[ $rc -eq 0 ] || exit $rc
done
