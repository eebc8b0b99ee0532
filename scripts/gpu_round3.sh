# round-1 GPU session 3: kernel microbench, 70B bench (cpu + gpu storage)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python scripts/kernel_bench.py --json gpurun_out/kernel_bench3.json > gpurun_out/kernel_bench3.log 2>&1
rc=$?; echo "kbench rc=$rc"; cat gpurun_out/kernel_bench3.log | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 2 --warmup 1 > gpurun_out/bench70b_cpu3.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -E "step|metric" gpurun_out/bench70b_cpu3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --storage gpu > gpurun_out/bench70b_gpu3.log 2>&1
rc=$?; echo "bench gpu rc=$rc"; grep -E "step|metric" gpurun_out/bench70b_gpu3.log
