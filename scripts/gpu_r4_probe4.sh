mkdir -p gpurun_out/r4_probe4 && PROBE_CALLS=3 timeout -k 10 300 python -u scripts/mem_probe.py > gpurun_out/r4_probe4/mem_probe.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "skinny" --timeout 150 --timeout-method thread > gpurun_out/r4_probe4/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/gemm_skinny_ab.py --ms 64,160 --blocks 256 > gpurun_out/r4_probe4/skinny_ab.log 2>&1
