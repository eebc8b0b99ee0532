mkdir -p gpurun_out/r4_moe && timeout -k 10 600 python -u -m pytest tests/test_moe_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r4_moe/tests.log 2>&1
