mkdir -p gpurun_out/r4_probe2 && timeout -k 10 300 python -u scripts/mem_probe.py > gpurun_out/r4_probe2/mem_probe.log 2>&1 || exit 1
timeout -k 10 1000 bash scripts/gpu_r4_gen.sh r4_gen2 || exit 1
