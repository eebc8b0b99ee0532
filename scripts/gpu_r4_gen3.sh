mkdir -p gpurun_out/r4_probe3 && PROBE_CALLS=4 timeout -k 10 300 python -u scripts/mem_probe.py > gpurun_out/r4_probe3/mem_probe.log 2>&1 || exit 1
timeout -k 10 1000 bash scripts/gpu_r4_gen.sh r4_gen3 || exit 1
