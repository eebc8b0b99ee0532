mkdir -p gpurun_out/r4_copy && timeout -k 10 200 python -u scripts/copy_probe.py > gpurun_out/r4_copy/copy_probe.log 2>&1
