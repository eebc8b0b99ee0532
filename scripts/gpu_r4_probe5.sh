mkdir -p gpurun_out/r4_probe5 && PROBE_CALLS=3 timeout -k 10 300 python -u scripts/mem_probe.py > gpurun_out/r4_probe5/mem_probe.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 4 --warmup 2 > gpurun_out/r4_probe5/bench.log 2>&1 || exit 1
