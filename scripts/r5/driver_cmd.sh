# the driver's exact headline command (20 timed steps after 5 warmup) on the final tree
set -o pipefail
O=gpurun_out/r5_driver_cmd
mkdir -p $O
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.log 2>&1 || exit 1
