set -o pipefail
mkdir -p gpurun_out/r5_copy
timeout -k 10 120 python -u scripts/copy_concurrency_probe.py > gpurun_out/r5_copy/probe2.log 2>&1 || exit 1
bash scripts/r5/poll.sh r5_poll
