set -o pipefail
O=gpurun_out/${1:-r4_bench}
mkdir -p $O
timeout -k 10 400 python -u bench.py --gpus 1 --steps 8 --warmup 2 > $O/bench.log 2>&1 || exit 1
