set -o pipefail
O=gpurun_out/r4_moebench
mkdir -p $O
timeout -k 10 400 python -u bench.py --model qwen1.5-moe-a2.7b --steps 4 --warmup 2 > $O/streamed.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --model qwen1.5-moe-a2.7b --steps 4 --warmup 2 --resident --storage gpu > $O/resident.log 2>&1 || exit 1
