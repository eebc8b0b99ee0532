# same-box config rows: headline (capped streamed), resident (config 5 per GPU), spill (storage=cpu with
# a token budget below the call's tokens: activations parked in pinned host RAM between layers)
set -o pipefail
O=gpurun_out/${1:-r4_configs}
mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 > $O/streamed_capped.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 4 --warmup 2 --resident --storage gpu > $O/resident.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --token-budget 16384 > $O/spill_tb16k.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 > $O/streamed_capped_2.log 2>&1 || exit 1
