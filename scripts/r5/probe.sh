# per-layer GPU timeline (CUDA events, no profiler): piece pool vs whole-layer slots at a 16k token
# budget under the 6 GB cap, and the pool at the headline
set -o pipefail
O=gpurun_out/${1:-r5_probe}
mkdir -p $O
timeout -k 10 300 python -u scripts/layer_timing_probe.py --token-budget 16384 > $O/pool_tb16k.txt 2>&1 || exit 1
FLS_PIECE_POOL=0 timeout -k 10 300 python -u scripts/layer_timing_probe.py --token-budget 16384 > $O/slots_tb16k.txt 2>&1 || exit 1
timeout -k 10 300 python -u scripts/layer_timing_probe.py > $O/pool_head.txt 2>&1 || exit 1
