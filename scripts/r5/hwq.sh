# HIP hardware queues (GPU_MAX_HW_QUEUES, 4 on the box): a copy stream that shares an in-order
# hardware queue with the compute stream blocks the compute behind its copies.  --token-budget
# 16384 under the cap (piece pool / whole-layer slots) and the headline at 4 vs 8 queues; then the
# decode attention microbenchmark
set -o pipefail
O=gpurun_out/${1:-r5_hwq}
mkdir -p $O
B="python -u bench.py --steps 3 --warmup 1"
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 $B --token-budget 16384 > $O/tb16k_q8.log 2>&1 || exit 1
timeout -k 10 300 $B --token-budget 16384 > $O/tb16k_q4.log 2>&1 || exit 1
GPU_MAX_HW_QUEUES=8 FLS_PIECE_POOL=0 timeout -k 10 300 $B --token-budget 16384 > $O/tb16k_slots_q8.log 2>&1 || exit 1
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 $B > $O/head_q8.log 2>&1 || exit 1
timeout -k 10 300 $B > $O/head_q4.log 2>&1 || exit 1
timeout -k 10 120 python -u scripts/attn_decode_bench.py > $O/attn_decode.log 2>&1 || exit 1
