# --token-budget 16384 under the cap, piece pool: does the MLP chunk (whole 14-15k-row micro-batch
# vs the slot plan's 9,216) explain the gap to whole-layer slots?  Same box as a slots run.
set -o pipefail
O=gpurun_out/${1:-r5_tb16k_chunk}
mkdir -p $O
B="python -u bench.py --steps 3 --warmup 1 --token-budget 16384"
timeout -k 10 300 $B --mlp-chunk 9216 > $O/pool_mc9216.log 2>&1 || exit 1
timeout -k 10 300 $B --mlp-chunk 12288 > $O/pool_mc12288.log 2>&1 || exit 1
timeout -k 10 300 $B > $O/pool.log 2>&1 || exit 1
FLS_PIECE_POOL=0 timeout -k 10 300 $B > $O/slots.log 2>&1 || exit 1
