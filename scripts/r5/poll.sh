# run-ahead waits by polling vs hipEventSynchronize, balanced micro-batches: 128 prompts and a 16k
# budget under the cap, same box
set -o pipefail
O=gpurun_out/${1:-r5_poll}
mkdir -p $O
B="python -u bench.py --warmup 1"
FLS_RUNAHEAD_ITEMS=6 FLS_RUNAHEAD_POLL=1 timeout -k 10 500 $B --steps 2 --prompts-per-gpu 128 > $O/p128_ra6_poll.log 2>&1 || exit 1
FLS_RUNAHEAD_ITEMS=0 timeout -k 10 500 $B --steps 2 --prompts-per-gpu 128 > $O/p128_ra0.log 2>&1 || exit 1
FLS_RUNAHEAD_ITEMS=6 FLS_RUNAHEAD_POLL=1 timeout -k 10 300 $B --steps 3 --token-budget 16384 > $O/tb16k_ra6_poll.log 2>&1 || exit 1
FLS_RUNAHEAD_ITEMS=0 FLS_RUNAHEAD_POLL=1 timeout -k 10 300 $B --steps 3 --token-budget 16384 > $O/tb16k_ra0_poll.log 2>&1 || exit 1
