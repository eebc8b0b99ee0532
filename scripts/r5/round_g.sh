# host run-ahead bounded per micro-batch compute: the spill regimes and the headline on one box,
# the envelope (pinned RAM / RSS), then the pool's segment trace
set -o pipefail
O=gpurun_out/r5_g
mkdir -p $O
B="python -u bench.py --steps 3 --warmup 1"
timeout -k 10 300 $B > $O/head.log 2>&1 || exit 1
timeout -k 10 500 $B --prompts-per-gpu 128 --steps 2 > $O/p128.log 2>&1 || exit 1
timeout -k 10 300 $B --token-budget 16384 > $O/tb16k.log 2>&1 || exit 1
bash scripts/r5/envelope.sh r5_envelope2 || exit 1
bash scripts/r5/seg_trace.sh r5_seg
