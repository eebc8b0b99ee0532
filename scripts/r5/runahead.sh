# host run-ahead bound (FLS_RUNAHEAD_ITEMS: 0 = two shards only, n = also n micro-batch computes):
# 128 prompts and a 16k token budget under the 6 GB cap, same box
set -o pipefail
O=gpurun_out/${1:-r5_runahead}
mkdir -p $O
B="python -u bench.py --warmup 1"
for n in 6 0 12; do
  FLS_RUNAHEAD_ITEMS=$n timeout -k 10 500 $B --steps 2 --prompts-per-gpu 128 > $O/p128_ra$n.log 2>&1 || exit 1
done
for n in 0 12; do
  FLS_RUNAHEAD_ITEMS=$n timeout -k 10 300 $B --steps 3 --token-budget 16384 > $O/tb16k_ra$n.log 2>&1 || exit 1
done
