# piece pool (default) vs whole-layer slots (FLS_PIECE_POOL=0) under the 6 GB cap, same box:
# headline, 128 prompts, 16k token budget
set -o pipefail
O=gpurun_out/${1:-r5_pool_ab}
mkdir -p $O
B="python -u bench.py --steps 3 --warmup 1"
for cfg in "head:" "p128:--prompts-per-gpu 128 --steps 2" "tb16k:--token-budget 16384"; do
  n=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 500 $B $args > $O/${n}_pool.log 2>&1 || exit 1
  FLS_PIECE_POOL=0 timeout -k 10 500 $B $args > $O/${n}_slots.log 2>&1 || exit 1
done
