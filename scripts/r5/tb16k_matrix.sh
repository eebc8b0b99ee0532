# --token-budget 16384 (3 micro-batches, one parked in host RAM per layer): where the capped run
# loses against the uncapped one, same box — piece pool off, a looser cap, two weight slots uncapped
set -o pipefail
O=gpurun_out/${1:-r5_tb16k}
mkdir -p $O
B="python -u bench.py --steps 3 --warmup 1 --token-budget 16384"
timeout -k 10 300 $B > $O/capped.log 2>&1 || exit 1
FLS_PIECE_POOL=0 timeout -k 10 300 $B > $O/capped_nopool.log 2>&1 || exit 1
timeout -k 10 300 $B --max-vram-gb 7 > $O/capped7.log 2>&1 || exit 1
timeout -k 10 300 $B --max-vram-gb 0 > $O/uncapped.log 2>&1 || exit 1
timeout -k 10 300 $B --max-vram-gb 0 --slots 2 > $O/uncapped_2slots.log 2>&1 || exit 1
FLS_QKV_FOLD=0 timeout -k 10 300 $B > $O/capped_nofold.log 2>&1 || exit 1
