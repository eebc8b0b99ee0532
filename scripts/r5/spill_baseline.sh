# round-5 starting point (HEAD of round 4) on one box: headline vs the spill regimes of VERDICT r4 #1
set -o pipefail
O=gpurun_out/${1:-r5_spill_base}
mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 > $O/headline.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --prompts-per-gpu 128 > $O/p128.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --token-budget 16384 > $O/tb16k.log 2>&1 || exit 1
