# pinned allocations during timed 128-prompt passes at two run-ahead bounds
set -o pipefail
O=gpurun_out/${1:-r5_allocs}
mkdir -p $O
for n in 0 6; do
  FLS_RUNAHEAD_ITEMS=$n timeout -k 10 500 python -u bench.py --warmup 1 --steps 2 --prompts-per-gpu 128 > $O/p128_ra$n.log 2>&1 || exit 1
done
