# interleaved same-box A/B of the headline bench: HEAD vs the round-3 tree (f22a617, checked out
# in ab_r3/ by `git worktree add ab_r3 f22a617` and built in place) on the driver's command
set -o pipefail
O=gpurun_out/${1:-r5_ab_r3}
R=$(pwd)
mkdir -p $O
for i in 1 2; do
  (cd ab_r3 && timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 > $R/$O/r3_$i.log 2>&1) || exit 1
  timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 > $O/head_$i.log 2>&1 || exit 1
done
