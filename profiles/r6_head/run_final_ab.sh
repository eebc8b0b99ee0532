# final headline A/B on one box: HEAD vs the round-5 tree (41fb1fc, ab_r5/), interleaved, driver
# command shape (steps 20 would be 90 s each: 10 here); --norm-fold on_landing and --no-prune-last
# rates; kernel trace + gaps of HEAD; envelope (O_DIRECT streamed, 128 prompts, 6 GB cap, 5 steps)
set -o pipefail
O=gpurun_out/${1:-r6_final}
R=$(pwd)
mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench_head_$i.log 2>&1 || exit 1
  (cd ab_r5 && timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $R/$O/bench_r5_$i.log 2>&1) || exit 1
done
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --norm-fold on_landing > $O/bench_onland.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-prune-last > $O/bench_noprune.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/head -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $R/$O/head.log 2>&1 || exit 1
cd $R
db=$(ls $O/head/*/run_results.db 2>/dev/null | head -1); [ -z "$db" ] && db=$(ls $O/head/run_results.db | head -1)
python3 scripts/rocpd_summary.py $db --embeds-per-pass 1 --json $O/head_passes.json > $O/head_summary.txt 2>&1 || exit 1
python3 scripts/rocpd_gaps.py $db --embeds-per-pass 1 --top 30 > $O/head_gaps.txt 2>&1 || exit 1
rm -f $db
