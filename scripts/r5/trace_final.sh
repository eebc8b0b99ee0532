# kernel traces of the 70B pass on the final tree: headline (one micro-batch) vs a 16k token budget
# (3 micro-batches, every state resident in its own ring slot), then a disk / RAM probe of the box
set -o pipefail
O=gpurun_out/${1:-r5_trace_final}
R=$(pwd)
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/head -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $R/$O/head.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/tb16k -o run -- python3 $R/bench.py --steps 2 --warmup 1 --token-budget 16384 > $R/$O/tb16k.log 2>&1 || exit 1
cd $R
for n in head tb16k; do
  db=$(ls $O/$n/*/run_results.db 2>/dev/null | head -1); [ -z "$db" ] && db=$(ls $O/$n/run_results.db | head -1)
  e=1; [ $n = tb16k ] && e=3
  python3 scripts/rocpd_summary.py $db --embeds-per-pass $e --json $O/${n}_passes.json > $O/${n}_summary.txt 2>&1 || exit 1
  rm -f $db
done
df -h /tmp $R > $O/disk.txt 2>&1; free -g >> $O/disk.txt 2>&1; nproc >> $O/disk.txt
