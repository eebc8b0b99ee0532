# data-parallel fan-out interference on one GPU: the headline pass with, after every weight piece,
# 7/8 of its bytes copied HBM -> HBM on the copy stream (the G = 8 all-gather's per-rank traffic), on
# the CUs (HIP blit kernel; a 32-workgroup kernel like RCCL's channels) and on the SDMA engines
set -o pipefail
O=gpurun_out/${1:-r6_dpi}
mkdir -p $O
for i in 1 2; do
  for m in none cu32 sdma blit; do
    timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --max-vram-gb 6.3 --emulate-dp-fanout $m > $O/bench_${m}_$i.log 2>&1 || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
for m in cu32 sdma; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OLDPWD/$O/tr_$m -o run -- python3 $OLDPWD/bench.py --steps 2 --warmup 1 --max-vram-gb 6.3 --emulate-dp-fanout $m > $OLDPWD/$O/tr_$m.log 2>&1 || exit 1
done
cd $OLDPWD
for m in cu32 sdma; do
  db=$(ls $O/tr_$m/*/run_results.db 2>/dev/null | head -1); [ -z "$db" ] && db=$(ls $O/tr_$m/run_results.db | head -1)
  python3 scripts/rocpd_summary.py $db --embeds-per-pass 1 > $O/tr_${m}_summary.txt 2>&1 || exit 1
  rm -f $db
done
