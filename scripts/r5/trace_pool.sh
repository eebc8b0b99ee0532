# --token-budget 16384 under the 6 GB cap: piece pool (default) vs whole-layer slots
# (FLS_PIECE_POOL=0), kernel traces with per-pass GPU busy / idle
set -o pipefail
O=gpurun_out/${1:-r5_trace_pool}
R=$(pwd)
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $R/$O/pool -o run -- python3 $R/bench.py --steps 2 --warmup 1 --token-budget 16384 > $R/$O/pool.log 2>&1 || exit 1
FLS_PIECE_POOL=0 timeout -k 10 400 rocprofv3 --kernel-trace -d $R/$O/slots -o run -- python3 $R/bench.py --steps 2 --warmup 1 --token-budget 16384 > $R/$O/slots.log 2>&1 || exit 1
cd $R
for n in pool slots; do
  db=$(ls $O/$n/*/run_results.db 2>/dev/null | head -1); [ -z "$db" ] && db=$(ls $O/$n/run_results.db | head -1)
  python3 scripts/rocpd_summary.py $db --embeds-per-pass 3 --json $O/${n}_passes.json > $O/${n}_summary.txt 2>&1 || exit 1
  cp $db /tmp/$n.db && rm -f $db
done
python3 scripts/rocpd_gaps.py /tmp/pool.db > $O/pool_gaps.txt 2>&1 || true
python3 scripts/rocpd_gaps.py /tmp/slots.db > $O/slots_gaps.txt 2>&1 || true
