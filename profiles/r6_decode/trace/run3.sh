# final tree: kernel traces of exact-reuse generation steps, 8 and 32 prompts (per-step breakdown)
set -o pipefail
O=gpurun_out/${1:-r6_decode_trace3}
R=$(pwd)
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for n in 8 32; do
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/$O/p$n -o run -- python3 $R/scripts/gen_exact_probe.py --prompts $n --gen 6 --only reuse > $R/$O/p$n.log 2>&1 || exit 1
done
cd $R
for n in 8 32; do
  db=$(ls $O/p$n/*/run_results.db 2>/dev/null | head -1); [ -z "$db" ] && db=$O/p$n/run_results.db
  python3 scripts/rocpd_summary.py $db --json $O/p${n}_summary.json > $O/p${n}_summary.txt 2>&1 || exit 1
  rm -f $db
done
