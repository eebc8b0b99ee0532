# kernel trace of 70B generation steps, 32 prompts, weights resident: exact reuse (default) and
# --exact_reuse false; per-step kernel breakdown with scripts/rocpd_summary.py (one embed per step)
set -o pipefail
O=gpurun_out/${1:-r6_decode_trace}
R=$(pwd)
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/$O/exact -o run -- python3 $R/scripts/gen_exact_probe.py --prompts 32 --gen 6 --only reuse --json $R/$O/exact.json > $R/$O/exact.log 2>&1 || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/$O/fast -o run -- python3 $R/scripts/gen_exact_probe.py --prompts 32 --gen 6 --only fast --json $R/$O/fast.json > $R/$O/fast.log 2>&1 || exit 1
cd $R
for arm in exact fast; do
  db=$(ls $O/$arm/*/run_results.db 2>/dev/null | head -1); [ -z "$db" ] && db=$O/$arm/run_results.db
  python3 scripts/rocpd_summary.py $db --json $O/${arm}_summary.json > $O/${arm}_summary.txt 2>&1 || exit 1
  rm -f $db
done
