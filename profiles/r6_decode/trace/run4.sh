# where an 8-prompt exact generation step idles (1.7-2 ms per step in trace/final): gaps of the last pass
set -o pipefail
O=gpurun_out/${1:-r6_decode_gaps}
R=$(pwd)
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace -d $R/$O/p8 -o run -- python3 $R/scripts/gen_exact_probe.py --prompts 8 --gen 6 --only reuse > $R/$O/p8.log 2>&1 || exit 1
cd $R
db=$(ls $O/p8/*/run_results.db 2>/dev/null | head -1); [ -z "$db" ] && db=$O/p8/run_results.db
python3 scripts/rocpd_gaps.py $db --embeds-per-pass 1 --top 20 > $O/gaps.txt 2>&1 || exit 1
rm -f $db
