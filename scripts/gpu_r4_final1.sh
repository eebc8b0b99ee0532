# config rows (streamed capped x2, resident, spill), GEMM PMC counters, headline kernel trace
set -o pipefail
timeout -k 10 1000 bash scripts/gpu_r4_configs.sh r4_configs || exit 1
timeout -k 10 400 bash scripts/pmc_r4.sh > gpurun_out/r4_pmc_run.log 2>&1 || exit 1
O=gpurun_out/r4_trace2
mkdir -p $O
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $R/$O/trace_bench.log 2>&1 || exit 1
cd $R
db=$(ls $O/trace/*/run_results.db 2>/dev/null | head -1); [ -z "$db" ] && db=$(ls $O/trace/run_results.db | head -1)
python3 scripts/rocpd_summary.py $db --json $O/trace_passes.json > $O/trace_summary.txt 2>&1 || exit 1
rm -f $db
