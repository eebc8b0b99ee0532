# GEMM attribution (PMC) + O-projection order / row-chunk sweep + config rows + headline trace
set -o pipefail
O=gpurun_out/r4_next
mkdir -p $O
timeout -k 10 240 python -u scripts/mem_probe.py > $O/mem_probe.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/gemm_v11_ab.py --only o_resid --orders 0,-8,4,7,14 --rows 0,21504 --rounds 3 > $O/o_sweep.log 2>&1 || exit 1
timeout -k 10 400 bash scripts/pmc_r4.sh > $O/pmc_run.log 2>&1 || exit 1
timeout -k 10 900 bash scripts/gpu_r4_configs.sh r4_configs > $O/configs_run.log 2>&1 || exit 1
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $R/$O/trace_bench.log 2>&1 || exit 1
cd $R
db=$(ls $O/trace/*/run_results.db 2>/dev/null | head -1); [ -z "$db" ] && db=$(ls $O/trace/run_results.db | head -1)
python3 scripts/rocpd_summary.py $db --json $O/trace_passes.json > $O/trace_summary.txt 2>&1 || exit 1
rm -f $db
