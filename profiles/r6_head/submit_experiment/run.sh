# pipelined calls (ShardedRunner.submit in bench.py): engine tests, a kernel trace (is the call-boundary
# gap gone?), then the driver command
set -o pipefail
O=gpurun_out/${1:-r6_submit}
R=$(pwd)
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 300 --timeout-method thread > $O/engine_tests.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/head -o run -- python3 $R/bench.py --steps 3 --warmup 1 > $R/$O/head.log 2>&1 || exit 1
cd $R
db=$(ls $O/head/*/run_results.db 2>/dev/null | head -1); [ -z "$db" ] && db=$(ls $O/head/run_results.db | head -1)
python3 scripts/rocpd_summary.py $db --embeds-per-pass 1 --json $O/head_passes.json > $O/head_summary.txt 2>&1 || exit 1
python3 scripts/rocpd_gaps.py $db --embeds-per-pass 1 --top 10 > $O/head_gaps.txt 2>&1 || exit 1
rm -f $db
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.log 2>&1 || exit 1
