# closing validation of the round-5 tree: GPU tests, smoke, headline, spill regimes, envelope, trace
set -o pipefail
O=gpurun_out/r5_final
R=$(pwd)
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
B="python -u bench.py --warmup 1"
timeout -k 10 300 $B --steps 4 > $O/head.log 2>&1 || exit 1
timeout -k 10 500 $B --steps 2 --prompts-per-gpu 128 > $O/p128.log 2>&1 || exit 1
timeout -k 10 300 $B --steps 3 --token-budget 16384 > $O/tb16k.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $R/$O/trace.log 2>&1 || exit 1
cd $R
db=$(ls $O/trace/*/run_results.db 2>/dev/null | head -1); [ -z "$db" ] && db=$(ls $O/trace/run_results.db | head -1)
python3 scripts/rocpd_summary.py $db --json $O/trace_passes.json > $O/trace_summary.txt 2>&1 || exit 1
rm -f $db
