# 16-wave row statistic + 8-wave mid blocks: bitwise kernel / engine tests, then the kernel trace of
# 32-prompt exact-reuse steps (per-step breakdown)
set -o pipefail
O=gpurun_out/${1:-r6_decode_trace2}
R=$(pwd)
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "row_ss or row_stat or small_m or row_rstd" > $O/kernel_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 300 --timeout-method thread > $O/engine_tests.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/$O/exact -o run -- python3 $R/scripts/gen_exact_probe.py --prompts 32 --gen 6 --only reuse --json $R/$O/exact.json > $R/$O/exact.log 2>&1 || exit 1
cd $R
db=$(ls $O/exact/*/run_results.db 2>/dev/null | head -1); [ -z "$db" ] && db=$O/exact/run_results.db
python3 scripts/rocpd_summary.py $db --json $O/exact_summary.json > $O/exact_summary.txt 2>&1 || exit 1
rm -f $db
