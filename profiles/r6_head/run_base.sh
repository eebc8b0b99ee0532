# round-6 first box: new tests (decode-graph eviction, residual-GEMM row partial sums), then the
# headline: HEAD (norm fold on landing, no row_rstd pass) vs HEAD --norm-fold prefolded vs the round-5
# tree (41fb1fc, ab_r5/), interleaved on one box; then a kernel trace of HEAD's default
set -o pipefail
O=gpurun_out/${1:-r6_base}
R=$(pwd)
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -x -v --timeout 200 --timeout-method thread -k "decode_graphs or speculative or row_sum_squares" > $O/tests.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > $O/bench_head_$i.log 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --norm-fold prefolded > $O/bench_prefold_$i.log 2>&1 || exit 1
  (cd ab_r5 && timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > $R/$O/bench_r5_$i.log 2>&1) || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/head -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $R/$O/head.log 2>&1 || exit 1
cd $R
db=$(ls $O/head/*/run_results.db 2>/dev/null | head -1); [ -z "$db" ] && db=$(ls $O/head/run_results.db | head -1)
python3 scripts/rocpd_summary.py $db --embeds-per-pass 1 --json $O/head_passes.json > $O/head_summary.txt 2>&1 || exit 1
rm -f $db
