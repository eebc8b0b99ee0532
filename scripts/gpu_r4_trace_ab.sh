# rocprofv3 kernel traces of the headline pass: round-3 GEMM path (v10) vs v11, same box
set -o pipefail
O=gpurun_out/${1:-r4_trace_ab}
mkdir -p $O
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
FLS_GEMM_V11=0 FLS_CHUNK_ALIGN=256 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/v10 -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $R/$O/v10.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/v11 -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $R/$O/v11.log 2>&1 || exit 1
cd $R
for v in v10 v11; do
  db=$(ls $O/$v/*/run_results.db 2>/dev/null | head -1); [ -z "$db" ] && db=$(ls $O/$v/run_results.db | head -1)
  python3 scripts/rocpd_summary.py $db --json $O/${v}_passes.json > $O/${v}_summary.txt 2>&1 || exit 1
  rm -f $db
done
