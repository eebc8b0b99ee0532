# Kernel + memory-copy timeline of the default 70B bench on the 48k-token micro-batch tree
# (2 timed steps): GPU idle gaps per step and the per-kernel breakdown.
set -o pipefail
O=gpurun_out/r2_trace48k
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/tr" -o bench -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 > "$GRAFT_REPO_ROOT/$O/bench.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit 1
cd "$GRAFT_REPO_ROOT" && python3 scripts/trace_gaps.py $O/tr > $O/gaps.txt 2>&1; echo "gaps rc=$?"; head -40 $O/gaps.txt
find $O/tr -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
find $O/tr -name "*kernel_trace.csv" -size +30M -delete
