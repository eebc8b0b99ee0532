# Kernel + memory-copy timeline of the default 70B bench (2 timed steps): GPU idle gaps per step.
set -o pipefail
O=gpurun_out/r2_trace
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
FLS_SPECULATIVE_PREFETCH=${SPEC:-0} timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$O/tr" -o bench -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 > "$GRAFT_REPO_ROOT/$O/bench.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit 1
cd "$GRAFT_REPO_ROOT" && python3 scripts/trace_gaps.py $O/tr > $O/gaps.txt 2>&1; echo "gaps rc=$?"; tail -70 $O/gaps.txt
