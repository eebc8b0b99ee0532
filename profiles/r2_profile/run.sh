# Round 2: full GPU tests (incl. 70B-geometry numerics), per-shape GEMM study vs hipBLASLt,
# rocprofv3 kernel breakdown of a resident 8-layer 70B bench.
set -o pipefail
O=gpurun_out/r2_profile
mkdir -p $O
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
echo "gputest rc=$? $(tail -1 $O/gputest.log)"
timeout -k 10 300 python -u scripts/kernel_bench.py --m 14336 --iters 20 --json $O/kernel_bench.json > $O/kernel_bench.log 2>&1
echo "kernel_bench rc=$?"; cut -c1-220 $O/kernel_bench.log | head -20
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof" -o bench8 -- python3 "$GRAFT_REPO_ROOT/bench.py" --num-layers 8 --resident --storage gpu --steps 3 --warmup 1 > "$GRAFT_REPO_ROOT/$O/prof_bench.log" 2>&1
echo "rocprof rc=$?"
find "$GRAFT_REPO_ROOT/$O/prof" -name "*kernel_stats.csv" | head -3
