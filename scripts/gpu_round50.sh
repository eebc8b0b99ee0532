# clean kernel breakdown of the 70B layer (resident weights: no H2D blits under the profiler)
set -o pipefail
mkdir -p gpurun_out/r50
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r50/prof -o run -- python bench.py --num-layers 8 --resident --storage gpu --steps 3 --warmup 1 > gpurun_out/r50/bench.log 2>&1
rc=$?; echo "rc=$rc"; tail -1 gpurun_out/r50/bench.log | cut -c1-300
find gpurun_out/r50/prof -name "*kernel_stats.csv" | head -3
