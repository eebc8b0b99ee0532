# canonical rocprof of the flagship (L8) with SDMA copies kept under the profiler
set -o pipefail
mkdir -p gpurun_out/r30
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_SDMA=1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r30/prof_l8 -o run -- python bench.py --steps 2 --warmup 1 --num-layers 8 > gpurun_out/r30/prof_l8.log 2>&1
echo "rocprof rc=$?"; grep metric gpurun_out/r30/prof_l8.log | cut -c1-200
